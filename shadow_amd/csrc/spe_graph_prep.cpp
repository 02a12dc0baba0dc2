// spe_graph_prep.cpp -- host-side ingest of a topology edge list into the
// device layout used by the gfx950 kernels.  This is boundary code: it
// validates the graph like the reference's topology_new and builds index
// structures (CSR, per-vertex rule constants); it performs no path computation.
//
// Reference behaviour restated here:
//   * validation: latency > 0, 0 <= loss <= 1        shd-topology.c:1026-1109
//   * completeness (_topology_isComplete)             shd-topology.c:435-537
//   * get_eid edge of a vertex pair: igraph keeps each vertex's incidence index
//     sorted by (neighbour asc, edge id desc) and get_eid takes the first match,
//     i.e. the HIGHEST edge id among parallel edges (see oracle/oracle.c header)
//   * SELF rule constants: first incident edge in igraph order with strictly
//     smaller latency; lat = 2.0*min, rel = r*r     shd-topology.c:1567-1626
//   * edge reliability factor 1.0f - p (f64)          shd-topology.c:422, 1582
#include "spe_internal.h"

#include <algorithm>
#include <cmath>
#include <numeric>

namespace spe {

static bool has_attr(double x) { return !std::isnan(x); }

int prepare_graph(const spe_graph_desc* d, HostGraph* hg, std::string* err) {
    if (!d || d->n_vertices <= 0 || d->n_edges < 0 || !d->edge_source || !d->edge_target ||
        !d->edge_latency || !d->edge_packetloss) {
        *err = "spe_graph_create: invalid descriptor";
        return SPE_EINVAL;
    }
    const int32_t n = d->n_vertices;
    const int64_t m = d->n_edges;
    hg->n = n;
    hg->m = m;
    hg->directed = d->directed != 0;
    hg->prefer_direct = d->prefer_direct != 0;

    double wmin = INFINITY, wsum = 0.0;
    for (int64_t e = 0; e < m; ++e) {
        const int32_t a = d->edge_source[e], b = d->edge_target[e];
        const double w = d->edge_latency[e], p = d->edge_packetloss[e];
        if (a < 0 || b < 0 || a >= n || b >= n) {
            *err = "edge " + std::to_string(e) + " has an endpoint out of range";
            return SPE_EINVAL;
        }
        if (!(w > 0.0) || !std::isfinite(w)) {
            *err = "edge " + std::to_string(e) + " latency must be > 0";
            return SPE_EINVAL;
        }
        if (!(p >= 0.0 && p <= 1.0)) {
            *err = "edge " + std::to_string(e) + " packetloss must be in [0,1]";
            return SPE_EINVAL;
        }
        wmin = std::min(wmin, w);
        wsum += w;
    }
    // fl(d + w) > d for every d <= wsum when w > wsum * 2^-53 (round to nearest even)
    hg->weight_floor_ok = (m == 0) || (wmin > std::ldexp(wsum, -52));

    hg->vfac.assign(n, NAN);
    for (int32_t v = 0; v < n; ++v) {
        const double p = d->vertex_packetloss ? d->vertex_packetloss[v] : NAN;
        if (has_attr(p)) hg->vfac[v] = 1.0 - p;
    }

    // ---- directed adjacency entries (from, to, eid), self-loops kept apart
    struct Ent {
        int32_t to, from;
        int64_t eid;
    };
    std::vector<Ent> ents;
    ents.reserve(static_cast<size_t>(hg->directed ? m : 2 * m));
    hg->loop_eid.assign(n, -1);
    for (int64_t e = 0; e < m; ++e) {
        const int32_t a = d->edge_source[e], b = d->edge_target[e];
        if (a == b) {
            if (e > hg->loop_eid[a]) hg->loop_eid[a] = e;  // get_eid(v,v): highest id
            continue;
        }
        ents.push_back({b, a, e});
        if (!hg->directed) ents.push_back({a, b, e});
    }
    hg->loop_w.assign(n, NAN);
    hg->loop_a.assign(n, NAN);
    for (int32_t v = 0; v < n; ++v) {
        const int64_t e = hg->loop_eid[v];
        if (e >= 0) {
            hg->loop_w[v] = d->edge_latency[e];
            hg->loop_a[v] = 1.0 - d->edge_packetloss[e];
        }
    }

    // ---- relaxation in-CSR: by (to, from); parallel edges merged
    std::sort(ents.begin(), ents.end(), [](const Ent& x, const Ent& y) {
        if (x.to != y.to) return x.to < y.to;
        if (x.from != y.from) return x.from < y.from;
        return x.eid > y.eid;  // first = highest id = get_eid's choice
    });
    hg->iptr.assign(static_cast<size_t>(n) + 1, 0);
    hg->icol.clear();
    hg->iw.clear();
    hg->ia.clear();
    hg->iwrep.clear();
    hg->ieid.clear();
    hg->multi_rep = false;
    for (size_t i = 0; i < ents.size();) {
        size_t j = i;
        double wrel = INFINITY;
        while (j < ents.size() && ents[j].to == ents[i].to && ents[j].from == ents[i].from) {
            wrel = std::min(wrel, d->edge_latency[ents[j].eid]);
            ++j;
        }
        const int64_t rep = ents[i].eid;
        const double wrep = d->edge_latency[rep];
        if (wrep != wrel) hg->multi_rep = true;
        hg->icol.push_back(ents[i].from);
        hg->iw.push_back(wrel);
        hg->ia.push_back(1.0 - d->edge_packetloss[rep]);
        hg->iwrep.push_back(wrep);
        hg->ieid.push_back(rep);
        hg->iptr[ents[i].to + 1]++;
        i = j;
    }
    if (hg->icol.size() >= (size_t)INT32_MAX) {
        *err = "graph too large for 32-bit adjacency offsets";
        return SPE_EUNSUPPORTED;
    }
    for (int32_t v = 0; v < n; ++v) hg->iptr[v + 1] += hg->iptr[v];

    // ---- out-CSR (frontier marking + DIRECT lookups): by (from, to)
    if (hg->directed) {
        std::vector<int64_t> idx(hg->icol.size());
        std::vector<int32_t> to_of(hg->icol.size());
        for (int32_t v = 0; v < n; ++v)
            for (int32_t k = hg->iptr[v]; k < hg->iptr[v + 1]; ++k) to_of[k] = v;
        std::iota(idx.begin(), idx.end(), 0);
        std::sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) {
            if (hg->icol[x] != hg->icol[y]) return hg->icol[x] < hg->icol[y];
            return to_of[x] < to_of[y];
        });
        hg->optr.assign(static_cast<size_t>(n) + 1, 0);
        hg->ocol.resize(idx.size());
        hg->orev.resize(idx.size());
        hg->owrep.resize(idx.size());
        hg->ow.resize(idx.size());
        hg->oarep.resize(idx.size());
        for (size_t i = 0; i < idx.size(); ++i) {
            hg->ocol[i] = to_of[idx[i]];
            hg->orev[i] = (int32_t)idx[i];
            hg->owrep[i] = hg->iwrep[idx[i]];
            hg->ow[i] = hg->iw[idx[i]];
            hg->oarep[i] = hg->ia[idx[i]];
            hg->optr[hg->icol[idx[i]] + 1]++;
        }
        for (int32_t v = 0; v < n; ++v) hg->optr[v + 1] += hg->optr[v];
    } else {
        // undirected: one CSR serves both directions; the reverse of entry
        // (x -> y) is the entry of x in y's (sorted) list
        hg->orev.resize(hg->icol.size());
        for (int32_t x = 0; x < n; ++x)
            for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k) {
                const int32_t y = hg->icol[k];
                const int32_t* b = hg->icol.data() + hg->iptr[y];
                const int32_t* e = hg->icol.data() + hg->iptr[y + 1];
                hg->orev[k] = (int32_t)(std::lower_bound(b, e, x) - hg->icol.data());
            }
    }

    // ---- SELF rule constants and completeness, both over incident(v, OUT)
    struct Inc {
        int32_t v, nb;
        int64_t eid;
    };
    std::vector<Inc> inc;
    inc.reserve(static_cast<size_t>(hg->directed ? m : 2 * m));
    std::vector<int64_t> inc_count(n, 0);
    for (int64_t e = 0; e < m; ++e) {
        const int32_t a = d->edge_source[e], b = d->edge_target[e];
        inc.push_back({a, b, e});
        inc_count[a]++;
        if (!hg->directed) {  // undirected: both endpoints (a self-loop twice)
            inc.push_back({b, a, e});
            inc_count[b]++;
        }
    }
    std::sort(inc.begin(), inc.end(), [](const Inc& x, const Inc& y) {
        if (x.v != y.v) return x.v < y.v;
        if (x.nb != y.nb) return x.nb < y.nb;
        return x.eid > y.eid;
    });
    hg->self_w2.assign(n, NAN);
    hg->self_a2.assign(n, NAN);
    hg->self_other.assign(n, -1);
    for (size_t i = 0; i < inc.size();) {
        const int32_t v = inc[i].v;
        double minLatency = 0.0, relMin = 0.0;
        int64_t best = -1;
        for (; i < inc.size() && inc[i].v == v; ++i) {
            const double w = d->edge_latency[inc[i].eid];
            if (minLatency == 0 || w < minLatency) {
                minLatency = w;
                relMin = 1.0 - d->edge_packetloss[inc[i].eid];
                best = inc[i].eid;
            }
        }
        if (best >= 0) {
            hg->self_w2[v] = 2.0 * minLatency;
            hg->self_a2[v] = relMin * relMin;
            const int32_t a = d->edge_source[best], b = d->edge_target[best];
            hg->self_other[v] = (a == v) ? b : a;
        }
    }
    bool complete = true;
    for (int32_t v = 0; v < n && complete; ++v) {
        int64_t cnt = inc_count[v];
        if (!hg->directed && hg->loop_eid[v] >= 0) cnt -= 1;
        if (cnt < n) complete = false;
    }
    hg->complete = complete;
    return SPE_OK;
}

void prune_pendants(HostGraph* hg, bool enable) {
    const int32_t n = hg->n;
    hg->fiptr = hg->iptr;
    hg->ficol = hg->icol;
    hg->fiw = hg->iw;
    hg->fia = hg->ia;
    hg->fiwrep = hg->iwrep;
    hg->fieid = hg->ieid;
    hg->core_id.resize(n);
    hg->anchor_core.assign(n, -1);
    std::vector<uint8_t> pend(n, 0);
    hg->pruned = false;
    if (enable && !hg->directed && n > 2) {
        for (int32_t v = 0; v < n; ++v) {
            if (hg->iptr[v + 1] - hg->iptr[v] != 1) continue;
            const int32_t c = hg->icol[hg->iptr[v]];
            if (hg->iptr[c + 1] - hg->iptr[c] >= 2) pend[v] = 1;   // anchor is not itself pendant
        }
        for (int32_t v = 0; v < n; ++v) hg->pruned |= pend[v] != 0;
    }
    if (!hg->pruned) {
        hg->nc = n;
        hg->corev.resize(n);
        for (int32_t v = 0; v < n; ++v) hg->core_id[v] = hg->corev[v] = v;
        return;
    }
    hg->corev.clear();
    for (int32_t v = 0; v < n; ++v) {
        hg->core_id[v] = pend[v] ? -1 : (int32_t)hg->corev.size();
        if (!pend[v]) hg->corev.push_back(v);
    }
    hg->nc = (int32_t)hg->corev.size();
    for (int32_t v = 0; v < n; ++v)
        if (pend[v]) hg->anchor_core[v] = hg->core_id[hg->icol[hg->iptr[v]]];
    // core in-CSR: core vertices, core neighbours only (relaxation ids; the
    // neighbour order is unchanged, so lists stay sorted by original = core id)
    std::vector<int32_t> iptr(1, 0), icol;
    std::vector<double> iw, ia, iwrep;
    std::vector<int64_t> ieid;
    for (int32_t c = 0; c < hg->nc; ++c) {
        const int32_t v = hg->corev[c];
        for (int32_t k = hg->fiptr[v]; k < hg->fiptr[v + 1]; ++k) {
            const int32_t u = hg->ficol[k];
            if (pend[u]) continue;
            icol.push_back(hg->core_id[u]);
            iw.push_back(hg->fiw[k]);
            ia.push_back(hg->fia[k]);
            iwrep.push_back(hg->fiwrep[k]);
            ieid.push_back(hg->fieid[k]);
        }
        iptr.push_back((int32_t)icol.size());
    }
    hg->iptr.swap(iptr);
    hg->icol.swap(icol);
    hg->iw.swap(iw);
    hg->ia.swap(ia);
    hg->iwrep.swap(iwrep);
    hg->ieid.swap(ieid);
    hg->orev.resize(hg->icol.size());
    for (int32_t x = 0; x < hg->nc; ++x)
        for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k) {
            const int32_t y = hg->icol[k];
            const int32_t* b = hg->icol.data() + hg->iptr[y];
            const int32_t* e = hg->icol.data() + hg->iptr[y + 1];
            hg->orev[k] = (int32_t)(std::lower_bound(b, e, x) - hg->icol.data());
        }
}

void contract_degree3(HostGraph* hg) {
    HostGraph::Contracted& cx = hg->cx;
    cx = HostGraph::Contracted{};
    if (hg->directed || hg->multi_rep) return;
    for (double f : hg->vfac)
        if (has_attr(f) && f != 1.0) return;   // the rows' path-order re-fold walks plain entries only
    const int32_t nc = hg->nc;
    if (nc < 8 || hg->n >= (1 << 29)) return;   // (a leg packs its first hop's id into 29 bits)
    std::vector<int32_t> pendants(nc, 0);
    for (int32_t v = 0; v < hg->n; ++v)
        if (hg->anchor_core[v] >= 0) pendants[hg->anchor_core[v]]++;
    cx.kid.assign(nc, 0);
    cx.rid.assign(nc, -1);
    std::vector<uint8_t> blocked(nc, 0);
    for (int32_t x = 0; x < nc; ++x) {   // greedy independent set in core order
        if (blocked[x] || pendants[x] || hg->iptr[x + 1] - hg->iptr[x] != 3) continue;
        bool ok = true;
        for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k) ok &= hg->icol[k] != x;
        if (!ok) continue;
        cx.rid[x] = (int32_t)cx.rcore.size();
        cx.rcore.push_back(x);
        blocked[x] = 1;
        for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k) blocked[hg->icol[k]] = 1;
    }
    // worth it only where it removes a good share of the rows: the contracted build
    // pays a few extra loads per visit and longer hub lists (C4's core, whose
    // degree-3 vertices nearly all anchor pendants, keeps 2 of 20k: not contracted)
    if (cx.rcore.empty() || (int64_t)cx.rcore.size() * 10 < (int64_t)nc) {
        cx = HostGraph::Contracted{};
        return;
    }
    for (int32_t c = 0; c < nc; ++c) {
        cx.kid[c] = cx.rid[c] >= 0 ? -1 : (int32_t)cx.kcore.size();
        if (cx.rid[c] < 0) cx.kcore.push_back(c);
    }
    cx.nk = (int32_t)cx.kcore.size();
    for (int32_t x : cx.rcore)
        for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k) {   // neighbours in core order = kept order
            cx.rnb.push_back(cx.kid[hg->icol[k]]);
            cx.rw.push_back(hg->iw[k]);
            cx.ra.push_back(hg->ia[k]);
        }
    // in-CSR over kept vertices
    auto find = [&](int32_t list_of, int32_t nb) {   // entry of nb in list_of's core list
        const int32_t* b = hg->icol.data() + hg->iptr[list_of];
        const int32_t* e = hg->icol.data() + hg->iptr[list_of + 1];
        return (int32_t)(std::lower_bound(b, e, nb) - hg->icol.data());
    };
    cx.ptr.assign(1, 0);
    for (int32_t kv = 0; kv < cx.nk; ++kv) {
        const int32_t v = cx.kcore[kv];
        for (int32_t k = hg->iptr[v]; k < hg->iptr[v + 1]; ++k) {
            const int32_t u = hg->icol[k];
            if (cx.rid[u] < 0) {   // plain edge u -> v
                cx.col.push_back(cx.kid[u]);
                cx.w1.push_back(hg->iw[k]);
                cx.w2.push_back(0.0);
                cx.a1.push_back(hg->ia[k]);
                cx.a2.push_back(1.0);
                cx.key.push_back(u);
                cx.via.push_back(-1);
            } else {               // u = x removed: a -> v via x for x's other neighbours a
                for (int32_t q = hg->iptr[u]; q < hg->iptr[u + 1]; ++q) {
                    const int32_t a = hg->icol[q];
                    if (a == v) continue;
                    const int32_t kax = find(u, a);   // edge a -> x is the entry of a in x's list
                    cx.col.push_back(cx.kid[a]);
                    cx.w1.push_back(hg->iw[kax]);
                    cx.w2.push_back(hg->iw[k]);       // x -> v: the entry of x in v's list
                    cx.a1.push_back(hg->ia[kax]);
                    cx.a2.push_back(hg->ia[k]);
                    cx.key.push_back(u);
                    cx.via.push_back(hg->corev[u]);
                }
            }
        }
        cx.ptr.push_back((int32_t)cx.col.size());
    }
    // Derivable sources: the removed vertices, then a greedy independent
    // set, in the contracted graph, of kept vertices x with at most DER_LEGS_KEPT
    // contracted entries, at most one removed neighbour and no pendant, fewest removed
    // neighbours and entries first.  x's legs are its contracted entries read as
    // paths FROM x (x -> u, or x -> y -> b through a removed neighbour y) plus the
    // direct edge to y as a one-target leg; a removed neighbour y of x then reaches
    // x's other neighbours through x (x has no lane): its legs are its two other
    // neighbours, each plain neighbour k of x as x's prefix y -> x -> k, and x itself
    // as a one-target leg.  Rows read only lanes (no derived source reads another).
#ifndef SPE_DER_KEPT_MAX
#define SPE_DER_KEPT_MAX 5      // contracted entries of a derived kept vertex
#endif
#ifndef SPE_DER_MAXDEP
#define SPE_DER_MAXDEP 1        // removed neighbours it may have (0 or 1)
#endif
#ifndef SPE_DER_DEP_PLAIN
#define SPE_DER_DEP_PLAIN 3     // with a removed neighbour: at most this many kept neighbours
#endif
    constexpr int32_t DER_LEGS_KEPT = SPE_DER_KEPT_MAX;
    cx.der.assign(nc, 0);
    for (int32_t x : cx.rcore) cx.der[x] = 1;
    auto nrem = [&](int32_t x) {
        int32_t r = 0;
        for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k) r += cx.rid[hg->icol[k]] >= 0;
        return r;
    };
    std::vector<int32_t> cand;
    for (int32_t x = 0; x < nc; ++x) {
        if (cx.rid[x] >= 0 || pendants[x]) continue;
        const int32_t kv = cx.kid[x];
        const int32_t cdeg = cx.ptr[kv + 1] - cx.ptr[kv];
        bool loop = false;
        for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k) loop |= hg->icol[k] == x;
        const int32_t r = nrem(x);
        const int32_t plain = hg->iptr[x + 1] - hg->iptr[x] - r;
        if (!loop && cdeg <= DER_LEGS_KEPT && r <= SPE_DER_MAXDEP && (r == 0 || plain <= SPE_DER_DEP_PLAIN))
            cand.push_back(x);
    }
    std::stable_sort(cand.begin(), cand.end(), [&](int32_t p, int32_t q) {
        const int32_t rp = nrem(p), rq = nrem(q);
        if (rp != rq) return rp < rq;
        return cx.ptr[cx.kid[p] + 1] - cx.ptr[cx.kid[p]] < cx.ptr[cx.kid[q] + 1] - cx.ptr[cx.kid[q]];
    });
    std::vector<uint8_t> near((size_t)nc, 0);   // contracted-adjacent to a derived kept vertex
    for (int32_t x : cand) {
        if (near[x]) continue;
        const int32_t kv = cx.kid[x];
        cx.der[x] = 1;
        ++cx.nd4;
        near[x] = 1;
        for (int32_t k = cx.ptr[kv]; k < cx.ptr[kv + 1]; ++k) near[cx.kcore[cx.col[k]]] = 1;
    }
    // the legs, in core-id space
    std::vector<int32_t> xnb((size_t)nc, -1);   // removed vertex -> its derived kept neighbour
    for (int32_t x = 0; x < nc; ++x)
        if (cx.der[x] && cx.rid[x] < 0)
            for (int32_t k = hg->iptr[x]; k < hg->iptr[x + 1]; ++k)
                if (cx.rid[hg->icol[k]] >= 0) xnb[hg->icol[k]] = x;
    cx.dptr.assign((size_t)nc + 1, 0);
    for (int32_t c = 0; c < nc; ++c) {
        if (cx.der[c]) {
            if (cx.rid[c] >= 0) {   // removed
                const int32_t x = xnb[c];
                for (int32_t k = hg->iptr[c]; k < hg->iptr[c + 1]; ++k) {
                    const int32_t u = hg->icol[k];
                    if (u != x) {
                        cx.dlegs.push_back({u, 0, hg->corev[u], 1, hg->iw[k], hg->ia[k]});
                        continue;
                    }
                    // through the derived x: x's plain neighbours, and x itself
                    for (int32_t q = hg->iptr[x]; q < hg->iptr[x + 1]; ++q) {
                        const int32_t kk = hg->icol[q];
                        if (cx.rid[kk] >= 0) continue;   // (x's only removed neighbour is c)
                        cx.dlegs.push_back({kk, 0, hg->corev[x], 2, hg->iw[k] + hg->iw[q], hg->ia[k] * hg->ia[q]});
                    }
                    cx.dlegs.push_back({-1, cx.kid[x], hg->corev[x], 1, hg->iw[k], hg->ia[k]});
                }
            } else {                // kept
                for (int32_t k = hg->iptr[c]; k < hg->iptr[c + 1]; ++k) {
                    const int32_t u = hg->icol[k];
                    if (cx.rid[u] < 0) {
                        cx.dlegs.push_back({u, 0, hg->corev[u], 1, hg->iw[k], hg->ia[k]});
                        continue;
                    }
                    for (int32_t q = hg->iptr[u]; q < hg->iptr[u + 1]; ++q) {   // c -> u -> b
                        const int32_t b = hg->icol[q];
                        if (b == c) continue;
                        cx.dlegs.push_back({b, 0, hg->corev[u], 2, hg->iw[k] + hg->iw[q], hg->ia[k] * hg->ia[q]});
                    }
                    cx.dlegs.push_back({-1, -2 - cx.rid[u], hg->corev[u], 1, hg->iw[k], hg->ia[k]});
                }
            }
        }
        cx.dptr[(size_t)c + 1] = (int32_t)cx.dlegs.size();
    }
    // reverse entries: (a -> v via x) <-> (v -> a via x)
    cx.rev.assign(cx.col.size(), -1);
    for (int32_t kv = 0; kv < cx.nk; ++kv)
        for (int32_t k = cx.ptr[kv]; k < cx.ptr[kv + 1]; ++k) {
            const int32_t a = cx.col[k];
            for (int32_t q = cx.ptr[a]; q < cx.ptr[a + 1]; ++q)
                if (cx.col[q] == kv && cx.via[q] == cx.via[k]) {
                    cx.rev[k] = q;
                    break;
                }
        }
    cx.active = true;
}

// Constants of the shared anchor trees (HostGraph::Share).  The relaxation sums
// weights in path order; when every weight is an integer multiple of 2^-q and
// n * max weight * 2^q < 2^53, every such sum is exact, so a source offset o
// shifts every offer, distance and tie by exactly o and the anchor's decisions are
// the source's.  Otherwise the batch engine checks each decision's margin against
// the rounding the offset can introduce (k_share_check, wmin / omax below).
void share_prep(HostGraph* hg) {
    HostGraph::Share& sh = hg->share;
    sh = HostGraph::Share{};
    // pendant sources (pruning) and contracted sources (derived from their three
    // neighbours' rows) are the two kinds of offset sources
    if (!(hg->pruned || hg->cx.active) || hg->directed || hg->multi_rep) return;
    for (double f : hg->vfac)
        if (!(std::isnan(f) || f == 1.0)) return;
    std::vector<double> ws(hg->iw.begin(), hg->iw.end());
    if (hg->cx.active) ws.insert(ws.end(), hg->cx.w2.begin(), hg->cx.w2.end());
    double omax = 0.0;
    for (int32_t v = 0; v < hg->n; ++v) {
        if (hg->core_id[(size_t)v] >= 0 || hg->anchor_core[(size_t)v] < 0) continue;
        const double w = hg->fiw[(size_t)hg->fiptr[(size_t)v]];
        omax = std::max(omax, w);
        ws.push_back(w);
    }
    if (hg->cx.active)   // a derived source's offset is one of its legs' prefixes (one or two edges)
        for (const HostGraph::Contracted::Leg& l : hg->cx.dlegs) {
            omax = std::max(omax, l.w);
            ws.push_back(l.w);
        }
    double wmin = INFINITY, wmax = 0.0;
    for (double w : hg->iw) wmin = std::min(wmin, w);
    for (double w : ws) {
        if (!(w >= 0.0) || !std::isfinite(w)) return;   // (weights are validated >= 0 at creation)
        wmax = std::max(wmax, w);
    }
    sh.eligible = true;
    // a shared / derived row multiplies a(s, c) * r_c(t) where the reference folds
    // ((1 a(s, c)) a_1) a_2 ... from the source (shd-topology.c:1415-1484): the same
    // bits only when every factor is 1 (no edge loss anywhere)
    sh.prod_exact = true;
    for (double a : hg->ia) sh.prod_exact = sh.prod_exact && a == 1.0;
    for (double a : hg->fia) sh.prod_exact = sh.prod_exact && a == 1.0;
    if (hg->cx.active)
        for (double a : hg->cx.a2) sh.prod_exact = sh.prod_exact && a == 1.0;
    sh.wmin = std::isfinite(wmin) ? wmin : 0.0;
    sh.omax = omax;
    for (int q = 0; q <= 20 && !sh.exact; ++q) {
        const double sc = std::ldexp(1.0, q);
        if (!((double)hg->n * (wmax * sc + 1.0) < 0x1p53)) break;
        bool ok = true;
        for (double w : ws)
            if (std::floor(w * sc) != w * sc) {
                ok = false;
                break;
            }
        sh.exact = ok;
    }
}

}  // namespace spe
