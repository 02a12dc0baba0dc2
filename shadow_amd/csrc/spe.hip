// spe.hip -- MI355X (gfx950) shortest-path engine for Shadow's topology routing.
//
// Replaces, for every attached (source, target) pair at once, what the
// reference computes lazily per cache miss in src/main/routing/shd-topology.c:
//   DIRECT  _topology_lookupDirectPath           :1862-1912
//   SSSP    _topology_computeSourcePaths          :1640-1860 (igraph Dijkstra :1741)
//           + _topology_computePathProperties     :1392-1508
//   SELF    _topology_computeShortestPathToSelf   :1530-1638
// and serves the per-packet queries (topology_getLatency/getReliability/
// isRoutable, :2048-2075) from an HBM-resident table.
//
// Kernels (all hand-written for CDNA4, wave64):
//   k_init_state   per-batch state reset (dist = +inf, parent = none)
//   k_seed         sources -> first frontier marks
//   k_relax        multi-source label-correcting relaxation over a dense
//                  frontier bitmap (wave-ballot compaction, no global counter):
//                  ONE WAVE = one vertex x 64 sources (lane = source).  Only
//                  in-neighbours that changed last round are read (their flags
//                  are ballot-scanned 64 at a time; 4 coalesced 512-B rows of the
//                  [vertex][64] state); the canonical parent (alt, dist[u], u)
//                  and the path-order reliability / hop count / first hop are
//                  carried with the distance, so converged state IS the row.
//   k_rows_sssp    state -> table rows (+ SELF / [s] rules, slow path-walk for
//                  targets with vertex loss or multigraph get_eid latencies)
//   k_rows_direct  complete graphs: every pair is the direct edge
//   k_direct_overlay  preferdirectpaths: adjacent pairs get the direct edge
//   k_sssp_lds     small graphs (<= 10,240 relaxation vertices): one workgroup per
//                  source row, relaxation state in LDS, rows written directly
//   k_owner_replay compat: the reference's first-writer-wins path cache
//   k_lookup       batched per-packet (s, t) -> (latency, reliability, ok)
//   k_min_latency  minimumPathLatency reduction
// plus the host side: graph upload, table build loop, on-disk table cache.
//
// Bit-exactness: every distance is the least fixpoint of
// d[v] = min_u fl(d[u] + w), which igraph's Dijkstra also computes (IEEE
// round-to-nearest addition is monotone); compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <queue>
#include <random>
#include <string>
#include <type_traits>
#include <vector>

#include "spe_internal.h"

#define WAVE 64
#define BLOCK 256

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define ABI_MSG(T) (std::string(T) + ".struct_size is not sizeof(" T ") of this libspe: the caller was built " \
                    "against another include/spe.h (set it with SPE_STRUCT_INIT)")

// FNV-1a 64 over raw bytes (table cache keys)
struct Fnv {
    uint64_t h = 1469598103934665603ull;
    void add(const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) {
            h ^= b[i];
            h *= 1099511628211ull;
        }
    }
    template <typename T>
    void val(const T& x) { add(&x, sizeof(x)); }
};

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return fail(SPE_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
    } while (0)

constexpr double INF = __builtin_inf();

struct DevGraph {
    int32_t n;               // relaxation vertices (the core when pendants are pruned)
    int32_t nrel;
    int32_t n_full;          // all vertices (original ids)
    const int32_t* iptr;
    const int32_t* icol;
    const int4* ipack;       // per in-entry, one 16-B load for the relaxation: {icol, orev | heavy[icol] << 31
                             // (undirected: the out-list is the in-list), iw as two 32-bit halves}
    const int32_t* irow;     // in-CSR entry -> its target vertex (flat edge passes)
    const uint32_t* ipair;   // nc <= 65535 only (LDS-engine graphs): (irow << 16) | icol, one 4-B load
    const double* iw;
    const double* ia;
    const double* iwrep;
    const int32_t* optr;
    const int32_t* ocol;
    const int32_t* orev;     // out-entry -> index of the same edge in the target's in-CSR list
    const double* owrep;
    const double* oarep;
    const double* ow;        // relaxation (lightest) weight per out-entry (== iw when undirected)
    int32_t undirected;      // out-CSR == in-CSR
    const uint8_t* heavy;    // [n] in-degree > 64
    const uint8_t* oheavy;   // [out entry] heavy[target]: which frontier buffer it goes to
    int32_t ablate;          // diagnostic only (SPE_ABLATE env): bit 0 = skip route records
    const double* vfac;
    const double* loop_w;
    const double* loop_a;
    const double* self_w2;
    const double* self_a2;
    const int32_t* self_other;
    // original <-> relaxation ids and the full in-CSR (pendant edges, DIRECT lookups)
    const int32_t* core_id;      // [n_full] -1 = pruned pendant
    const int32_t* corev;        // [n]
    const int32_t* anchor_core;  // [n_full]
    const int32_t* fiptr;
    const double* fiw;
    const double* fia;
    const double* fiwrep;
    // optional per-edge auxiliary attribute of the get_eid edge (spe_graph_set_edge_aux)
    const double* iaux;          // [relaxation in-CSR entry]
    const double* fiaux;         // [full in-CSR entry]
    const int32_t* dptr;         // DIRECT lookups: full out-CSR
    const int32_t* dcol;
    const double* dwrep;
    const double* darep;
    // Degree-3 contraction (spe_graph.devx, the batch engine's graph when the
    // table runs on it; NULL in the plain graph).  Relaxation ids are then the kept
    // vertices; entry k offers fl(fl(d[icol[k]] + iw[k]) + xw2[k]) (xw2 = 0 for a plain
    // edge: the same bits as one add), its parent of record is core vertex xkey[k] (x
    // for a shortcut), and the route multiplies ia[k] then xa2[k] and adds 1 + (xvia >= 0)
    // hops.  A removed vertex's rows come from its three neighbours (rnb / rw / ra).
    const double* xw2;
    const double* xa2;
    const int32_t* xkey;
    const int32_t* xvia;         // original id of x, -1 for a plain edge
    const int32_t* xrm;          // [n_full] removed index, -1 otherwise
    const int32_t* rnb;          // [3 removed] kept ids of the neighbours (increasing)
    const double* rw;
    const double* ra;
};

struct RowMode {
    int32_t complete;
    int32_t prefer;
    int32_t self_mode;
    int32_t multi_rep;
    int32_t directed;
};

// Per-lane route record carried with the distance: the path-order reliability
// fold (starting at the source factor) and (hops, first hop).  16 B so a parent
// lookup is ONE 16-B access per lane (lanes with the same parent coalesce).
struct alignas(16) Route {
    double r;
    int32_t h;
    int32_t f;
};

// Relaxation state of one batch, [lane group][vertex][L lanes] (lane = source).
// A lane group of L sources is the unit that shares a frontier; a wave holds
// 64/L subgroups and so relaxes 64/L (group, vertex) items at once.
struct State {
    double* D;        // distance
    int32_t* P;       // in-CSR index of the chosen parent edge, -1 none
    Route* RT;        // route record
};

typedef double dvec2 __attribute__((ext_vector_type(2)));

struct Table {
    double2* lr;      // {latency, reliability}: one 16-B record, so a lookup is one HBM line
    int32_t* next;
    uint16_t* hops;
    int32_t A;
    int32_t* prev;    // owner-replay mode only: vertex before the target on the path
    double* aux;      // want_aux only: path-order sum of the edges' auxiliary attribute
};

__device__ __forceinline__ bool has_attr(double x) { return !__builtin_isnan(x); }

__device__ __forceinline__ size_t tidx(int32_t sb_local, int32_t A, int32_t j, int32_t lane) {
    return ((size_t)sb_local * (size_t)A + (size_t)j) * WAVE + (size_t)lane;
}

template <int L>
struct Sub {
    static constexpr int V = WAVE / L;                                   // subgroups per wave
    static constexpr uint64_t MASK = (L == 64) ? ~0ull : ((1ull << L) - 1);
    static constexpr int INFL = (L == 64) ? 8 : (L == 32 ? 6 : 4);       // neighbour rows in flight per subgroup
};

template <int L>
__device__ __forceinline__ size_t sidx(int32_t g, int32_t n, int32_t v, int32_t j) {
    return ((size_t)g * (size_t)n + (size_t)v) * L + (size_t)j;
}

// value of `x` held by lane `src` (same subgroup, active)
template <int L>
__device__ __forceinline__ int32_t sub_get(int32_t x, int32_t src) {
    if constexpr (L == 64) return __builtin_amdgcn_readlane(x, src);
    else return __shfl(x, src);
}

template <int L>
__device__ __forceinline__ double sub_get_d(double x, int32_t src) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    const uint32_t lo = (uint32_t)sub_get<L>((int32_t)(uint32_t)b, src);
    const uint32_t hi = (uint32_t)sub_get<L>((int32_t)(uint32_t)(b >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ----------------------------------------------------------------- kernels

// One lane group per blockIdx.y; threads stride over its [n][L] block with a
// stride that is a multiple of L, so each thread keeps one lane (one source)
// and resolves that source's constants once.  Stores only: D, P per element,
// the route record on the source's own (and pruned source's anchor) row.
template <int L>
__global__ __launch_bounds__(BLOCK) void k_init_state(int32_t n, int32_t groups, const int32_t* __restrict__ srcv,
                                                      const double* __restrict__ vfac, DevGraph G, State st) {
    static_assert(BLOCK % L == 0, "the stride must keep the lane");
    const int32_t g = blockIdx.y;
    const int64_t per = (int64_t)n * L;
    const int32_t j = threadIdx.x & (L - 1);
    const int32_t s = srcv[g * L + j];   // original id, -1 = padding lane
    int32_t sc = -1, anc = -1, kx = -1, rm = -1;
    double r0 = 1.0;
    if (s >= 0) {
        const double fs = vfac[s];
        r0 = has_attr(fs) ? 1.0 * fs : 1.0;  // (1 * (1 - p_src)), shd-topology.c:1428-1430
        sc = G.core_id[s];
        if (sc < 0) {
            anc = G.anchor_core[s];
            kx = G.fiptr[s];
            if (G.xrm) rm = G.xrm[s];   // a contracted source: its three edges seed the relaxation
        }
    }
    int32_t rn0 = -1, rn1 = -1, rn2 = -1;
    if (rm >= 0) {
        rn0 = G.rnb[3 * rm];
        rn1 = G.rnb[3 * rm + 1];
        rn2 = G.rnb[3 * rm + 2];
    }
    const size_t base = (size_t)g * (size_t)per;
    for (int64_t x = (int64_t)blockIdx.x * BLOCK + threadIdx.x; x < per; x += (int64_t)gridDim.x * BLOCK) {
        const int32_t v = (int32_t)(x / L);
        const size_t i = base + (size_t)x;
        double d = INF;
        int32_t p = -1;
        if (v == sc) {
            d = 0.0;
            Route rt;
            rt.r = r0;
            rt.h = 0;
            rt.f = -1;
            st.RT[i] = rt;
        } else if (v == anc) {
            // pruned pendant source: Dijkstra's first step s -> anchor, fixed (every
            // path leaves through it); P = -2 marks "parent is the pendant source"
            d = 0.0 + G.fiw[kx];
            p = -2;
            Route rt;
            rt.r = r0 * G.fia[kx];
            rt.h = 1;
            rt.f = G.corev[v];
            st.RT[i] = rt;
        } else if (rm >= 0 && (v == rn0 || v == rn1 || v == rn2)) {
            // contracted source: its first edge to each neighbour, an offer like any
            // other (a shorter path through another neighbour replaces it); P = -2 as
            // for a pendant source: the parent is the source itself, which wins ties
            const int32_t q = v == rn0 ? 0 : (v == rn1 ? 1 : 2);
            d = 0.0 + G.rw[3 * rm + q];
            p = -2;
            Route rt;
            rt.r = r0 * G.ra[3 * rm + q];
            rt.h = 1;
            rt.f = G.corev[v];
            st.RT[i] = rt;
        }
        st.D[i] = d;
        st.P[i] = p;
    }
}

// Change propagation.  When (group, u) changes in round r, it sets, for every
// out-edge u -> x, the frontier mark of (group, x) and the in-edge flag of the
// mirrored in-CSR entry (reverse index G.orev) in round r+1's buffers.  A vertex
// then sees WHICH of its in-neighbours changed with one coalesced byte load per
// L in-edges, without dereferencing the neighbour ids first.
struct Flags {
    uint8_t* mark_cur;     // [group][vertex]   light-vertex frontier of this round (consumed)
    uint8_t* mark_next;
    uint8_t* hmark_cur;    // [group][vertex]   heavy-vertex frontier (in-degree > 64)
    uint8_t* hmark_next;
    uint8_t* in_cur;       // [group][in-CSR entry] changed in-neighbour (consumed)
    uint8_t* in_next;
    int32_t* any_changed;  // set when some vertex changed this round
    const int32_t* prev_changed;   // the previous round's flag: 0 = converged, the round is a no-op
};

// Delta-stepping schedule (SPE_DELTA=<ms>, experimental): each lane
// group relaxes only offers below its bucket bound; a row whose lanes saw larger
// offers is parked (pending) with the smallest of them, and when the group's round
// changes nothing its bound moves to that offer + Delta and its parked rows are
// rescanned over every in-edge.  Converges to the same fixpoint (every edge is
// eventually offered with no bound in the way), so rows are unchanged.
struct DeltaState {
    double* bound;               // [lane group] current bucket bound
    unsigned long long* minrej;  // [lane group] smallest deferred offer (f64 bits) since the last advance
    double* pending;             // [lane group][vertex] smallest deferred offer of a parked row (>= 1e300: none)
    int32_t* gchanged;           // [lane group] some lane of the group changed this round
};

__device__ __forceinline__ double wave_min_f64(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o));
    return x;
}

// after a (group, v) item: park it if an offer was deferred, flag the group's change
__device__ __forceinline__ void delta_note(const DeltaState& ds, int32_t g, int32_t n, int32_t v, double rej,
                                           bool any, bool item, int32_t lane) {
    const double r = wave_min_f64(rej);
    if (item && lane == 0) {
        if (r < INF) {   // (g, v) is this wave's alone within a round: plain read-modify-write
            double* pv = ds.pending + (size_t)g * n + v;
            *pv = fmin(*pv, r);
            atomicMin(&ds.minrej[g], (unsigned long long)__double_as_longlong(r));
        }
        if (any) ds.gchanged[g] = 1;
    }
}

__global__ __launch_bounds__(BLOCK) void k_delta_init(int32_t groups, double delta, DeltaState ds) {
    const int32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= groups) return;
    ds.bound[g] = delta;
    ds.minrej[g] = 0x7FF0000000000000ull;   // +inf
    ds.gchanged[g] = 0;
}

// After round r: a lane group that changed nothing and has parked rows moves its
// bound to (smallest deferred offer + Delta) -- empty buckets are skipped -- and
// puts the parked rows whose smallest deferred offer is now below the bound into
// round r+1's frontier with all their in-edges flagged; the others stay parked
// (their minimum becomes the group's next one).  One workgroup per lane group.
__global__ __launch_bounds__(BLOCK) void k_delta_advance(int32_t n, int32_t nrel, double delta, DevGraph G,
                                                         DeltaState ds, uint8_t* mark_next, uint8_t* in_next,
                                                         int32_t* any_changed) {
    __shared__ int32_t go;
    __shared__ double bnd;
    __shared__ unsigned long long left;
    const int32_t g = blockIdx.x;
    if (threadIdx.x == 0) {
        const unsigned long long mr = ds.minrej[g];
        go = ds.gchanged[g] == 0 && mr != 0x7FF0000000000000ull;
        if (go) {
            bnd = __longlong_as_double((long long)mr) + delta;
            ds.bound[g] = bnd;
            *any_changed = 1;
        }
        left = 0x7FF0000000000000ull;
        ds.gchanged[g] = 0;
    }
    __syncthreads();
    if (!go) return;
    double keep = INF;
    for (int32_t v = threadIdx.x; v < n; v += BLOCK) {
        double* pv = ds.pending + (size_t)g * n + v;
        const double p = *pv;
        if (p >= 1e300) continue;
        if (p >= bnd) {
            keep = fmin(keep, p);
            continue;
        }
        *pv = 1e301;
        mark_next[(size_t)g * n + v] = 1;
        for (int32_t k = G.iptr[v]; k < G.iptr[v + 1]; ++k) in_next[(size_t)g * nrel + k] = 1;
    }
    keep = wave_min_f64(keep);
    if ((threadIdx.x & (WAVE - 1)) == 0 && keep < INF)
        atomicMin(&left, (unsigned long long)__double_as_longlong(keep));
    __syncthreads();
    if (threadIdx.x == 0) ds.minrej[g] = left;
}

// One wave per source entry (a hub source's out-list spreads over the lanes).
template <int L>
__global__ __launch_bounds__(BLOCK) void k_seed(int32_t n, int32_t groups, const int32_t* __restrict__ srcv,
                                                DevGraph G, uint8_t* mark, uint8_t* hmark, uint8_t* in_flags) {
    const int32_t i = __builtin_amdgcn_readfirstlane((int32_t)((blockIdx.x * BLOCK + threadIdx.x) >> 6));
    const int32_t lane = threadIdx.x & (WAVE - 1);
    if (i >= groups * L) return;
    const int32_t s0 = srcv[i];
    if (s0 < 0) return;
    const int32_t sc = G.core_id[s0];
    const int32_t g = i / L;
    const int32_t rm = (sc < 0 && G.xrm) ? G.xrm[s0] : -1;
    // rows holding the source's first values: its own, its pendant anchor, or (a
    // contracted source) its three neighbours
    for (int32_t q = 0; q < (rm >= 0 ? 3 : 1); ++q) {
        const int32_t s = rm >= 0 ? G.rnb[3 * rm + q] : (sc >= 0 ? sc : G.anchor_core[s0]);
        for (int32_t k = G.optr[s] + lane; k < G.optr[s + 1]; k += WAVE) {
            (G.oheavy[k] ? hmark : mark)[(size_t)g * n + G.ocol[k]] = 1;
            in_flags[(size_t)g * G.nrel + G.orev[k]] = 1;
        }
    }
}

// Lexicographic candidate update (alt, d[u], u) against the running best of one
// lane.  Ties against the current parent resolve with the parent's CURRENT
// distance; an offer from the current parent itself (kk == bk) refreshes it.
// The stored parent P is read lazily (PK_UNREAD): only an offer EQUAL to the
// current distance (a refresh from the parent, or a tie) needs it; most offers
// are strictly better or worse, so most visits skip the 256-B P row.
constexpr int32_t PK_UNREAD = -3;

// Lexicographic key comparisons are written branch-free (bitwise & / | on bools,
// then selects).  The short-circuit form `a < A || (a == A && (b < B || ...))`
// followed by several assignments was miscompiled by the gfx950 backend (ROCm
// 7.2): with a wave-uniform last key, the tie branch's lanes took the new
// distance fields but kept the OLD parent entry / vertex, so a tie won on
// (d[u], u) recorded the wrong parent (found on decimal-latency graphs, whose
// f64 sums tie).  Selects leave the compiler no such branch to merge.
__device__ __forceinline__ bool lex_less3(double a, double b, int32_t c, double A, double B, int32_t C) {
    return (a < A) | ((a == A) & ((b < B) | ((b == B) & (c < C))));
}
__device__ __forceinline__ bool lex_less2(double b, int32_t c, double B, int32_t C) {
    return (b < B) | ((b == B) & (c < C));
}

struct Best {
    double bd;     // best alt (= distance)
    int32_t bk;    // in-CSR index of the parent edge (PK_UNREAD: the stored one, not read yet)
    int32_t bu;    // parent vertex (-1: not resolved yet)
    double bdu;    // parent distance (-1: not resolved yet)
    bool need;     // the parent's (R, H, F) must be (re)gathered
    int32_t pold;  // the stored parent once read (PK_UNREAD until then)
    size_t rv;     // this lane's state index (for the lazy P read)
};

template <int L>
__device__ __forceinline__ void offer(Best& b, const DevGraph& G, const State& st, int32_t g, int32_t n, int32_t j,
                                      int32_t kk, int32_t u, double du, double alt) {
    bool better = false;
    if (alt < b.bd) {
        better = true;
    } else if (alt == b.bd) {
        if (b.bk == PK_UNREAD) b.bk = b.pold = st.P[b.rv];
        if (kk == b.bk) {
#ifdef SPE_DIAGNOSTICS   // experiments only: SPE_ABLATE bit 1 skips parent refreshes (inexact)
            if (G.ablate & 2) return;
#endif
            b.need = true;
            b.bdu = du;
            b.bu = u;
        } else if (b.bk >= 0) {   // (bk = -2: fixed seed from a pendant source, never tied)
            if (b.bu < 0) b.bu = G.icol[b.bk];
            if (b.bdu < 0.0) b.bdu = st.D[sidx<L>(g, n, b.bu, j)];
            better = lex_less2(du, u, b.bdu, b.bu);
        }
    }
    b.bd = better ? alt : b.bd;
    b.bk = better ? kk : b.bk;
    b.bu = better ? u : b.bu;
    b.bdu = better ? du : b.bdu;
    b.need = b.need | better;
}

// offer<L> on the contracted graph (the heavy combine): b.bu holds the parent-of-
// record key (a core id), b.bdu its distance; two shortcuts through the same x
// tie-break on their kept vertices (d[a], a).
template <int L>
__device__ __forceinline__ void offer_x(Best& b, const DevGraph& G, const State& st, int32_t g, int32_t n, int32_t j,
                                        int32_t kk, int32_t key, double drec, double alt) {
    bool better = false;
    if (alt < b.bd) {
        better = true;
    } else if (alt == b.bd) {
        if (b.bk == PK_UNREAD) b.bk = b.pold = st.P[b.rv];
        if (kk == b.bk) {
            b.need = true;
            b.bdu = drec;
            b.bu = key;
        } else if (b.bk >= 0) {
            const int4 po = G.ipack[b.bk];
            if (b.bu < 0) b.bu = G.xkey[b.bk];
            if (b.bdu < 0.0) {
                const double da = st.D[sidx<L>(g, n, po.x, j)];
                b.bdu = (po.y & 0x40000000) ? da + __hiloint2double(po.w, po.z) : da;
            }
            better = lex_less2(drec, key, b.bdu, b.bu);
            if (drec == b.bdu && key == b.bu) {   // same x: x's own canonical parent decides
                const int32_t an = G.ipack[kk].x, ao = po.x;
                const double dn = st.D[sidx<L>(g, n, an, j)], dd = st.D[sidx<L>(g, n, ao, j)];
                better = lex_less2(dn, an, dd, ao);
            }
        }
    }
    b.bd = better ? alt : b.bd;
    b.bk = better ? kk : b.bk;
    b.bu = better ? key : b.bu;
    b.bdu = better ? drec : b.bdu;
    b.need = b.need | better;
}

// Flagged candidates of one L-entry chunk [c0, c0+L) of a vertex's in-list.
// `sm` = subgroup-relative mask of flagged entries (subgroup-uniform); rows of
// the flagged neighbours are gathered INFL at a time; f(kk, u, du, alt) is
// called for lanes where the candidate is a valid improvement path.
template <int L, int INFL, typename F>
__device__ __forceinline__ void scan_chunk(uint64_t sm, int32_t c0, int32_t base, int32_t u_j, double w_j, int32_t g,
                                           int32_t n, int32_t j, bool active, const State& st, F&& f) {
    while (sm) {
        int32_t us[INFL], ks[INFL];
        double ws[INFL], dus[INFL];
#pragma unroll
        for (int q = 0; q < INFL; ++q) {
            us[q] = -1;
            if (sm) {
                const int32_t b = __builtin_ctzll(sm);
                sm &= sm - 1;
                us[q] = sub_get<L>(u_j, base + b);
                ws[q] = sub_get_d<L>(w_j, base + b);
                ks[q] = c0 + b;
            }
        }
#pragma unroll
        for (int q = 0; q < INFL; ++q)
            if (us[q] >= 0) {   // uniform row base (L = 64: SGPRs) + per-lane offset: no 64-bit VGPR address per row
                const double* row = st.D + ((size_t)g * (size_t)n + (size_t)us[q]) * L;
                dus[q] = row[j];
            }
#pragma unroll
        for (int q = 0; q < INFL; ++q) {
            if (us[q] < 0) continue;
            const double alt = dus[q] + ws[q];
            if (active && alt > dus[q]) f(ks[q], us[q], dus[q], alt);
        }
    }
}

// Gather the chosen parent's (R, H, F), write the lane's state if it changed.
template <int L>
__device__ __forceinline__ bool finish_vertex(Best& b, const DevGraph& G, const State& st, int32_t g, int32_t n,
                                              int32_t j, int32_t v, int32_t s, size_t rv, double d_old) {
    bool changed = false;
    // need with b.bd == d_old implies an equal offer, which read the stored parent
    const int32_t p_old = b.pold;
    if (b.need && G.xw2) {   // contracted graph (heavy combine): route from the entry's kept vertex
        const int32_t ga = G.icol[b.bk];
        const int32_t via = G.xvia[b.bk];
        const Route pu = st.RT[sidx<L>(g, n, ga, j)];
        Route nr;
        nr.r = (pu.r * G.ia[b.bk]) * G.xa2[b.bk];
        nr.h = pu.h + (via >= 0 ? 2 : 1);
        nr.f = (ga == s) ? (via >= 0 ? via : G.corev[v]) : pu.f;
        if (d_old == INF || b.bd != d_old || b.bk != p_old) {
            changed = true;
        } else {
            const Route old = st.RT[rv];
            changed = (nr.r != old.r) || (nr.h != old.h) || (nr.f != old.f);
        }
        if (changed) {
            st.D[rv] = b.bd;
            st.P[rv] = b.bk;
            st.RT[rv] = nr;
        }
        return changed;
    }
    if (b.need) {
        if (b.bu < 0) b.bu = G.icol[b.bk];
        if (G.ablate & 1) {   // diagnostic only: distances + parents, no route records
            changed = (d_old == INF || b.bd != d_old || b.bk != p_old);
            if (changed) {
                st.D[rv] = b.bd;
                st.P[rv] = b.bk;
            }
            return changed;
        }
        const Route pu = st.RT[sidx<L>(g, n, b.bu, j)];
        Route nr;
        nr.r = pu.r * G.ia[b.bk];
        nr.h = pu.h + 1;
        nr.f = (b.bu == s) ? G.corev[v] : pu.f;
        if (d_old == INF || b.bd != d_old || b.bk != p_old) {
            changed = true;
        } else {   // same parent, same distance: did the parent's route change?
            const Route old = st.RT[rv];
            changed = (nr.r != old.r) || (nr.h != old.h) || (nr.f != old.f);
        }
        if (changed) {
            st.D[rv] = b.bd;
            st.P[rv] = b.bk;
            st.RT[rv] = nr;
        }
    }
    return changed;
}

// (group, v) changed: flag its out-edges for the next round (L lanes of the subgroup).
template <int L>
__device__ __forceinline__ void mark_out(const DevGraph& G, int32_t g, int32_t n, int32_t v, int32_t j,
                                         const Flags& fl) {
    const int32_t o0 = G.optr[v], o1 = G.optr[v + 1];
    for (int32_t k = o0 + j; k < o1; k += L) {
        (G.oheavy[k] ? fl.hmark_next : fl.mark_next)[(size_t)g * n + G.ocol[k]] = 1;
        fl.in_next[(size_t)g * G.nrel + G.orev[k]] = 1;
    }
}

// Relaxation of one light (in-degree <= 64) item e = g * n + v by one subgroup
// (lane j = source g*L + j); e < 0: this subgroup has no item (it still takes
// part in the wave-wide ballots).  Returns this lane's "changed".
template <int L, int INFL, bool DELTA = false>
__device__ __forceinline__ bool relax_item(int64_t e, int32_t n, int32_t j, int32_t base,
                                           const int32_t* __restrict__ srcv, const DevGraph& G, const State& st,
                                           const Flags& fl, const DeltaState& ds) {
    int32_t g = 0, v = 0, k0 = 0, k1 = 0, s = -1;
    double d_old = INF;
    int32_t p_old = -1;
    if (e >= 0) {
        g = (int32_t)(e / n);
        v = (int32_t)(e - (int64_t)g * n);
        k0 = G.iptr[v];
        k1 = G.iptr[v + 1];
        s = srcv[g * L + j];
    }
    const size_t rv = sidx<L>(g, n, v, j);
    if (e >= 0) {
        d_old = st.D[rv];
        p_old = d_old < INF ? PK_UNREAD : -1;   // an unreached lane has no parent (k_init_state)
    }
    const bool active = (e >= 0) && (s != -1) && (s != v);
    Best b{d_old, p_old, -1, -1.0, false, p_old, rv};
    const double bnd = (DELTA && e >= 0) ? ds.bound[g] : INF;
    double rej = INF;
    // undirected graphs: the out-list IS the in-list; a single-chunk vertex keeps
    // what marking needs (neighbour, reverse entry, heavy bit) in registers
    int32_t u_last = 0, orev_last = 0;
    bool heavy_last = false, ok_last = false;
    for (int32_t c0 = k0; c0 < k1; c0 += L) {   // subgroup-uniform trip count
        const int32_t k = c0 + j;
        const bool ok = k < k1;
        const int4 pk = ok ? G.ipack[k] : make_int4(0, 0, 0, 0);
        const int32_t u_j = pk.x;
        const double w_j = __hiloint2double(pk.w, pk.z);
        const size_t fo = (size_t)g * G.nrel + k;
        const bool f = ok && fl.in_cur[fo] != 0;
        if (G.undirected && ok) {
            orev_last = pk.y & 0x7FFFFFFF;
            heavy_last = pk.y < 0;
        }
        u_last = u_j;
        ok_last = ok;
        if (f) fl.in_cur[fo] = 0;   // consumed
        const uint64_t sm = (__ballot(f) >> base) & Sub<L>::MASK;
        scan_chunk<L, INFL>(sm, c0, base, u_j, w_j, g, n, j, active, st,
                            [&](int32_t kk, int32_t u, double du, double alt) {
                                if (DELTA && alt >= bnd) {   // beyond the group's bucket: deferred
                                    rej = fmin(rej, alt);
                                    return;
                                }
                                offer<L>(b, G, st, g, n, j, kk, u, du, alt);
                            });
    }
    bool changed = false;
    if (e >= 0) changed = finish_vertex<L>(b, G, st, g, n, j, v, s, rv, d_old);
    const bool any = ((__ballot(changed) >> base) & Sub<L>::MASK) != 0;
    if constexpr (DELTA) delta_note(ds, g, n, v, rej, any, e >= 0, j);   // L == 64 only (host-enforced)
    if (any) {
        if (G.undirected && k1 - k0 <= L) {
            if (ok_last) {
                (heavy_last ? fl.hmark_next : fl.mark_next)[(size_t)g * n + u_last] = 1;
                fl.in_next[(size_t)g * G.nrel + orev_last] = 1;
            }
        } else {
            mark_out<L>(G, g, n, v, j, fl);
        }
    }
    return changed;
}

__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
           (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

// nonzero bytes of w -> bit per byte
__device__ __forceinline__ uint32_t byte_mask(uint64_t w) {
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) m |= ((w >> (8 * q)) & 0xFF) ? (1u << q) : 0u;
    return m;
}

// One relaxation round over the dense light-frontier bitmap.  Work unit = 8
// consecutive (group, vertex) flags read as one 64-bit word; the wave's V
// subgroups take its marked items V at a time (V = 64/L items in flight per
// wave).  XCD-aware split (speed only, never correctness): blocks are dealt
// round-robin over the 8 XCDs, so blocks with equal blockIdx % 8 share an L2;
// each such class gets one contiguous eighth of the (group, vertex) space.
template <int L, int INFL, int OCC = 1, bool DELTA = false>
__global__ __launch_bounds__(BLOCK, OCC) void k_relax(int32_t total, int32_t n, const int32_t* __restrict__ srcv,
                                                 DevGraph G, State st, Flags fl, DeltaState ds) {
    if (*fl.prev_changed == 0) return;   // converged: rounds are enqueued ahead of the host's check
    constexpr int V = Sub<L>::V;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int32_t sub = lane / L, j = lane % L, base = sub * L;
    uint64_t* words = reinterpret_cast<uint64_t*>(fl.mark_cur);
    const int64_t all_units = ((int64_t)total + 7) >> 3;   // mark buffers padded to 8 bytes
    const int32_t xcd = blockIdx.x & 7;
    const int64_t waves_per_xcd = ((int64_t)(gridDim.x >> 3) * BLOCK) >> 6;
    const int64_t wave = (int64_t)(blockIdx.x >> 3) * (BLOCK / WAVE) +
                         __builtin_amdgcn_readfirstlane((int32_t)(threadIdx.x >> 6));   // uniform: SGPRs
    const int64_t lo = all_units * xcd / 8, hi = all_units * (xcd + 1) / 8;
    bool wrote = false;
    int64_t u8 = lo + wave;
    uint64_t w_ahead = u8 < hi ? words[u8] : 0;
    for (; u8 < hi; u8 += waves_per_xcd) {
        const uint64_t w = uniform_u64(w_ahead);
        const int64_t nx = u8 + waves_per_xcd;
        w_ahead = nx < hi ? words[nx] : 0;
        if (!w) continue;
        if (lane == 0) words[u8] = 0;   // taken
        uint32_t bm = byte_mask(w);
        while (bm) {
            // subgroup `sub` takes the sub-th marked byte of the next V
            uint32_t t = bm;
            int32_t mine = -1;
#pragma unroll
            for (int q = 0; q < V; ++q) {
                if (!t) break;
                const int32_t bit = __builtin_ctz(t);
                t &= t - 1;
                if (q == sub) mine = bit;
            }
            bm = t;
            int64_t e = mine >= 0 ? u8 * 8 + mine : -1;
            if (e >= total) e = -1;
            wrote |= relax_item<L, INFL, DELTA>(e, n, j, base, srcv, G, st, fl, ds);
        }
    }
    if (__ballot(wrote) && lane == 0) *fl.any_changed = 1;   // at most one plain store per wave
}

// Heavy vertices: their in-neighbour lists are cut into 64-entry segments; one
// subgroup per (group, segment) computes the lexicographic best changed
// candidate of its segment (no comparison with the stored state).
struct HeavyPlan {
    int32_t nseg;                 // segments over all heavy vertices
    int32_t nheavy;
    const int32_t* seg_vertex;    // [nseg]
    const int32_t* seg_begin;     // [nseg] in-CSR start of the segment
    const int32_t* heavy_vertex;  // [nheavy]
    const int32_t* heavy_seg0;    // [nheavy + 1] segment range of each heavy vertex
};

struct Partial {                  // [group][segment][L]
    double* alt;
    double* du;
    int2* uk;                     // (u, k), u = -1: no candidate
};

template <int L, int INFL = Sub<L>::INFL>
__global__ __launch_bounds__(BLOCK) void k_heavy_partial(int32_t groups, int32_t n, const int32_t* __restrict__ srcv,
                                                         DevGraph G, State st, HeavyPlan hp, Partial pp, Flags fl) {
    if (*fl.prev_changed == 0) return;
    constexpr int V = Sub<L>::V;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int32_t sub = lane / L, j = lane % L, base = sub * L;
    const int64_t nsub = (((int64_t)gridDim.x * BLOCK) >> 6) * V;
    const int64_t items = (int64_t)groups * hp.nseg;
    const int64_t first = ((((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6) * V) + sub;
    const int64_t rounds = (items + nsub - 1) / nsub;   // wave-uniform loop count
    for (int64_t r = 0; r < rounds; ++r) {
        const int64_t it = first + r * nsub;
        bool item = it < items;
        int32_t g = 0, sgi = 0, v = 0;
        if (item) {
            g = (int32_t)(it / hp.nseg);
            sgi = (int32_t)(it - (int64_t)g * hp.nseg);
            v = hp.seg_vertex[sgi];
            item = fl.hmark_cur[(size_t)g * n + v] != 0;
        }
        int32_t kb = 0, ke = 0, s = -1;
        if (item) {
            kb = hp.seg_begin[sgi];
            ke = min(kb + WAVE, G.iptr[v + 1]);
            s = srcv[g * L + j];
        }
        const bool active = item && (s != -1) && (s != v);
        double ba = INF, bdu = INF;
        int32_t bu = -1, bk = -1;
        for (int32_t c0 = kb; c0 < ke; c0 += L) {
            const int32_t k = c0 + j;
            const bool ok = k < ke;
            const int4 pk = ok ? G.ipack[k] : make_int4(0, 0, 0, 0);
            const int32_t u_j = pk.x;
            const double w_j = __hiloint2double(pk.w, pk.z);
            const size_t fo = (size_t)g * G.nrel + k;
            const bool f = ok && fl.in_cur[fo] != 0;
            if (f) fl.in_cur[fo] = 0;
            const uint64_t sm = (__ballot(f) >> base) & Sub<L>::MASK;
            scan_chunk<L, INFL>(sm, c0, base, u_j, w_j, g, n, j, active, st,
                          [&](int32_t kk, int32_t u, double du, double alt) {
                              const bool better = lex_less3(alt, du, u, ba, bdu, bu);
                              ba = better ? alt : ba;
                              bdu = better ? du : bdu;
                              bu = better ? u : bu;
                              bk = better ? kk : bk;
                          });
        }
        if (item) {
            const size_t o = ((size_t)g * hp.nseg + sgi) * L + j;
            pp.alt[o] = ba;
            pp.du[o] = bdu;
            pp.uk[o] = make_int2(bu, bk);
        }
    }
}

// Combine the segment partials of each marked heavy (group, v) into its state.
template <int L>
__global__ __launch_bounds__(BLOCK) void k_heavy_combine(int32_t groups, int32_t n, const int32_t* __restrict__ srcv,
                                                         DevGraph G, State st, HeavyPlan hp, Partial pp, Flags fl) {
    if (*fl.prev_changed == 0) return;
    constexpr int V = Sub<L>::V;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int32_t sub = lane / L, j = lane % L, base = sub * L;
    const int64_t nsub = (((int64_t)gridDim.x * BLOCK) >> 6) * V;
    const int64_t items = (int64_t)groups * hp.nheavy;
    const int64_t first = ((((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6) * V) + sub;
    const int64_t rounds = (items + nsub - 1) / nsub;
    bool wrote = false;
    for (int64_t r = 0; r < rounds; ++r) {
        const int64_t it = first + r * nsub;
        bool item = it < items;
        int32_t g = 0, h = 0, v = 0;
        if (item) {
            g = (int32_t)(it / hp.nheavy);
            h = (int32_t)(it - (int64_t)g * hp.nheavy);
            v = hp.heavy_vertex[h];
            item = fl.hmark_cur[(size_t)g * n + v] != 0;
        }
        bool changed = false;
        if (item) {
            const int32_t s = srcv[g * L + j];
            const size_t rv = sidx<L>(g, n, v, j);
            const double d_old = st.D[rv];
            const int32_t p_old = st.P[rv];
            Best b{d_old, p_old, -1, -1.0, false, p_old, rv};
            for (int32_t sgi = hp.heavy_seg0[h]; sgi < hp.heavy_seg0[h + 1]; ++sgi) {
                const size_t o = ((size_t)g * hp.nseg + sgi) * L + j;
                const int2 uk = pp.uk[o];
                if (uk.x >= 0) offer<L>(b, G, st, g, n, j, uk.y, uk.x, pp.du[o], pp.alt[o]);
            }
            if (j == 0) fl.hmark_cur[(size_t)g * n + v] = 0;
            changed = finish_vertex<L>(b, G, st, g, n, j, v, s, rv, d_old);
        }
        const bool any = ((__ballot(changed) >> base) & Sub<L>::MASK) != 0;
        if (any) {
            mark_out<L>(G, g, n, v, j, fl);
            wrote = true;
        }
    }
    if (__ballot(wrote) && lane == 0) *fl.any_changed = 1;
}

// ---- L = 64 * M sources per relaxation row, M > 1: each thread holds M lanes
// (j = lane, lane + 64, ...).  A row visit's fixed costs (frontier word, CSR
// chunk, in-edge flags, out-edge marks) are then shared by 64 M sources while
// the per-source work (the lanes of each neighbour row read, the own row, the
// route gathers and writes) scales with M; a CPU model of the schedule
// (tools/sim_schedules.py) and the measured L = 32 / 64 ratio put the lines
// touched per source ~13 % below L = 64 at L = 128.

template <int M, int INFL, typename F>
__device__ __forceinline__ void scan_chunk_m(uint64_t sm, int32_t c0, int32_t u_j, double w_j, int32_t g, int32_t n,
                                             int32_t lane, const bool (&active)[M], const State& st, F&& f) {
    constexpr int L = WAVE * M;
    while (sm) {
        int32_t us[INFL], ks[INFL];
        double ws[INFL], dus[INFL][M];
#pragma unroll
        for (int q = 0; q < INFL; ++q) {
            us[q] = -1;
            if (sm) {
                const int32_t b = __builtin_ctzll(sm);
                sm &= sm - 1;
                us[q] = __builtin_amdgcn_readlane(u_j, b);
                ws[q] = sub_get_d<WAVE>(w_j, b);
                ks[q] = c0 + b;
            }
        }
#pragma unroll
        for (int q = 0; q < INFL; ++q)
            if (us[q] >= 0) {
                const double* row = st.D + ((size_t)g * (size_t)n + (size_t)us[q]) * L;
#pragma unroll
                for (int m = 0; m < M; ++m) dus[q][m] = row[lane + m * WAVE];
            }
#pragma unroll
        for (int q = 0; q < INFL; ++q) {
            if (us[q] < 0) continue;
#pragma unroll
            for (int m = 0; m < M; ++m) {
                const double alt = dus[q][m] + ws[q];
                if (active[m] && alt > dus[q][m]) f(m, ks[q], us[q], dus[q][m], alt);
            }
        }
    }
}

// finish_vertex for the M lanes a thread carries: every lane's parent id, then
// every lane's parent route / edge factor / old route, are requested together,
// so the M lanes wait for two memory round trips instead of 2 M.
template <int M>
__device__ __forceinline__ bool finish_vertex_m(Best (&b)[M], const DevGraph& G, const State& st, int32_t g, int32_t n,
                                                int32_t lane, int32_t v, const int32_t (&s)[M],
                                                const double (&d_old)[M]) {
    constexpr int L = WAVE * M;
#pragma unroll
    for (int m = 0; m < M; ++m)
        if (b[m].need && b[m].bu < 0) b[m].bu = G.icol[b[m].bk];
    Route pu[M], old[M];
    double ia[M];
    bool same[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        same[m] = false;
        if (b[m].need) {
            pu[m] = st.RT[sidx<L>(g, n, b[m].bu, lane + m * WAVE)];
            ia[m] = G.ia[b[m].bk];
            // need with bd == d_old implies an equal offer, which read the stored parent
            same[m] = !(d_old[m] == INF || b[m].bd != d_old[m] || b[m].bk != b[m].pold);
            if (same[m]) old[m] = st.RT[b[m].rv];
        }
    }
    bool changed = false;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        if (!b[m].need) continue;
        Route nr;
        nr.r = pu[m].r * ia[m];
        nr.h = pu[m].h + 1;
        nr.f = (b[m].bu == s[m]) ? G.corev[v] : pu[m].f;
        const bool ch = !same[m] || nr.r != old[m].r || nr.h != old[m].h || nr.f != old[m].f;
        if (ch) {
            st.D[b[m].rv] = b[m].bd;
            st.P[b[m].rv] = b[m].bk;
            st.RT[b[m].rv] = nr;
        }
        changed |= ch;
    }
    return changed;
}

template <int M, int INFL, bool DELTA = false>
__device__ __forceinline__ bool relax_item_m(int64_t e, int32_t n, int32_t lane, const int32_t* __restrict__ srcv,
                                             const DevGraph& G, const State& st, const Flags& fl,
                                             const DeltaState& ds) {
    constexpr int L = WAVE * M;
    int32_t g = 0, v = 0, k0 = 0, k1 = 0;
    if (e >= 0) {
        g = (int32_t)(e / n);
        v = (int32_t)(e - (int64_t)g * n);
        k0 = G.iptr[v];
        k1 = G.iptr[v + 1];
    }
    Best b[M];
    int32_t s[M];
    double d_old[M];
    bool active[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int32_t j = lane + m * WAVE;
        s[m] = e >= 0 ? srcv[g * L + j] : -1;
        const size_t rv = sidx<L>(g, n, v, j);
        d_old[m] = e >= 0 ? st.D[rv] : INF;
        const int32_t p = d_old[m] < INF ? PK_UNREAD : -1;
        b[m] = Best{d_old[m], p, -1, -1.0, false, p, rv};
        active[m] = (e >= 0) && (s[m] != -1) && (s[m] != v);
    }
    const double bnd = (DELTA && e >= 0) ? ds.bound[g] : INF;
    double rej = INF;
    int32_t u_last = 0, orev_last = 0;
    bool heavy_last = false, ok_last = false;
    for (int32_t c0 = k0; c0 < k1; c0 += WAVE) {   // wave-uniform trip count
        const int32_t k = c0 + lane;
        const bool ok = k < k1;
        const int4 pk = ok ? G.ipack[k] : make_int4(0, 0, 0, 0);
        const int32_t u_j = pk.x;
        const double w_j = __hiloint2double(pk.w, pk.z);
        const size_t fo = (size_t)g * G.nrel + k;
        const bool f = ok && fl.in_cur[fo] != 0;
        if (G.undirected && ok) {
            orev_last = pk.y & 0x7FFFFFFF;
            heavy_last = pk.y < 0;
        }
        u_last = u_j;
        ok_last = ok;
        if (f) fl.in_cur[fo] = 0;   // consumed
        const uint64_t sm = __ballot(f);
        scan_chunk_m<M, INFL>(sm, c0, u_j, w_j, g, n, lane, active, st,
                              [&](int m, int32_t kk, int32_t u, double du, double alt) {
                                  if (DELTA && alt >= bnd) {   // beyond the group's bucket: deferred
                                      rej = fmin(rej, alt);
                                      return;
                                  }
                                  offer<L>(b[m], G, st, g, n, lane + m * WAVE, kk, u, du, alt);
                              });
    }
    bool changed = false;
    if (e >= 0) {
        if (G.ablate) {   // diagnostic builds only
#pragma unroll
            for (int m = 0; m < M; ++m)
                changed |= finish_vertex<L>(b[m], G, st, g, n, lane + m * WAVE, v, s[m], b[m].rv, d_old[m]);
        } else {
            changed = finish_vertex_m<M>(b, G, st, g, n, lane, v, s, d_old);
        }
    }
    if constexpr (DELTA) delta_note(ds, g, n, v, rej, __ballot(changed) != 0, e >= 0, lane);
    if (__ballot(changed)) {
        if (G.undirected && k1 - k0 <= WAVE) {
            if (ok_last) {
                (heavy_last ? fl.hmark_next : fl.mark_next)[(size_t)g * n + u_last] = 1;
                fl.in_next[(size_t)g * G.nrel + orev_last] = 1;
            }
        } else {
            mark_out<WAVE>(G, g, n, v, lane, fl);
        }
    }
    return changed;
}

template <int M, int INFL, int OCC = 1, bool DELTA = false>
__global__ __launch_bounds__(BLOCK, OCC) void k_relax_m(int32_t total, int32_t n, const int32_t* __restrict__ srcv,
                                                      DevGraph G, State st, Flags fl, DeltaState ds) {
    if (*fl.prev_changed == 0) return;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    uint64_t* words = reinterpret_cast<uint64_t*>(fl.mark_cur);
    const int64_t all_units = ((int64_t)total + 7) >> 3;
    const int32_t xcd = blockIdx.x & 7;
    const int64_t waves_per_xcd = ((int64_t)(gridDim.x >> 3) * BLOCK) >> 6;
    const int64_t wave = (int64_t)(blockIdx.x >> 3) * (BLOCK / WAVE) +
                         __builtin_amdgcn_readfirstlane((int32_t)(threadIdx.x >> 6));   // uniform: SGPRs
    const int64_t lo = all_units * xcd / 8, hi = all_units * (xcd + 1) / 8;
    bool wrote = false;
    int64_t u8 = lo + wave;
    uint64_t w_ahead = u8 < hi ? words[u8] : 0;
    for (; u8 < hi; u8 += waves_per_xcd) {
        const uint64_t w = uniform_u64(w_ahead);
        const int64_t nx = u8 + waves_per_xcd;
        w_ahead = nx < hi ? words[nx] : 0;
        if (!w) continue;
        if (lane == 0) words[u8] = 0;   // taken
        for (uint32_t bm = byte_mask(w); bm; bm &= bm - 1) {
            int64_t e = u8 * 8 + __builtin_ctz(bm);
            if (e >= total) e = -1;
            wrote |= relax_item_m<M, INFL, DELTA>(e, n, lane, srcv, G, st, fl, ds);
        }
    }
    if (__ballot(wrote) && lane == 0) *fl.any_changed = 1;
}

// ---- k_relax_s: the 128-lane relaxation with LDS-staged neighbour rows.
// k_relax_m's item is a chain of dependent memory round trips (frontier word ->
// in-CSR bounds -> in-list chunk and flags -> neighbour rows INFL at a time ->
// parent routes), and the kernel spends ~80 % of its wave cycles waiting on
// them.  Two of those trips go here:
//  * the in-CSR bounds of a frontier unit's eight vertices are fetched with the
//    unit's frontier word, one unit ahead, so an item issues its own distance
//    row, its in-list chunk and its in-edge flags in ONE round trip;
//  * the flagged neighbours' distance rows (1 KB each: 128 lanes x f64) are
//    gathered straight into a per-wave LDS ring by LDS-DMA
//    (global_load_lds_dwordx4: one wave instruction per row, no VGPR
//    destination), NS rows per round trip instead of INFL register-staged rows,
//    so a light vertex's flagged in-neighbours (4-5 on C3) arrive together and
//    the kernel holds fewer live registers.
// Offers, finish and marks are k_relax_m's (same canonical keys, same routes):
// the relaxation order changes nothing in the fixpoint.
// The ring kernel's per-lane relaxation state, leaner than Best: the lane's
// state index is recomputed where needed and the stored distance is not kept --
// whether the finish must write follows from two bits (the distance dropped; the
// lane was unreached) and the stored parent, read lazily as before.
struct Lean {
    double bd;      // best distance so far (starts at the stored one)
    double bdu;     // distance of the chosen parent (-1: not resolved yet)
    int32_t bk;     // in-CSR entry of the parent edge (PK_UNREAD / -1 none / -2 pendant seed)
    int32_t bu;     // parent vertex (-1: not resolved yet)
    int32_t pold;   // the stored parent once read (PK_UNREAD until then)
    uint32_t fl;    // LEAN_NEED | LEAN_DROP | LEAN_INF
};
constexpr uint32_t LEAN_NEED = 1u, LEAN_DROP = 2u, LEAN_INF = 4u;

template <int L>
__device__ __forceinline__ void offer_lean(Lean& b, const DevGraph& G, const State& st, int32_t g, int32_t n, int32_t v,
                                           int32_t j, int32_t kk, int32_t u, double du, double alt) {
    bool better = false;
    if (alt < b.bd) {
        better = true;
        b.fl |= LEAN_DROP;
    } else if (alt == b.bd) {
        if (b.bk == PK_UNREAD) b.bk = b.pold = st.P[sidx<L>(g, n, v, j)];
        if (kk == b.bk) {   // the current parent re-offers: refresh its route
            b.fl |= LEAN_NEED;
            b.bdu = du;
            b.bu = u;
        } else if (b.bk >= 0) {   // exact tie: canonical (d[u], u)
            if (b.bu < 0) b.bu = G.icol[b.bk];
            if (b.bdu < 0.0) b.bdu = st.D[sidx<L>(g, n, b.bu, j)];
            better = lex_less2(du, u, b.bdu, b.bu);
        }
    }
    b.bd = better ? alt : b.bd;
    b.bk = better ? kk : b.bk;
    b.bu = better ? u : b.bu;
    b.bdu = better ? du : b.bdu;
    b.fl |= better ? LEAN_NEED : 0u;
}

// finish_vertex_m on Lean lanes (same routes, same writes)
template <int M>
__device__ __forceinline__ bool finish_lean(Lean (&b)[M], const DevGraph& G, const State& st, int32_t g, int32_t n,
                                            int32_t lane, int32_t v, const int32_t (&s)[M]) {
    constexpr int L = WAVE * M;
    Route pu[M], old[M];
    double ia[M];
    bool same[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        same[m] = false;
        if (b[m].fl & LEAN_NEED) {
            pu[m] = st.RT[sidx<L>(g, n, b[m].bu, lane + m * WAVE)];
            ia[m] = G.ia[b[m].bk];
            // a refresh or a tie (no drop, reached before) read the stored parent
            same[m] = !(b[m].fl & (LEAN_DROP | LEAN_INF)) && b[m].bk == b[m].pold;
            if (same[m]) old[m] = st.RT[sidx<L>(g, n, v, lane + m * WAVE)];
        }
    }
    bool changed = false;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        if (!(b[m].fl & LEAN_NEED)) continue;
        Route nr;
        nr.r = pu[m].r * ia[m];
        nr.h = pu[m].h + 1;
        nr.f = (b[m].bu == s[m]) ? G.corev[v] : pu[m].f;
        const bool ch = !same[m] || nr.r != old[m].r || nr.h != old[m].h || nr.f != old[m].f;
        if (ch) {
            const size_t rv = sidx<L>(g, n, v, lane + m * WAVE);
            st.D[rv] = b[m].bd;
            st.P[rv] = b[m].bk;
            st.RT[rv] = nr;
        }
        changed |= ch;
    }
    return changed;
}

// Lean lanes on the degree-3 contracted graph (DevGraph.xw2 != NULL): an entry's
// parent of record (the canonical key) is core vertex xkey[k] -- x for a shortcut a ->
// v via x, whose distance is fl(d[a] + w1) -- while its route is gathered from the
// kept vertex a = icol[k].  Two shortcuts through the same x tie-break on x's own
// canonical parent: (d[a], a).
struct LeanX {
    double bd;
    double bdu;     // distance of the parent of record (-1: not resolved yet)
    int32_t bk;
    int32_t bu;     // kept vertex the route is gathered from (-1: not resolved yet)
    int32_t bkey;   // core id of the parent of record
    int32_t pold;
    uint32_t fl;
};

template <int L>
__device__ __forceinline__ void offer_leanx(LeanX& b, const DevGraph& G, const State& st, int32_t g, int32_t n,
                                            int32_t v, int32_t j, int32_t kk, int32_t u, int32_t key, double du,
                                            double drec, double alt) {
    bool better = false;
    if (alt < b.bd) {
        better = true;
        b.fl |= LEAN_DROP;
    } else if (alt == b.bd) {
        if (b.bk == PK_UNREAD) b.bk = b.pold = st.P[sidx<L>(g, n, v, j)];
        if (kk == b.bk) {
            b.fl |= LEAN_NEED;
            b.bdu = drec;
            b.bu = u;
            b.bkey = key;
        } else if (b.bk >= 0) {
            const int4 pb = G.ipack[b.bk];
            if (b.bu < 0) {
                b.bu = pb.x;
                b.bkey = G.xkey[b.bk];
            }
            const double da = st.D[sidx<L>(g, n, b.bu, j)];
            if (b.bdu < 0.0) b.bdu = (pb.y & 0x40000000) ? da + __hiloint2double(pb.w, pb.z) : da;
            better = (drec < b.bdu) | ((drec == b.bdu) & ((key < b.bkey) | ((key == b.bkey) & lex_less2(du, u, da, b.bu))));
        }
    }
    b.bd = better ? alt : b.bd;
    b.bk = better ? kk : b.bk;
    b.bu = better ? u : b.bu;
    b.bkey = better ? key : b.bkey;
    b.bdu = better ? drec : b.bdu;
    b.fl |= better ? LEAN_NEED : 0u;
}

template <int M>
__device__ __forceinline__ bool finish_leanx(LeanX (&b)[M], const DevGraph& G, const State& st, int32_t g, int32_t n,
                                             int32_t lane, int32_t v, const int32_t (&s)[M]) {
    constexpr int L = WAVE * M;
    Route pu[M], old[M];
    double a1[M], a2[M];
    int32_t via[M];
    bool same[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        same[m] = false;
        if (b[m].fl & LEAN_NEED) {
            pu[m] = st.RT[sidx<L>(g, n, b[m].bu, lane + m * WAVE)];
            a1[m] = G.ia[b[m].bk];
            a2[m] = G.xa2[b[m].bk];
            via[m] = G.xvia[b[m].bk];
            same[m] = !(b[m].fl & (LEAN_DROP | LEAN_INF)) && b[m].bk == b[m].pold;
            if (same[m]) old[m] = st.RT[sidx<L>(g, n, v, lane + m * WAVE)];
        }
    }
    bool changed = false;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        if (!(b[m].fl & LEAN_NEED)) continue;
        Route nr;
        nr.r = (pu[m].r * a1[m]) * a2[m];   // the path order: edge a -> x, then x -> v
        nr.h = pu[m].h + (via[m] >= 0 ? 2 : 1);
        nr.f = (b[m].bu == s[m]) ? (via[m] >= 0 ? via[m] : G.corev[v]) : pu[m].f;
        const bool ch = !same[m] || nr.r != old[m].r || nr.h != old[m].h || nr.f != old[m].f;
        if (ch) {
            const size_t rv = sidx<L>(g, n, v, lane + m * WAVE);
            st.D[rv] = b[m].bd;
            st.P[rv] = b[m].bk;
            st.RT[rv] = nr;
        }
        changed |= ch;
    }
    return changed;
}

template <int NS>
struct RelaxRing {
    double row[NS][2 * WAVE];   // one wave's LDS slots: 128 lanes of one neighbour row each
};

template <int NS, bool CX = false>
__device__ __forceinline__ bool relax_item_s(int64_t e, int32_t k0, int32_t k1, int32_t n, int32_t lane,
                                             const int32_t* __restrict__ srcv, const DevGraph& G, const State& st,
                                             const Flags& fl, RelaxRing<NS>* ring) {
    constexpr int M = 2, L = WAVE * M;
    using LaneT = typename std::conditional<CX, LeanX, Lean>::type;
    int32_t g = 0, v = 0;
    if (e >= 0) {
        g = (int32_t)(e / n);
        v = (int32_t)(e - (int64_t)g * n);
    } else {
        k0 = k1 = 0;
    }
    // round trip 1: sources, own row, in-list chunk, in-edge flags (all independent)
    const int32_t k = k0 + lane;
    const bool ok = k < k1;   // light vertex: in-degree <= 64, one chunk
    const int4 pk = ok ? G.ipack[k] : make_int4(0, 0, 0, 0);
    const size_t fo = (size_t)g * G.nrel + k;
    const bool f = ok && fl.in_cur[fo] != 0;
    double w2_j = 0.0;   // CX: second weight and parent-of-record key of the lane's entry
    int32_t key_j = 0;
    if constexpr (CX) {
        if (ok) {
            w2_j = G.xw2[k];
            key_j = G.xkey[k];
        }
    }
    LaneT b[M];
    int32_t s[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int32_t j = lane + m * WAVE;
        s[m] = e >= 0 ? srcv[g * L + j] : -1;
        b[m].bd = e >= 0 ? st.D[sidx<L>(g, n, v, j)] : INF;
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const bool reached = b[m].bd < INF;
        b[m].bk = b[m].pold = reached ? PK_UNREAD : -1;
        b[m].bu = -1;
        b[m].bdu = -1.0;
        b[m].fl = reached ? 0u : LEAN_INF;
        if constexpr (CX) b[m].bkey = -1;
    }
    const int32_t u_j = pk.x;
    const double w_j = __hiloint2double(pk.w, pk.z);
    if (f) fl.in_cur[fo] = 0;   // consumed
    uint64_t sm = __ballot(f);
    // round trip 2..: the flagged rows, NS per trip, into this wave's LDS ring
    const double* gbase = st.D + (size_t)g * (size_t)n * L;
    while (sm) {
        int32_t bs[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            bs[q] = -1;
            if (sm) {
                bs[q] = __builtin_ctzll(sm);
                sm &= sm - 1;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous trip's LDS reads are done
#pragma unroll
        for (int q = 0; q < NS; ++q)
            if (bs[q] >= 0) {
                const int32_t u = __builtin_amdgcn_readlane(u_j, bs[q]);
                const double* src = gbase + (size_t)u * L + 2 * lane;   // 16 B per lane: the whole 1-KB row
                __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)&ring->row[q][0], 16, 0, 0);
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            if (bs[q] < 0) continue;
            const int32_t u = __builtin_amdgcn_readlane(u_j, bs[q]);
            const double w = sub_get_d<WAVE>(w_j, bs[q]);
            const int32_t kk = k0 + bs[q];
            if constexpr (CX) {
                const double w2 = sub_get_d<WAVE>(w2_j, bs[q]);
                const int32_t key = __builtin_amdgcn_readlane(key_j, bs[q]);
                const bool sc = (__builtin_amdgcn_readlane(pk.y, bs[q]) & 0x40000000) != 0;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const double du = ring->row[q][lane + m * WAVE];
                    const double dx = du + w;           // the shortcut's x (a plain edge: the offer)
                    const double alt = dx + w2;         // + 0.0 for a plain edge: the same bits
                    const bool active = s[m] != -1 && s[m] != v;
                    if (active && alt > du)
                        offer_leanx<L>(b[m], G, st, g, n, v, lane + m * WAVE, kk, u, key, du, sc ? dx : du, alt);
                }
            } else {
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const double du = ring->row[q][lane + m * WAVE];
                    const double alt = du + w;
                    const bool active = s[m] != -1 && s[m] != v;   // (e < 0: s = -1)
                    if (active && alt > du) offer_lean<L>(b[m], G, st, g, n, v, lane + m * WAVE, kk, u, du, alt);
                }
            }
            // one slot's values live at a time: the next slot's LDS reads are not hoisted
            // above these offers (holding all NS rows in VGPRs costs occupancy)
            asm volatile("" ::: "memory");
        }
    }
    bool changed = false;
    if constexpr (CX) {
        if (e >= 0) changed = finish_leanx<M>(b, G, st, g, n, lane, v, s);
    } else {
        if (e >= 0) changed = finish_lean<M>(b, G, st, g, n, lane, v, s);
    }
    if (__ballot(changed)) {
        if (G.undirected) {   // the out-list IS the in-list: marks from registers
            if (ok) {
                const int32_t orev = pk.y & (CX ? 0x3FFFFFFF : 0x7FFFFFFF);
                (pk.y < 0 ? fl.hmark_next : fl.mark_next)[(size_t)g * n + u_j] = 1;
                fl.in_next[(size_t)g * G.nrel + orev] = 1;
            }
        } else {
            mark_out<WAVE>(G, g, n, v, lane, fl);
        }
    }
    return changed;
}

// in-CSR bounds (iptr[v], iptr[v + 1]) of item e = unit * 8 + lane, lanes 0..7
__device__ __forceinline__ int2 unit_bounds(int64_t unit, int32_t lane, int32_t total, int32_t n, const int32_t* iptr) {
    const int64_t e = unit * 8 + lane;
    if (lane >= 8 || e >= total) return make_int2(0, 0);
    const int32_t v = (int32_t)(e % n);
    return make_int2(iptr[v], iptr[v + 1]);
}

template <int NS, int OCC = 1, bool CX = false>
__global__ __launch_bounds__(BLOCK, OCC) void k_relax_s(int32_t total, int32_t n, const int32_t* __restrict__ srcv,
                                                      DevGraph G, State st, Flags fl) {
    __shared__ RelaxRing<NS> rings[BLOCK / WAVE];
    if (*fl.prev_changed == 0) return;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    // wave-uniform values made provably uniform (readfirstlane): the ring base, the
    // unit cursor and the (group, vertex) division then live in SGPRs, not VGPRs
    const int32_t wib = __builtin_amdgcn_readfirstlane((int32_t)(threadIdx.x >> 6));
    RelaxRing<NS>* ring = &rings[wib];
    uint64_t* words = reinterpret_cast<uint64_t*>(fl.mark_cur);
    const int64_t all_units = ((int64_t)total + 7) >> 3;
    const int32_t xcd = blockIdx.x & 7;
    const int64_t waves_per_xcd = ((int64_t)(gridDim.x >> 3) * BLOCK) >> 6;
    const int64_t wave = (int64_t)(blockIdx.x >> 3) * (BLOCK / WAVE) + wib;
    const int64_t lo = all_units * xcd / 8, hi = all_units * (xcd + 1) / 8;
    bool wrote = false;
    int64_t u8 = lo + wave;
    uint64_t w_ahead = u8 < hi ? words[u8] : 0;
    int2 b_ahead = u8 < hi ? unit_bounds(u8, lane, total, n, G.iptr) : make_int2(0, 0);
    for (; u8 < hi; u8 += waves_per_xcd) {
        const uint64_t w = uniform_u64(w_ahead);
        const int2 bnd = b_ahead;
        const int64_t nx = u8 + waves_per_xcd;
        w_ahead = nx < hi ? words[nx] : 0;
        b_ahead = nx < hi ? unit_bounds(nx, lane, total, n, G.iptr) : make_int2(0, 0);
        if (!w) continue;
        if (lane == 0) words[u8] = 0;   // taken
        for (uint32_t bm = byte_mask(w); bm; bm &= bm - 1) {
            const int32_t bit = __builtin_ctz(bm);
            int64_t e = u8 * 8 + bit;
            if (e >= total) e = -1;
            const int32_t k0 = __builtin_amdgcn_readlane(bnd.x, bit);
            const int32_t k1 = __builtin_amdgcn_readlane(bnd.y, bit);
            wrote |= relax_item_s<NS, CX>(e, k0, k1, n, lane, srcv, G, st, fl, ring);
        }
    }
    if (__ballot(wrote) && lane == 0) *fl.any_changed = 1;
}

#ifndef SPE_HEAVY_CX_INFL
#define SPE_HEAVY_CX_INFL 2   // flagged rows per round trip of the contracted heavy partial (A/B: 2 / 3 / 4 / 5 -> 61 / 68 / 72 / 72 ms of heavy passes per two C3 tables)
#endif
template <int M, int INFL, bool CX = false>
__global__ __launch_bounds__(BLOCK) void k_heavy_partial_m(int32_t groups, int32_t n, const int32_t* __restrict__ srcv,
                                                           DevGraph G, State st, HeavyPlan hp, Partial pp, Flags fl) {
    if (*fl.prev_changed == 0) return;
    constexpr int L = WAVE * M;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int64_t nw = ((int64_t)gridDim.x * BLOCK) >> 6;
    const int64_t items = (int64_t)groups * hp.nseg;
    const int64_t first = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
    for (int64_t it = first; it < items; it += nw) {   // wave-uniform
        const int32_t g = (int32_t)(it / hp.nseg);
        const int32_t sgi = (int32_t)(it - (int64_t)g * hp.nseg);
        const int32_t v = hp.seg_vertex[sgi];
        if (!fl.hmark_cur[(size_t)g * n + v]) continue;
        const int32_t kb = hp.seg_begin[sgi];
        const int32_t ke = min(kb + WAVE, G.iptr[v + 1]);
        bool active[M];
        double ba[M], bdu[M];
        int32_t bu[M], bk[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int32_t s = srcv[g * L + lane + m * WAVE];
            active[m] = (s != -1) && (s != v);
            ba[m] = INF;
            bdu[m] = INF;
            bu[m] = -1;
            bk[m] = -1;
        }
        const int32_t k = kb + lane;
        const bool ok = k < ke;
        const int4 pk = ok ? G.ipack[k] : make_int4(0, 0, 0, 0);
        const size_t fo = (size_t)g * G.nrel + k;
        const bool f = ok && fl.in_cur[fo] != 0;
        if (f) fl.in_cur[fo] = 0;
        if constexpr (CX) {   // contracted graph: shortcut entries, keys (alt, d[parent], parent, d[a], a)
            const double w2_j = ok ? G.xw2[k] : 0.0;
            const int32_t key_j = ok ? G.xkey[k] : 0;
            const double w1_j = __hiloint2double(pk.w, pk.z);
            double bda[M];
            int32_t bua[M];
#pragma unroll
            for (int m = 0; m < M; ++m) {
                bda[m] = INF;
                bua[m] = -1;
            }
            for (uint64_t sm = __ballot(f); sm;) {
                // INFL flagged rows per memory round trip (as scan_chunk_m)
                int32_t bs[INFL];
                double dus[INFL][M];
#pragma unroll
                for (int q = 0; q < INFL; ++q) {
                    bs[q] = -1;
                    if (sm) {
                        bs[q] = __builtin_ctzll(sm);
                        sm &= sm - 1;
                    }
                }
#pragma unroll
                for (int q = 0; q < INFL; ++q)
                    if (bs[q] >= 0) {
                        const int32_t u = __builtin_amdgcn_readlane(pk.x, bs[q]);
                        const double* row = st.D + ((size_t)g * (size_t)n + (size_t)u) * L;
#pragma unroll
                        for (int m = 0; m < M; ++m) dus[q][m] = row[lane + m * WAVE];
                    }
#pragma unroll
                for (int q = 0; q < INFL; ++q) {
                if (bs[q] < 0) continue;
                const int32_t b = bs[q];
                const int32_t u = __builtin_amdgcn_readlane(pk.x, b);
                const double w1 = sub_get_d<WAVE>(w1_j, b), w2 = sub_get_d<WAVE>(w2_j, b);
                const int32_t key = __builtin_amdgcn_readlane(key_j, b);
                const bool sc = (__builtin_amdgcn_readlane(pk.y, b) & 0x40000000) != 0;
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const double du = dus[q][m];
                    const double dx = du + w1, alt = dx + w2, drec = sc ? dx : du;
                    if (!(active[m] && alt > du)) continue;
                    const bool better =
                        (alt < ba[m]) |
                        ((alt == ba[m]) & ((drec < bdu[m]) | ((drec == bdu[m]) & ((key < bu[m]) |
                                                                                  ((key == bu[m]) & lex_less2(du, u, bda[m], bua[m]))))));
                    ba[m] = better ? alt : ba[m];
                    bdu[m] = better ? drec : bdu[m];
                    bu[m] = better ? key : bu[m];
                    bk[m] = better ? kb + b : bk[m];
                    bda[m] = better ? du : bda[m];
                    bua[m] = better ? u : bua[m];
                }
                }
            }
        } else {
            scan_chunk_m<M, INFL>(__ballot(f), kb, pk.x, __hiloint2double(pk.w, pk.z), g, n, lane, active, st,
                                  [&](int m, int32_t kk, int32_t u, double du, double alt) {
                                      const bool better = lex_less3(alt, du, u, ba[m], bdu[m], bu[m]);
                                      ba[m] = better ? alt : ba[m];
                                      bdu[m] = better ? du : bdu[m];
                                      bu[m] = better ? u : bu[m];
                                      bk[m] = better ? kk : bk[m];
                                  });
        }
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const size_t o = ((size_t)g * hp.nseg + sgi) * L + lane + m * WAVE;
            pp.alt[o] = ba[m];
            pp.du[o] = bdu[m];
            pp.uk[o] = make_int2(bu[m], bk[m]);
        }
    }
}

template <int M, bool CX = false>
__global__ __launch_bounds__(BLOCK) void k_heavy_combine_m(int32_t groups, int32_t n, const int32_t* __restrict__ srcv,
                                                           DevGraph G, State st, HeavyPlan hp, Partial pp, Flags fl) {
    if (*fl.prev_changed == 0) return;
    constexpr int L = WAVE * M;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int64_t nw = ((int64_t)gridDim.x * BLOCK) >> 6;
    const int64_t items = (int64_t)groups * hp.nheavy;
    const int64_t first = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
    bool wrote = false;
    for (int64_t it = first; it < items; it += nw) {   // wave-uniform
        const int32_t g = (int32_t)(it / hp.nheavy);
        const int32_t h = (int32_t)(it - (int64_t)g * hp.nheavy);
        const int32_t v = hp.heavy_vertex[h];
        if (!fl.hmark_cur[(size_t)g * n + v]) continue;
        bool changed = false;
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int32_t j = lane + m * WAVE;
            const int32_t s = srcv[g * L + j];
            const size_t rv = sidx<L>(g, n, v, j);
            const double d_old = st.D[rv];
            const int32_t p_old = st.P[rv];
            Best b{d_old, p_old, -1, -1.0, false, p_old, rv};
            for (int32_t sgi = hp.heavy_seg0[h]; sgi < hp.heavy_seg0[h + 1]; ++sgi) {
                const size_t o = ((size_t)g * hp.nseg + sgi) * L + j;
                const int2 uk = pp.uk[o];
                if (uk.x < 0) continue;
                if constexpr (CX) offer_x<L>(b, G, st, g, n, j, uk.y, uk.x, pp.du[o], pp.alt[o]);
                else offer<L>(b, G, st, g, n, j, uk.y, uk.x, pp.du[o], pp.alt[o]);
            }
            changed |= finish_vertex<L>(b, G, st, g, n, j, v, s, rv, d_old);
        }
        if (lane == 0) fl.hmark_cur[(size_t)g * n + v] = 0;
        if (__ballot(changed)) {
            mark_out<WAVE>(G, g, n, v, lane, fl);
            wrote = true;
        }
    }
    if (__ballot(wrote) && lane == 0) *fl.any_changed = 1;
}

// (s, s) entry: DIRECT self-loop, the row's [s] path, or the SELF rule.
__device__ __forceinline__ void self_entry(const DevGraph& G, const RowMode& md, int32_t s, double& L_,
                                           double& R, int32_t& N, int32_t& H) {
    const double fs = G.vfac[s];
    const double lw = G.loop_w[s];
    const bool loop = has_attr(lw);
    if (md.complete && !loop) return;                    // get_eid(s, s) fails: unroutable
    if ((md.complete || md.prefer) && loop) {            // _topology_lookupDirectPath(s, s)
        double r = 1.0;
        if (has_attr(fs)) r *= fs;
        if (has_attr(fs)) r *= fs;
        r *= G.loop_a[s];
        L_ = 0.0 + lw;
        R = r;
        N = s;
        H = 1;
    } else if (md.self_mode == SPE_SELF_ROW && loop) {   // path [s], shd-topology.c:1456-1484
        double r = 1.0;
        if (has_attr(fs)) r *= fs;
        r *= G.loop_a[s];
        double l = 0.0 + lw;
        if (l == 0) l = 1;
        L_ = l;
        R = r;
        N = s;
        H = 1;
    } else if (G.self_other[s] >= 0) {                   // SELF rule
        L_ = G.self_w2[s];
        R = G.self_a2[s];
        N = G.self_other[s];
        H = 2;
    }
}

// DIRECT (s, t != s): first edge s->t in the out-CSR (merged, get_eid's edge).
__device__ __forceinline__ bool direct_entry(const DevGraph& G, int32_t s, int32_t t, double& L_, double& R,
                                             int32_t& N, int32_t& H) {
    int32_t lo = G.dptr[s], hi = G.dptr[s + 1];
    while (lo < hi) {
        const int32_t mid = lo + ((hi - lo) >> 1);
        if (G.dcol[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= G.dptr[s + 1] || G.dcol[lo] != t) return false;
    const double fs = G.vfac[s], ft = G.vfac[t];
    double r = 1.0;
    if (has_attr(fs)) r *= fs;
    if (has_attr(ft)) r *= ft;
    r *= G.darep[lo];
    L_ = 0.0 + G.dwrep[lo];
    R = r;
    N = t;
    H = 1;
    return true;
}

// per-target constants of the row passes (host-built, SlotInfo[A]): one 32-B
// uniform load per target instead of a chain of dependent graph lookups
struct alignas(16) SlotInfo {
    int32_t t;      // attached vertex (original id)
    int32_t c;      // relaxation vertex the row reads: t itself or its pendant anchor
    int32_t kt;     // full in-CSR entry of t's pendant edge, -1 if t is a relaxation vertex
    int32_t fast;   // 1: t's vertex factor is absent or 1.0 (no path-order re-fold for it)
    double pw;      // latency of the pendant edge (relaxation weight), 0 otherwise
    double pa;      // 1 - p of the pendant edge (get_eid edge), 1 otherwise
};

// Path-order sum 0.0 + a_1 + a_2 + ... of the auxiliary edge attribute along the
// row's path to core vertex c (then the pendant target edge kt, if any), as the
// offline completion tool sums a path's jitters (compute-topology-paths.py:27-33).
// The path is walked back from c through the parent edges; up to 64 core edges
// are kept and folded forward, longer paths re-walk per edge (O(h^2)).
template <int L>
__device__ double aux_fold(const DevGraph& G, const State& st, int32_t g, int32_t n, int32_t j, int32_t s,
                           int32_t c, int32_t kt) {
    constexpr int KMAX = 64;
    int32_t ks[KMAX];
    int32_t nk = 0;
    bool pend_src = false, overflow = false;
    for (int32_t x = c;;) {
        const int32_t k = st.P[sidx<L>(g, n, x, j)];
        if (k == -1) break;             // x is the (core) source
        if (k == -2) {                  // x is the anchor of a pruned source: s -> x
            pend_src = true;
            break;
        }
        if (nk < KMAX) ks[nk] = k;
        else overflow = true;
        ++nk;
        x = G.icol[k];
    }
    double a = 0.0;
    if (pend_src) a += G.fiaux[G.fiptr[s]];
    if (!overflow) {
        for (int32_t q = nk - 1; q >= 0; --q) a += G.iaux[ks[q]];
    } else {
        for (int32_t q = nk - 1; q >= 0; --q) {   // edge q (0 = the last one, into c)
            int32_t x = c;
            for (int32_t r = 0; r < q; ++r) x = G.icol[st.P[sidx<L>(g, n, x, j)]];
            a += G.iaux[st.P[sidx<L>(g, n, x, j)]];
        }
    }
    if (kt >= 0) a += G.fiaux[kt];
    return a;
}

// State -> table rows.  One wave per (64-source block of the batch, target
// slot): lane l = source b*64 + l, i.e. lane group b*(64/L) + l/L, lane l%L.
#ifndef ROWS_ITEMS
#define ROWS_ITEMS 2
#endif
// SHARE (shared anchor trees): the state lanes are the batch's roots; rli[b * 64 + l]
// = {state lane of source b * 64 + l's root, its first hop (the anchor) or -1 for a
// core source} and rwa[.] = {pendant edge latency w, f_s * (1 - p)}: a pruned pendant
// source's row is its anchor's with the edge folded in front (latency w + d,
// reliability (f_s a) r, one more hop, first hop the anchor).
// (Here only for contracted shared tables; plain ones take k_rows_shared_lds.)
template <int L, bool AUX, bool SHARE = false>
__global__ __launch_bounds__(BLOCK) void k_rows_sssp(int32_t n, int32_t blocks, int32_t sb0,
                                                     const int32_t* __restrict__ srcv,
                                                     const SlotInfo* __restrict__ slots, DevGraph G,
                                                     RowMode md, State st, Table tb,
                                                     const int2* __restrict__ rli = nullptr,
                                                     const double2* __restrict__ rwa = nullptr) {
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int64_t items_all = (int64_t)blocks * tb.A;
    // XCD-contiguous slices (grid a multiple of 8; workgroups are dealt round-robin
    // over the 8 XCDs): one XCD's waves take consecutive items, so targets that
    // share a pendant anchor (adjacent slots) read that anchor's state row from
    // the same L2 instead of one XCD each.
    const bool xs = (gridDim.x & 7) == 0;
    const int32_t xcd = xs ? (int32_t)(blockIdx.x & 7) : 0;
    const int64_t nwaves = xs ? (((int64_t)(gridDim.x >> 3) * BLOCK) >> 6) : (((int64_t)gridDim.x * BLOCK) >> 6);
    const int64_t lo = xs ? items_all * xcd / 8 : 0;
    const int64_t items = xs ? items_all * (xcd + 1) / 8 : items_all;
    const int64_t wave0 = xs ? ((((int64_t)(blockIdx.x >> 3) * BLOCK + threadIdx.x) >> 6))
                             : ((((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6));
    // Two items per trip: every load both need (slot constants, source, the
    // target row's distance and route) is issued before either one's stores,
    // so a trip waits for two memory round trips, not four.
    struct In {
        int32_t b, jt, s;
        SlotInfo si;
        double dc;
        Route rc;
        int2 ri;       // SHARE: (root's state lane, first hop of a pendant source or -1)
    };
    constexpr int NI = ROWS_ITEMS;
    // SHARE: items run over tiles of BT consecutive source blocks, the blocks fastest:
    // the ~10 blocks whose sources share one lane group of roots then read a target's
    // root row from L2 one after the other instead of once per block sweep (each
    // item still writes one whole 1-KB record segment)
    constexpr int BT = SHARE ? 8 : 1;
    auto load1 = [&](int64_t i0, In (&dst)[NI]) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int64_t it = i0 + q * nwaves;
            In& x = dst[q];
            x.b = -1;
            if (it < items) {
                if constexpr (BT > 1) {
                    const int64_t tile = it / ((int64_t)BT * tb.A);
                    const int32_t b0 = (int32_t)tile * BT;
                    const int32_t bt = min(BT, blocks - b0);
                    const int64_t r = it - tile * BT * (int64_t)tb.A;
                    x.jt = (int32_t)(r / bt);
                    x.b = b0 + (int32_t)(r - (int64_t)x.jt * bt);
                } else {
                    x.b = (int32_t)(it / tb.A);
                    x.jt = (int32_t)(it - (int64_t)x.b * tb.A);
                }
                x.si = slots[x.jt];
                x.s = srcv[x.b * WAVE + lane];
                if constexpr (SHARE) x.ri = rli[x.b * WAVE + lane];
            }
        }
    };
    for (int64_t it0 = lo + wave0; it0 < items; it0 += NI * nwaves) {
        In in[NI];
        load1(it0, in);
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            In& x = in[q];
            x.dc = INF;
            if (x.b >= 0 && x.s >= 0 && x.si.t != x.s) {
                const int32_t sl = SHARE ? x.ri.x : x.b * WAVE + lane;   // state lane
                const int32_t g = sl / L, j = sl % L;
                if (x.si.c >= 0) {
                    const size_t rt = sidx<L>(g, n, x.si.c, j);
                    x.dc = st.D[rt];
                    x.rc = st.RT[rt];
                } else {   // a contracted target: the best of its three neighbours (d, then d[u], then u)
                    const int32_t r = -2 - x.si.c;
                    const int32_t u0 = G.rnb[3 * r], u1 = G.rnb[3 * r + 1], u2 = G.rnb[3 * r + 2];
                    const double d0 = st.D[sidx<L>(g, n, u0, j)], d1 = st.D[sidx<L>(g, n, u1, j)],
                                 d2 = st.D[sidx<L>(g, n, u2, j)];
                    const double a0 = d0 + G.rw[3 * r], a1 = d1 + G.rw[3 * r + 1], a2 = d2 + G.rw[3 * r + 2];
                    int32_t q = d0 < INF ? 0 : -1;
                    double bd = d0 < INF ? a0 : INF, bu = d0;
                    const bool t1 = (d1 < INF) & ((a1 < bd) | ((a1 == bd) & (d1 < bu)));   // (branch-free: lex_less3)
                    q = t1 ? 1 : q;
                    bd = t1 ? a1 : bd;
                    bu = t1 ? d1 : bu;
                    const bool t2 = (d2 < INF) & ((a2 < bd) | ((a2 == bd) & (d2 < bu)));
                    q = t2 ? 2 : q;
                    bd = t2 ? a2 : bd;
                    bu = t2 ? d2 : bu;
                    if (q >= 0) {
                        const Route rc = st.RT[sidx<L>(g, n, G.rnb[3 * r + q], j)];
                        x.dc = bd;
                        x.rc.r = rc.r * G.ra[3 * r + q];
                        x.rc.h = rc.h + 1;
                        x.rc.f = (rc.h == 0) ? x.si.t : rc.f;   // the neighbour is the source itself
                    }
                }
                if constexpr (SHARE) {
                    if (x.ri.y >= 0 && x.dc < INF) {   // a pruned pendant source: s -> anchor, then the root's path
                        const double2 wa = rwa[x.b * WAVE + lane];
                        x.dc = wa.x + x.dc;
                        x.rc.r = wa.y * x.rc.r;
                        x.rc.h = x.rc.h + 1;
                        x.rc.f = x.ri.y;
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const In& x = in[q];
            if (x.b < 0) continue;
            const int32_t b = x.b, jt = x.jt, s = x.s;
            const SlotInfo& si = x.si;
            const int32_t t = si.t;
            const int32_t g = (b * WAVE + lane) / L, j = (b * WAVE + lane) % L;   // (!SHARE: the re-fold walks)
            double Lt = -1.0, R = -1.0, AX = -1.0;
            int32_t N = -1, H = 0, PV = -1;
            if (s >= 0) {
                if (t == s) {
                    self_entry(G, md, s, Lt, R, N, H);
                    PV = (H == 2) ? N : (H > 0 ? s : -1);
                    AX = 0.0;
                } else {
                    // a pruned pendant target is one edge past its anchor: Dijkstra's
                    // d[t] = d[c] + w, parent c (its only candidate)
                    const int32_t c = si.c;
                    const int32_t kt = si.kt;
                    const size_t rt = sidx<L>(g, n, c, j);
                    const double dc = x.dc;
                    if (dc < INF) {
                        const Route rc = x.rc;
                        double d = dc;
                        Route rr = rc;
                        if (kt >= 0) {
                            d = dc + si.pw;
                            rr.r = rc.r * si.pa;
                            rr.h = rc.h + 1;
                            rr.f = (rc.h == 0) ? t : rc.f;   // c is the source itself
                        }
                        const bool fast = si.fast && !md.multi_rep;
                        if (fast) {
                            Lt = d;
                            R = rr.r;
                        } else {
                            // path-order re-fold, shd-topology.c:1413-1493 (rare: vertex loss on
                            // the target, or multigraph get_eid latencies).  Edge i of the path
                            // (1 = leaves the source) is found by walking back from t.
                            const double fs = G.vfac[s];
                            const double ft = G.vfac[t];
                            double l = 0.0, r = 1.0;
                            if (has_attr(fs)) r *= fs;
                            if (has_attr(ft)) r *= ft;
                            const int32_t h = rr.h;
                            for (int32_t i = 1; i <= h; ++i) {
                                int32_t back = h - i;   // edges to step over from the end
                                double ew, ea;
                                if (kt >= 0 && back == 0) {
                                    ew = G.fiwrep[kt];
                                    ea = G.fia[kt];
                                } else {
                                    int32_t x = c;
                                    if (kt >= 0) back -= 1;
                                    for (int32_t q = 0; q < back; ++q) x = G.icol[st.P[sidx<L>(g, n, x, j)]];
                                    const int32_t k = st.P[sidx<L>(g, n, x, j)];
                                    if (k >= 0) {
                                        ew = G.iwrep[k];
                                        ea = G.ia[k];
                                    } else {   // -2: the pendant source's edge into its anchor
                                        ew = G.fiwrep[G.fiptr[s]];
                                        ea = G.fia[G.fiptr[s]];
                                    }
                                }
                                l += ew;
                                r *= ea;
                            }
                            Lt = l;
                            R = r;
                        }
                        if (Lt == 0) Lt = 1;   // shd-topology.c:1833-1837
                        if constexpr (AUX) AX = aux_fold<L>(G, st, g, n, j, s, c, kt);
                        N = rr.f;
                        H = rr.h;
                        if (tb.prev) {
                            if (kt >= 0) {
                                PV = G.corev[c];
                            } else {
                                const int32_t pk = st.P[rt];
                                PV = pk >= 0 ? G.corev[G.icol[pk]] : s;   // -2: parent is the pendant source
                            }
                        }
                    }
                }
            }
            const size_t o = tidx(sb0 + b, tb.A, jt, lane);
            // the table is written once and not read during the build: stream it
            dvec2 e;
            e.x = Lt;
            e.y = R;
            __builtin_nontemporal_store(e, reinterpret_cast<dvec2*>(tb.lr + o));
            __builtin_nontemporal_store(N, tb.next + o);
            __builtin_nontemporal_store((uint16_t)(H > 65535 ? 65535 : H), tb.hops + o);
            if (tb.prev) tb.prev[o] = PV;
            if constexpr (AUX) tb.aux[o] = AX;
        }
    }
}


// Shared anchor trees, rows through LDS (plain relaxation graph, fast targets): a
// workgroup takes a tile of RT_B (16) consecutive source blocks x RT_T (4) consecutive
// targets.  The tile's sources read the root lanes [r0, r1] (rng[tile], host-built;
// roots are numbered in first-appearance order, so a tile's ~100 roots are
// consecutive lanes), so the workgroup first stages those lanes' distance and route
// for its RT_T targets in LDS -- every load of the tile in flight at once, one
// memory round trip -- and then writes the tile's 64-lane records from LDS (each
// wave one source block's targets in order: contiguous 1-KB record segments).
// A tile whose lane span exceeds RT_R takes the per-lane gathers of k_rows_sssp.
#ifndef SPE_RT_B
#define SPE_RT_B 16
#endif
#ifndef SPE_RT_T
#define SPE_RT_T 4
#endif
constexpr int RT_B = SPE_RT_B, RT_T = SPE_RT_T, RT_R = 24 * SPE_RT_B;

template <int L>
__global__ __launch_bounds__(BLOCK) void k_rows_shared_lds(int32_t n, int32_t blocks, int32_t sb0,
                                                           const int32_t* __restrict__ srcv,
                                                           const SlotInfo* __restrict__ slots, DevGraph G,
                                                           RowMode md, State st, Table tb,
                                                           const int2* __restrict__ rli,
                                                           const double2* __restrict__ rwa,
                                                           const int2* __restrict__ rng) {
    __shared__ double sD[RT_T][RT_R];
    __shared__ Route sR[RT_T][RT_R];
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int32_t wib = __builtin_amdgcn_readfirstlane((int32_t)(threadIdx.x >> 6));
    const int32_t ntiles = (blocks + RT_B - 1) / RT_B;
    const int32_t ntc = (tb.A + RT_T - 1) / RT_T;
    const int64_t work = (int64_t)ntiles * ntc;
    for (int64_t w = blockIdx.x; w < work; w += gridDim.x) {   // workgroup-uniform
        const int32_t tile = (int32_t)(w / ntc);
        const int32_t jt0 = (int32_t)(w - (int64_t)tile * ntc) * RT_T;
        const int32_t b0 = tile * RT_B, nb = min(RT_B, blocks - b0);
        const int32_t nt = min(RT_T, tb.A - jt0);
        const int2 rr = rng[tile];
        const int32_t nr = rr.y - rr.x + 1;
        const bool staged = nr > 0 && nr <= RT_R;
        if (staged) {
            for (int32_t i = threadIdx.x; i < nt * nr; i += BLOCK) {
                const int32_t tl = i / nr, q = i - tl * nr;
                const int32_t c = slots[jt0 + tl].c;
                const int32_t R = rr.x + q;
                double d = INF;
                Route rt{1.0, 0, -1};
                if (c >= 0) {
                    const size_t x = sidx<L>(R / L, n, c, R % L);
                    d = st.D[x];
                    rt = st.RT[x];
                }
                sD[tl][q] = d;
                sR[tl][q] = rt;
            }
        }
        __syncthreads();
        for (int32_t bl = wib; bl < nb; bl += BLOCK / WAVE) {
            const int32_t b = b0 + bl;
            const int32_t s = srcv[b * WAVE + lane];
            const int2 ri = rli[b * WAVE + lane];
            const double2 wa = rwa[b * WAVE + lane];
            for (int32_t tl = 0; tl < nt; ++tl) {
                const int32_t jt = jt0 + tl;
                const SlotInfo si = slots[jt];
                double Lt = -1.0, R = -1.0;
                int32_t N = -1, H = 0;
                if (s >= 0) {
                    if (si.t == s) {
                        self_entry(G, md, s, Lt, R, N, H);
                    } else {
                        double dc = INF;
                        Route rc{1.0, 0, -1};
                        if (staged) {
                            dc = sD[tl][ri.x - rr.x];
                            rc = sR[tl][ri.x - rr.x];
                        } else if (si.c >= 0) {
                            const size_t x = sidx<L>(ri.x / L, n, si.c, ri.x % L);
                            dc = st.D[x];
                            rc = st.RT[x];
                        }
                        if (dc < INF) {
                            if (ri.y >= 0) {   // a pruned pendant source: s -> anchor, then the root's path
                                dc = wa.x + dc;
                                rc.r = wa.y * rc.r;
                                rc.h = rc.h + 1;
                                rc.f = ri.y;
                            }
                            double d = dc;
                            Route rt2 = rc;
                            if (si.kt >= 0) {   // a pruned pendant target: one edge past its anchor
                                d = dc + si.pw;
                                rt2.r = rc.r * si.pa;
                                rt2.h = rc.h + 1;
                                rt2.f = (rc.h == 0) ? si.t : rc.f;
                            }
                            Lt = d == 0 ? 1.0 : d;   // shd-topology.c:1833-1837
                            R = rt2.r;
                            N = rt2.f;
                            H = rt2.h;
                        }
                    }
                }
                const size_t o = tidx(sb0 + b, tb.A, jt, lane);
                dvec2 e;
                e.x = Lt;
                e.y = R;
                __builtin_nontemporal_store(e, reinterpret_cast<dvec2*>(tb.lr + o));
                __builtin_nontemporal_store(N, tb.next + o);
                __builtin_nontemporal_store((uint16_t)(H > 65535 ? 65535 : H), tb.hops + o);
            }
        }
        __syncthreads();   // the next tile's staging overwrites sD / sR
    }
}

// Contracted shared tables: derived rows.  The relaxation lanes are
// the batch's roots (kept core sources, pendant anchors); a contracted source x (a
// removed degree-3 vertex whose three neighbours are all roots of the batch) takes
// no lane: every path from x leaves through one of its neighbours u_i, so
//   d_x(t) = min_i fl(w(x, u_i) + d_{u_i}(t)),  next hop u*, hops 1 + h_{u*}(t),
//   reliability a(x, u*) r_{u*}(t)
// (shd-topology.c:1741 runs one Dijkstra per source instead).  x's route is u*'s
// route behind the edge x -> u* exactly when u* wins by more than the rounding
// both sums carry and u*'s own decisions hold for the offset w(x, u*)
// (k_share_check); a source where the first test fails is flagged in `sunsafe`
// and its block is rebuilt one lane per source.  A removed TARGET y reads its three
// neighbours in the root's row (best by (d, d[u], u), as k_rows_sssp); for a
// source with an offset (pendant or derived) that choice is margin-checked too.
// Items are (tile of TT targets, source block) with the target tile slowest and
// XCD-contiguous: an XCD's resident waves work on the same few targets, so the
// state columns the derived sources gather (every root lane at those vertices)
// stay in that XCD's L2, and each wave writes TT consecutive 1-KB segments.
// One record per derived source, every per-source constant of its first legs
// (coalesced 16-B loads; no per-lane gathers from the graph or the lane -> vertex
// map).  A removed source has three legs, a degree-4 one four (lane -1: none).
constexpr int DER_K = 4;
struct alignas(16) DerivedSrc {
    int32_t lane[DER_K];   // root lanes of the neighbours, in core in-list order
    int32_t hop[DER_K];    // the neighbours' original ids (the first hop through each)
    double w[DER_K];       // latency of the edge x -> neighbour
    double a[DER_K];       // its 1 - p
};

__device__ __forceinline__ bool near_tie(double best, double alt, double wmin, double omax, double hmax) {
    const double h = wmin > 0.0 ? fmin(hmax, alt / wmin + 3.0) : hmax;
    return alt - best <= 4.5 * h * 0x1p-53 * (omax + alt);
}

// A root lane's value at a target: the relaxation vertex c's distance, or for a
// removed target (c = -2 - r) the expanded entry k_expand_removed wrote (the best
// of its three neighbours, its sign the margin flag); `tight` when an offset could
// change that choice (runner-up within the margin of k_share_check) -- only asked
// for sources with an offset.
struct RootVal {
    double d;
    bool tight;
};

template <int L>
__device__ __forceinline__ RootVal root_val(const State& st, const double* __restrict__ DX, int32_t n, int32_t nr,
                                            int32_t sl, int32_t c, bool check) {
    RootVal o;
    const int32_t g = sl / L, j = sl - (sl / L) * L;
    if (c >= 0) {
        o.d = st.D[sidx<L>(g, n, c, j)];
        o.tight = false;
    } else {
        const double x = DX[sidx<L>(g, nr, -2 - c, j)];
        o.d = __builtin_fabs(x);
        o.tight = check && __builtin_signbit(x);
    }
    return o;
}

// the route record a row continues: the relaxation state's, or a removed target's
// expanded one (the edge past the neighbour already folded in)
template <int L>
__device__ __forceinline__ const Route* root_route(const State& st, const Route* __restrict__ RTX, int32_t n,
                                                   int32_t nr, int32_t sl, int32_t c) {
    const int32_t g = sl / L, j = sl - (sl / L) * L;
    return c >= 0 ? st.RT + sidx<L>(g, n, c, j) : RTX + sidx<L>(g, nr, -2 - c, j);
}

// Contracted shared tables: every (root lane, removed vertex) entry once, before the
// rows -- the best of the removed vertex's three neighbours by (d, d[u], u) as
// k_rows_sssp chooses it, with the route one edge past that neighbour, and (sums
// not exact) the sign bit set when a runner-up is within the margin of an offset
// source (near_tie).  The rows kernel then reads one entry where every source that
// reads the lane (its own, and each derived source next to it: a hub's lane is read
// by thousands) re-did three gathers and the choice.  One wave per (lane group,
// removed vertex): three coalesced neighbour rows in, one row of DX and of RTX out.
template <int L>
__global__ __launch_bounds__(BLOCK) void k_expand_removed(int32_t groups, int32_t n, int32_t nr, DevGraph G, State st,
                                                          double* __restrict__ DX, Route* __restrict__ RTX,
                                                          const int32_t* __restrict__ rorig, int32_t check,
                                                          double wmin, double omax, double hmax) {
    constexpr int M = L / WAVE;
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int64_t items = (int64_t)groups * nr;
    const int64_t nw = ((int64_t)gridDim.x * BLOCK) >> 6;
    for (int64_t it = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6; it < items; it += nw) {   // wave-uniform
        const int32_t g = (int32_t)(it / nr), r = (int32_t)(it - (it / nr) * nr);
        const int32_t u0 = G.rnb[3 * r], u1 = G.rnb[3 * r + 1], u2 = G.rnb[3 * r + 2];
        const double w0 = G.rw[3 * r], w1 = G.rw[3 * r + 1], w2 = G.rw[3 * r + 2];
        double d0[M], d1[M], d2[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int32_t j = lane + m * WAVE;
            d0[m] = st.D[sidx<L>(g, n, u0, j)];
            d1[m] = st.D[sidx<L>(g, n, u1, j)];
            d2[m] = st.D[sidx<L>(g, n, u2, j)];
        }
        int32_t qq[M];
        double bb[M];
        bool tt[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const double a0 = d0[m] + w0, a1 = d1[m] + w1, a2 = d2[m] + w2;
            int32_t q = d0[m] < INF ? 0 : -1;
            double bd = d0[m] < INF ? a0 : INF, bu = d0[m];
            const bool t1 = (d1[m] < INF) & ((a1 < bd) | ((a1 == bd) & (d1[m] < bu)));   // (branch-free: lex_less3)
            q = t1 ? 1 : q;
            bd = t1 ? a1 : bd;
            bu = t1 ? d1[m] : bu;
            const bool t2 = (d2[m] < INF) & ((a2 < bd) | ((a2 == bd) & (d2[m] < bu)));
            q = t2 ? 2 : q;
            bd = t2 ? a2 : bd;
            bool t = false;
            if (check && q >= 0) {
                if (q != 0 && d0[m] < INF) t |= near_tie(bd, a0, wmin, omax, hmax);
                if (q != 1 && d1[m] < INF) t |= near_tie(bd, a1, wmin, omax, hmax);
                if (q != 2 && d2[m] < INF) t |= near_tie(bd, a2, wmin, omax, hmax);
            }
            qq[m] = q;
            bb[m] = bd;
            tt[m] = t;
        }
        Route rc[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            rc[m] = Route{1.0, 0, -1};
            if (qq[m] >= 0) rc[m] = st.RT[sidx<L>(g, n, qq[m] == 0 ? u0 : (qq[m] == 1 ? u1 : u2), lane + m * WAVE)];
        }
        const int32_t yo = rorig[r];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const size_t o = sidx<L>(g, nr, r, lane + m * WAVE);
            Route x = rc[m];
            if (qq[m] >= 0) {   // one edge past the neighbour taken
                x.r = rc[m].r * G.ra[3 * r + qq[m]];
                x.h = rc[m].h + 1;
                x.f = (rc[m].h == 0) ? yo : rc[m].f;   // the neighbour is the lane's root itself
            }
            DX[o] = qq[m] < 0 ? INF : (tt[m] ? -bb[m] : bb[m]);
            RTX[o] = x;
        }
    }
}

#ifndef SPE_DERIVED_TT
#define SPE_DERIVED_TT 3
#endif
// Each item's TT targets go through the load chain together -- slot constants
// (scalar), then every root-lane distance, then the chosen route records, then the
// stores -- so a wave waits for three memory round trips per item, not three per
// target (the stores could alias the state as far as the compiler knows, so
// target-at-a-time code serialises every target's chain behind the last one's stores).
#ifndef SPE_DERIVED_OCC
#define SPE_DERIVED_OCC 1
#endif
template <int L, int TT>
__global__ __launch_bounds__(BLOCK, SPE_DERIVED_OCC) void k_rows_derived(int32_t n, int32_t blocks, int32_t sb0,
                                                        const int32_t* __restrict__ srcv,
                                                        const SlotInfo* __restrict__ slots, DevGraph G,
                                                        RowMode md, State st, Table tb,
                                                        const int2* __restrict__ rli,
                                                        const double2* __restrict__ rwa,
                                                        const DerivedSrc* __restrict__ der,
                                                        const double* __restrict__ DX,
                                                        const Route* __restrict__ RTX, int32_t nr, double wmin,
                                                        double omax, double hmax, int32_t exact,
                                                        uint8_t* __restrict__ sunsafe) {
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int32_t ntt = (tb.A + TT - 1) / TT;
    const int64_t items_all = (int64_t)ntt * blocks;
    const bool xs = (gridDim.x & 7) == 0;
    const int32_t xcd = xs ? (int32_t)(blockIdx.x & 7) : 0;
    const int64_t nwaves = xs ? (((int64_t)(gridDim.x >> 3) * BLOCK) >> 6) : (((int64_t)gridDim.x * BLOCK) >> 6);
    const int64_t lo = xs ? items_all * xcd / 8 : 0;
    const int64_t items = xs ? items_all * (xcd + 1) / 8 : items_all;
    const int64_t wave0 = xs ? ((((int64_t)(blockIdx.x >> 3) * BLOCK + threadIdx.x) >> 6))
                             : ((((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6));
    for (int64_t it = lo + wave0; it < items; it += nwaves) {   // wave-uniform
        const int32_t tt = (int32_t)(it / blocks);
        const int32_t b = (int32_t)(it - (int64_t)tt * blocks);
        const int32_t s = srcv[b * WAVE + lane];
        const int2 ri = rli[b * WAVE + lane];
        const bool pend = ri.y >= 0, derv = ri.y <= -2;
        // the source's candidate first legs: a kept source reads its root lane with
        // offset 0 (core) or its pendant edge; a derived one its neighbours' lanes
        int32_t rl[DER_K], hq[DER_K];
        double wq[DER_K], aq[DER_K];
#pragma unroll
        for (int k = 0; k < DER_K; ++k) {
            rl[k] = k == 0 ? ri.x : -1;
            wq[k] = k == 0 ? 0.0 : INF;
            aq[k] = 1.0;
            hq[k] = -1;
        }
        if (pend) {
            const double2 wa = rwa[b * WAVE + lane];
            wq[0] = wa.x;
            aq[0] = wa.y;
            hq[0] = ri.y;
        }
        if (derv) {
            const DerivedSrc dx = der[-2 - ri.y];
#pragma unroll
            for (int k = 0; k < DER_K; ++k) {
                rl[k] = dx.lane[k];
                wq[k] = dx.w[k];
                aq[k] = dx.a[k];
                hq[k] = dx.hop[k];
            }
        }
        const bool chk = (pend || derv) && !exact;
        bool bad = false;
        SlotInfo si[TT];
        int32_t sc[TT];
        bool live[TT];
#pragma unroll
        for (int tl = 0; tl < TT; ++tl) {
            const int32_t jt = tt * TT + tl;
            si[tl] = slots[jt < tb.A ? jt : tb.A - 1];
            sc[tl] = si[tl].c;
            live[tl] = jt < tb.A && s >= 0 && si[tl].t != s;
        }
        RootVal v[TT][DER_K];
#pragma unroll
        for (int tl = 0; tl < TT; ++tl)
#pragma unroll
            for (int k = 0; k < DER_K; ++k) {
                if (live[tl] && rl[k] >= 0) {
                    v[tl][k] = root_val<L>(st, DX, n, nr, rl[k], sc[tl], chk);
                } else {
                    v[tl][k].d = INF;
                    v[tl][k].tight = false;
                }
            }
        // the first leg: min_k fl(w_k + d_k) (strict: the first of equal sums; a tie
        // flags the source anyway).  The winner's fields by selects (constant indices).
        double dd[TT];
        int32_t bk[TT], bl[TT];
#pragma unroll
        for (int tl = 0; tl < TT; ++tl) {
            double o[DER_K];
#pragma unroll
            for (int k = 0; k < DER_K; ++k) o[k] = wq[k] + v[tl][k].d;
            int32_t bi = 0;
            double bo = o[0];
#pragma unroll
            for (int k = 1; k < DER_K; ++k) {
                const bool tk = o[k] < bo;
                bi = tk ? k : bi;
                bo = tk ? o[k] : bo;
            }
            int32_t sl = 0;
            bool tg = false;
#pragma unroll
            for (int k = 0; k < DER_K; ++k) {
                sl = k == bi ? rl[k] : sl;
                tg = k == bi ? v[tl][k].tight : tg;
            }
            if (bo < INF) {
                if (derv) {   // u* must beat the other first hops by more than rounding (exact sums: strictly)
#pragma unroll
                    for (int k = 0; k < DER_K; ++k) {
                        if (exact) bad |= (k != bi) & (o[k] <= bo);
                        else if (k != bi && o[k] < INF) bad |= near_tie(bo, o[k], wmin, omax, hmax);
                    }
                }
                bad |= tg;
            }
            dd[tl] = bo;
            bk[tl] = bi;
            bl[tl] = sl < 0 ? 0 : sl;
        }
        Route rc[TT];
#pragma unroll
        for (int tl = 0; tl < TT; ++tl) {
            rc[tl] = Route{1.0, 0, -1};
            if (dd[tl] < INF) rc[tl] = *root_route<L>(st, RTX, n, nr, bl[tl], sc[tl]);
        }
#pragma unroll
        for (int tl = 0; tl < TT; ++tl) {
            const int32_t jt = tt * TT + tl;
            if (jt >= tb.A) break;
            const SlotInfo& sv = si[tl];
            double Lt = -1.0, R = -1.0;
            int32_t N = -1, H = 0;
            if (s >= 0) {
                if (sv.t == s) {
                    self_entry(G, md, s, Lt, R, N, H);
                } else if (dd[tl] < INF) {
                    const int32_t bi = bk[tl];
                    double d = dd[tl];
                    Route rt = rc[tl];
                    int32_t hop = -1;
                    double apre = 1.0;
#pragma unroll
                    for (int k = 0; k < DER_K; ++k) {
                        hop = k == bi ? hq[k] : hop;
                        apre = k == bi ? aq[k] : apre;
                    }
                    if (hop >= 0) {   // an offset source: its first edge in front
                        rt.r = apre * rt.r;
                        rt.h = rt.h + 1;
                        rt.f = hop;
                    }
                    if (sv.kt >= 0) {   // a pruned pendant target: one edge past its anchor
                        d = d + sv.pw;
                        rt.r = rt.r * sv.pa;
                        rt.f = (rt.h == 0) ? sv.t : rt.f;
                        rt.h = rt.h + 1;
                    }
                    Lt = d == 0 ? 1.0 : d;   // shd-topology.c:1833-1837
                    R = rt.r;
                    N = rt.f;
                    H = rt.h;
                }
            }
            const size_t o = tidx(sb0 + b, tb.A, jt, lane);
            dvec2 e;
            e.x = Lt;
            e.y = R;
            __builtin_nontemporal_store(e, reinterpret_cast<dvec2*>(tb.lr + o));
            __builtin_nontemporal_store(N, tb.next + o);
            __builtin_nontemporal_store((uint16_t)(H > 65535 ? 65535 : H), tb.hops + o);
        }
        if (bad) sunsafe[b * WAVE + lane] = 1;
    }
}

// Shared anchor trees: after a batch's relaxation over its roots, flag every root
// some of whose parent decisions a source offset could change.  A source s with
// offset o (its pendant edge, o <= omax) sums every path in the same order as its
// root but from o instead of 0; along a path of h edges each sum is within
// h u (o + d) of o + the exact sum (u = 2^-53), so a vertex whose parent's offer
// beats every other in-entry's offer alt by more than 4.5 H u (omax + alt) -- H
// bounding the edge count, alt / wmin + 3 -- keeps that parent, without a
// tie-break, for every such source; then every source's tree is the root's (DESIGN
// §4.1).  The test is per entry (alt - d - bound(alt) grows with alt, so the
// smallest competing offer fails it first), so in-lists split freely: one wave per
// (lane group, light vertex) or (lane group, 64-entry segment of a heavy vertex),
// four neighbour rows per round trip.
template <int L>
__global__ __launch_bounds__(BLOCK) void k_share_check(int32_t groups, int32_t n, const int32_t* __restrict__ srcv,
                                                       DevGraph G, State st, HeavyPlan hp, double wmin, double omax,
                                                       double hmax, uint8_t* __restrict__ unsafe) {
    constexpr int M = L > WAVE ? L / WAVE : 1;
    static_assert(L >= WAVE, "one lane group per wave");
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int64_t nw = ((int64_t)gridDim.x * BLOCK) >> 6;
    const int64_t light = (int64_t)groups * n;
    const int64_t items = light + (int64_t)groups * hp.nseg;
    for (int64_t it = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6; it < items; it += nw) {   // wave-uniform
        int32_t g, v, k0, k1;
        if (it < light) {
            g = (int32_t)(it / n);
            v = (int32_t)(it - (int64_t)g * n);
            k0 = G.iptr[v];
            k1 = G.iptr[v + 1];
            if (k1 - k0 > WAVE) continue;   // heavy: its segments below
        } else {
            const int64_t q = it - light;
            g = (int32_t)(q / hp.nseg);
            const int32_t sg = (int32_t)(q - (int64_t)g * hp.nseg);
            v = hp.seg_vertex[sg];
            k0 = hp.seg_begin[sg];
            k1 = min(k0 + WAVE, G.iptr[v + 1]);
        }
        double d[M];
        int32_t pk[M];
        bool act[M], any = false, bad[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const int32_t j = lane + m * WAVE;
            const size_t i = sidx<L>(g, n, v, j);
            d[m] = st.D[i];
            pk[m] = st.P[i];
            act[m] = srcv[g * L + j] >= 0 && d[m] < INF && pk[m] != -1;   // (-1: the root itself)
            bad[m] = false;
            any |= act[m];
        }
        if (!__ballot(any)) continue;
        const int32_t k = k0 + lane;
        const bool ok = k < k1;
        const int4 pkk = ok ? G.ipack[k] : make_int4(0, 0, 0, 0);
        const double w_j = __hiloint2double(pkk.w, pkk.z);
        const double w2_j = (G.xw2 && ok) ? G.xw2[k] : 0.0;
        const int32_t cnt = k1 - k0;
        for (int32_t q = 0; q < cnt; q += 4) {
            double du[4][M];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int32_t u = __builtin_amdgcn_readlane(pkk.x, min(q + r, cnt - 1));
#pragma unroll
                for (int m = 0; m < M; ++m) du[r][m] = st.D[sidx<L>(g, n, u, lane + m * WAVE)];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (q + r >= cnt) break;
                const double w = sub_get_d<WAVE>(w_j, q + r), w2 = sub_get_d<WAVE>(w2_j, q + r);
#pragma unroll
                for (int m = 0; m < M; ++m) {
                    const double alt = (du[r][m] + w) + w2;   // the relaxation's fold (+ 0.0: one add)
                    if (!act[m] || k0 + q + r == pk[m] || !(alt < INF)) continue;
                    const double h = wmin > 0.0 ? fmin(hmax, alt / wmin + 3.0) : hmax;
                    bad[m] |= alt - d[m] <= 4.5 * h * 0x1p-53 * (omax + alt);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < M; ++m)
            if (bad[m]) unsafe[(size_t)g * L + lane + m * WAVE] = 1;
    }
}

__global__ __launch_bounds__(BLOCK) void k_rows_direct(int32_t groups, int32_t sb0,
                                                       const int32_t* __restrict__ srcv,
                                                       const int32_t* __restrict__ slot_vertex, DevGraph G,
                                                       RowMode md, Table tb) {
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int64_t nwaves = ((int64_t)gridDim.x * BLOCK) >> 6;
    const int64_t items = (int64_t)groups * tb.A;
    for (int64_t it = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6; it < items; it += nwaves) {
        const int32_t g = (int32_t)(it / tb.A);
        const int32_t j = (int32_t)(it - (int64_t)g * tb.A);
        const int32_t t = slot_vertex[j];
        const int32_t s = srcv[g * WAVE + lane];
        double L = -1.0, R = -1.0;
        int32_t N = -1, H = 0;
        if (s >= 0) {
            if (t == s) self_entry(G, md, s, L, R, N, H);
            else direct_entry(G, s, t, L, R, N, H);
        }
        const size_t o = tidx(sb0 + g, tb.A, j, lane);
        tb.lr[o] = make_double2(L, R);
        tb.next[o] = N;
        tb.hops[o] = (uint16_t)H;
        if (tb.prev) tb.prev[o] = (H == 2) ? N : (H > 0 ? s : -1);
    }
}

// preferdirectpaths: every attached neighbour t of s takes the direct edge.
__global__ __launch_bounds__(BLOCK) void k_direct_overlay(int32_t groups, int32_t sb0,
                                                          const int32_t* __restrict__ srcv,
                                                          const int32_t* __restrict__ vertex_slot, DevGraph G,
                                                          Table tb) {
    const int32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= groups * WAVE) return;
    const int32_t g = i / WAVE, lane = i % WAVE;
    const int32_t s = srcv[i];
    if (s < 0) return;
    const double fs = G.vfac[s];
    for (int32_t k = G.dptr[s]; k < G.dptr[s + 1]; ++k) {
        const int32_t t = G.dcol[k];
        const int32_t j = vertex_slot[t];
        if (j < 0) continue;
        const double ft = G.vfac[t];
        double r = 1.0;
        if (has_attr(fs)) r *= fs;
        if (has_attr(ft)) r *= ft;
        r *= G.darep[k];
        const size_t o = tidx(sb0 + g, tb.A, j, lane);
        tb.lr[o] = make_double2(0.0 + G.dwrep[k], r);
        tb.next[o] = t;
        tb.hops[o] = 1;
        if (tb.prev) tb.prev[o] = s;
    }
}

// ------------------------------------------------------------------------
// LDS engine: one workgroup per source row with the row's relaxation state
// resident in LDS.  For graphs up to 10,240 relaxation vertices (Shadow's own
// topologies, C2) this replaces the 64-lane HBM-resident batch relaxation.
// Per source row:
//   1. push Bellman-Ford over a changed-vertex bitset: LDS 64-bit atomic min on
//      the distance bits (non-negative doubles order as integers); a wave takes
//      64 vertices and spreads their out-edges over its lanes (wave_expand), so
//      a round costs one global round trip per 64 edges, not one per edge;
//   2. canonical parent = argmin (d[u], u) over {u : fl(d[u] + w) == d[v]},
//      in-edges spread over lanes the same way, per-vertex argmin in LDS;
//   3. latencies of every target (d is final);
//   4. top-down over the parent tree by hop level, entirely in LDS: every
//      thread keeps its vertices' parent and parent-edge factor in registers and
//      a level settles each vertex whose parent settled in the previous one:
//      hops, the path-order reliability fold r(v) = r(parent) * (1 - p_e) and
//      the first hop, each computed once from the parent's final values;
//   5. reliability / next hop / hops of every target into the SB64 table.
// Distances are the least fixpoint of d[v] = min fl(d[u] + w), as in the batch
// engine, so rows are bit-identical (tests/test_gpu_lds.py).
constexpr int LDS_T = 1024;                 // threads per workgroup (16 waves)
constexpr int LDS_WAVES = LDS_T / WAVE;
constexpr int LDS_MAX_BYTES = 160 * 1024 - 1024;   // dynamic share; the rest covers static __shared__
constexpr int LDS_WL = 256;                 // per-wave marked-vertex list of the push pass
#ifndef LDS_WIN_N
#define LDS_WIN_N 3
#endif
constexpr int LDS_WIN = LDS_WIN_N;          // 64-edge windows per global round trip of the push pass
constexpr int LDS_CAND_BYTES = LDS_WAVES * (LDS_WL * 4 + LDS_WIN * WAVE);   // push lists + owner maps (H space)

__host__ __device__ constexpr size_t lds_align(size_t b) { return (b + 15) & ~(size_t)15; }
// D f64 | X i32 (out-row starts, then parent entry) | H u16 / argmin scratch | 2 bitsets
__host__ __device__ constexpr size_t lds_hs_bytes(int32_t nc) {
    return lds_align((size_t)nc * 2) > (size_t)LDS_CAND_BYTES ? lds_align((size_t)nc * 2) : (size_t)LDS_CAND_BYTES;
}
__host__ __device__ constexpr size_t lds_bytes(int32_t nc) {
    return lds_align((size_t)nc * 8) + lds_align((size_t)nc * 4) + lds_hs_bytes(nc) +
           2 * lds_align((size_t)((nc + 31) / 32) * 4);
}

// per-workgroup global scratch: the parent entries, kept for pass 5's rare
// path walks once the LDS parent array holds first hops
struct LdsScratch {
    int32_t* par;       // [grid][nc] in-CSR entry of each vertex's parent edge
};

// vertices per thread of the tree pass (registers): the LDS engine takes graphs
// of at most LDS_VPT * LDS_T = 10,240 relaxation vertices (C2's 9,998 fit; the
// register budget of 4 waves per SIMD leaves no room for 11)
constexpr int LDS_VPT = 10;

__device__ __forceinline__ int32_t par_vertex(const DevGraph& G, int32_t k) { return G.icol[k]; }

// Inclusive prefix sum over the wave in DPP (row shifts, then the two row
// broadcasts of the GFX9 DPP set): six VALU ops, where a shuffle-based scan is
// six dependent ds_bpermute round trips through the LDS crossbar.
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);    // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);    // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);    // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);    // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Spread the edges of up to 64 owner lanes (lane l owns `deg` consecutive
// items) over the wave's lanes, 64 at a time.  body(ok, o, off) runs with the
// whole wave (so it may shuffle): item `off` of owner lane `o`, ok = a real item.
template <typename F>
__device__ __forceinline__ void wave_expand(int32_t lane, int32_t deg, F&& body) {
    const int32_t incl = wave_incl_scan(deg);
    const int32_t total = __builtin_amdgcn_readlane(incl, WAVE - 1);
    const int32_t excl = incl - deg;
    for (int32_t base = 0; base < total; base += WAVE) {
        const int32_t e = base + lane;
        int32_t o = 0;
#pragma unroll
        for (int step = WAVE / 2; step; step >>= 1) {
            const int32_t y = __shfl(incl, o + step - 1);
            if (y <= e) o += step;
        }
        const int32_t off = e - __shfl(excl, o);
        body(e < total, o, off, base, excl, incl);
    }
}

// Workgroup-wide OR with ONE barrier (__syncthreads_or costs three): call ix
// ORs into flag[ix % 3] and thread 0 clears flag[(ix + 2) % 3], which every
// thread read before this call's barrier and nobody writes before call ix + 2.
// ix must be workgroup-uniform and increase by one per call; flags start zero.
__device__ __forceinline__ bool wg_any(bool p, uint32_t& ix, int32_t* flag) {
    const uint32_t k = ix % 3u;
    if (__ballot(p) && (threadIdx.x & (WAVE - 1)) == 0) flag[k] = 1;
    __syncthreads();
    const bool r = flag[k] != 0;
    if (threadIdx.x == 0) flag[(k + 2u) % 3u] = 0;
    ++ix;
    return r;
}

__global__ __launch_bounds__(LDS_T) void k_sssp_lds(int32_t slot0, int32_t slot1, const SlotInfo* __restrict__ slots,
                                                     int32_t blk0, DevGraph G, RowMode md, Table tb, LdsScratch sc_,
                                                     unsigned long long* __restrict__ dbg) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int32_t nc = G.n;
    const int32_t nw = (nc + 31) / 32;
    double* D = reinterpret_cast<double*>(smem);
    unsigned long long* Db = reinterpret_cast<unsigned long long*>(smem);
    int32_t* X = reinterpret_cast<int32_t*>(smem + lds_align((size_t)nc * 8));
    unsigned char* hs = smem + lds_align((size_t)nc * 8) + lds_align((size_t)nc * 4);
    uint16_t* H = reinterpret_cast<uint16_t*>(hs);
    uint32_t* F0 = reinterpret_cast<uint32_t*>(hs + lds_hs_bytes(nc));
    uint32_t* F1 = F0 + lds_align((size_t)nw * 4) / 4;
    // after the latency pass the distance space holds the reliability fold and X
    // (parent, first hop); the parent entries move to Xg
    double* Rl = D;
    __shared__ int32_t s_any[3];
    uint32_t syncix = 0;
    const int32_t tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid / WAVE;
    if (tid < 3) s_any[tid] = 0;   // (the first slot's init barrier publishes it)
    const unsigned long long INF_BITS = 0x7FF0000000000000ull;
    const int32_t oend = G.optr[nc];
    // Workgroups are dealt round-robin over the 8 XCDs; give the workgroups of
    // one XCD consecutive slots so the partial 512-B SB64 segments each row
    // writes meet in the same L2 before write-back.
    const int32_t gx = gridDim.x;
    const int32_t bx = (gx % 8 == 0) ? (blockIdx.x % 8) * (gx / 8) + blockIdx.x / 8 : blockIdx.x;
    int32_t* Xg = sc_.par + (size_t)blockIdx.x * nc;
    for (int32_t slot = slot0 + bx; slot < slot1; slot += gx) {
        const int32_t s = slots[slot].t;
        unsigned long long tph = dbg && tid == 0 ? wall_clock64() : 0, nround = 0, nlev = 0;
#define LDS_PHASE(i)                                                        \
    if (dbg && tid == 0) {                                                  \
        const unsigned long long now = wall_clock64();                      \
        atomicAdd(&dbg[i], now - tph);                                      \
        tph = now;                                                          \
    }
        const int32_t sc = G.core_id[s];
        const int32_t seed = sc >= 0 ? sc : G.anchor_core[s];
        for (int32_t v = tid; v < nc; v += LDS_T) {
            Db[v] = INF_BITS;
            X[v] = G.optr[v];
        }
        for (int32_t w = tid; w < nw; w += LDS_T) {
            F0[w] = 0;
            F1[w] = 0;
        }
        __syncthreads();
        if (tid == 0) {
            // pruned pendant source: its first step s -> anchor is fixed (see k_init_state)
            D[seed] = sc >= 0 ? 0.0 : 0.0 + G.fiw[G.fiptr[s]];
            F0[seed >> 5] = 1u << (seed & 31);
        }
        __syncthreads();
        LDS_PHASE(0)
        // 1. push relaxation to the fixpoint.  Each wave reads 64 bitset words at
        // once (words wave, wave+16, ...), lists their marked vertices (up to
        // 256), then spreads the listed vertices' out-edges over its lanes, two
        // 64-edge windows per global round trip.
        uint32_t* cur = F0;
        uint32_t* nxt = F1;
        int32_t* wl = reinterpret_cast<int32_t*>(hs) + wave * LDS_WL;   // H space is idle here
        uint8_t* om = hs + LDS_WAVES * LDS_WL * 4 + wave * LDS_WIN * WAVE;
        for (;;) {
            bool any = false;
            int32_t cnt = 0;   // wave-uniform list length
            unsigned long long tfl = 0;
            auto flush = [&]() {
                const unsigned long long tf0 = (dbg && tid == 0) ? wall_clock64() : 0;
                for (int32_t lb = 0; lb < cnt; lb += WAVE) {
                const int32_t v = lb + lane < cnt ? wl[lb + lane] : -1;
                int32_t k0 = 0, deg = 0;
                double dv = 0.0;
                if (v >= 0) {
                    k0 = X[v];
                    deg = (v + 1 < nc ? X[v + 1] : oend) - k0;
                    dv = D[v];
                }
                const int32_t incl = wave_incl_scan(deg);
                const int32_t total = __builtin_amdgcn_readlane(incl, WAVE - 1);
                const int32_t excl = incl - deg;
                for (int32_t base = 0; base < total; base += LDS_WIN * WAVE) {
                    int32_t x[LDS_WIN];
                    double cand[LDS_WIN], du[LDS_WIN];
                    bool ok[LDS_WIN];
                    // owner map of this window: each lane stamps its own edges
                    for (int32_t i = max(excl, base), ie = min(incl, base + LDS_WIN * WAVE); i < ie; ++i)
                        om[i - base] = (uint8_t)lane;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                    for (int h = 0; h < LDS_WIN; ++h) {
                        const int32_t e = base + h * WAVE + lane;
                        const int32_t o = e < total ? om[e - base] : 0;
                        ok[h] = e < total;
                        // unconditional loads (index clamped): every window's edges
                        // are in flight together, one wait for all of them
                        const int32_t kr = __shfl(k0, o) + e - __shfl(excl, o);
                        const int32_t k = ok[h] ? kr : 0;
                        du[h] = __shfl(dv, o);
                        x[h] = G.ocol[k];
                        cand[h] = G.ow[k];
                    }
#pragma unroll
                    for (int h = 0; h < LDS_WIN; ++h) cand[h] += du[h];
#pragma unroll
                    for (int h = 0; h < LDS_WIN; ++h) {
                        if (!ok[h]) continue;
                        const unsigned long long cb = (unsigned long long)__double_as_longlong(cand[h]);
                        if (cb < atomicMin(&Db[x[h]], cb)) {
                            atomicOr(&nxt[x[h] >> 5], 1u << (x[h] & 31));
                            any = true;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();   // owner map reads done before the next stamps
                }
                }
                cnt = 0;
                if (dbg && tid == 0) tfl += wall_clock64() - tf0;
            };
            for (int32_t w0 = wave; w0 < nw; w0 += LDS_WAVES * WAVE) {
                const int32_t wi = w0 + lane * LDS_WAVES;
                uint32_t W = wi < nw ? cur[wi] : 0u;
                uint64_t pend = __ballot(W != 0);
                if (!pend) continue;
                if (W) cur[wi] = 0;   // consumed (each word belongs to one wave)
                while (pend) {
                    const bool mine = (pend >> lane) & 1ull;
                    const int32_t c = mine ? __popc(W) : 0;
                    const int32_t incl = wave_incl_scan(c);
                    const bool fit = mine && incl <= LDS_WL - cnt;   // a prefix of the pending lanes
                    const uint64_t fm = __ballot(fit);
                    if (!fm) {   // list full: process it, then retry
                        flush();
                        continue;
                    }
                    if (fit) {
                        int32_t pos = cnt + incl - c;
                        for (uint32_t x = W; x; x &= x - 1) wl[pos++] = wi * 32 + __builtin_ctz(x);
                    }
                    cnt += __builtin_amdgcn_readlane(incl, 63 - __builtin_clzll(fm));
                    pend &= ~fm;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if (pend) flush();
                }
            }
            if (cnt) flush();
            ++nround;
            const unsigned long long tb0 = (dbg && tid == 0) ? wall_clock64() : 0;
            const bool more = wg_any(any, syncix, s_any);
            if (dbg && tid == 0) {
                atomicAdd(&dbg[11], tfl);
                atomicAdd(&dbg[12], wall_clock64() - tb0);
            }
            if (!more) break;
            uint32_t* tmp = cur;
            cur = nxt;
            nxt = tmp;
        }
        LDS_PHASE(1)
#ifdef SPE_LDS_PUSH_ONLY   // timing build (tools/gpu_pushonly.sh): the push alone, no rows
        continue;
#endif
        // 2. canonical parents: X[v] = in-CSR entry, -1 none (source), -2 pendant seed.
        // One flat pass over the in-CSR registers every valid candidate
        // (fl(d[u] + w) == d[v] > d[u]); a vertex with exactly one takes it, a
        // vertex with several (exact ties) rescans its in-list for argmin (d[u], u).
        // (Recording the push's improving edge and validating it instead was
        // measured slower: Gauss-Seidel reads make a vertex re-offer the value it
        // already gave, so equal offers cannot tell ties apart.)
        // Candidate counts are u16 halves of the (idle) H space, bumped by
        // non-returning LDS adds: a returning atomic per candidate would put an
        // LDS round trip on every valid in-entry.
        uint32_t* CNT = reinterpret_cast<uint32_t*>(hs);
        for (int32_t v = tid; v < nc; v += LDS_T) X[v] = (v == seed) ? (sc >= 0 ? -1 : -2) : -1;
        for (int32_t w = tid; w < (nc + 1) / 2; w += LDS_T) CNT[w] = 0;
        __syncthreads();
        {
            const int32_t m_rel = G.iptr[nc];
#ifndef LDS_PARENT_U
#define LDS_PARENT_U 8
#endif
            constexpr int U = LDS_PARENT_U;
            for (int32_t e0 = tid; e0 < m_rel; e0 += U * LDS_T) {
                int32_t u[U], v[U];
                double w[U];
#pragma unroll
                for (int q = 0; q < U; ++q) {   // unconditional (clamped) loads: all U in flight
                    const int32_t e = min(e0 + q * LDS_T, m_rel - 1);
                    const uint32_t uv = G.ipair[e];   // 12 B per entry instead of 16
                    u[q] = (int32_t)(uv & 0xFFFFu);
                    v[q] = (int32_t)(uv >> 16);
                    w[q] = G.iw[e];
                }
#pragma unroll
                for (int q = 0; q < U; ++q)
                    if (e0 + q * LDS_T >= m_rel) u[q] = -1;
#pragma unroll
                for (int q = 0; q < U; ++q) {
                    if (u[q] < 0 || v[q] == seed) continue;
                    const double du = D[u[q]], dv = D[v[q]];
                    const double alt = du + w[q];
                    if (du < INF && alt == dv && alt > du) {
                        X[v[q]] = e0 + q * LDS_T;   // the only writer unless the count says tie
                        atomicAdd(&CNT[v[q] >> 1], 1u << ((v[q] & 1) * 16));
                    }
                }
            }
        }
        __syncthreads();
        for (int32_t v = tid; v < nc; v += LDS_T) {   // exact ties: canonical argmin (d[u], u)
            if (((CNT[v >> 1] >> ((v & 1) * 16)) & 0xFFFFu) < 2u) continue;
            const double dv = D[v];
            double bdu = INF;
            int32_t bu = -1, bk = -1;
            for (int32_t k = G.iptr[v]; k < G.iptr[v + 1]; ++k) {
                const int32_t u = G.icol[k];
                const double du = D[u];
                if (!(du < INF)) continue;
                const double alt = du + G.iw[k];
                if (alt == dv && alt > du && (du < bdu || (du == bdu && u < bu))) {
                    bdu = du;
                    bu = u;
                    bk = k;
                }
            }
            X[v] = bk;
        }
        __syncthreads();
        LDS_PHASE(2)
        // 3. latencies (distances are final); unreachable targets complete here
        const int32_t sb_local = slot / WAVE - blk0, lane_s = slot % WAVE;
        // Targets go UR at a time: their slot records (and in pass 5 the next-hop
        // ids) are loaded together, one memory round trip per UR targets.
        constexpr int UR = 4;
        for (int32_t j0 = tid; j0 < tb.A; j0 += UR * LDS_T) {
        SlotInfo sv[UR];
#pragma unroll
        for (int q = 0; q < UR; ++q) sv[q] = slots[min(j0 + q * LDS_T, tb.A - 1)];
#pragma unroll
        for (int q = 0; q < UR; ++q) {
            const int32_t j = j0 + q * LDS_T;
            const SlotInfo& si = sv[q];
            if (j >= tb.A || si.t == s) continue;
            const size_t o = tidx(sb_local, tb.A, j, lane_s);
            if (Db[si.c] == INF_BITS) {
                tb.lr[o] = make_double2(-1.0, -1.0);
                tb.next[o] = -1;
                tb.hops[o] = 0;
                if (tb.prev) tb.prev[o] = -1;
            } else if (!md.multi_rep) {
                double l = si.kt >= 0 ? D[si.c] + si.pw : D[si.c];
                if (l == 0) l = 1;   // shd-topology.c:1833-1837
                tb.lr[o].x = l;
            }
        }
        }
        __syncthreads();
        LDS_PHASE(3)
        // 4. hops, first hop and the reliability fold over the parent tree.
        // Thread-owned vertices v = tid + i * LDS_T keep (parent, 1 - p of the
        // parent edge) in registers (relaxation-vertex ids: nc <= LDS_VPT * LDS_T
        // < 2^16).  Hops and first hop are integers, so pointer jumping gets them
        // exactly in ~log2(depth) rounds: W[v] = (jump << 16) | dist, "jump is
        // dist hops above v", ends at the terminal vertices (the seed's children
        // for a core source, the anchor seed for a pruned pendant source), whose
        // jump is themselves; then jump = the first hop and hops = dist + 1.  The
        // reliability product must fold in path order, so it runs top-down, one
        // barrier per hop level, each vertex at the level known from its hops.
        // X becomes W, then PF: first hop (high 16 bits, 0xFFFF = none) | parent.
        uint32_t* PF = reinterpret_cast<uint32_t*>(X);
        __shared__ uint32_t s_maxh;
        double pa[LDS_VPT];
        uint16_t par[LDS_VPT];
        uint32_t w[LDS_VPT];
        uint32_t todo = 0;
        const int32_t tpar = sc >= 0 ? seed : -1;   // a parent that makes its child terminal
#pragma unroll
        for (int i = 0; i < LDS_VPT; ++i) {
            const int32_t v = tid + i * LDS_T;
            int32_t k = -1;
            if (v < nc) {
                k = X[v];
                Xg[v] = k;
            }
            pa[i] = (double)k;   // the parent entry for now; its factor is loaded below
            par[i] = k >= 0 ? (uint16_t)par_vertex(G, k) : (uint16_t)0;
            if (k >= 0) todo |= 1u << i;
            w[i] = k < 0 ? ((v == seed && sc < 0) ? ((uint32_t)seed << 16) : 0xFFFFFFFFu)
                         : ((int32_t)par[i] == tpar ? ((uint32_t)v << 16) : (((uint32_t)par[i] << 16) | 1u));
        }
        if (tid == 0) s_maxh = 0;
        __syncthreads();   // every X read before W overwrites it
        uint32_t act = 0;
#pragma unroll
        for (int i = 0; i < LDS_VPT; ++i) {
            const int32_t v = tid + i * LDS_T;
            if (v < nc) PF[v] = w[i];
            if (((todo >> i) & 1u) && (w[i] >> 16) != (uint32_t)v) act |= 1u << i;
        }
        __syncthreads();
        LDS_PHASE(4)
        // parent-edge factors: requested here, first needed by the level pass, so
        // their latency hides behind the pointer jumping (unconditional, clamped)
#pragma unroll
        for (int i = 0; i < LDS_VPT; ++i) pa[i] = G.ia[((todo >> i) & 1u) ? (int32_t)pa[i] : 0];
        {
            auto wload = [&](uint32_t j) -> uint32_t {
                return __hip_atomic_load(PF + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            // in place and asynchronous: any (jump, dist) pair read is valid, so
            // composing with a newer one only shortens the chain
            for (;;) {
                uint32_t wj[LDS_VPT];
#pragma unroll
                for (int i = 0; i < LDS_VPT; ++i) wj[i] = ((act >> i) & 1u) ? wload(w[i] >> 16) : 0u;
#pragma unroll
                for (int i = 0; i < LDS_VPT; ++i) {
                    if (!((act >> i) & 1u)) continue;
                    const uint32_t j = w[i] >> 16;
                    if ((wj[i] >> 16) == j) {   // j is terminal: done
                        act &= ~(1u << i);
                    } else {
                        w[i] = (wj[i] & 0xFFFF0000u) | ((w[i] + wj[i]) & 0xFFFFu);
                        __hip_atomic_store(PF + tid + i * LDS_T, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (!wg_any(act != 0, syncix, s_any)) break;
            }
            uint32_t hmax = 0;
#pragma unroll
            for (int i = 0; i < LDS_VPT; ++i) {
                if (!((todo >> i) & 1u)) continue;
                const int32_t v = tid + i * LDS_T;
                const uint32_t h = (w[i] & 0xFFFFu) + 1u;
                H[v] = (uint16_t)h;
                PF[v] = (w[i] & 0xFFFF0000u) | par[i];
                w[i] = h;
                hmax = max(hmax, h);
            }
#pragma unroll
            for (int i = 0; i < LDS_VPT; ++i) {   // no parent: the seed or unreachable
                const int32_t v = tid + i * LDS_T;
                if (v < nc && !((todo >> i) & 1u)) {
                    H[v] = v == seed ? (sc >= 0 ? 0 : 1) : 0xFFFF;
                    PF[v] = (v == seed && sc < 0) ? (((uint32_t)seed << 16) | 0xFFFFu) : 0xFFFFFFFFu;
                }
            }
            for (int d = 1; d < WAVE; d <<= 1) hmax = max(hmax, (uint32_t)__shfl_xor((int)hmax, d));
            if (lane == 0 && hmax) atomicMax(&s_maxh, hmax);
            if (tid == 0) {
                const double fs = G.vfac[s];
                const double r0 = has_attr(fs) ? 1.0 * fs : 1.0;   // shd-topology.c:1428-1430
                Rl[seed] = sc >= 0 ? r0 : r0 * G.fia[G.fiptr[s]];
            }
            __syncthreads();
            const uint32_t levels = s_maxh;
            for (uint32_t l = 1; l <= levels; ++l) {
#pragma unroll
                for (int i = 0; i < LDS_VPT; ++i)
                    if (((todo >> i) & 1u) && w[i] == l) Rl[tid + i * LDS_T] = Rl[par[i]] * pa[i];
                __syncthreads();
            }
            nlev = levels;
        }
        LDS_PHASE(5)
        // 5. reliability, next hop, hops (+ latency re-fold for multigraphs)
        for (int32_t j0 = tid; j0 < tb.A; j0 += UR * LDS_T) {
        SlotInfo sv[UR];
        int32_t nh[UR];
#pragma unroll
        for (int q = 0; q < UR; ++q) sv[q] = slots[min(j0 + q * LDS_T, tb.A - 1)];
#pragma unroll
        for (int q = 0; q < UR; ++q) {
            const uint32_t fc = PF[sv[q].c] >> 16;
            nh[q] = G.corev[fc == 0xFFFFu ? 0u : fc];
        }
#pragma unroll
        for (int q = 0; q < UR; ++q) {
            const int32_t j = j0 + q * LDS_T;
            if (j >= tb.A) continue;
            const SlotInfo& si = sv[q];
            const int32_t t = si.t;
            const size_t o = tidx(sb_local, tb.A, j, lane_s);
            if (t == s) {
                double Lt = -1.0, R = -1.0;
                int32_t N = -1, Hh = 0;
                self_entry(G, md, s, Lt, R, N, Hh);
                tb.lr[o] = make_double2(Lt, R);
                tb.next[o] = N;
                tb.hops[o] = (uint16_t)Hh;
                if (tb.prev) tb.prev[o] = (Hh == 2) ? N : (Hh > 0 ? s : -1);
                continue;
            }
            const int32_t c = si.c, kt = si.kt;
            const uint16_t hc = H[c];
            if (hc == 0xFFFF) continue;   // unreachable: written in pass 3
            const int32_t Hh = hc + (kt >= 0 ? 1 : 0);
            double R;
            if (si.fast) {   // t's vertex factor absent or 1.0
                R = Rl[c] * si.pa;   // pa = 1.0 for relaxation vertices (exact)
            } else {   // ((1 * fs) * ft) * a1 * a2 ... : the target factor comes second
                const double ft = G.vfac[t];
                const double fs = G.vfac[s];
                double r = 1.0;
                if (has_attr(fs)) r *= fs;
                r *= ft;
                for (int32_t i = 1; i <= Hh; ++i) {
                    int32_t back = Hh - i;
                    double ea;
                    if (kt >= 0 && back == 0) {
                        ea = si.pa;
                    } else {
                        int32_t x = c;
                        if (kt >= 0) back -= 1;
                        for (int32_t q = 0; q < back; ++q) x = par_vertex(G, Xg[x]);
                        ea = Xg[x] >= 0 ? G.ia[Xg[x]] : G.fia[G.fiptr[s]];
                    }
                    r *= ea;
                }
                R = r;
            }
            if (md.multi_rep) {   // path-order re-fold of the get_eid latencies
                double l = 0.0;
                for (int32_t i = 1; i <= Hh; ++i) {
                    int32_t back = Hh - i;
                    double ew;
                    if (kt >= 0 && back == 0) {
                        ew = G.fiwrep[kt];
                    } else {
                        int32_t x = c;
                        if (kt >= 0) back -= 1;
                        for (int32_t q = 0; q < back; ++q) x = par_vertex(G, Xg[x]);
                        ew = Xg[x] >= 0 ? G.iwrep[Xg[x]] : G.fiwrep[G.fiptr[s]];
                    }
                    l += ew;
                }
                if (l == 0) l = 1;
                tb.lr[o].x = l;
            }
            tb.lr[o].y = R;
            const uint32_t fc = PF[c] >> 16;
            tb.next[o] = kt >= 0 && hc == 0 ? t : (fc == 0xFFFFu ? -1 : nh[q]);
            tb.hops[o] = (uint16_t)Hh;
            if (tb.prev) tb.prev[o] = kt >= 0 ? G.corev[c] : (Xg[c] >= 0 ? G.corev[par_vertex(G, Xg[c])] : s);
        }
        }
        __syncthreads();
        LDS_PHASE(6)
        if (dbg && tid == 0) {
            atomicAdd(&dbg[8], nround);
            atomicAdd(&dbg[9], nlev);
            atomicAdd(&dbg[10], 1ull);
        }
    }
#undef LDS_PHASE
}

// Owner replay (compat with the reference's first-writer-wins path cache,
// _topology_shouldStorePath shd-topology.c:1292-1321 + the either-direction
// lookup of _topology_getPathEntry :1952-2034): for each unordered slot pair,
// the source that ran first stores its path if it is not DIRECT and routable,
// the second stores only if the first did not; a non-DIRECT query answers its
// own stored path, else the reverse one (same latency / reliability / hops; next
// hop = the vertex before the querier on the owner's path when undirected, -1
// when directed), else fails.  One lane per pair (i < j): lane = i of a
// 64-slot block, wave = (block, j).
__device__ __forceinline__ bool has_edge(const DevGraph& G, int32_t a, int32_t b) {
    int32_t lo = G.dptr[a], hi = G.dptr[a + 1];
    while (lo < hi) {
        const int32_t mid = lo + ((hi - lo) >> 1);
        if (G.dcol[mid] < b) lo = mid + 1;
        else hi = mid;
    }
    return lo < G.dptr[a + 1] && G.dcol[lo] == b;
}

__global__ __launch_bounds__(BLOCK) void k_owner_replay(int32_t A, const int32_t* __restrict__ rank,
                                                        const int32_t* __restrict__ slot_vertex, DevGraph G,
                                                        RowMode md, Table tb) {
    const int32_t lane = threadIdx.x & (WAVE - 1);
    const int64_t nblk = (A + WAVE - 1) / WAVE;
    const int64_t items = nblk * A;
    const int64_t nwaves = ((int64_t)gridDim.x * BLOCK) >> 6;
    for (int64_t it = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6; it < items; it += nwaves) {
        const int32_t bi = (int32_t)(it / A);
        const int32_t j = (int32_t)(it - (int64_t)bi * A);
        const int32_t i = bi * WAVE + lane;
        if (i >= A || i >= j) continue;
        const int32_t vi = slot_vertex[i], vj = slot_vertex[j];
        const bool dij = md.prefer && has_edge(G, vi, vj);   // DIRECT, never cached
        const bool dji = md.prefer && has_edge(G, vj, vi);
        const size_t oij = tidx(bi, A, j, lane);
        const size_t oji = tidx(j / WAVE, A, i, j % WAVE);
        const bool i_first = rank[i] < rank[j];
        const size_t of = i_first ? oij : oji, oo = i_first ? oji : oij;
        const bool dfo = i_first ? dij : dji, dof = i_first ? dji : dij;
        const double2 ef = tb.lr[of], eo = tb.lr[oo];
        const double lf = ef.x, lo_ = eo.x;
        const bool sf = !dfo && lf > -1.0;                 // first runner stored (f, o)
        const bool so = !dof && lo_ > -1.0 && !sf;         // second stored (o, f)
        const double rf = ef.y, ro = eo.y;
        const uint16_t hf = tb.hops[of], ho = tb.hops[oo];
        const int32_t pf = tb.prev[of], po = tb.prev[oo];
        if (!dfo && !sf) {   // (f, o) answers the reverse path or fails
            tb.lr[of] = make_double2(so ? lo_ : -1.0, so ? ro : -1.0);
            tb.hops[of] = so ? ho : 0;
            tb.next[of] = (so && !md.directed) ? po : -1;
        }
        if (!dof && !so) {   // (o, f)
            tb.lr[oo] = make_double2(sf ? lf : -1.0, sf ? rf : -1.0);
            tb.hops[oo] = sf ? hf : 0;
            tb.next[oo] = (sf && !md.directed) ? pf : -1;
        }
    }
}


// Whole-table self-check (spe_table_check): one thread per SB64 entry (s, t),
// s != t.  Counters: [0] pairs, [1] unroutable, [2] bad values, [3] next hop not
// adjacent to s, [4] hop checks, [5] hop mismatches, [6] symmetry checks, [7]
// symmetry mismatches, [8] max relative asymmetry (f64 bits), [9] first bad pair
// (s << 32 | t, ~0 = none).  The checks are the per-target walk's consequences
// (shd-topology.c:1790-1849): the next hop is the path's second vertex, so it is
// adjacent to s, and on unique shortest paths hops(s, t) = 1 + hops(next, t);
// on an undirected graph lat(s, t) and lat(t, s) sum the same edges in opposite
// orders.
__device__ __forceinline__ void check_bad(unsigned long long* c, int32_t s, int32_t t) {
    atomicCAS(&c[9], ~0ull, ((unsigned long long)(uint32_t)s << 32) | (uint32_t)t);
}

__global__ __launch_bounds__(BLOCK) void k_table_check(int32_t A, const int32_t* __restrict__ slot_vertex,
                                                       const int32_t* __restrict__ vertex_slot, DevGraph G,
                                                       int32_t undirected, int32_t hop_rule, Table tb,
                                                       unsigned long long* __restrict__ c) {
    const int64_t total = (int64_t)((A + WAVE - 1) / WAVE) * A * WAVE;
    unsigned long long n[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double worst = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < total; i += (int64_t)gridDim.x * BLOCK) {
        const int32_t b = (int32_t)(i / ((int64_t)A * WAVE));
        const int64_t rem = i - (int64_t)b * A * WAVE;
        const int32_t ts = (int32_t)(rem / WAVE), ss = b * WAVE + (int32_t)(rem % WAVE);
        if (ss >= A || ss == ts) continue;
        ++n[0];
        const double2 e = tb.lr[i];
        if (!(e.x > -1.0)) {
            ++n[1];
            continue;
        }
        const int32_t sv = slot_vertex[ss], tv = slot_vertex[ts];
        const int32_t nx = tb.next[i];
        const int32_t h = tb.hops[i];
        bool bad = false;
        if (!(e.x > 0.0) || !(e.y > 0.0 && e.y <= 1.0) || h < 1 || nx < 0 || nx >= G.n_full) {
            ++n[2];
            bad = true;
        } else {
            if (!has_edge(G, sv, nx)) {
                ++n[3];
                bad = true;
            }
            const int32_t xs = vertex_slot[nx];
            if (hop_rule && xs >= 0 && nx != tv) {
                ++n[4];
                const int32_t h2 = tb.hops[tidx(xs / WAVE, A, ts, xs % WAVE)];
                if (h != 1 + h2) {
                    ++n[5];
                    bad = true;
                }
            }
            if (undirected) {
                ++n[6];
                const double2 r = tb.lr[tidx(ts / WAVE, A, ss, ts % WAVE)];
                const double dl = fabs(e.x - r.x) / e.x, dr = fabs(e.y - r.y) / e.y;
                const double d = fmax(dl, dr);
                worst = fmax(worst, d);
                if (!(d <= 1e-12)) {
                    ++n[7];
                    bad = true;
                }
            }
        }
        if (bad) check_bad(c, ss, ts);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        unsigned long long v = n[k];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & (WAVE - 1)) == 0 && v) atomicAdd(&c[k], v);
    }
    for (int o = 32; o > 0; o >>= 1) worst = fmax(worst, __shfl_xor(worst, o));
    if ((threadIdx.x & (WAVE - 1)) == 0 && worst > 0.0) atomicMax(&c[8], (unsigned long long)__double_as_longlong(worst));
}

template <int NT>
__global__ __launch_bounds__(BLOCK) void k_lookup(const int2* __restrict__ pairs, int64_t q, int32_t blk0,
                                                  int32_t blk1, Table tb, double* __restrict__ lat,
                                                  double* __restrict__ rel, uint8_t* __restrict__ ok) {
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < q; i += (int64_t)gridDim.x * BLOCK) {
        const int2 p = pairs[i];
        const int32_t sb = p.x >> 6;
        double L = -1.0, R = -1.0;
        if (p.x >= 0 && p.y >= 0 && p.y < tb.A && sb >= blk0 && sb < blk1) {
            const size_t o = tidx(sb - blk0, tb.A, p.y, p.x & (WAVE - 1));
            if constexpr (NT) {   // no L2 allocation for a record that is never re-read
                const dvec2 e = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(tb.lr + o));
                L = e.x;
                R = e.y;
            } else {
                const double2 e = tb.lr[o];
                L = e.x;
                R = e.y;
            }
        }
        if constexpr (NT) {
            __builtin_nontemporal_store(L, lat + i);
            __builtin_nontemporal_store(R, rel + i);
        } else {
            lat[i] = L;
            rel[i] = R;
        }
        ok[i] = L > -1.0 ? 1 : 0;   // topology_isRoutable: getLatency > -1
    }
}

// SB64 elements ((block - blk0) * A + t) * 64 + lane; lanes of the last block at
// or past A are padding (no source) and never count
__global__ __launch_bounds__(BLOCK) void k_min_latency(const double2* __restrict__ lr, int64_t elems, int32_t A,
                                                       int32_t blk0, unsigned long long* out) {
    double m = INF;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < elems; i += (int64_t)gridDim.x * BLOCK) {
        const int64_t slot = (i / ((int64_t)A * WAVE) + blk0) * WAVE + (i & (WAVE - 1));
        if (slot >= A) continue;
        const double l = lr[i].x;
        if (l > -1.0 && l < m) m = l;
    }
    for (int off = 32; off > 0; off >>= 1) m = fmin(m, __shfl_xor(m, off));
    if ((threadIdx.x & (WAVE - 1)) == 0 && m < INF)
        atomicMin(out, (unsigned long long)__double_as_longlong(m));  // positive doubles order as integers
}


// ------------------------------------------------------------------------
// Blocked min-plus Floyd-Warshall (the north star's dense C2 algorithm), kept as
// a measured comparison engine and an independent distance check: distances
// over the relaxation graph in FW association order (so within rounding of,
// not bit-equal to, the path-order folds the table holds) plus a next hop
// derived from them.  64 x 64 tiles, 256 threads, 4 x 4 elements per thread;
// per pivot block kb: the diagonal tile, then its row / column panels, then
// every other tile as a 64-deep min-plus product from two LDS-staged panels.
// FP64 VALU bound (add + min per relaxation; no MFMA: (min, +) is no FMA).
#define FWB 64
__device__ __forceinline__ void fw_load(double (*T)[FWB + 1], const double* __restrict__ D, int64_t ld, int32_t bi,
                                        int32_t bj) {
    for (int32_t e = threadIdx.x; e < FWB * FWB; e += 256) {
        const int32_t r = e / FWB, c = e % FWB;
        T[r][c] = D[((int64_t)bi * FWB + r) * ld + (int64_t)bj * FWB + c];
    }
}
__device__ __forceinline__ void fw_store(double (*T)[FWB + 1], double* __restrict__ D, int64_t ld, int32_t bi,
                                         int32_t bj) {
    for (int32_t e = threadIdx.x; e < FWB * FWB; e += 256) {
        const int32_t r = e / FWB, c = e % FWB;
        D[((int64_t)bi * FWB + r) * ld + (int64_t)bj * FWB + c] = T[r][c];
    }
}

__global__ __launch_bounds__(256) void k_fw_init(int32_t n, int64_t ld, DevGraph G, double* __restrict__ D) {
    const int64_t total = ld * ld;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int64_t i = e / ld, j = e % ld;
        D[e] = (i == j) ? 0.0 : INF;
    }
}
__global__ __launch_bounds__(256) void k_fw_edges(int32_t nrel, int64_t ld, DevGraph G, double* __restrict__ D) {
    const int32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k < nrel) D[(int64_t)G.icol[k] * ld + G.irow[k]] = G.iw[k];   // merged: one entry per ordered pair
}

// phase 1 (diagonal tile, launch with one block, b0 = 0) and phase 2 (its row /
// column panels, a second launch with b0 = 1): sequential in k
__global__ __launch_bounds__(256) void k_fw_panel(int32_t kb, int32_t nb, int64_t ld, double* __restrict__ D,
                                                  int32_t b0) {
    __shared__ double Dk[FWB][FWB + 1];
    __shared__ double T[FWB][FWB + 1];
    const int32_t b = b0 + blockIdx.x;   // 0: diagonal; 1..nb-1: row panel; nb..2nb-2: column panel
    fw_load(Dk, D, ld, kb, kb);
    __syncthreads();
    if (b == 0) {
        for (int32_t k = 0; k < FWB; ++k) {
            for (int32_t e = threadIdx.x; e < FWB * FWB; e += 256) {
                const int32_t r = e / FWB, c = e % FWB;
                const double a = Dk[r][k] + Dk[k][c];
                if (a < Dk[r][c]) Dk[r][c] = a;
            }
            __syncthreads();
        }
        fw_store(Dk, D, ld, kb, kb);
        return;
    }
    const bool row = b < nb;
    int32_t o = row ? b - 1 : b - nb;
    if (o >= kb) ++o;   // skip the diagonal
    if (row) fw_load(T, D, ld, kb, o);
    else fw_load(T, D, ld, o, kb);
    __syncthreads();
    for (int32_t k = 0; k < FWB; ++k) {
        for (int32_t e = threadIdx.x; e < FWB * FWB; e += 256) {
            const int32_t r = e / FWB, c = e % FWB;
            const double a = row ? Dk[r][k] + T[k][c] : T[r][k] + Dk[k][c];
            if (a < T[r][c]) T[r][c] = a;
        }
        __syncthreads();
    }
    if (row) fw_store(T, D, ld, kb, o);
    else fw_store(T, D, ld, o, kb);
}

// phase 3: every tile off the pivot row / column, 4 x 4 per thread in registers
__global__ __launch_bounds__(256) void k_fw_rest(int32_t kb, int32_t nb, int64_t ld, double* __restrict__ D) {
    __shared__ __align__(16) double At[FWB][FWB];   // At[k][r] = D(bi, kb)[r][k]
    __shared__ __align__(16) double Bk[FWB][FWB];   // Bk[k][c] = D(kb, bj)[k][c]
    int32_t bi = blockIdx.x / (nb - 1), bj = blockIdx.x % (nb - 1);
    if (bi >= kb) ++bi;
    if (bj >= kb) ++bj;
    for (int32_t e = threadIdx.x; e < FWB * FWB; e += 256) {
        const int32_t r = e / FWB, c = e % FWB;
        At[c][r] = D[((int64_t)bi * FWB + r) * ld + (int64_t)kb * FWB + c];
        Bk[r][c] = D[((int64_t)kb * FWB + r) * ld + (int64_t)bj * FWB + c];
    }
    const int32_t tx = threadIdx.x % 16, ty = threadIdx.x / 16;
    double d[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) d[r][c] = D[((int64_t)bi * FWB + ty * 4 + r) * ld + (int64_t)bj * FWB + tx * 4 + c];
    __syncthreads();
#pragma unroll 4
    for (int32_t k = 0; k < FWB; ++k) {
        const double2 a01 = *reinterpret_cast<const double2*>(&At[k][ty * 4]);
        const double2 a23 = *reinterpret_cast<const double2*>(&At[k][ty * 4 + 2]);
        const double2 b01 = *reinterpret_cast<const double2*>(&Bk[k][tx * 4]);
        const double2 b23 = *reinterpret_cast<const double2*>(&Bk[k][tx * 4 + 2]);
        const double a[4] = {a01.x, a01.y, a23.x, a23.y}, bb[4] = {b01.x, b01.y, b23.x, b23.y};
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) d[r][c] = fmin(d[r][c], a[r] + bb[c]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) D[((int64_t)bi * FWB + ty * 4 + r) * ld + (int64_t)bj * FWB + tx * 4 + c] = d[r][c];
}

// next hop from the closure: argmin over out-neighbours u of i of w(i,u) + D[u][j]
// (first minimum in out-list order); -1 when j is unreachable, j itself for i == j
__global__ __launch_bounds__(256) void k_fw_next(int32_t n, int64_t ld, DevGraph G, const double* __restrict__ D,
                                                 int32_t* __restrict__ nxt) {
    const int64_t total = (int64_t)n * n;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int32_t i = (int32_t)(e / n), j = (int32_t)(e % n);
        int32_t best = -1;
        if (i == j) {
            best = i;
        } else if (D[(int64_t)i * ld + j] < INF) {
            double bv = INF;
            for (int32_t k = G.optr[i]; k < G.optr[i + 1]; ++k) {
                const int32_t u = G.ocol[k];
                const double v = G.ow[k] + D[(int64_t)u * ld + j];
                if (v < bv) {
                    bv = v;
                    best = u;
                }
            }
        }
        nxt[(int64_t)i * n + j] = best;
    }
}

// ---- FW engine: the closure carries the (latency, reliability, next-hop) triple.
// D(i,j) distance, R(i,j) product of the edge factors (1 - p) of the path in FW's
// association order, N(i,j) the relaxation in-CSR entry of the path's FIRST edge
// (i -> y, y = irow[N]).  An update through pivot k (strict <, so the lowest k of
// a tie wins) sets D = D(i,k) + D(k,j), R = R(i,k) * R(k,j), N = N(i,k).  The
// table rows are then re-folded in path order from the walk along N
// (k_fw_state), which is what makes them bit-exact; R itself agrees with the
// path-order product only to rounding (tests: 1e-12 relative).
struct Fw3 {
    double* D;
    double* R;
    int32_t* N;
};
constexpr int FW3_LDS = 4 * FWB * FWB * 8 + FWB * FWB * 4;   // 144 KiB dynamic LDS (panel kernel)
constexpr int FW3_REST_LDS = FW3_LDS / 2;                      // 72 KiB: the rest kernel stages 32-deep halves
constexpr int64_t FW_MAX_N = 32768;   // FW engine: 20 B x n^2 of closure (21 GB at the cap)

__global__ __launch_bounds__(256) void k_fw3_init(int64_t ld, Fw3 M) {
    const int64_t total = ld * ld;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const bool diag = (e / ld) == (e % ld);
        M.D[e] = diag ? 0.0 : INF;
        M.R[e] = diag ? 1.0 : 0.0;
        M.N[e] = -1;
    }
}
__global__ __launch_bounds__(256) void k_fw3_edges(int32_t nrel, int64_t ld, DevGraph G, Fw3 M) {
    const int32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= nrel) return;
    const int32_t u = G.icol[k], v = G.irow[k];
    if (u == v) return;   // a loop never shortens a path (D(u,u) = 0)
    const int64_t e = (int64_t)u * ld + v;   // merged: one in-entry per ordered pair
    M.D[e] = G.iw[k];
    M.R[e] = G.ia[k];
    M.N[e] = k;
}

extern __shared__ __align__(16) unsigned char fw3_smem[];

// Phases 1 and 2 of pivot block kb.  X = the left operand tile (D, R, N), Y = the
// right one (D, R): diagonal: X = Y = the pivot tile, updated in place; row panel
// (kb, o): X = pivot, Y = the panel (its N in registers); column panel (o, kb):
// X = the panel, Y = pivot.  Row and column k of the updated tile do not change
// in step k (D(k,k) = 0), so in-place updates between barriers are race-free.
// Row blocks [rb0, rb1) are this launch's (a device's share of the closure's rows
// in the multi-device build; [0, nb) otherwise): the column panel covers only
// those, skipping the pivot block.
__device__ __forceinline__ int32_t fw_row_block(int32_t idx, int32_t kb, int32_t rb0, int32_t rb1) {
    const int32_t o = rb0 + idx;
    return (kb >= rb0 && kb < rb1 && o >= kb) ? o + 1 : o;
}

__global__ __launch_bounds__(256) void k_fw3_panel(int32_t kb, int32_t nb, int64_t ld, Fw3 M, int32_t b0,
                                                   int32_t rb0, int32_t rb1) {
    double* XD = reinterpret_cast<double*>(fw3_smem);
    double* XR = XD + FWB * FWB;
    double* YD = XR + FWB * FWB;
    double* YR = YD + FWB * FWB;
    int32_t* XN = reinterpret_cast<int32_t*>(YR + FWB * FWB);
    const int32_t b = b0 + blockIdx.x;
    const int32_t mode = b == 0 ? 0 : (b < nb ? 1 : 2);   // 0 diagonal, 1 row panel, 2 column panel
    int32_t o = b - 1;
    if (mode == 1 && o >= kb) ++o;
    if (mode == 2) o = fw_row_block(b - nb, kb, rb0, rb1);
    const int32_t xi = mode == 2 ? o : kb, xj = kb;   // X tile
    const int32_t yi = kb, yj = mode == 1 ? o : kb;   // Y tile
    int32_t myN[16];
    for (int32_t q = 0; q < 16; ++q) {
        const int32_t e = threadIdx.x + 256 * q, r = e / FWB, c = e % FWB;
        const int64_t gx = ((int64_t)xi * FWB + r) * ld + (int64_t)xj * FWB + c;
        XD[e] = M.D[gx];
        XR[e] = M.R[gx];
        XN[e] = M.N[gx];
        if (mode) {
            const int64_t gy = ((int64_t)yi * FWB + r) * ld + (int64_t)yj * FWB + c;
            YD[e] = M.D[gy];
            YR[e] = M.R[gy];
            if (mode == 1) myN[q] = M.N[gy];
        }
    }
    __syncthreads();
    const double* RD = mode ? YD : XD;   // right operand
    const double* RR = mode ? YR : XR;
    for (int32_t k = 0; k < FWB; ++k) {
#pragma unroll 4
        for (int32_t q = 0; q < 16; ++q) {
            const int32_t e = threadIdx.x + 256 * q, r = e / FWB, c = e % FWB;
            const double a = XD[r * FWB + k] + RD[k * FWB + c];
            if (mode == 1) {
                if (a < YD[e]) {
                    YD[e] = a;
                    YR[e] = XR[r * FWB + k] * RR[k * FWB + c];
                    myN[q] = XN[r * FWB + k];
                }
            } else if (a < XD[e]) {
                XR[e] = XR[r * FWB + k] * RR[k * FWB + c];
                XN[e] = XN[r * FWB + k];
                XD[e] = a;
            }
        }
        __syncthreads();
    }
    for (int32_t q = 0; q < 16; ++q) {
        const int32_t e = threadIdx.x + 256 * q, r = e / FWB, c = e % FWB;
        if (mode == 1) {
            const int64_t gy = ((int64_t)yi * FWB + r) * ld + (int64_t)yj * FWB + c;
            M.D[gy] = YD[e];
            M.R[gy] = YR[e];
            M.N[gy] = myN[q];
        } else {
            const int64_t gx = ((int64_t)xi * FWB + r) * ld + (int64_t)xj * FWB + c;
            M.D[gx] = XD[e];
            M.R[gx] = XR[e];
            M.N[gx] = XN[e];
        }
    }
}

// Phase 3: every tile off the pivot row / column, a 64-deep (min, +) product of
// the two LDS-staged panels carrying R and N; 4 x 4 elements per thread.
__global__ __launch_bounds__(256) void k_fw3_rest(int32_t kb, int32_t nb, int64_t ld, Fw3 M, int32_t rb0,
                                                  int32_t rb1) {
    // the 64-deep product in two 32-deep halves: 72 KiB of panels, two workgroups per CU
    constexpr int KH = FWB / 2;
    double* AD = reinterpret_cast<double*>(fw3_smem);   // [k][r] of tile (bi, kb), this half's k
    double* AR = AD + KH * FWB;
    double* BD = AR + KH * FWB;                          // [k][c] of tile (kb, bj)
    double* BR = BD + KH * FWB;
    int32_t* AN = reinterpret_cast<int32_t*>(BR + KH * FWB);
    const int32_t bi = fw_row_block(blockIdx.x / (nb - 1), kb, rb0, rb1);
    int32_t bj = blockIdx.x % (nb - 1);
    if (bj >= kb) ++bj;
    const int32_t tx = threadIdx.x % 16, ty = threadIdx.x / 16;
    double d[4][4], rr[4][4];
    int32_t nn[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int64_t gi = ((int64_t)bi * FWB + ty * 4 + r) * ld + (int64_t)bj * FWB + tx * 4 + c;
            d[r][c] = M.D[gi];
            rr[r][c] = M.R[gi];
            nn[r][c] = M.N[gi];
        }
    for (int32_t h = 0; h < 2; ++h) {
        if (h) __syncthreads();   // the first half's panels are read
        for (int32_t e = threadIdx.x; e < KH * FWB; e += 256) {
            const int32_t r = e / KH, c = e % KH;      // A: row r of the tile, column h*KH + c
            const int64_t ga = ((int64_t)bi * FWB + r) * ld + (int64_t)kb * FWB + h * KH + c;
            AD[c * FWB + r] = M.D[ga];
            AR[c * FWB + r] = M.R[ga];
            AN[c * FWB + r] = M.N[ga];
            const int32_t rb = e / FWB, cb = e % FWB;  // B: row h*KH + rb of the pivot panel
            const int64_t gb = ((int64_t)kb * FWB + h * KH + rb) * ld + (int64_t)bj * FWB + cb;
            BD[e] = M.D[gb];
            BR[e] = M.R[gb];
        }
        __syncthreads();
#pragma unroll 2
        for (int32_t k = 0; k < KH; ++k) {
            const double2 a01 = *reinterpret_cast<const double2*>(&AD[k * FWB + ty * 4]);
            const double2 a23 = *reinterpret_cast<const double2*>(&AD[k * FWB + ty * 4 + 2]);
            const double2 b01 = *reinterpret_cast<const double2*>(&BD[k * FWB + tx * 4]);
            const double2 b23 = *reinterpret_cast<const double2*>(&BD[k * FWB + tx * 4 + 2]);
            const double a[4] = {a01.x, a01.y, a23.x, a23.y};
            const double bb[4] = {b01.x, b01.y, b23.x, b23.y};
            double x[4][4];
            bool up[4][4], any = false;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    x[r][c] = a[r] + bb[c];
                    up[r][c] = x[r][c] < d[r][c];
                    any |= up[r][c];
                }
            // Improvements get rare after the first pivots: the reliability and
            // first-edge panels are read from LDS, and the products and selects done,
            // only by waves with an improvement at this k (the common step is the
            // distance-only closure's: two panel reads, add + compare).
            if (__ballot(any)) {
                const double2 r01 = *reinterpret_cast<const double2*>(&AR[k * FWB + ty * 4]);
                const double2 r23 = *reinterpret_cast<const double2*>(&AR[k * FWB + ty * 4 + 2]);
                const int4 an4 = *reinterpret_cast<const int4*>(&AN[k * FWB + ty * 4]);
                const double2 s01 = *reinterpret_cast<const double2*>(&BR[k * FWB + tx * 4]);
                const double2 s23 = *reinterpret_cast<const double2*>(&BR[k * FWB + tx * 4 + 2]);
                const double ar[4] = {r01.x, r01.y, r23.x, r23.y}, br[4] = {s01.x, s01.y, s23.x, s23.y};
                const int32_t an[4] = {an4.x, an4.y, an4.z, an4.w};
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        d[r][c] = up[r][c] ? x[r][c] : d[r][c];
                        rr[r][c] = up[r][c] ? ar[r] * br[c] : rr[r][c];
                        nn[r][c] = up[r][c] ? an[r] : nn[r][c];
                    }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int64_t gi = ((int64_t)bi * FWB + ty * 4 + r) * ld + (int64_t)bj * FWB + tx * 4 + c;
            M.D[gi] = d[r][c];
            M.R[gi] = rr[r][c];
            M.N[gi] = nn[r][c];
        }
}

// FW engine: the batch state (D, P, RT per (group, vertex, lane), as the batch
// engine's relaxation leaves it) from the closure, by walking each (source,
// vertex) path along N and folding it in path order from the source: latency
// 0.0 + w1 + w2 + ..., reliability from the source factor, hops, first hop, and
// the last edge as the parent entry.  On graphs without equal-length paths the
// walk is the Dijkstra tree path, so the rows k_rows_sssp writes from this state
// are the batch engine's, bit for bit.  Workgroup = 64 vertices x one group;
// wave w walks lanes (sources) w, w+4, ...; a lane's 64 walks start on one N row.
__global__ __launch_bounds__(256) void k_fw_state(int32_t n, int64_t ld, const int32_t* __restrict__ srcv,
                                                  const int32_t* __restrict__ srcc, DevGraph G, Fw3 M, State st) {
    const int32_t g = blockIdx.y;
    const int32_t v = blockIdx.x * WAVE + (threadIdx.x & (WAVE - 1));
    if (v >= n) return;   // no barriers below
    for (int32_t j = threadIdx.x >> 6; j < WAVE; j += (int32_t)(blockDim.x >> 6)) {
        const int32_t s0 = srcv[g * WAVE + j];
        const int32_t sc = srcc[g * WAVE + j];
        const size_t i = sidx<WAVE>(g, n, v, j);
        double d = INF;
        int32_t p = -1;
        Route rt{1.0, 0, -1};
        bool wr = false;
        if (s0 >= 0) {
            const double fs = G.vfac[s0];
            double r = has_attr(fs) ? 1.0 * fs : 1.0;   // shd-topology.c:1428-1430
            int32_t x, h = 0, f = -1, p0 = -1;
            double d0 = 0.0;
            if (sc >= 0) {
                x = sc;
            } else {   // pruned pendant source: its edge into the anchor comes first
                x = G.anchor_core[s0];
                const int32_t kx = G.fiptr[s0];
                d0 = 0.0 + G.fiw[kx];
                r = r * G.fia[kx];
                h = 1;
                f = G.corev[x];
                p0 = -2;
            }
            if (v == x) {
                d = d0;
                p = p0;
                rt = Route{r, h, f};
                wr = true;
            } else if (M.D[(int64_t)x * ld + v] < INF) {
                double dd = d0;
                int32_t pp = p0;
                for (int32_t step = 0; step < n && x != v; ++step) {
                    const int32_t k = M.N[(int64_t)x * ld + v];
                    if (k < 0) break;
                    const int32_t y = G.irow[k];
                    dd = dd + G.iw[k];
                    r = r * G.ia[k];
                    ++h;
                    if (f < 0) f = G.corev[y];
                    pp = k;
                    x = y;
                }
                if (x == v) {
                    d = dd;
                    p = pp;
                    rt = Route{r, h, f};
                    wr = true;
                }
            }
        }
        st.D[i] = d;
        st.P[i] = p;
        if (wr) st.RT[i] = rt;
    }
}
}  // namespace

// ================================================================== host side

struct spe_graph {
    spe::HostGraph hg;
    uint64_t key = 0;              // hash of the graph description (table cache key)
    int32_t device = 0;
    std::vector<double> aux_edge;  // spe_graph_set_edge_aux values per edge (re-uploaded by clones)
    DevGraph dev{};
    HeavyPlan hp{};
    const uint8_t* d_heavy = nullptr;
    DevGraph devx{};               // degree-3 contracted relaxation graph (hg.cx.active), batch engine
    HeavyPlan hpx{};
    std::vector<void*> allocs;
};

struct spe_table {
    spe_graph* g = nullptr;
    uint64_t key = 0;              // on-disk cache key (spe_table_key)
    int32_t A = 0;
    int32_t blk0 = 0, blk1 = 0;
    int32_t row_base = 0;          // the block tb's pointers start at (blk0; spe_table_build_blocks_into moves it)
    int32_t groups = 8;            // 64-source blocks per batch
    int32_t lanes = 16;            // sources per lane group (L)
    int32_t engine = SPE_ENGINE_BATCH;   // resolved engine
    int32_t relax_kernel = SPE_RELAX_REGISTER;   // resolved SPE_RELAX_* (batch engine)
    int32_t infl = 8;              // neighbour rows per round trip (register: in flight per wave; ring: LDS slots)
    bool trace = false;            // per-launch times to stderr while profiling (spe_table_opts.trace)
    unsigned long long* d_lds_dbg = nullptr;       // diagnostic (SPE_LDS_DEBUG): LDS engine phase clocks
#ifdef SPE_DIAGNOSTICS
    bool lds_debug = getenv("SPE_LDS_DEBUG") != nullptr;   // diagnostic builds only
#else
    static constexpr bool lds_debug = false;
#endif
    int32_t occ = 0;               // waves/SIMD the relaxation kernel is held to (0 = compiler's choice)
    // the batch engine's relaxation graph: the core, or its degree-3 contraction (cx)
    bool cx = false;
    const DevGraph* bG = nullptr;
    const HeavyPlan* bhp = nullptr;
    int32_t bn = 0;                // relaxation vertices (state rows per lane group)
    int32_t bm = 0;                // relaxation in-entries
    RowMode md{};
    bool ext = false;
    bool built = false;              // every owned block holds its rows
    std::vector<uint8_t> blk_built;  // per owned block (spe_table_build_blocks builds ranges)
    spe::MultiDev* multi = nullptr;  // a multi-device table: everything below is unused
    Table tb{};
    int32_t* d_slot_vertex = nullptr;
    SlotInfo* d_slots = nullptr;   // row passes (both engines): per-target constants
    LdsScratch lsc{};              // LDS engine: per-workgroup parent-entry scratch
    int32_t lds_grid = 0;          // LDS engine: workgroups per launch (scratch is sized for it)
    int32_t* d_rank = nullptr;     // owner replay: position of each slot in the source-run order
    int32_t* d_vertex_slot = nullptr;
    std::vector<int32_t> attached;
    // workspace
    State st{};
    uint8_t* inflag[2] = {nullptr, nullptr};
    uint8_t* mark[2] = {nullptr, nullptr};
    uint8_t* hmark[2] = {nullptr, nullptr};
    Partial pp{};
    int32_t* counts = nullptr;   // per round: 1 if any vertex changed
    int32_t max_iters = 0;
    int32_t last_rounds = 0;      // rounds the previous batch needed (sizes the next chunk)
    int32_t* d_srcv = nullptr;     // batch sources, original ids (-1 = padding)
    int32_t* d_srcc = nullptr;     // relaxation ids (-2 = pruned pendant source, -1 = padding)
    int32_t* h_srcv = nullptr;     // pinned staging for both
    int32_t* h_counts = nullptr;
    unsigned long long* d_min = nullptr;
    hipStream_t stream = nullptr;
    // batch engine: the rows of batch i (rows_stream) overlap batch i+1's
    // relaxation (stream) on the other state / source buffer
    bool overlap = false;
    State st_buf[2]{};
    int32_t* srcv_buf[2] = {nullptr, nullptr};
    int32_t* srcc_buf[2] = {nullptr, nullptr};
    hipStream_t rows_stream = nullptr;
    hipEvent_t ev_relaxed = nullptr;
    hipEvent_t ev_rows[2] = {nullptr, nullptr};
    bool rows_pending[2] = {false, false};
    spe_build_stats stats{};
    std::vector<void*> allocs;
    // profiling: one event pair per launch, resolved after each batch's sync
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    struct Rec {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<Rec> pending;
    size_t ev_next = 0;
    spe_kernel_profile kp{};
    std::vector<int32_t> h_hist;
    // FW engine: the closure (D, R, N over the relaxation graph, ld x ld), computed
    // by the first build and kept for the table's lifetime
    Fw3 fw{};
    int64_t fw_ld = 0;
    bool fw_done = false;
    // experimental Delta-stepping schedule of the batch engine (SPE_DELTA=<ms> at creation)
    double delta = 0.0;
    DeltaState ds{};
    // shared anchor trees (batch engine): relaxation lanes = the batch's
    // roots; rows per source through rlane
    bool share = false;
    bool share_off = false;        // this build runs one lane per source (fallback, source trees)
    int32_t* rsrc_buf[2] = {nullptr, nullptr};    // per source slot of the batch: original id (-1 pad)
    int2* rli_buf[2] = {nullptr, nullptr};        // per source slot: {root's state lane, first hop / -1}
    double2* rwa_buf[2] = {nullptr, nullptr};     // per source slot: {pendant latency, f_s (1 - p)}
    int2* rng_buf[2] = {nullptr, nullptr};        // per tile of RT_B source blocks: root lane span
    unsigned char* h_rows = nullptr;   // pinned staging for the three (owned blocks x 64 x 28 B)
    uint8_t* d_unsafe = nullptr;   // per root lane: k_share_check's flag
    uint8_t* h_unsafe = nullptr;
    // contracted shared tables: derived sources (k_rows_derived)
    DerivedSrc* d_der = nullptr;   // per derived source of the batch
    DerivedSrc* h_der = nullptr;   // pinned staging
    uint8_t* d_sunsafe = nullptr;  // per source slot of the batch: a derived row's margin failed
    double* d_dx = nullptr;        // [lane group][removed vertex][L]: expanded entries (k_expand_removed)
    Route* d_rtx = nullptr;
    const int32_t* d_rorig = nullptr;   // [removed] original id
    int32_t nr = 0;
    uint8_t* h_sunsafe = nullptr;
    bool derive = false;           // contracted sources take their neighbours' roots (no lane)
    // spe_lookup_batch_host / spe_table_get: device + pinned staging, grown on demand,
    // one caller at a time (the topology shim queries from several worker threads)
    struct HostLookup {
        std::mutex mu;
        int32_t device = -1;
        hipStream_t stream = nullptr;
        int64_t cap = 0;
        int2* d_pairs = nullptr;
        double* d_lat = nullptr;
        double* d_rel = nullptr;
        uint8_t* d_ok = nullptr;
        int2* h_pairs = nullptr;
        double* h_lat = nullptr;
        double* h_rel = nullptr;
        uint8_t* h_ok = nullptr;
        unsigned char* h_entry = nullptr;   // spe_table_get: 16 + 4 + 2 B read back with one sync
    };
    HostLookup* hlk = new HostLookup();
};

namespace {

template <typename T>
int dev_alloc(std::vector<void*>& allocs, T** p, size_t count) {
    void* q = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(&q, count * sizeof(T));
    if (e != hipSuccess)
        return fail(SPE_ENOMEM, "hipMalloc(" + std::to_string(count * sizeof(T)) + " B): " + hipGetErrorString(e));
    allocs.push_back(q);
    *p = static_cast<T*>(q);
    return SPE_OK;
}

template <typename T>
int dev_upload(std::vector<void*>& allocs, const std::vector<T>& h, const T** out) {
    T* p = nullptr;
    int r = dev_alloc(allocs, &p, h.size());
    if (r) return r;
    if (!h.empty()) HIP_TRY(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = p;
    return SPE_OK;
}

int check_device(int32_t device) {
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0) return fail(SPE_ENODEV, "no HIP device visible");
    if (device < 0 || device >= cnt) return fail(SPE_EINVAL, "device index out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SPE_ENODEV, std::string("libspe is built for gfx950, device is ") + prop.gcnArchName);
    HIP_TRY(hipSetDevice(device));
    return SPE_OK;
}

// The relaxation shapes instantiated in relax_to_convergence (keep in sync).
#define RELAX_DEFAULT_128 SPE_RELAX_LDS_RING
#define RELAX_RING_NS 5   // 5 LDS slots per wave at 7 waves / SIMD
bool relax_shape_supported(int32_t lanes, int32_t kernel, int32_t infl, int32_t occ, bool delta) {
    if (delta) return true;   // fixed shapes
    if (lanes == 64) return infl == 8 && occ <= 1;
    if (kernel == SPE_RELAX_LDS_RING)
        return (infl == 4 && occ == 8) || (infl == 5 && occ == 7) || (infl == 6 && occ == 6);
    return (infl == 4 && occ <= 1) || (infl == 2 && (occ <= 1 || occ == 6));
}

int grid_for(int64_t work_items, int64_t per_block, int cap = 8192) {
    int64_t b = (work_items + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

}  // namespace

static int graph_upload(spe_graph* g);

int spe::set_error(int code, const std::string& msg) { return fail(code, msg); }

extern "C" {

const char* spe_last_error(void) { return g_err.c_str(); }

int spe_device_count(int32_t* out) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    if (out) *out = c;
    return SPE_OK;
}

int spe_graph_create(const spe_graph_desc* desc, int32_t device, spe_graph** out) {
    if (!out) return fail(SPE_EINVAL, "out is NULL");
    if (desc && desc->struct_size != sizeof(spe_graph_desc)) return fail(SPE_EINVAL, ABI_MSG("spe_graph_desc"));
    *out = nullptr;
    auto* g = new spe_graph();
    std::string err;
    int r = spe::prepare_graph(desc, &g->hg, &err);
    if (r) {
        delete g;
        return fail(r, err);
    }
    r = check_device(device);
    if (r) {
        delete g;
        return r;
    }
    g->device = device;
    {   // everything in the description that can change a row
        Fnv f;
        f.val(desc->n_vertices);
        f.val(desc->n_edges);
        const size_t m = (size_t)desc->n_edges;
        f.add(desc->edge_source, m * sizeof(int32_t));
        f.add(desc->edge_target, m * sizeof(int32_t));
        f.add(desc->edge_latency, m * sizeof(double));
        f.add(desc->edge_packetloss, m * sizeof(double));
        const int32_t has_v = desc->vertex_packetloss != nullptr;
        f.val(has_v);
        if (has_v) f.add(desc->vertex_packetloss, (size_t)desc->n_vertices * sizeof(double));
        f.val(desc->directed);
        f.val(desc->prefer_direct);
        g->key = f.h;
    }
    spe::prune_pendants(&g->hg, desc->keep_pendants == 0);
    spe::contract_degree3(&g->hg);
    spe::share_prep(&g->hg);
    r = graph_upload(g);
    if (r) {
        spe_graph_free(g);
        return r;
    }
    *out = g;
    return SPE_OK;
}

}  // extern "C"

// Device copy of a prepared host graph (spe_graph_create, and the other devices
// of a multi-device table).  On failure the caller frees g.
static int graph_upload(spe_graph* g) {
    int r = SPE_OK;
    const spe::HostGraph& h = g->hg;
    DevGraph& d = g->dev;
    d.n = h.nc;
    d.n_full = h.n;
    d.nrel = (int32_t)h.icol.size();
#ifdef SPE_DIAGNOSTICS   // experiments only: SPE_ABLATE bit 0 skips route records (inexact rows)
    d.ablate = getenv("SPE_ABLATE") ? atoi(getenv("SPE_ABLATE")) : 0;
#else
    d.ablate = 0;
#endif
#define UPBASE d
#define UP(field, src)                                   \
    do {                                                 \
        r = dev_upload(g->allocs, src, &UPBASE.field);   \
        if (r) return r;                                 \
    } while (0)
    UP(iptr, h.iptr);
    UP(icol, h.icol);
    {
        std::vector<int32_t> irow(h.icol.size());
        for (int32_t v = 0; v < h.nc; ++v)
            for (int32_t k = h.iptr[v]; k < h.iptr[v + 1]; ++k) irow[k] = v;
        r = dev_upload(g->allocs, irow, &d.irow);
        if (r) return r;
        d.ipair = nullptr;
        if (h.nc <= 65535) {
            std::vector<uint32_t> ip(h.icol.size());
            for (size_t k = 0; k < ip.size(); ++k) ip[k] = ((uint32_t)irow[k] << 16) | (uint32_t)h.icol[k];
            r = dev_upload(g->allocs, ip, &d.ipair);
            if (r) return r;
        }
    }
    UP(iw, h.iw);
    UP(ia, h.ia);
    UP(iwrep, h.iwrep);
    UP(orev, h.orev);
    if (h.directed) {
        UP(optr, h.optr);
        UP(ocol, h.ocol);
        UP(owrep, h.owrep);
        UP(oarep, h.oarep);
        UP(ow, h.ow);
        d.undirected = 0;
    } else {
        d.optr = d.iptr;
        d.ocol = d.icol;
        d.owrep = d.iwrep;
        d.oarep = d.ia;
        d.ow = d.iw;
        d.undirected = 1;
    }
    UP(vfac, h.vfac);
    UP(loop_w, h.loop_w);
    UP(loop_a, h.loop_a);
    UP(self_w2, h.self_w2);
    UP(self_a2, h.self_a2);
    UP(self_other, h.self_other);
    UP(core_id, h.core_id);
    UP(corev, h.corev);
    UP(anchor_core, h.anchor_core);
    UP(fiptr, h.fiptr);
    UP(fiw, h.fiw);
    UP(fia, h.fia);
    UP(fiwrep, h.fiwrep);
    if (h.directed) {
        d.dptr = d.optr;
        d.dcol = d.ocol;
        d.dwrep = d.owrep;
        d.darep = d.oarep;
    } else if (!h.pruned) {
        d.dptr = d.iptr;
        d.dcol = d.icol;
        d.dwrep = d.iwrep;
        d.darep = d.ia;
    } else {
        d.dptr = d.fiptr;
        UP(dcol, h.ficol);
        d.dwrep = d.fiwrep;
        d.darep = d.fia;
    }
    {   // heavy-vertex segment plan (in-degree > 64), over the relaxation graph
        std::vector<uint8_t> heavy(h.nc, 0);
        std::vector<int32_t> seg_vertex, seg_begin, heavy_vertex, heavy_seg0;
        for (int32_t v = 0; v < h.nc; ++v) {
            const int32_t k0 = h.iptr[v], k1 = h.iptr[v + 1];
            if (k1 - k0 <= WAVE) continue;
            heavy[v] = 1;
            heavy_vertex.push_back(v);
            heavy_seg0.push_back((int32_t)seg_vertex.size());
            for (int32_t k = k0; k < k1; k += WAVE) {
                seg_vertex.push_back(v);
                seg_begin.push_back(k);
            }
        }
        heavy_seg0.push_back((int32_t)seg_vertex.size());
        g->hp.nseg = (int32_t)seg_vertex.size();
        g->hp.nheavy = (int32_t)heavy_vertex.size();
#undef UPBASE
#define UPBASE g->hp
        UP(seg_vertex, seg_vertex);
        UP(seg_begin, seg_begin);
        UP(heavy_vertex, heavy_vertex);
        UP(heavy_seg0, heavy_seg0);
#undef UPBASE
        r = dev_upload(g->allocs, heavy, &g->d_heavy);
        if (r) return r;
        d.heavy = g->d_heavy;
        const std::vector<int32_t>& oc = h.directed ? h.ocol : h.icol;
        std::vector<uint8_t> oheavy(oc.size());
        for (size_t k = 0; k < oc.size(); ++k) oheavy[k] = heavy[oc[k]];
        r = dev_upload(g->allocs, oheavy, &d.oheavy);
        if (r) return r;
        std::vector<int4> pack(std::max<size_t>(1, h.icol.size()));
        for (size_t k = 0; k < h.icol.size(); ++k) {
            uint64_t wb;
            std::memcpy(&wb, &h.iw[k], sizeof wb);
            const int32_t rev = h.directed ? 0 : (h.orev[k] | (heavy[h.icol[k]] ? (int32_t)0x80000000 : 0));
            pack[k] = make_int4(h.icol[k], rev, (int32_t)(uint32_t)wb, (int32_t)(uint32_t)(wb >> 32));
        }
        r = dev_upload(g->allocs, pack, &d.ipack);
        if (r) return r;
    }
#undef UP
    if (h.cx.active) {   // the batch engine's contracted relaxation graph (shares the rest of dev)
        const spe::HostGraph::Contracted& cx = h.cx;
        DevGraph& x = g->devx;
        x = d;
        x.n = cx.nk;
        x.nrel = (int32_t)cx.col.size();
        x.ipair = nullptr;
        x.iaux = x.fiaux = nullptr;
#define UPX(field, src)                                  \
    do {                                                 \
        r = dev_upload(g->allocs, src, &x.field);        \
        if (r) return r;                                 \
    } while (0)
        UPX(iptr, cx.ptr);
        UPX(icol, cx.col);
        UPX(iw, cx.w1);
        UPX(ia, cx.a1);
        UPX(orev, cx.rev);
        UPX(xw2, cx.w2);
        UPX(xa2, cx.a2);
        UPX(xkey, cx.key);
        UPX(xvia, cx.via);
        UPX(rnb, cx.rnb);
        UPX(rw, cx.rw);
        UPX(ra, cx.ra);
        x.iwrep = x.iw;   // (contraction needs no multigraph representatives)
        x.optr = x.iptr;
        x.ocol = x.icol;
        x.owrep = x.iw;
        x.oarep = x.ia;
        x.ow = x.iw;
        {
            std::vector<int32_t> irow(cx.col.size()), cid(h.n, -1), anc(h.n, -1), rm(h.n, -1);
            for (int32_t v = 0; v < cx.nk; ++v)
                for (int32_t k = cx.ptr[v]; k < cx.ptr[v + 1]; ++k) irow[k] = v;
            std::vector<int32_t> corev(cx.nk);
            for (int32_t k = 0; k < cx.nk; ++k) corev[k] = h.corev[cx.kcore[k]];
            for (int32_t v = 0; v < h.n; ++v) {
                const int32_t c = h.core_id[v];
                if (c >= 0) {
                    cid[v] = cx.kid[c];
                    rm[v] = cx.rid[c];
                } else if (h.anchor_core[v] >= 0) {
                    anc[v] = cx.kid[h.anchor_core[v]];   // (no removed vertex anchors a pendant)
                }
            }
            UPX(irow, irow);
            UPX(corev, corev);
            UPX(core_id, cid);
            UPX(anchor_core, anc);
            UPX(xrm, rm);
        }
#undef UPX
        std::vector<uint8_t> heavy(cx.nk, 0);
        std::vector<int32_t> seg_vertex, seg_begin, heavy_vertex, heavy_seg0;
        for (int32_t v = 0; v < cx.nk; ++v) {
            const int32_t k0 = cx.ptr[v], k1 = cx.ptr[v + 1];
            if (k1 - k0 <= WAVE) continue;
            heavy[v] = 1;
            heavy_vertex.push_back(v);
            heavy_seg0.push_back((int32_t)seg_vertex.size());
            for (int32_t k = k0; k < k1; k += WAVE) {
                seg_vertex.push_back(v);
                seg_begin.push_back(k);
            }
        }
        heavy_seg0.push_back((int32_t)seg_vertex.size());
        g->hpx.nseg = (int32_t)seg_vertex.size();
        g->hpx.nheavy = (int32_t)heavy_vertex.size();
        if ((r = dev_upload(g->allocs, seg_vertex, &g->hpx.seg_vertex))) return r;
        if ((r = dev_upload(g->allocs, seg_begin, &g->hpx.seg_begin))) return r;
        if ((r = dev_upload(g->allocs, heavy_vertex, &g->hpx.heavy_vertex))) return r;
        if ((r = dev_upload(g->allocs, heavy_seg0, &g->hpx.heavy_seg0))) return r;
        if ((r = dev_upload(g->allocs, heavy, &x.heavy))) return r;
        std::vector<uint8_t> oheavy(cx.col.size());
        for (size_t k = 0; k < cx.col.size(); ++k) oheavy[k] = heavy[cx.col[k]];
        if ((r = dev_upload(g->allocs, oheavy, &x.oheavy))) return r;
        // bit 31: the target of the reverse entry is heavy; bit 30: a shortcut entry
        std::vector<int4> pack(std::max<size_t>(1, cx.col.size()));
        for (size_t k = 0; k < cx.col.size(); ++k) {
            uint64_t wb;
            std::memcpy(&wb, &cx.w1[k], sizeof wb);
            const int32_t rev = cx.rev[k] | (cx.via[k] >= 0 ? 0x40000000 : 0) | (heavy[cx.col[k]] ? (int32_t)0x80000000 : 0);
            pack[k] = make_int4(cx.col[k], rev, (int32_t)(uint32_t)wb, (int32_t)(uint32_t)(wb >> 32));
        }
        if ((r = dev_upload(g->allocs, pack, &x.ipack))) return r;
    }
    if (!g->aux_edge.empty()) {   // the auxiliary attribute, if set (spe_graph_set_edge_aux)
        std::vector<double> ia(h.ieid.size()), fa(h.fieid.size());
        for (size_t k = 0; k < ia.size(); ++k) ia[k] = g->aux_edge[h.ieid[k]];
        for (size_t k = 0; k < fa.size(); ++k) fa[k] = g->aux_edge[h.fieid[k]];
        if (ia.empty()) ia.push_back(0.0);
        if (fa.empty()) fa.push_back(0.0);
        if ((r = dev_upload(g->allocs, ia, &g->dev.iaux))) return r;
        if ((r = dev_upload(g->allocs, fa, &g->dev.fiaux))) return r;
    }
    return SPE_OK;
}

int spe::graph_clone(const spe_graph* g, int32_t device, spe_graph** out) {
    *out = nullptr;
    int r = check_device(device);
    if (r) return r;
    auto* c = new spe_graph();
    c->hg = g->hg;
    c->key = g->key;
    c->device = device;
    c->aux_edge = g->aux_edge;
    r = graph_upload(c);
    if (r) {
        spe_graph_free(c);
        return r;
    }
    *out = c;
    return SPE_OK;
}

extern "C" {

int spe_graph_set_edge_aux(spe_graph* g, const double* edge_aux) {
    if (!g || (!edge_aux && g->hg.m > 0)) return fail(SPE_EINVAL, "NULL argument");
    HIP_TRY(hipSetDevice(g->device));
    const spe::HostGraph& h = g->hg;
    for (int64_t e = 0; e < h.m; ++e)
        if (!std::isfinite(edge_aux[e])) return fail(SPE_EINVAL, "edge " + std::to_string(e) + " aux value is not finite");
    g->aux_edge.assign(edge_aux, edge_aux + h.m);
    std::vector<double> ia(h.ieid.size()), fa(h.fieid.size());
    for (size_t k = 0; k < ia.size(); ++k) ia[k] = edge_aux[h.ieid[k]];
    for (size_t k = 0; k < fa.size(); ++k) fa[k] = edge_aux[h.fieid[k]];
    if (ia.empty()) ia.push_back(0.0);
    if (fa.empty()) fa.push_back(0.0);
    if (int r = dev_upload(g->allocs, ia, &g->dev.iaux)) return r;
    if (int r = dev_upload(g->allocs, fa, &g->dev.fiaux)) return r;
    return SPE_OK;
}

int spe_graph_info_get(const spe_graph* g, spe_graph_info* out) {
    if (!g || !out) return fail(SPE_EINVAL, "NULL argument");
    if (out->struct_size != sizeof(spe_graph_info)) return fail(SPE_EINVAL, ABI_MSG("spe_graph_info"));
    out->n_vertices = g->hg.n;
    out->n_edges = g->hg.m;
    out->n_relax_entries = (int64_t)g->hg.icol.size();
    out->n_relax_vertices = g->hg.nc;
    out->directed = g->hg.directed;
    out->prefer_direct = g->hg.prefer_direct;
    out->complete = g->hg.complete;
    out->parallel_latency_differs = g->hg.multi_rep;
    out->weight_floor_ok = g->hg.weight_floor_ok;
    out->device = g->device;
    out->sums_exact = g->hg.share.eligible && g->hg.share.exact;
    return SPE_OK;
}

int spe_graph_self_path(const spe_graph* g, int32_t v, spe_entry* out) {
    if (!g || !out) return fail(SPE_EINVAL, "NULL argument");
    const spe::HostGraph& h = g->hg;
    if (v < 0 || v >= h.n) return fail(SPE_EINVAL, "vertex out of range");
    if (h.self_other[(size_t)v] < 0) {
        *out = spe_entry{-1.0, -1.0, -1, 0};
    } else {
        *out = spe_entry{h.self_w2[(size_t)v], h.self_a2[(size_t)v], h.self_other[(size_t)v], 2};
    }
    return SPE_OK;
}

int spe_graph_adjacent(const spe_graph* g, int32_t from, int32_t to, int32_t* out) {
    if (!g || !out) return fail(SPE_EINVAL, "NULL argument");
    const spe::HostGraph& h = g->hg;
    if (from < 0 || from >= h.n || to < 0 || to >= h.n) return fail(SPE_EINVAL, "vertex out of range");
    if (from == to) {   // self-loops are kept out of the CSRs (get_eid(v, v): loop_eid)
        *out = h.loop_eid[(size_t)from] >= 0 ? 1 : 0;
        return SPE_OK;
    }
    // the out-CSR of a directed graph (never pruned), the full original-id in-CSR
    // of an undirected one (symmetric: search the list of `to` for `from`)
    const std::vector<int32_t>& ptr = h.directed ? h.optr : h.fiptr;
    const std::vector<int32_t>& col = h.directed ? h.ocol : h.ficol;
    const int32_t row = h.directed ? from : to, key = h.directed ? to : from;
    *out = std::binary_search(col.begin() + ptr[(size_t)row], col.begin() + ptr[(size_t)row + 1], key) ? 1 : 0;
    return SPE_OK;
}

int spe_graph_edge(const spe_graph* g, int32_t from, int32_t to, double* latency, double* reliability) {
    if (!g) return fail(SPE_EINVAL, "NULL argument");
    const spe::HostGraph& h = g->hg;
    if (from < 0 || from >= h.n || to < 0 || to >= h.n) return fail(SPE_EINVAL, "vertex out of range");
    double w = NAN, a = NAN;
    if (from == to) {
        if (h.loop_eid[(size_t)from] >= 0) {
            w = h.loop_w[(size_t)from];
            a = h.loop_a[(size_t)from];
        }
    } else {
        const std::vector<int32_t>& ptr = h.directed ? h.optr : h.fiptr;
        const std::vector<int32_t>& col = h.directed ? h.ocol : h.ficol;
        const int32_t row = h.directed ? from : to, key = h.directed ? to : from;
        const auto b = col.begin() + ptr[(size_t)row], e = col.begin() + ptr[(size_t)row + 1];
        const auto it = std::lower_bound(b, e, key);
        if (it != e && *it == key) {
            const size_t k = (size_t)(it - col.begin());
            w = h.directed ? h.owrep[k] : h.fiwrep[k];
            a = h.directed ? h.oarep[k] : h.fia[k];
        }
    }
    if (std::isnan(w)) return fail(SPE_EINVAL, "no such edge");
    if (latency) *latency = w;
    if (reliability) *reliability = a;
    return SPE_OK;
}

int spe_order_sources(const spe_graph* g, const int32_t* attached, int32_t n_attached, int32_t* order_out) {
    if (!g || (n_attached > 0 && (!attached || !order_out))) return fail(SPE_EINVAL, "NULL argument");
    if (n_attached < 0) return fail(SPE_EINVAL, "negative n_attached");
    const spe::HostGraph& h = g->hg;
    // relaxation vertex of every source (a pruned pendant's anchor, else itself)
    std::vector<int32_t> rv((size_t)n_attached);
    std::vector<int32_t> distinct;
    for (int32_t i = 0; i < n_attached; ++i) {
        const int32_t v = attached[i];
        if (v < 0 || v >= h.n) return fail(SPE_EINVAL, "attached vertex out of range");
        rv[(size_t)i] = h.core_id[v] >= 0 ? h.core_id[v] : h.anchor_core[v];
        if (rv[(size_t)i] >= 0) distinct.push_back(rv[(size_t)i]);
    }
    std::sort(distinct.begin(), distinct.end());
    distinct.erase(std::unique(distinct.begin(), distinct.end()), distinct.end());
    // Voronoi cells of ceil(A / 64) seeded-random centres over the relaxation
    // graph (multi-source Dijkstra on the in-CSR): a 64-source block then holds
    // sources that are close to one another, whose lanes advance in similar rounds
    const int32_t per_cell = WAVE;   // cells of 16..512 sources measured flat within +-4 %
    const size_t K = std::min(distinct.size(), (size_t)((n_attached + per_cell - 1) / per_cell));
    std::vector<int32_t> cell((size_t)h.nc, INT32_MAX);
    std::vector<double> dist((size_t)h.nc, INF);
    if (K > 0 && !h.complete) {
        std::vector<int32_t> c = distinct;
        std::mt19937_64 rng(0x5eed);
        std::shuffle(c.begin(), c.end(), rng);
        using QE = std::pair<double, int32_t>;
        std::priority_queue<QE, std::vector<QE>, std::greater<QE>> pq;
        for (size_t i = 0; i < K; ++i) {
            cell[(size_t)c[i]] = (int32_t)i;
            dist[(size_t)c[i]] = 0.0;
            pq.push({0.0, c[i]});
        }
        while (!pq.empty()) {
            const QE e = pq.top();
            pq.pop();
            const int32_t x = e.second;
            if (e.first > dist[(size_t)x]) continue;
            for (int32_t k = h.iptr[(size_t)x]; k < h.iptr[(size_t)x + 1]; ++k) {
                const int32_t u = h.icol[(size_t)k];
                const double du = e.first + h.iw[(size_t)k];
                if (du < dist[(size_t)u]) {
                    dist[(size_t)u] = du;
                    cell[(size_t)u] = cell[(size_t)x];
                    pq.push({du, u});
                }
            }
        }
    }
    struct Key {
        int32_t cell;
        double d;
        int32_t r, v;
    };
    std::vector<Key> key((size_t)n_attached);
    for (int32_t i = 0; i < n_attached; ++i) {
        const int32_t r = rv[(size_t)i];
        key[(size_t)i] = r >= 0 ? Key{cell[(size_t)r], dist[(size_t)r], r, attached[i]}
                                : Key{INT32_MAX, INF, INT32_MAX, attached[i]};
    }
    std::sort(key.begin(), key.end(), [](const Key& a, const Key& b) {
        if (a.cell != b.cell) return a.cell < b.cell;
        if (a.d != b.d) return a.d < b.d;
        if (a.r != b.r) return a.r < b.r;
        return a.v < b.v;
    });
    for (int32_t i = 0; i < n_attached; ++i) order_out[i] = key[(size_t)i].v;
    return SPE_OK;
}

void spe_graph_free(spe_graph* g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    for (void* p : g->allocs) (void)hipFree(p);
    delete g;
}

int spe_table_create(spe_graph* g, const int32_t* attached, int32_t n_attached, const spe_table_opts* opts,
                     spe_table** out) {
    if (!g || !attached || n_attached <= 0 || !out) return fail(SPE_EINVAL, "spe_table_create: bad arguments");
    *out = nullptr;
    HIP_TRY(hipSetDevice(g->device));
    const int32_t n_full = g->hg.n;
    const int32_t n = g->hg.nc;   // relaxation state is over the core
    std::vector<int32_t> vslot(n_full, -1);
    for (int32_t i = 0; i < n_attached; ++i) {
        const int32_t v = attached[i];
        if (v < 0 || v >= n_full) return fail(SPE_EINVAL, "attached vertex out of range");
        if (vslot[v] >= 0) return fail(SPE_EINVAL, "attached vertices must be unique");
        vslot[v] = i;
    }
    spe_table_opts o{};
    o.struct_size = sizeof(spe_table_opts);
    if (opts) {
        if (opts->struct_size != sizeof(spe_table_opts)) return fail(SPE_EINVAL, ABI_MSG("spe_table_opts"));
        o = *opts;
    }
    const int32_t nblk_all = (n_attached + WAVE - 1) / WAVE;
    // every argument check before the first allocation (nothing to unwind)
    if (o.block_begin != 0 || o.block_end != 0) {
        if (o.block_begin < 0 || o.block_end > nblk_all || o.block_begin > o.block_end)
            return fail(SPE_EINVAL, "block range out of bounds");
    }
    if (o.owner_rank && (o.block_begin != 0 || (o.block_end != 0 && o.block_end != nblk_all)))
        return fail(SPE_EUNSUPPORTED, "owner replay needs a table that owns every source block");
    if ((o.ext_latrel || o.ext_next_hop || o.ext_hops) && !(o.ext_latrel && o.ext_next_hop && o.ext_hops))
        return fail(SPE_EINVAL, "external storage needs all three fields");
    if (o.devices && o.n_devices < 1) return fail(SPE_EINVAL, "n_devices must be >= 1 with a device list");
    auto* t = new spe_table();
    t->g = g;
    t->A = n_attached;
    t->attached.assign(attached, attached + n_attached);
    t->blk0 = 0;
    t->blk1 = nblk_all;
    if (o.block_begin != 0 || o.block_end != 0) {
        t->blk0 = o.block_begin;
        t->blk1 = o.block_end;
    }
    t->row_base = t->blk0;
    const bool force = o.force_sssp != 0;
    {   // table cache key: graph, attached set, and every option that changes a row
        Fnv f;
        const char fmt[] = "spe-table-v1 latrel+next+hops SB64";
        f.add(fmt, sizeof(fmt));
        f.val(g->key);
        f.val(n_attached);
        f.add(attached, (size_t)n_attached * sizeof(int32_t));
        f.val(o.self_mode);
        const int32_t fs = force;
        f.val(fs);
        f.val(t->blk0);
        f.val(t->blk1);
        const int32_t has_owner = o.owner_rank != nullptr;
        f.val(has_owner);
        const int32_t aux = o.want_aux != 0;
        f.val(aux);
        const int32_t exact_src = o.exact_sources != 0;   // shared anchor trees change the last bits
        f.val(exact_src);
        if (has_owner) f.add(o.owner_rank, (size_t)n_attached * sizeof(int32_t));
        t->key = f.h;
    }
    if (o.devices) {   // one process, several devices (spe_multi.cpp)
        int r = spe::multi_create(g, attached, n_attached, o, &t->multi);
        if (r) {
            delete t;
            return r;
        }
        *out = t;
        return SPE_OK;
    }
    t->md.complete = g->hg.complete && !force;
    t->md.prefer = g->hg.prefer_direct && !force;
    if (o.want_aux) {   // the aux fold walks the batch engine's parent edges: SSSP rows only
        if (!g->dev.iaux) {
            delete t;
            return fail(SPE_ESTATE, "want_aux: no auxiliary edge attribute (spe_graph_set_edge_aux)");
        }
        if (t->md.complete || t->md.prefer || o.owner_rank) {
            delete t;
            return fail(SPE_EUNSUPPORTED, "want_aux needs SSSP rows (force_sssp on complete/preferdirect graphs, "
                                          "no owner replay)");
        }
        if (o.engine == SPE_ENGINE_LDS) {
            delete t;
            return fail(SPE_EUNSUPPORTED, "want_aux runs on the batch engine");
        }
        o.engine = SPE_ENGINE_BATCH;
    }
    t->md.self_mode = o.self_mode;
    t->md.multi_rep = g->hg.multi_rep;
    t->md.directed = g->hg.directed;
    // groups per launch: ~10M (group, vertex) rows per relaxation round.  Fewer,
    // larger batches cut the rounds a table takes (each batch converges in ~the
    // same count) and the near-empty tail rounds of each batch.  Same-box sweeps
    // (tools/gpu_groups_big.sh): C3 46 / 98 / 196 / 261 / 391 / 782 groups ->
    // 89-94k / 98.9k / 101.5k / 102.3k / 98.5k / 98.8k sources/s (one or two
    // batches lose the rows / relaxation overlap); C4 64 / 196 / 391 -> 278k /
    // 315k / 335k.  Batches are balanced; the state (n * 64 * 28 B per group, held
    // twice: the rows of one batch overlap the next batch's relaxation) must fit
    // the device's free HBM next to the table (the table and 4 GB kept free).
    int32_t groups = o.groups_per_launch;
    const int32_t owned = std::max(1, t->blk1 - t->blk0);
    if (groups <= 0) {
        const double per_group = 2.0 * ((double)n * WAVE * 28.0 + 4.0 * n + 2.0 * (double)g->hg.icol.size());
        double want = std::max(1.0, std::round(1.0e7 / std::max(1, n)));
        size_t free_b = 0, total_b = 0;
        if (hipSetDevice(g->device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
            const bool ext = o.ext_latrel || o.ext_next_hop || o.ext_hops;
            const double rec = 22.0 + (o.owner_rank ? 4.0 : 0.0) + (o.want_aux ? 8.0 : 0.0);
            const double table_b = ext ? 0.0 : (double)owned * n_attached * WAVE * rec;
            const double ldf = std::ceil(std::max(1, n) / 64.0) * 64.0;   // FW engine: its closure, 20 B x ld^2
            const double closure_b = o.engine == SPE_ENGINE_FW ? 20.0 * ldf * ldf : 0.0;
            const double budget = (double)free_b - table_b - closure_b - 4.0e9;
            want = std::min(want, std::max(1.0, budget / per_group));
        } else {
            want = std::min(want, 6.0e9 / per_group);
        }
        const int32_t w = (int32_t)std::min<double>(want, owned);
        const int32_t batches = (owned + w - 1) / w;
        groups = (owned + batches - 1) / batches;
        if (groups > 1 && groups % 2 && groups + 1 <= w) ++groups;   // even: no padding lanes at L = 128
    }
    t->groups = std::max(1, std::min(groups, owned));
    // sources per lane group (shared frontier); 64/L groups per 64-source block
    int32_t lanes = o.lanes_per_group;
    // default: 128 sources per relaxation row (2 per thread) when every full build
    // launch covers an even or a large block count, else 64.
    // Same-box A/B, three pairs: C3 +1.4..2.1 %, C4 within +-0.5 %.
    // (an odd launch pads one block of empty lanes: 1 / (groups + 1) extra work)
    if (lanes <= 0) lanes = (t->groups >= 2 && (t->groups % 2 == 0 || t->groups >= 32)) ? 128 : 64;
    if (lanes != 64 && lanes != 128) {
        delete t;
        return fail(SPE_EINVAL, "lanes_per_group must be 64 or 128");
    }
    t->lanes = lanes;
    {
        const bool fits = lds_bytes(g->hg.nc) <= (size_t)LDS_MAX_BYTES && g->hg.nc <= LDS_VPT * LDS_T;
        int32_t e = o.engine;
        if (e == SPE_ENGINE_FW && !t->md.complete && (int64_t)g->hg.nc > FW_MAX_N) {
            delete t;
            return fail(SPE_EUNSUPPORTED, "relaxation graph too large for the FW engine (n^2 closure)");
        }
        if (e == SPE_ENGINE_LDS && !fits) {
            delete t;
            return fail(SPE_EUNSUPPORTED, "relaxation graph too large for the LDS engine");
        }
        t->engine = (e == SPE_ENGINE_AUTO) ? (fits ? SPE_ENGINE_LDS : SPE_ENGINE_BATCH) : e;
        if (t->engine == SPE_ENGINE_LDS && !t->md.complete) {
            // no HBM state: one launch covers every owned block (unless asked otherwise)
            if (o.groups_per_launch <= 0) t->groups = std::max(1, t->blk1 - t->blk0);
            const hipError_t fe = hipFuncSetAttribute((const void*)k_sssp_lds,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      (int)lds_bytes(g->hg.nc));
            if (fe != hipSuccess) {
                delete t;
                return fail(SPE_EHIP, std::string("hipFuncSetAttribute(k_sssp_lds): ") + hipGetErrorString(fe));
            }
        }
    }
    if (t->engine == SPE_ENGINE_FW) t->lanes = lanes = WAVE;   // its state walk writes 64-lane rows
    // relaxation kernel and its shape.  64 lanes: k_relax, 8 rows in flight.  128
    // lanes: k_relax_s (LDS ring, RELAX_RING_NS rows per trip) or k_relax_m (2 rows
    // in flight held to 6 waves / SIMD).  Unsupported shapes are refused.
    // (the kernel / rows / waves tuning applies to 128-lane rows; 64-lane rows run k_relax as measured)
    t->delta = o.delta_ms > 0.0 ? o.delta_ms : 0.0;
    const bool wide = lanes == 128;
    t->relax_kernel = !wide ? SPE_RELAX_REGISTER
                            : (o.relax_kernel != SPE_RELAX_AUTO ? o.relax_kernel
                                                                : (t->delta == 0.0 ? RELAX_DEFAULT_128 : SPE_RELAX_REGISTER));
    if (t->relax_kernel == SPE_RELAX_LDS_RING && t->delta > 0.0) {
        delete t;
        return fail(SPE_EUNSUPPORTED, "the LDS-ring relaxation runs 128-lane rows without the Delta schedule");
    }
    // waves_per_simd 0 = the default for the shape, 1 = the compiler's choice
    if (t->relax_kernel == SPE_RELAX_LDS_RING) {
        t->infl = o.rows_in_flight > 0 ? o.rows_in_flight : RELAX_RING_NS;
        t->occ = o.waves_per_simd > 0 ? o.waves_per_simd : (t->infl == 4 ? 8 : t->infl == 5 ? 7 : t->infl == 6 ? 6 : 1);
    } else if (!wide) {
        t->infl = 8;
        t->occ = 1;
    } else {
        t->infl = o.rows_in_flight > 0 ? o.rows_in_flight : 2;
        t->occ = o.waves_per_simd > 0 ? o.waves_per_simd : (t->infl == 2 ? 6 : 1);
        if (t->delta > 0.0) {   // the Delta schedule's own instantiations
            t->infl = lanes == 64 ? 8 : 4;
            t->occ = 0;
        }
    }
    if (!relax_shape_supported(t->lanes, t->relax_kernel, t->infl, t->occ, t->delta > 0.0)) {
        delete t;
        return fail(SPE_EUNSUPPORTED, "relaxation shape (rows_in_flight, waves_per_simd) not built");
    }
    // degree-3 contraction: the LDS-ring batch relaxation of SSSP rows,
    // without the compat modes that walk parent edges (owner replay, aux fold)
    t->cx = g->hg.cx.active && !o.no_contract && t->engine == SPE_ENGINE_BATCH && !t->md.complete &&
            t->lanes == 128 && t->relax_kernel == SPE_RELAX_LDS_RING && t->infl == RELAX_RING_NS && t->occ == 7 &&
            t->delta == 0.0 && !o.owner_rank && !o.want_aux;
    t->bG = t->cx ? &g->devx : &g->dev;
    t->bhp = t->cx ? &g->hpx : &g->hp;
    t->bn = t->cx ? g->hg.cx.nk : g->hg.nc;
    t->bm = t->cx ? (int32_t)g->hg.cx.col.size() : (int32_t)g->hg.icol.size();
    // shared anchor trees: pendant sources relax as their anchor
    t->share = !o.exact_sources && g->hg.share.eligible && t->engine == SPE_ENGINE_BATCH && !t->md.complete &&
               !o.owner_rank && !o.want_aux && t->delta == 0.0;
    if (t->share) {   // some offset source: a pruned pendant, or (contracted tables) a removed vertex
        bool any = false;
        for (int32_t i = t->blk0 * WAVE; i < std::min(n_attached, t->blk1 * WAVE) && !any; ++i) {
            const int32_t c = g->hg.core_id[(size_t)attached[i]];
            any = c < 0 || (t->cx && g->hg.cx.der[(size_t)c]);
        }
        t->share = any;
    }
    t->derive = t->share && t->cx;
    if (t->share && o.groups_per_launch <= 0) {
        // lane groups per batch for shared tables: every root of the owned range in one
        // relaxation when the state fits (the rows of a contracted source read its
        // neighbours' lanes, so they must be in its batch).  Roots: each core source and
        // pendant anchor once, a contracted source none when its three neighbours are
        // roots (derived), else its own lane.  State held once (no rows overlap).
        const spe::HostGraph& h = g->hg;
        std::vector<uint8_t> isroot((size_t)std::max(1, h.nc), 0);
        int64_t roots = 0;
        const int32_t s0 = t->blk0 * WAVE, s1 = std::min(n_attached, t->blk1 * WAVE);
        for (int32_t i = s0; i < s1; ++i) {
            const int32_t v = attached[i];
            int32_t c = h.core_id[(size_t)v];
            if (c < 0) c = h.anchor_core[(size_t)v];
            else if (t->cx && h.cx.der[(size_t)c]) continue;
            if (c >= 0 && !isroot[(size_t)c]) {
                isroot[(size_t)c] = 1;
                ++roots;
            }
        }
        if (t->cx)
            for (int32_t i = s0; i < s1; ++i) {
                const int32_t c = h.core_id[(size_t)attached[i]];
                if (c < 0 || !h.cx.der[(size_t)c]) continue;
                bool all = true;
                for (int32_t k = h.iptr[(size_t)c]; k < h.iptr[(size_t)c + 1]; ++k) all &= isroot[(size_t)h.icol[(size_t)k]] != 0;
                if (!all) ++roots;
            }
        const int32_t need = (int32_t)std::max<int64_t>(1, (roots + WAVE - 1) / WAVE);
        const double per_group = (double)t->bn * WAVE * 28.0 + 4.0 * t->bn + 2.0 * std::max(1, t->bm) +
                                 (t->derive ? (double)h.cx.rcore.size() * WAVE * 24.0 : 0.0);
        double cap = (double)need;
        size_t free_b = 0, total_b = 0;
        if (hipSetDevice(g->device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
            const bool ext = o.ext_latrel || o.ext_next_hop || o.ext_hops;
            const double table_b = ext ? 0.0 : (double)owned * n_attached * WAVE * 22.0;
            cap = std::max(1.0, ((double)free_b - table_b - 4.0e9) / per_group);
        }
        const int32_t w = (int32_t)std::min<double>(need, cap);
        const int32_t batches = (need + w - 1) / w;
        int32_t gg = (need + batches - 1) / batches;
        if (t->lanes == 128 && gg > 1 && gg % 2) ++gg;   // no padding lanes at L = 128
        t->groups = std::max(1, std::min(gg, owned));
    }
    t->trace = o.trace != 0;
    t->tb.A = n_attached;
    const size_t elems = (size_t)(t->blk1 - t->blk0) * n_attached * WAVE;
    int r = SPE_OK;
#define TRY(x)                  \
    do {                        \
        r = (x);                \
        if (r) {                \
            spe_table_free(t);  \
            return r;           \
        }                       \
    } while (0)
    if (o.ext_latrel || o.ext_next_hop || o.ext_hops) {
        t->ext = true;
        t->built = o.ext_filled != 0;
        t->tb.lr = (double2*)o.ext_latrel;
        t->tb.next = (int32_t*)o.ext_next_hop;
        t->tb.hops = (uint16_t*)o.ext_hops;
    } else {
        TRY(dev_alloc(t->allocs, &t->tb.lr, elems));
        TRY(dev_alloc(t->allocs, &t->tb.next, elems));
        TRY(dev_alloc(t->allocs, &t->tb.hops, elems));
    }
    if (o.owner_rank) {   // owner replay needs every source row in this table (checked above)
        std::vector<int32_t> rk(o.owner_rank, o.owner_rank + n_attached);
        const int32_t* tmpr = nullptr;
        TRY(dev_upload(t->allocs, rk, &tmpr));
        t->d_rank = const_cast<int32_t*>(tmpr);
        TRY(dev_alloc(t->allocs, &t->tb.prev, elems));
    }
    if (o.want_aux) TRY(dev_alloc(t->allocs, &t->tb.aux, elems));
    const std::vector<int32_t> sv(attached, attached + n_attached);
    const int32_t* tmp = nullptr;
    TRY(dev_upload(t->allocs, sv, &tmp));
    t->d_slot_vertex = const_cast<int32_t*>(tmp);
    TRY(dev_upload(t->allocs, vslot, &tmp));
    t->d_vertex_slot = const_cast<int32_t*>(tmp);
    if (!t->md.complete) {
        const spe::HostGraph& h = g->hg;
        std::vector<SlotInfo> si(n_attached);
        for (int32_t j = 0; j < n_attached; ++j) {
            const int32_t v = attached[j];
            SlotInfo& x = si[j];
            x.t = v;
            const double ft = h.vfac[v];
            x.fast = (std::isnan(ft) || ft == 1.0) ? 1 : 0;
            if (h.core_id[v] >= 0) {
                x.c = h.core_id[v];
                x.kt = -1;
                x.pw = 0.0;
                x.pa = 1.0;
            } else {
                x.c = h.anchor_core[v];
                x.kt = h.fiptr[v];
                x.pw = h.fiw[x.kt];
                x.pa = h.fia[x.kt];
            }
            // contracted tables: kept ids; a removed target reads its three neighbours
            // (c = -2 - removed index)
            if (t->cx) x.c = h.cx.kid[x.c] >= 0 ? h.cx.kid[x.c] : -2 - h.cx.rid[x.c];
        }
        const SlotInfo* tsi = nullptr;
        TRY(dev_upload(t->allocs, si, &tsi));
        t->d_slots = const_cast<SlotInfo*>(tsi);
    }
    if (!t->md.complete && t->engine == SPE_ENGINE_LDS) {
        const spe::HostGraph& h = g->hg;
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device);
        const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, LDS_MAX_BYTES / lds_bytes(h.nc)));
        t->lds_grid = cus * per_cu;
        const size_t per = (size_t)t->lds_grid * std::max(1, h.nc);
        TRY(dev_alloc(t->allocs, &t->lsc.par, per));
    }
    const size_t G = (size_t)t->groups;
    // lane groups per batch (L > 64: a group spans L / 64 blocks; an odd tail is padded)
    const size_t GL = t->lanes <= WAVE ? G * (WAVE / t->lanes) : (G * WAVE + t->lanes - 1) / t->lanes;
    const size_t GW = GL * (size_t)t->lanes;   // source entries per batch (>= G * 64: padding lanes)
    if (!t->md.complete && t->engine == SPE_ENGINE_BATCH) {
        const size_t se = GW * (size_t)t->bn;
        // (shared tables relax and write rows on one stream: one state buffer)
        t->overlap = o.no_overlap == 0 && !t->share;
        for (int i = 0; i < (t->overlap ? 2 : 1); ++i) {
            TRY(dev_alloc(t->allocs, &t->st_buf[i].D, se));
            TRY(dev_alloc(t->allocs, &t->st_buf[i].P, se));
            TRY(dev_alloc(t->allocs, &t->st_buf[i].RT, se));
        }
        t->st = t->st_buf[0];
        const size_t nrel = std::max<size_t>(1, (size_t)t->bm);
        TRY(dev_alloc(t->allocs, &t->inflag[0], GL * nrel));
        TRY(dev_alloc(t->allocs, &t->inflag[1], GL * nrel));
        TRY(dev_alloc(t->allocs, &t->mark[0], (GL * t->bn + 8) & ~(size_t)7));
        TRY(dev_alloc(t->allocs, &t->mark[1], (GL * t->bn + 8) & ~(size_t)7));
        TRY(dev_alloc(t->allocs, &t->hmark[0], GL * t->bn));
        TRY(dev_alloc(t->allocs, &t->hmark[1], GL * t->bn));
        const size_t pe = GW * std::max<size_t>(1, (size_t)t->bhp->nseg);
        TRY(dev_alloc(t->allocs, &t->pp.alt, pe));
        TRY(dev_alloc(t->allocs, &t->pp.du, pe));
        TRY(dev_alloc(t->allocs, &t->pp.uk, pe));
        t->max_iters = 4 * t->bn + 64;
        TRY(dev_alloc(t->allocs, &t->counts, (size_t)t->max_iters + 2));
        if (t->delta > 0.0) {
            t->max_iters = 64 * t->bn + 4096;   // buckets add rounds
            TRY(dev_alloc(t->allocs, &t->counts, (size_t)t->max_iters + 2));
            TRY(dev_alloc(t->allocs, &t->ds.bound, GL));
            TRY(dev_alloc(t->allocs, &t->ds.minrej, GL));
            TRY(dev_alloc(t->allocs, &t->ds.gchanged, GL));
            TRY(dev_alloc(t->allocs, &t->ds.pending, GL * t->bn));
        }
    }
    if (!t->md.complete && t->engine == SPE_ENGINE_FW) {
        const size_t se = GW * n;
        TRY(dev_alloc(t->allocs, &t->st_buf[0].D, se));
        TRY(dev_alloc(t->allocs, &t->st_buf[0].P, se));
        TRY(dev_alloc(t->allocs, &t->st_buf[0].RT, se));
        t->st = t->st_buf[0];
        t->fw_ld = ((int64_t)std::max(1, n) + FWB - 1) / FWB * FWB;
        const size_t ll = (size_t)t->fw_ld * (size_t)t->fw_ld;
        TRY(dev_alloc(t->allocs, &t->fw.D, ll));
        TRY(dev_alloc(t->allocs, &t->fw.R, ll));
        TRY(dev_alloc(t->allocs, &t->fw.N, ll));
    }
    for (int i = 0; i < (t->overlap ? 2 : 1); ++i) {
        TRY(dev_alloc(t->allocs, &t->srcv_buf[i], GW));
        TRY(dev_alloc(t->allocs, &t->srcc_buf[i], GW));
    }
    t->d_srcv = t->srcv_buf[0];
    t->d_srcc = t->srcc_buf[0];
    TRY(dev_alloc(t->allocs, &t->d_min, 1));
    const size_t owned_slots = (size_t)std::max(1, t->blk1 - t->blk0) * WAVE;
    if (t->share) {
        for (int i = 0; i < (t->overlap ? 2 : 1); ++i) {
            TRY(dev_alloc(t->allocs, &t->rsrc_buf[i], owned_slots));
            TRY(dev_alloc(t->allocs, &t->rli_buf[i], owned_slots));
            TRY(dev_alloc(t->allocs, &t->rwa_buf[i], owned_slots));
            TRY(dev_alloc(t->allocs, &t->rng_buf[i], owned_slots / WAVE / RT_B + 2));
        }
        TRY(dev_alloc(t->allocs, &t->d_unsafe, GW));
        if (t->derive) {
            TRY(dev_alloc(t->allocs, &t->d_der, owned_slots));
            TRY(dev_alloc(t->allocs, &t->d_sunsafe, owned_slots));
            const spe::HostGraph& h = g->hg;
            t->nr = (int32_t)h.cx.rcore.size();
            const size_t sx = GW * (size_t)std::max(1, t->nr);
            TRY(dev_alloc(t->allocs, &t->d_dx, sx));
            TRY(dev_alloc(t->allocs, &t->d_rtx, sx));
            std::vector<int32_t> ro((size_t)std::max(1, t->nr), -1);
            for (int32_t r = 0; r < t->nr; ++r) ro[(size_t)r] = h.corev[(size_t)h.cx.rcore[(size_t)r]];
            TRY(dev_upload(t->allocs, ro, &t->d_rorig));
        }
    }
#undef TRY
    // every failure from here on releases what was allocated (spe_table_free)
#define HTRY(expr)                                                                         \
    do {                                                                                   \
        const hipError_t _e = (expr);                                                      \
        if (_e != hipSuccess) {                                                            \
            spe_table_free(t);                                                             \
            return fail(SPE_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
        }                                                                                  \
    } while (0)
    HTRY(hipHostMalloc((void**)&t->h_srcv, 2 * GW * sizeof(int32_t), hipHostMallocDefault));
    if (t->share) {
        HTRY(hipHostMalloc((void**)&t->h_rows,
                           owned_slots * (sizeof(double2) + sizeof(int2) + sizeof(int32_t)) +
                               (owned_slots / WAVE / RT_B + 2) * sizeof(int2),
                           hipHostMallocDefault));
        HTRY(hipHostMalloc((void**)&t->h_unsafe, GW, hipHostMallocDefault));
        if (t->derive) {
            HTRY(hipHostMalloc((void**)&t->h_der, owned_slots * sizeof(DerivedSrc), hipHostMallocDefault));
            HTRY(hipHostMalloc((void**)&t->h_sunsafe, owned_slots, hipHostMallocDefault));
        }
    }
    HTRY(hipHostMalloc((void**)&t->h_counts, std::max<size_t>(64, (size_t)t->max_iters + 2) * sizeof(int32_t),
                       hipHostMallocDefault));
    HTRY(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
    if (t->overlap) {
        HTRY(hipStreamCreateWithFlags(&t->rows_stream, hipStreamNonBlocking));
        HTRY(hipEventCreateWithFlags(&t->ev_relaxed, hipEventDisableTiming));
        HTRY(hipEventCreateWithFlags(&t->ev_rows[0], hipEventDisableTiming));
        HTRY(hipEventCreateWithFlags(&t->ev_rows[1], hipEventDisableTiming));
    }
#undef HTRY
    t->blk_built.assign((size_t)(t->blk1 - t->blk0), t->built ? 1 : 0);
    *out = t;
    return SPE_OK;
}

// Event bracketing around a launch (no-op unless profiling is enabled).
struct LaunchTimer {
    spe_table* t;
    hipStream_t s;
    int kind;
    hipEvent_t a = nullptr, b = nullptr;
    LaunchTimer(spe_table* t_, hipStream_t s_, int kind_) : t(t_), s(s_), kind(kind_) {
        if (!t->prof) return;
        if (t->ev_next + 2 > t->ev_pool.size()) {
            for (int i = 0; i < 256; ++i) {
                hipEvent_t e;
                if (hipEventCreate(&e) != hipSuccess) return;
                t->ev_pool.push_back(e);
            }
        }
        a = t->ev_pool[t->ev_next++];
        b = t->ev_pool[t->ev_next++];
        (void)hipEventRecord(a, s);
    }
    ~LaunchTimer() {
        if (!a) return;
        (void)hipEventRecord(b, s);
        t->pending.push_back({kind, a, b});
    }
};

// all = false: only records whose end event has completed (the rows stream may
// still run); the pool is recycled once nothing is pending.
static int resolve_profile(spe_table* t, bool all = true) {
    std::vector<spe_table::Rec> keep;
    for (auto& r : t->pending) {
        if (!all && hipEventQuery(r.b) != hipSuccess) {
            keep.push_back(r);
            continue;
        }
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, r.a, r.b));
        t->kp.ms[r.kind] += ms;
        t->kp.launches[r.kind] += 1;
        if (t->trace) fprintf(stderr, "spe-trace %d %.4f\n", r.kind, ms);
    }
    t->pending.swap(keep);
    if (t->pending.empty()) t->ev_next = 0;
    return SPE_OK;
}

extern "C++" {
// The FW engine's closure (D, R, N) over the relaxation graph, ld x ld, enqueued on s.
static int fw3_closure(const spe_graph* g, Fw3 M, int64_t ld, hipStream_t s) {
    const int32_t nb = (int32_t)(ld / FWB);
    HIP_TRY(hipFuncSetAttribute((const void*)k_fw3_panel, hipFuncAttributeMaxDynamicSharedMemorySize, FW3_LDS));
    HIP_TRY(hipFuncSetAttribute((const void*)k_fw3_rest, hipFuncAttributeMaxDynamicSharedMemorySize, FW3_REST_LDS));
    k_fw3_init<<<grid_for(ld * ld, 256, 16384), 256, 0, s>>>(ld, M);
    const int32_t nrel = (int32_t)g->hg.icol.size();
    if (nrel > 0) k_fw3_edges<<<(nrel + 255) / 256, 256, 0, s>>>(nrel, ld, g->dev, M);
    // padding rows / columns stay +inf off the diagonal: they never shorten a path
    for (int32_t kb = 0; kb < nb; ++kb) {
        k_fw3_panel<<<1, 256, FW3_LDS, s>>>(kb, nb, ld, M, 0, 0, nb);
        if (nb > 1) k_fw3_panel<<<2 * nb - 2, 256, FW3_LDS, s>>>(kb, nb, ld, M, 1, 0, nb);
        if (nb > 1) k_fw3_rest<<<(nb - 1) * (nb - 1), 256, FW3_REST_LDS, s>>>(kb, nb, ld, M, 0, nb);
    }
    HIP_TRY(hipGetLastError());
    return SPE_OK;
}

// ---- the multi-device FW closure (spe_multi.cpp drives it): 1-D
// row blocks per device; per pivot block the owner relaxes the diagonal tile and
// the pivot row panel, the panel is broadcast, and every device relaxes its own
// rows' column panel and remaining tiles.
namespace spe {
int fw_part(spe_table* t, FwPart* out) {
    if (!t || t->engine != SPE_ENGINE_FW || t->md.complete || !t->fw.D) return set_error(SPE_EINVAL, "not an FW-engine table");
    out->D = t->fw.D;
    out->R = t->fw.R;
    out->N = t->fw.N;
    out->ld = t->fw_ld;
    out->device = t->g->device;
    out->stream = t->stream;
    out->done = &t->fw_done;
    return SPE_OK;
}
int fw_init(const spe_graph* g, const FwPart& p) {
    HIP_TRY(hipSetDevice(p.device));
    HIP_TRY(hipFuncSetAttribute((const void*)k_fw3_panel, hipFuncAttributeMaxDynamicSharedMemorySize, FW3_LDS));
    HIP_TRY(hipFuncSetAttribute((const void*)k_fw3_rest, hipFuncAttributeMaxDynamicSharedMemorySize, FW3_REST_LDS));
    hipStream_t s = (hipStream_t)p.stream;
    const Fw3 M{p.D, p.R, p.N};
    k_fw3_init<<<grid_for(p.ld * p.ld, 256, 16384), 256, 0, s>>>(p.ld, M);
    const int32_t nrel = (int32_t)g->hg.icol.size();
    if (nrel > 0) k_fw3_edges<<<(nrel + 255) / 256, 256, 0, s>>>(nrel, p.ld, g->dev, M);
    HIP_TRY(hipGetLastError());
    return SPE_OK;
}
int fw_pivot_owner(const FwPart& p, int32_t kb) {
    HIP_TRY(hipSetDevice(p.device));
    const int32_t nb = (int32_t)(p.ld / FWB);
    hipStream_t s = (hipStream_t)p.stream;
    const Fw3 M{p.D, p.R, p.N};
    k_fw3_panel<<<1, 256, FW3_LDS, s>>>(kb, nb, p.ld, M, 0, 0, nb);
    if (nb > 1) k_fw3_panel<<<nb - 1, 256, FW3_LDS, s>>>(kb, nb, p.ld, M, 1, 0, nb);   // row panel only
    HIP_TRY(hipGetLastError());
    return SPE_OK;
}
int fw_pivot_rows(const FwPart& p, int32_t kb, int32_t rb0, int32_t rb1) {
    HIP_TRY(hipSetDevice(p.device));
    const int32_t nb = (int32_t)(p.ld / FWB);
    const int32_t rows = (rb1 - rb0) - ((kb >= rb0 && kb < rb1) ? 1 : 0);
    if (rows <= 0 || nb < 2) return SPE_OK;
    hipStream_t s = (hipStream_t)p.stream;
    const Fw3 M{p.D, p.R, p.N};
    k_fw3_panel<<<rows, 256, FW3_LDS, s>>>(kb, nb, p.ld, M, nb, rb0, rb1);   // column panel, own rows
    k_fw3_rest<<<rows * (nb - 1), 256, FW3_REST_LDS, s>>>(kb, nb, p.ld, M, rb0, rb1);
    HIP_TRY(hipGetLastError());
    return SPE_OK;
}
}  // namespace spe

template <int L, int INFL, int OCC = 1, bool DELTA = false, bool RING = false>
static int relax_to_convergence_l(spe_table* t, int32_t blocks, hipStream_t s) {
    static_assert(!RING || (L == 2 * WAVE && !DELTA), "the LDS-ring kernel runs 128-lane rows, no Delta schedule");
    constexpr int M = L > WAVE ? L / WAVE : 1;    // lanes per thread
    const spe_graph* g = t->g;
    const int32_t n = t->bn;      // the batch engine's relaxation graph (core or contracted)
    const int32_t nrel = t->bm;
    const DevGraph& G = *t->bG;
    const HeavyPlan& HP = *t->bhp;
    const int32_t groups = M > 1 ? (blocks + M - 1) / M : blocks * (WAVE / L);    // lane groups
    const int64_t total = (int64_t)groups * n;
    // one resident wave per hardware slot (no second wave of late blocks), multiple of 8 (XCD split)
    int per_cu = 0, cus = 0;
    const void* kfn;
    if constexpr (RING) kfn = t->cx ? (const void*)k_relax_s<INFL, OCC, true> : (const void*)k_relax_s<INFL, OCC>;
    else if constexpr (M > 1) kfn = (const void*)k_relax_m<M, INFL, OCC, DELTA>;
    else kfn = (const void*)k_relax<L, INFL, OCC, DELTA>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, BLOCK, 0) != hipSuccess || per_cu < 1)
        per_cu = 4;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || cus < 1) cus = 256;
    const int relax_grid = (grid_for((total + 7) / 8 * WAVE, BLOCK, per_cu * cus) + 7) & ~7;
    HIP_TRY(hipMemsetAsync(t->counts, 0, sizeof(int32_t) * ((size_t)t->max_iters + 2), s));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)t->counts, 1, 1, s));   // round 0 (the sources) changed
    for (int i = 0; i < 2; ++i) {   // consumers clear what they read; this only guards a failed batch
        HIP_TRY(hipMemsetAsync(t->inflag[i], 0, (size_t)groups * std::max(1, nrel), s));
        HIP_TRY(hipMemsetAsync(t->mark[i], 0, ((size_t)total + 8) & ~(size_t)7, s));
        HIP_TRY(hipMemsetAsync(t->hmark[i], 0, (size_t)total, s));
    }
    {
        LaunchTimer lt(t, s, SPE_K_INIT);
        const dim3 ig(grid_for((int64_t)n * L, BLOCK, std::max(8, 16384 / std::max(1, (int)groups))), groups);
        k_init_state<L><<<ig, BLOCK, 0, s>>>(n, groups, t->d_srcv, G.vfac, G, t->st);
    }
    if constexpr (DELTA) {
        HIP_TRY(hipMemsetAsync(t->ds.pending, 0x7F, sizeof(double) * (size_t)total, s));   // 1.4e306: none
        k_delta_init<<<(groups + BLOCK - 1) / BLOCK, BLOCK, 0, s>>>(groups, t->delta, t->ds);
    }
    {
        LaunchTimer lt(t, s, SPE_K_SEED);
        // the sources "changed in round 0": their out-edges form round 1's frontier
        // (Delta: heavy vertices stay in the light frontier, relaxed by the same kernel)
        k_seed<L><<<(int)(((int64_t)groups * L * WAVE + BLOCK - 1) / BLOCK), BLOCK, 0, s>>>(n, groups, t->d_srcv, G, t->mark[1],
                                                                     DELTA ? t->mark[1] : t->hmark[1], t->inflag[1]);
    }
    const int64_t subs_per_wave = M > 1 ? 1 : WAVE / L;
    // Rounds are enqueued in chunks sized by the previous batch's round count
    // (batches of one graph converge in similar counts); rounds after the
    // converged one exit at once, so one host check per batch is typical.
    int32_t it = 1;
    int32_t chunk = t->last_rounds > 0 ? t->last_rounds + 1 : 8;
    for (;;) {
        for (int32_t q = 0; q < chunk; ++q, ++it) {
            if (it > t->max_iters) return fail(SPE_ESTATE, "relaxation did not converge");
            Flags fl{t->mark[it & 1],   t->mark[(it + 1) & 1],   t->hmark[it & 1],
                     t->hmark[(it + 1) & 1], t->inflag[it & 1], t->inflag[(it + 1) & 1], t->counts + it,
                     t->counts + it - 1};
            if constexpr (DELTA) fl.hmark_next = fl.mark_next;   // heavy rows relaxed by k_relax too
            {
                LaunchTimer lt(t, s, SPE_K_RELAX);
                if constexpr (RING) {
                    if (t->cx)
                        k_relax_s<INFL, OCC, true><<<relax_grid, BLOCK, 0, s>>>((int32_t)total, n, t->d_srcc, G, t->st, fl);
                    else
                        k_relax_s<INFL, OCC><<<relax_grid, BLOCK, 0, s>>>((int32_t)total, n, t->d_srcc, G, t->st, fl);
                }
                else if constexpr (M > 1)
                    k_relax_m<M, INFL, OCC, DELTA><<<relax_grid, BLOCK, 0, s>>>((int32_t)total, n, t->d_srcc, G,
                                                                                t->st, fl, t->ds);
                else
                    k_relax<L, INFL, OCC, DELTA><<<relax_grid, BLOCK, 0, s>>>((int32_t)total, n, t->d_srcc, G,
                                                                              t->st, fl, t->ds);
            }
            if constexpr (DELTA) {
                k_delta_advance<<<groups, BLOCK, 0, s>>>(n, nrel, t->delta, G, t->ds, fl.mark_next, fl.in_next,
                                                         t->counts + it);
            } else if (HP.nheavy > 0) {
                LaunchTimer lt(t, s, SPE_K_HEAVY);
                const int64_t pw = ((int64_t)groups * HP.nseg + subs_per_wave - 1) / subs_per_wave;
                const int64_t cw = ((int64_t)groups * HP.nheavy + subs_per_wave - 1) / subs_per_wave;
                if constexpr (M > 1) {
                    if (t->cx) {
                        k_heavy_partial_m<M, SPE_HEAVY_CX_INFL, true><<<grid_for(pw * WAVE, BLOCK, 4096), BLOCK, 0, s>>>(
                            groups, n, t->d_srcc, G, t->st, HP, t->pp, fl);
                        k_heavy_combine_m<M, true><<<grid_for(cw * WAVE, BLOCK, 4096), BLOCK, 0, s>>>(
                            groups, n, t->d_srcc, G, t->st, HP, t->pp, fl);
                    } else {
                        k_heavy_partial_m<M, INFL><<<grid_for(pw * WAVE, BLOCK, 4096), BLOCK, 0, s>>>(
                            groups, n, t->d_srcc, G, t->st, HP, t->pp, fl);
                        k_heavy_combine_m<M><<<grid_for(cw * WAVE, BLOCK, 4096), BLOCK, 0, s>>>(
                            groups, n, t->d_srcc, G, t->st, HP, t->pp, fl);
                    }
                } else {
                    k_heavy_partial<L><<<grid_for(pw * WAVE, BLOCK, 4096), BLOCK, 0, s>>>(groups, n, t->d_srcc, G,
                                                                                          t->st, HP, t->pp, fl);
                    k_heavy_combine<L><<<grid_for(cw * WAVE, BLOCK, 4096), BLOCK, 0, s>>>(groups, n, t->d_srcc, G,
                                                                                          t->st, HP, t->pp, fl);
                }
            }
        }
        HIP_TRY(hipMemcpyAsync(t->h_counts, t->counts, sizeof(int32_t) * (size_t)it, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        t->stats.launches += chunk;
        if (t->h_counts[it - 1] == 0) break;
        chunk = 2;
    }
    // the first round that changed nothing ends the relaxation (work accounting)
    int32_t rounds = 1;
    while (rounds < it && t->h_counts[rounds] != 0) ++rounds;
    t->stats.active_rounds += rounds - 1;
    t->stats.iterations += rounds;
    t->last_rounds = rounds;
    return SPE_OK;
}

static int relax_to_convergence(spe_table* t, int32_t blocks, hipStream_t s) {
    if (t->delta > 0.0)   // measured slower
        return t->lanes == 128 ? relax_to_convergence_l<128, 4, 1, true>(t, blocks, s)
                               : relax_to_convergence_l<64, 8, 1, true>(t, blocks, s);
    if (t->lanes == 64) return relax_to_convergence_l<64, 8>(t, blocks, s);
    if (t->relax_kernel == SPE_RELAX_LDS_RING) {
        if (t->infl == 4) return relax_to_convergence_l<128, 4, 8, false, true>(t, blocks, s);
        if (t->infl == 6) return relax_to_convergence_l<128, 6, 6, false, true>(t, blocks, s);
        return relax_to_convergence_l<128, 5, 7, false, true>(t, blocks, s);
    }
    if (t->infl == 4) return relax_to_convergence_l<128, 4>(t, blocks, s);
    return t->occ == 6 ? relax_to_convergence_l<128, 2, 6>(t, blocks, s) : relax_to_convergence_l<128, 2>(t, blocks, s);
}

static void launch_rows_sssp(spe_table* t, int grid, int32_t blocks, int32_t sb0, hipStream_t s) {
#define ROWS(LL)                                                                                              \
    do {                                                                                                      \
        if (t->tb.aux)                                                                                        \
            k_rows_sssp<LL, true><<<grid, BLOCK, 0, s>>>(t->bn, blocks, sb0, t->d_srcv, t->d_slots, *t->bG,   \
                                                         t->md, t->st, t->tb);                                \
        else                                                                                                  \
            k_rows_sssp<LL, false><<<grid, BLOCK, 0, s>>>(t->bn, blocks, sb0, t->d_srcv, t->d_slots,          \
                                                          *t->bG, t->md, t->st, t->tb);                       \
    } while (0)
    switch (t->lanes) {
        case 128: ROWS(128); break;
        default: ROWS(64); break;
    }
#undef ROWS
}
#ifndef SPE_SHARED_ROWS_LDS
#define SPE_SHARED_ROWS_LDS 1
#endif
static void launch_rows_shared(spe_table* t, int grid, int32_t blocks, int32_t sb0, hipStream_t s,
                               const int32_t* rsrc, const int2* rli, const double2* rwa, const int2* rng) {
    if (SPE_SHARED_ROWS_LDS && !t->cx) {   // (contracted targets read three rows: the gather kernel)
        const int64_t work = (int64_t)((blocks + RT_B - 1) / RT_B) * ((t->A + RT_T - 1) / RT_T);
        const int g = (int)std::max<int64_t>(1, std::min<int64_t>(work, 2048));
        if (t->lanes == 128)
            k_rows_shared_lds<128><<<g, BLOCK, 0, s>>>(t->bn, blocks, sb0, rsrc, t->d_slots, *t->bG, t->md, t->st,
                                                       t->tb, rli, rwa, rng);
        else
            k_rows_shared_lds<64><<<g, BLOCK, 0, s>>>(t->bn, blocks, sb0, rsrc, t->d_slots, *t->bG, t->md, t->st,
                                                      t->tb, rli, rwa, rng);
        return;
    }
    if (t->lanes == 128)
        k_rows_sssp<128, false, true><<<grid, BLOCK, 0, s>>>(t->bn, blocks, sb0, rsrc, t->d_slots, *t->bG, t->md,
                                                              t->st, t->tb, rli, rwa);
    else
        k_rows_sssp<64, false, true><<<grid, BLOCK, 0, s>>>(t->bn, blocks, sb0, rsrc, t->d_slots, *t->bG, t->md,
                                                             t->st, t->tb, rli, rwa);
}
}  // extern "C++"

int spe_table_build(spe_table* t, void* stream) {
    if (!t) return fail(SPE_EINVAL, "NULL table");
    if (t->multi) {
        const int r = spe::multi_build(t->multi, &t->stats);
        t->built = r == SPE_OK && spe::multi_built(t->multi);
        return r;
    }
    int r = spe_table_build_blocks(t, t->blk0, t->blk1, stream);
    if (r || !t->d_rank || t->md.complete) return r;
    hipStream_t s = stream ? (hipStream_t)stream : t->stream;
    const int64_t items = (int64_t)((t->A + WAVE - 1) / WAVE) * t->A;
    k_owner_replay<<<grid_for(items * WAVE, BLOCK, 8192), BLOCK, 0, s>>>(t->A, t->d_rank, t->d_slot_vertex,
                                                                        t->g->dev, t->md, t->tb);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    return SPE_OK;
}

static int build_blocks_impl(spe_table* t, int32_t block_begin, int32_t block_end, void* stream);

int spe_table_build_blocks(spe_table* t, int32_t block_begin, int32_t block_end, void* stream) {
    if (!t) return fail(SPE_EINVAL, "NULL table");
    if (t->multi) return fail(SPE_EUNSUPPORTED, "a multi-device table builds whole (spe_table_build)");
    if (block_begin < t->blk0 || block_end > t->blk1 || block_begin > block_end)
        return fail(SPE_EINVAL, "block range not owned by this table");
    const int r = build_blocks_impl(t, block_begin, block_end, stream);
    if (r) return r;
    for (int32_t b = block_begin; b < block_end; ++b) t->blk_built[(size_t)(b - t->blk0)] = 1;
    t->built = std::all_of(t->blk_built.begin(), t->blk_built.end(), [](uint8_t x) { return x != 0; });
    return SPE_OK;
}

int spe_table_build_blocks_into(spe_table* t, int32_t block_begin, int32_t block_end, void* latrel, void* next_hop,
                                void* hops, void* stream) {
    if (!t) return fail(SPE_EINVAL, "NULL table");
    if (t->multi) return fail(SPE_EUNSUPPORTED, "a multi-device table builds whole (spe_table_build)");
    if (block_begin < t->blk0 || block_end > t->blk1 || block_begin > block_end)
        return fail(SPE_EINVAL, "block range not owned by this table");
    if (!latrel || !next_hop || !hops) return fail(SPE_EINVAL, "spe_table_build_blocks_into needs all three fields");
    if (t->tb.prev || t->tb.aux) return fail(SPE_EUNSUPPORTED, "owner-replay / want_aux tables build in place");
    const Table keep = t->tb;
    const int32_t keep_base = t->row_base;
    t->tb.lr = (double2*)latrel;
    t->tb.next = (int32_t*)next_hop;
    t->tb.hops = (uint16_t*)hops;
    t->row_base = block_begin;
    const int r = build_blocks_impl(t, block_begin, block_end, stream);
    t->tb = keep;
    t->row_base = keep_base;
    return r;   // the table's own storage is untouched: nothing is marked built
}

// Shared anchor trees and derived rows: a batch's relaxation lanes
// are its ROOTS -- each core source, and the anchor of each pruned pendant source,
// once -- and the rows kernel gives every source its root's row (a pendant
// source's with its edge in front).  On a contracted graph a removed source whose
// three neighbours are all roots of the call's range takes no lane (derived, see
// k_rows_derived); any other removed source relaxes on its own lane.  Batches are
// cut at block boundaries into about equal root counts.  Where the weights' sums
// are not exact, k_share_check flags roots whose decisions an offset could change;
// the blocks holding an offset source (pendant or derived) of a flagged root, or a
// source whose derived row failed its own margin (sunsafe), are rebuilt with one
// lane per source.
static int build_shared(spe_table* t, int32_t block_begin, int32_t block_end, hipStream_t s) {
    const spe_graph* g = t->g;
    const spe::HostGraph& h = g->hg;
    const int32_t L = t->lanes;
    const int32_t cap = t->groups * WAVE;   // root lanes one batch's state holds
    const int32_t s_end = std::min(t->A, block_end * WAVE);
    // per slot: root core id (core source, pendant anchor, or a removed source itself),
    // or -3 for a derived source, -1 padding
    // derivable sources (h.cx.der: removed vertices, degree-4 kept ones); neighbour q
    // of such a source = entry q of its core in-list (G.rnb order for a removed one)
    auto removed = [&](int32_t c) { return t->derive && c >= 0 && h.cx.der[(size_t)c]; };
    auto ndeg = [&](int32_t c) { return h.iptr[(size_t)c + 1] - h.iptr[(size_t)c]; };
    auto nbr = [&](int32_t c, int q) { return h.icol[(size_t)h.iptr[(size_t)c] + q]; };
    std::vector<int32_t> tag((size_t)std::max(1, h.nc), -1), lane_of((size_t)std::max(1, h.nc), -1);
    // the call's non-derived roots: a removed source is derivable iff its three neighbours are among them
    int32_t total = 0;
    for (int32_t i = block_begin * WAVE; i < s_end; ++i) {
        const int32_t v = t->attached[(size_t)i];
        const int32_t c0 = h.core_id[(size_t)v];
        const int32_t c = c0 >= 0 ? c0 : h.anchor_core[(size_t)v];
        if (c >= 0 && !removed(c) && tag[(size_t)c] < 0) {
            tag[(size_t)c] = 0;
            ++total;
        }
    }
    std::vector<uint8_t> derivable((size_t)std::max(0, s_end - block_begin * WAVE), 0);
    for (int32_t i = block_begin * WAVE; i < s_end; ++i) {
        const int32_t c = h.core_id[(size_t)t->attached[(size_t)i]];
        if (!removed(c)) continue;
        bool all = true;
        for (int q = 0; q < ndeg(c); ++q) all &= tag[(size_t)nbr(c, q)] == 0;
        derivable[(size_t)(i - block_begin * WAVE)] = all;
        if (!all) ++total;
    }
    auto root_of = [&](int32_t slot) -> int32_t {
        const int32_t v = t->attached[(size_t)slot];
        const int32_t c0 = h.core_id[(size_t)v];
        if (c0 >= 0 && removed(c0) && derivable[(size_t)(slot - block_begin * WAVE)]) return -3;
        return c0 >= 0 ? c0 : h.anchor_core[(size_t)v];
    };
    const int32_t nb = std::max(1, (total + cap - 1) / cap);
    const int32_t target = (total + nb - 1) / nb;
    std::fill(tag.begin(), tag.end(), -1);
    std::vector<int32_t> roots, deferred;
    std::vector<uint8_t> bad((size_t)std::max(1, h.nc), 0);
    std::vector<uint8_t> dk((size_t)(block_end - block_begin) * WAVE, 0);   // per slot of the batch: derived
    const spe::HostGraph::Share& sh = h.share;
    for (int32_t b = block_begin, bid = 0; b < block_end; ++bid) {
        HIP_TRY(hipStreamSynchronize(s));   // the pinned staging is reused per batch
        roots.clear();
        int32_t e = b;
        auto add = [&](int32_t c) {
            if (c >= 0 && tag[(size_t)c] != bid) {
                tag[(size_t)c] = bid;
                lane_of[(size_t)c] = (int32_t)roots.size();
                roots.push_back(c);
            }
        };
        // The roots of the blocks' other sources first (the cut counts those), then each
        // derivable source of the batch: derived when at most one of its neighbours is
        // not yet a root of the batch (that one becomes a root: no more lanes than the
        // source's own), else on its own lane -- small batches would otherwise re-relax
        // hubs batch after batch.  A batch the second step would overflow is cut before
        // the block that overflows and assembled again (one block always fits: each of
        // its sources costs at most one lane).
        const int32_t limit = bid + 1 >= nb ? cap : std::min(target, cap);
        int32_t e_max = block_end;
        for (;;) {
            roots.clear();
            e = b;
            while (e < e_max) {
                const size_t before = roots.size();
                for (int32_t l = 0; l < WAVE; ++l) {
                    const int32_t slot = e * WAVE + l;
                    if (slot >= t->A) break;
                    const int32_t c = root_of(slot);
                    if (c != -3) add(c);
                }
                // this block starts the next batch (the last planned batch takes the rest up to `cap`)
                if (e > b && (int32_t)roots.size() > limit) {
                    for (size_t i = before; i < roots.size(); ++i) tag[(size_t)roots[i]] = -1;
                    roots.resize(before);
                    break;
                }
                ++e;
            }
            std::fill(dk.begin(), dk.begin() + (size_t)(e - b) * WAVE, 0);
            int32_t over = -1;
            for (int32_t i = 0; i < (e - b) * WAVE && over < 0; ++i) {
                const int32_t slot = b * WAVE + i;
                if (slot >= t->A || root_of(slot) != -3) continue;
                const int32_t x = h.core_id[(size_t)t->attached[(size_t)slot]];
                int32_t miss = 0;
                for (int q = 0; q < ndeg(x); ++q) miss += tag[(size_t)nbr(x, q)] != bid;
                if (miss > 0 && (int32_t)roots.size() >= cap) {
                    over = b + i / WAVE;
                    break;
                }
                if (miss <= 1) {
                    for (int q = 0; q < ndeg(x); ++q) add(nbr(x, q));
                    dk[(size_t)i] = 1;
                } else {
                    add(x);
                }
            }
            if (over < 0) break;
            for (int32_t c : roots) tag[(size_t)c] = -1;
            e_max = std::max(b + 1, over);
        }
        const int32_t R = (int32_t)roots.size();
        if (R > cap) return fail(SPE_ESTATE, "shared batch exceeds the state (one block's roots > groups * 64)");
        const int32_t nblk = e - b;
        // relaxation lanes: the roots (core sources of the batch engine's state)
        const int32_t bpg = std::max(1, L / WAVE);
        const int32_t rb = std::max(1, (R + WAVE - 1) / WAVE);
        const int32_t pb = (rb + bpg - 1) / bpg * bpg;
        for (int32_t i = 0; i < pb * WAVE; ++i) {
            const int32_t c = i < R ? roots[(size_t)i] : -1;
            t->h_srcv[i] = c < 0 ? -1 : h.corev[(size_t)c];
            int32_t cc = c;
            if (t->cx && c >= 0) cc = h.cx.kid[(size_t)c] >= 0 ? h.cx.kid[(size_t)c] : -2;
            t->h_srcv[pb * WAVE + i] = cc;
        }
        // rows: every source slot of blocks [b, e), its root's lane and pendant prefix,
        // or (derived) its record of neighbour lanes
        const size_t ns = (size_t)nblk * WAVE;
        double2* hw = reinterpret_cast<double2*>(t->h_rows);
        int2* hl = reinterpret_cast<int2*>(hw + ns);
        int32_t* hr = reinterpret_cast<int32_t*>(hl + ns);
        int32_t nder = 0;
        for (int32_t i = 0; i < nblk * WAVE; ++i) {
            const int32_t slot = b * WAVE + i;
            int32_t c = slot < t->A ? root_of(slot) : -1;
            if (c == -3 && !dk[(size_t)i]) c = h.core_id[(size_t)t->attached[(size_t)slot]];   // on its own lane
            const int32_t v = (slot < t->A && c != -1) ? t->attached[(size_t)slot] : -1;
            hr[i] = v;
            hw[i] = make_double2(0.0, 1.0);
            if (c == -3) {
                const int32_t x = h.core_id[(size_t)v];
                DerivedSrc d;
                for (int q = 0; q < DER_K; ++q) {
                    const bool on = q < ndeg(x);
                    const size_t k = on ? (size_t)h.iptr[(size_t)x] + q : 0;
                    d.lane[q] = on ? lane_of[(size_t)nbr(x, q)] : -1;
                    d.hop[q] = on ? h.corev[(size_t)nbr(x, q)] : -1;
                    d.w[q] = on ? h.iw[k] : INF;
                    d.a[q] = on ? h.ia[k] : 1.0;
                }
                t->h_der[nder] = d;
                hl[i] = make_int2(d.lane[0], -2 - nder);
                ++nder;
                continue;
            }
            hl[i] = make_int2(c >= 0 ? lane_of[(size_t)c] : -1, -1);
            if (v >= 0 && h.core_id[(size_t)v] < 0) {   // pendant: the edge s -> anchor in front
                const int32_t kx = h.fiptr[(size_t)v];
                const double fs = h.vfac[(size_t)v];
                hl[i].y = h.corev[(size_t)h.anchor_core[(size_t)v]];
                hw[i] = make_double2(h.fiw[(size_t)kx], (std::isnan(fs) ? 1.0 : 1.0 * fs) * h.fia[(size_t)kx]);
            }
        }
        // per tile of RT_B blocks: the span of root lanes its sources read (k_rows_shared_lds)
        const int32_t ntile = (nblk + RT_B - 1) / RT_B;
        int2* hg = reinterpret_cast<int2*>(hr + ns);
        for (int32_t k = 0; k < ntile; ++k) {
            int32_t lo = INT32_MAX, hi = -1;
            for (int32_t i = k * RT_B * WAVE; i < std::min(nblk, (k + 1) * RT_B) * WAVE; ++i)
                if (hl[i].x >= 0) {
                    lo = std::min(lo, hl[i].x);
                    hi = std::max(hi, hl[i].x);
                }
            hg[k] = hi >= 0 ? make_int2(lo, hi) : make_int2(0, -1);
        }
        int32_t* d_rsrc = t->rsrc_buf[0];
        int2* d_rli = t->rli_buf[0];
        double2* d_rwa = t->rwa_buf[0];
        int2* d_rng = t->rng_buf[0];
        HIP_TRY(hipMemcpyAsync(t->d_srcv, t->h_srcv, sizeof(int32_t) * pb * WAVE, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(t->d_srcc, t->h_srcv + pb * WAVE, sizeof(int32_t) * pb * WAVE, hipMemcpyHostToDevice,
                               s));
        HIP_TRY(hipMemcpyAsync(d_rsrc, hr, sizeof(int32_t) * ns, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_rli, hl, sizeof(int2) * ns, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_rwa, hw, sizeof(double2) * ns, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(d_rng, hg, sizeof(int2) * ntile, hipMemcpyHostToDevice, s));
        if (nder > 0) HIP_TRY(hipMemcpyAsync(t->d_der, t->h_der, sizeof(DerivedSrc) * nder, hipMemcpyHostToDevice, s));
        int r = relax_to_convergence(t, rb, s);
        if (r) return r;
        t->stats.relaxed_lanes += R;
        t->stats.derived_sources += nder;
        bool any_bad = false;
        if (!sh.exact) {
            const int32_t groups = L > WAVE ? pb / bpg : pb * (WAVE / L);
            HIP_TRY(hipMemsetAsync(t->d_unsafe, 0, (size_t)groups * L, s));
            {
                LaunchTimer lt(t, s, SPE_K_HEAVY);   // (accounted with the heavy-vertex passes)
                const int grid = grid_for((int64_t)groups * (t->bn + t->bhp->nseg) * WAVE, BLOCK, 8192);
                const double hmax = (double)h.n + 2.0;
                if (L == 128)
                    k_share_check<128><<<grid, BLOCK, 0, s>>>(groups, t->bn, t->d_srcv, *t->bG, t->st, *t->bhp,
                                                              sh.wmin, sh.omax, hmax, t->d_unsafe);
                else
                    k_share_check<64><<<grid, BLOCK, 0, s>>>(groups, t->bn, t->d_srcv, *t->bG, t->st, *t->bhp,
                                                             sh.wmin, sh.omax, hmax, t->d_unsafe);
            }
            HIP_TRY(hipMemcpyAsync(t->h_unsafe, t->d_unsafe, (size_t)R, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            for (int32_t i = 0; i < R; ++i)
                if (t->h_unsafe[i]) {
                    bad[(size_t)roots[(size_t)i]] = 1;
                    any_bad = true;
                }
        }
        const int32_t sb0 = b - t->row_base;
        {
            LaunchTimer lt(t, s, SPE_K_ROWS);
            if (t->derive) {
                HIP_TRY(hipMemsetAsync(t->d_sunsafe, 0, ns, s));
                const double hmax = (double)h.n + 2.0;
                if (t->nr > 0) {
                    const int32_t groups = pb / bpg;   // (L = 128: contracted tables)
                    const int grid = grid_for((int64_t)groups * t->nr * WAVE, BLOCK, 8192);
                    k_expand_removed<128><<<grid, BLOCK, 0, s>>>(groups, t->bn, t->nr, *t->bG, t->st, t->d_dx,
                                                                 t->d_rtx, t->d_rorig, sh.exact ? 0 : 1, sh.wmin,
                                                                 sh.omax, hmax);
                }
                const int64_t items = (int64_t)((t->A + SPE_DERIVED_TT - 1) / SPE_DERIVED_TT) * nblk;
                const int grid = (grid_for(items * WAVE, BLOCK, 8192) + 7) & ~7;
                k_rows_derived<128, SPE_DERIVED_TT><<<grid, BLOCK, 0, s>>>(
                    t->bn, nblk, sb0, d_rsrc, t->d_slots, *t->bG, t->md, t->st, t->tb, d_rli, d_rwa, t->d_der,
                    t->d_dx, t->d_rtx, t->nr, sh.wmin, sh.omax, hmax, sh.exact ? 1 : 0, t->d_sunsafe);
            } else {
                launch_rows_shared(t, grid_for((int64_t)nblk * t->A * WAVE, BLOCK, 8192), nblk, sb0, s, d_rsrc,
                                   d_rli, d_rwa, d_rng);
            }
        }
        if (t->md.prefer) {
            LaunchTimer lt(t, s, SPE_K_DIRECT);
            k_direct_overlay<<<(nblk * WAVE + BLOCK - 1) / BLOCK, BLOCK, 0, s>>>(nblk, sb0, d_rsrc, t->d_vertex_slot,
                                                                                 g->dev, t->tb);
        }
        HIP_TRY(hipGetLastError());
        bool any_sunsafe = false;
        if (t->derive) {
            HIP_TRY(hipMemcpyAsync(t->h_sunsafe, t->d_sunsafe, ns, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            for (size_t i = 0; i < ns && !any_sunsafe; ++i) any_sunsafe = t->h_sunsafe[i] != 0;
        }
        if (any_bad || any_sunsafe)
            for (int32_t blk = b; blk < e; ++blk)
                for (int32_t l = 0; l < WAVE; ++l) {
                    const int32_t slot = blk * WAVE + l;
                    if (slot >= t->A) break;
                    const size_t i = (size_t)(slot - b * WAVE);
                    bool d = any_sunsafe && t->h_sunsafe[i];
                    const int32_t v = t->attached[(size_t)slot];
                    int32_t c = root_of(slot);
                    if (c == -3 && !dk[i]) c = h.core_id[(size_t)v];
                    if (!d && any_bad) {
                        // an offset source of a flagged root (a core source is its own root: exact)
                        if (c == -3) {
                            const int32_t x = h.core_id[(size_t)v];
                            for (int q = 0; q < ndeg(x); ++q) d |= bad[(size_t)nbr(x, q)] != 0;
                        } else if (c >= 0 && h.core_id[(size_t)v] != c) {
                            d = bad[(size_t)c] != 0;
                        }
                    }
                    if (d) {
                        deferred.push_back(blk);
                        break;
                    }
                }
        if (t->prof) {
            HIP_TRY(hipStreamSynchronize(s));
            r = resolve_profile(t, true);
            if (r) return r;
        }
        b = e;
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (!deferred.empty()) {   // one lane per source for the flagged blocks
        std::sort(deferred.begin(), deferred.end());
        deferred.erase(std::unique(deferred.begin(), deferred.end()), deferred.end());
        spe_build_stats keep = t->stats;
        t->share_off = true;
        int r = SPE_OK;
        for (size_t i = 0; i < deferred.size() && !r;) {
            size_t j = i + 1;
            while (j < deferred.size() && deferred[j] == deferred[j - 1] + 1) ++j;
            r = build_blocks_impl(t, deferred[i], deferred[j - 1] + 1, s);
            keep.iterations += t->stats.iterations;
            keep.active_rounds += t->stats.active_rounds;
            keep.launches += t->stats.launches;
            keep.relaxed_lanes += t->stats.relaxed_lanes;
            keep.fallback_blocks += deferred[j - 1] + 1 - deferred[i];
            i = j;
        }
        t->share_off = false;
        t->stats = keep;
        if (r) return r;
    }
    return SPE_OK;
}

static int build_blocks_impl(spe_table* t, int32_t block_begin, int32_t block_end, void* stream) {
    HIP_TRY(hipSetDevice(t->g->device));
    if (t->trace)   // where the relaxation state lives (run-to-run placement studies)
        for (int i = 0; i < 2; ++i)
            fprintf(stderr, "spe-trace-buf %d D %p P %p RT %p in %p mark %p\n", i, (void*)t->st_buf[i].D,
                    (void*)t->st_buf[i].P, (void*)t->st_buf[i].RT, (void*)t->inflag[i], (void*)t->mark[i]);
    hipStream_t s = stream ? (hipStream_t)stream : t->stream;
    const auto t0 = std::chrono::steady_clock::now();
    const spe_graph* g = t->g;
    t->stats = spe_build_stats{};
    const bool ovl = t->overlap && !t->md.complete && t->engine == SPE_ENGINE_BATCH;
    hipStream_t rs = ovl ? t->rows_stream : s;
    if (t->share && !t->share_off) {
        // one stream: the rows kernel's grid holds every CU slot while it runs, so a
        // concurrent relaxation of the next batch only queues behind it (the launches
        // between them wait for slots); one batch of every root, then its rows, was
        // as fast or faster (C4 0.1275 vs 0.130 s, same box, two passes)
        const int r = build_shared(t, block_begin, block_end, s);
        if (r) return r;
        t->stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        t->stats.n_devices = 1;
        return SPE_OK;
    }
    int buf = 0;
    for (int32_t b = block_begin; b < block_end; b += t->groups) {
        const int32_t groups = std::min(t->groups, block_end - b);
        HIP_TRY(hipStreamSynchronize(s));   // h_srcv is reused per batch
        if (ovl) {   // this batch's buffers: free once the rows two batches back are written
            t->st = t->st_buf[buf];
            t->d_srcv = t->srcv_buf[buf];
            t->d_srcc = t->srcc_buf[buf];
            if (t->rows_pending[buf]) HIP_TRY(hipStreamWaitEvent(s, t->ev_rows[buf], 0));
        }
        // blocks of source entries: a lane group of L > 64 spans L / 64 blocks, so
        // an odd tail is padded with empty (-1) blocks
        const int32_t bpg = std::max(1, t->lanes / WAVE);
        const int32_t pb = (groups + bpg - 1) / bpg * bpg;
        for (int32_t gi = 0; gi < pb; ++gi)
            for (int32_t l = 0; l < WAVE; ++l) {
                const int32_t slot = (b + gi) * WAVE + l;
                const int32_t v = (gi < groups && slot < t->A) ? t->attached[slot] : -1;
                t->h_srcv[gi * WAVE + l] = v;
                int32_t c = v < 0 ? -1 : (g->hg.core_id[v] >= 0 ? g->hg.core_id[v] : -2);
                if (t->cx && c >= 0) c = g->hg.cx.kid[c] >= 0 ? g->hg.cx.kid[c] : -2;   // (a contracted source: -2)
                t->h_srcv[(pb + gi) * WAVE + l] = c;
            }
        HIP_TRY(hipMemcpyAsync(t->d_srcv, t->h_srcv, sizeof(int32_t) * pb * WAVE, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(t->d_srcc, t->h_srcv + pb * WAVE, sizeof(int32_t) * pb * WAVE,
                               hipMemcpyHostToDevice, s));
        const int32_t sb0 = b - t->row_base;
        const int64_t items = (int64_t)groups * t->A;
        const int row_grid = grid_for(items * WAVE, BLOCK, 8192);
        if (t->md.complete) {
            LaunchTimer lt(t, s, SPE_K_DIRECT);
            k_rows_direct<<<row_grid, BLOCK, 0, s>>>(groups, sb0, t->d_srcv, t->d_slot_vertex, g->dev, t->md, t->tb);
        } else if (t->engine == SPE_ENGINE_LDS) {
            {
                LaunchTimer lt(t, s, SPE_K_LDS);
                const int32_t s0 = b * WAVE, s1 = std::min(t->A, (b + groups) * WAVE);
                const size_t bytes = lds_bytes(g->hg.nc);
                int grid = std::min(s1 - s0, t->lds_grid);
                if (grid >= 8) grid -= grid % 8;   // whole XCD rounds (see k_sssp_lds's slot order)
                if (t->lds_debug && !t->d_lds_dbg) {
                    if (int r = dev_alloc(t->allocs, &t->d_lds_dbg, 16)) return r;
                    HIP_TRY(hipMemset(t->d_lds_dbg, 0, 16 * sizeof(unsigned long long)));
                }
                k_sssp_lds<<<std::max(1, grid), LDS_T, bytes, s>>>(s0, s1, t->d_slots, t->row_base, g->dev, t->md, t->tb,
                                                                   t->lsc, t->d_lds_dbg);
                if (t->d_lds_dbg) {
                    unsigned long long h[16];
                    HIP_TRY(hipStreamSynchronize(s));
                    HIP_TRY(hipMemcpy(h, t->d_lds_dbg, sizeof(h), hipMemcpyDeviceToHost));
                    const double nsrc = (double)std::max(1ull, h[10]);
                    fprintf(stderr, "spe-lds sources %llu rounds/src %.1f levels/src %.1f us/src: init %.1f push %.1f "
                            "parent %.1f lat %.1f tree-build %.1f tree-pass %.1f rows %.1f | push: wave0 flush %.1f barrier %.1f\n", h[10], h[8] / nsrc, h[9] / nsrc,
                            h[0] / nsrc / 100.0, h[1] / nsrc / 100.0, h[2] / nsrc / 100.0, h[3] / nsrc / 100.0,
                            h[4] / nsrc / 100.0, h[5] / nsrc / 100.0, h[6] / nsrc / 100.0, h[11] / nsrc / 100.0,
                            h[12] / nsrc / 100.0);
                }
            }
            if (t->md.prefer) {
                LaunchTimer lt(t, s, SPE_K_DIRECT);
                k_direct_overlay<<<(groups * WAVE + BLOCK - 1) / BLOCK, BLOCK, 0, s>>>(
                    groups, sb0, t->d_srcv, t->d_vertex_slot, g->dev, t->tb);
            }
        } else if (t->engine == SPE_ENGINE_FW) {
            if (!t->fw_done) {
                LaunchTimer lt(t, s, SPE_K_FW);
                if (int r = fw3_closure(g, t->fw, t->fw_ld, s)) return r;
                t->fw_done = true;
            }
            {
                LaunchTimer lt(t, s, SPE_K_FW);
                k_fw_state<<<dim3((g->hg.nc + WAVE - 1) / WAVE, groups), BLOCK, 0, s>>>(
                    g->hg.nc, t->fw_ld, t->d_srcv, t->d_srcc, g->dev, t->fw, t->st);
            }
            {
                LaunchTimer lt(t, s, SPE_K_ROWS);
                launch_rows_sssp(t, row_grid, groups, sb0, s);
            }
            if (t->md.prefer) {
                LaunchTimer lt(t, s, SPE_K_DIRECT);
                k_direct_overlay<<<(groups * WAVE + BLOCK - 1) / BLOCK, BLOCK, 0, s>>>(
                    groups, sb0, t->d_srcv, t->d_vertex_slot, g->dev, t->tb);
            }
        } else {
            int r = relax_to_convergence(t, groups, s);
            if (r) return r;
            t->stats.relaxed_lanes += std::max(0, std::min(t->A, (b + groups) * WAVE) - b * WAVE);
            if (ovl) {
                HIP_TRY(hipEventRecord(t->ev_relaxed, s));
                HIP_TRY(hipStreamWaitEvent(rs, t->ev_relaxed, 0));
            }
            {
                LaunchTimer lt(t, rs, SPE_K_ROWS);
                launch_rows_sssp(t, row_grid, groups, sb0, rs);
            }
            if (t->md.prefer) {
                LaunchTimer lt(t, rs, SPE_K_DIRECT);
                k_direct_overlay<<<(groups * WAVE + BLOCK - 1) / BLOCK, BLOCK, 0, rs>>>(
                    groups, sb0, t->d_srcv, t->d_vertex_slot, g->dev, t->tb);
            }
            if (ovl) {
                HIP_TRY(hipEventRecord(t->ev_rows[buf], rs));
                t->rows_pending[buf] = true;
                buf ^= 1;
            }
        }
        HIP_TRY(hipGetLastError());
        if (t->prof) {
            HIP_TRY(hipStreamSynchronize(s));
            int r = resolve_profile(t, !ovl);
            if (r) return r;
        }
    }
    if (ovl) {
        HIP_TRY(hipStreamSynchronize(rs));
        t->rows_pending[0] = t->rows_pending[1] = false;
        t->st = t->st_buf[0];
        t->d_srcv = t->srcv_buf[0];
        t->d_srcc = t->srcc_buf[0];
        if (t->prof) {
            int r = resolve_profile(t);
            if (r) return r;
        }
    }
    HIP_TRY(hipStreamSynchronize(s));
    t->stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    t->stats.n_devices = 1;
    return SPE_OK;
}

int spe_table_profile_enable(spe_table* t, int32_t enable) {
    if (!t) return fail(SPE_EINVAL, "NULL table");
    if (t->multi) return spe::multi_profile_enable(t->multi, enable);
    t->prof = enable != 0;
    t->kp = spe_kernel_profile{};
    t->pending.clear();
    t->ev_next = 0;
    return SPE_OK;
}

int spe_table_profile_get(const spe_table* t, spe_kernel_profile* out) {
    if (!t || !out) return fail(SPE_EINVAL, "NULL argument");
    if (t->multi) return spe::multi_profile_get(t->multi, out);
    *out = t->kp;
    return SPE_OK;
}

int spe_table_build_stats(const spe_table* t, spe_build_stats* out) {
    if (!t || !out) return fail(SPE_EINVAL, "NULL argument");
    if (out->struct_size != sizeof(spe_build_stats)) return fail(SPE_EINVAL, ABI_MSG("spe_build_stats"));
    *out = t->stats;
    out->struct_size = sizeof(spe_build_stats);
    return SPE_OK;
}

int spe_table_layout_get(const spe_table* t, spe_table_layout* out) {
    if (!t || !out) return fail(SPE_EINVAL, "NULL argument");
    if (out->struct_size != sizeof(spe_table_layout)) return fail(SPE_EINVAL, ABI_MSG("spe_table_layout"));
    if (t->multi) return spe::multi_layout(t->multi, out);
    out->n_devices = 1;
    out->device = t->g->device;
    out->n_attached = t->A;
    out->block_begin = t->blk0;
    out->block_end = t->blk1;
    out->elems = (int64_t)(t->blk1 - t->blk0) * t->A * WAVE;
    out->latrel = t->tb.lr;
    out->next_hop = t->tb.next;
    out->hops = t->tb.hops;
    out->groups_per_launch = t->groups;
    out->engine = t->engine;
    out->lanes_per_group = t->lanes;
    out->relax_kernel = t->relax_kernel;
    out->contracted_vertices = t->cx ? t->bn : 0;
    out->shared_sources = t->share ? 1 : 0;
    return SPE_OK;
}

}  // extern "C"

// Staging of the host-side lookups (caller holds h->mu): a stream on `device` and
// room for `q` queries (0: only the single-entry buffer).
static int host_lookup_reserve(spe_table::HostLookup* h, int32_t device, int64_t q) {
    if (h->device < 0) {
        HIP_TRY(hipSetDevice(device));
        HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        HIP_TRY(hipHostMalloc((void**)&h->h_entry, 64, hipHostMallocDefault));
        h->device = device;
    }
    HIP_TRY(hipSetDevice(h->device));
    if (q <= h->cap) return SPE_OK;
    for (void* p : {(void*)h->d_pairs, (void*)h->d_lat, (void*)h->d_rel, (void*)h->d_ok})
        if (p) HIP_TRY(hipFree(p));
    for (void* p : {(void*)h->h_pairs, (void*)h->h_lat, (void*)h->h_rel, (void*)h->h_ok})
        if (p) HIP_TRY(hipHostFree(p));
    h->d_pairs = nullptr;
    h->d_lat = h->d_rel = nullptr;
    h->d_ok = nullptr;
    h->h_pairs = nullptr;
    h->h_lat = h->h_rel = nullptr;
    h->h_ok = nullptr;
    h->cap = 0;
    HIP_TRY(hipMalloc(&h->d_pairs, (size_t)q * sizeof(int2)));
    HIP_TRY(hipMalloc(&h->d_lat, (size_t)q * sizeof(double)));
    HIP_TRY(hipMalloc(&h->d_rel, (size_t)q * sizeof(double)));
    HIP_TRY(hipMalloc(&h->d_ok, (size_t)q));
    HIP_TRY(hipHostMalloc((void**)&h->h_pairs, (size_t)q * sizeof(int2), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&h->h_lat, (size_t)q * sizeof(double), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&h->h_rel, (size_t)q * sizeof(double), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&h->h_ok, (size_t)q, hipHostMallocDefault));
    h->cap = q;
    return SPE_OK;
}

extern "C" {

int spe_table_get(const spe_table* t, int32_t s_slot, int32_t t_slot, spe_entry* out) {
    if (!t || !out) return fail(SPE_EINVAL, "NULL argument");
    if (t->multi) {
        if (!t->built) return fail(SPE_ESTATE, "table not built");
        return spe::multi_get(t->multi, s_slot, t_slot, out);
    }
    if (s_slot < 0 || s_slot >= t->A || t_slot < 0 || t_slot >= t->A) return fail(SPE_EINVAL, "slot out of range");
    const int32_t sb = s_slot / WAVE;
    if (sb < t->blk0 || sb >= t->blk1) return fail(SPE_EINVAL, "source row not owned by this table");
    if (!t->blk_built[(size_t)(sb - t->blk0)]) return fail(SPE_ESTATE, "source row not built");
    HIP_TRY(hipSetDevice(t->g->device));
    const size_t o = ((size_t)(sb - t->blk0) * t->A + t_slot) * WAVE + (s_slot % WAVE);
    // the three fields read back into pinned memory on one stream, one synchronisation
    spe_table::HostLookup* hl = t->hlk;
    std::lock_guard<std::mutex> lock(hl->mu);
    if (int r = host_lookup_reserve(hl, t->g->device, 0)) return r;
    unsigned char* b = hl->h_entry;
    HIP_TRY(hipMemcpyAsync(b, t->tb.lr + o, sizeof(double2), hipMemcpyDeviceToHost, hl->stream));
    HIP_TRY(hipMemcpyAsync(b + 16, t->tb.next + o, sizeof(int32_t), hipMemcpyDeviceToHost, hl->stream));
    HIP_TRY(hipMemcpyAsync(b + 20, t->tb.hops + o, sizeof(uint16_t), hipMemcpyDeviceToHost, hl->stream));
    HIP_TRY(hipStreamSynchronize(hl->stream));
    double2 e;
    uint16_t h = 0;
    std::memcpy(&e, b, sizeof e);
    std::memcpy(&out->next_hop, b + 16, sizeof(int32_t));
    std::memcpy(&h, b + 20, sizeof h);
    out->latency = e.x;
    out->reliability = e.y;
    out->hops = h;
    return SPE_OK;
}

// SB64 block -> 64 row-major rows, on the device (a 64 x 64 LDS tile per
// workgroup: coalesced reads of the 64 interleaved sources, coalesced row writes).
__global__ __launch_bounds__(256) void k_sb64_rows(int32_t A, const double2* __restrict__ lr,
                                                   const int32_t* __restrict__ nx, const uint16_t* __restrict__ hp,
                                                   const double* __restrict__ ax, double* __restrict__ olat,
                                                   double* __restrict__ orel, int32_t* __restrict__ onext,
                                                   int32_t* __restrict__ ohops, double* __restrict__ oaux) {
    __shared__ double T0[64][65], T1[64][65];
    __shared__ int32_t I0[64][65], I1[64][65];
    const int32_t j0 = blockIdx.x * 64;
    for (int32_t e = threadIdx.x; e < 64 * 64; e += 256) {   // e = (target jj, lane l), lane fastest
        const int32_t jj = e / 64, l = e % 64, j = j0 + jj;
        if (j >= A) continue;
        const size_t o = (size_t)j * WAVE + l;
        if (olat || orel) {
            const double2 v = lr[o];
            T0[l][jj] = v.x;
            T1[l][jj] = v.y;
        }
        if (oaux) T0[l][jj] = ax[o];
        if (onext) I0[l][jj] = nx[o];
        if (ohops) I1[l][jj] = hp[o];
    }
    __syncthreads();
    for (int32_t e = threadIdx.x; e < 64 * 64; e += 256) {   // e = (lane l, target jj), target fastest
        const int32_t l = e / 64, jj = e % 64, j = j0 + jj;
        if (j >= A) continue;
        const size_t o = (size_t)l * A + j;
        if (olat) olat[o] = T0[l][jj];
        if (orel) orel[o] = T1[l][jj];
        if (oaux) oaux[o] = T0[l][jj];
        if (onext) onext[o] = I0[l][jj];
        if (ohops) ohops[o] = I1[l][jj];
    }
}

// Owned rows [row_begin, row_end) to host, row-major: each 64-source block is
// transposed on the device, then copied as one contiguous span per field.
// (aux is requested alone: it shares the first staging tile with latency.)
static int download_rows(const spe_table* t, int32_t row_begin, int32_t row_end, double* latency,
                         double* reliability, int32_t* next_hop, int32_t* hops, double* aux) {
    if (!t) return fail(SPE_EINVAL, "NULL table");
    if (row_begin < t->blk0 * WAVE || row_end > std::min(t->A, t->blk1 * WAVE) || row_begin > row_end)
        return fail(SPE_EINVAL, "row range not owned by this table");
    for (int32_t b = row_begin / WAVE; b < (row_end + WAVE - 1) / WAVE; ++b)
        if (!t->blk_built[(size_t)(b - t->blk0)]) return fail(SPE_ESTATE, "rows not built");
    if (row_begin == row_end) return SPE_OK;
    HIP_TRY(hipSetDevice(t->g->device));
    const int32_t A = t->A;
    const size_t blk_elems = (size_t)A * WAVE;
    std::vector<void*> tmp;
    double *dl = nullptr, *dr = nullptr, *da = nullptr;
    int32_t *dn = nullptr, *dh = nullptr;
    int r = SPE_OK;
    if (latency && !r) r = dev_alloc(tmp, &dl, blk_elems);
    if (reliability && !r) r = dev_alloc(tmp, &dr, blk_elems);
    if (aux && !r) r = dev_alloc(tmp, &da, blk_elems);
    if (next_hop && !r) r = dev_alloc(tmp, &dn, blk_elems);
    if (hops && !r) r = dev_alloc(tmp, &dh, blk_elems);
    hipStream_t s = t->stream;
    for (int32_t b = row_begin / WAVE; !r && b < (row_end + WAVE - 1) / WAVE; ++b) {
        const size_t off = (size_t)(b - t->blk0) * blk_elems;
        k_sb64_rows<<<(A + 63) / 64, 256, 0, s>>>(A, t->tb.lr + off, t->tb.next + off, t->tb.hops + off,
                                                  aux ? t->tb.aux + off : nullptr, dl, dr, dn, dh, da);
        if (hipGetLastError() != hipSuccess) {
            r = fail(SPE_EHIP, "k_sb64_rows launch");
            break;
        }
        // the rows of this block inside [row_begin, row_end)
        const int32_t r0 = std::max(row_begin, b * WAVE), r1 = std::min(row_end, (b + 1) * WAVE);
        const size_t src = (size_t)(r0 - b * WAVE) * A, dst = (size_t)(r0 - row_begin) * A;
        const size_t cnt = (size_t)(r1 - r0) * A;
        auto cp = [&](void* h, const void* d, size_t esz) -> int {
            if (!h) return SPE_OK;
            if (hipMemcpyAsync((char*)h + dst * esz, (const char*)d + src * esz, cnt * esz, hipMemcpyDeviceToHost,
                               s) != hipSuccess)
                return fail(SPE_EHIP, "hipMemcpyAsync (download)");
            return SPE_OK;
        };
        r = cp(latency, dl, 8);
        if (!r) r = cp(reliability, dr, 8);
        if (!r) r = cp(aux, da, 8);
        if (!r) r = cp(next_hop, dn, 4);
        if (!r) r = cp(hops, dh, 4);
        if (!r && hipStreamSynchronize(s) != hipSuccess) r = fail(SPE_EHIP, "download sync");
    }
    (void)hipStreamSynchronize(s);
    for (void* p : tmp) (void)hipFree(p);
    return r;
}

int spe_table_download(const spe_table* t, int32_t row_begin, int32_t row_end, double* latency,
                       double* reliability, int32_t* next_hop, int32_t* hops) {
    if (t && t->multi) {
        if (!t->built) return fail(SPE_ESTATE, "table not built");
        return spe::multi_download(t->multi, row_begin, row_end, latency, reliability, next_hop, hops);
    }
    return download_rows(t, row_begin, row_end, latency, reliability, next_hop, hops, nullptr);
}

int spe_table_download_aux(const spe_table* t, int32_t row_begin, int32_t row_end, double* aux) {
    if (!t || !aux) return fail(SPE_EINVAL, "NULL argument");
    if (t->multi) return fail(SPE_EUNSUPPORTED, "multi-device tables have no aux field");
    if (!t->tb.aux) return fail(SPE_ESTATE, "table was created without want_aux");
    return download_rows(t, row_begin, row_end, nullptr, nullptr, nullptr, nullptr, aux);
}

int spe_lookup_batch(const spe_table* t, const int32_t* d_pairs, int64_t q, double* d_latency,
                     double* d_reliability, uint8_t* d_ok, void* stream) {
    if (!t || (q > 0 && (!d_pairs || !d_latency || !d_reliability || !d_ok))) return fail(SPE_EINVAL, "bad arguments");
    if (!t->built) return fail(SPE_ESTATE, "table not built");
    if (q == 0) return SPE_OK;
    return spe_lookup_batch_replica(t, 0, d_pairs, q, d_latency, d_reliability, d_ok, stream);
}

int spe_lookup_batch_replica(const spe_table* t, int32_t replica, const int32_t* d_pairs, int64_t q,
                             double* d_latency, double* d_reliability, uint8_t* d_ok, void* stream) {
    if (!t || (q > 0 && (!d_pairs || !d_latency || !d_reliability || !d_ok))) return fail(SPE_EINVAL, "bad arguments");
    if (!t->built) return fail(SPE_ESTATE, "table not built");
    if (q == 0) return SPE_OK;
    if (t->multi) return spe::multi_lookup(t->multi, replica, d_pairs, q, d_latency, d_reliability, d_ok, stream);
    if (replica != 0) return fail(SPE_EINVAL, "a single-device table has one replica (0)");
    HIP_TRY(hipSetDevice(t->g->device));
    hipStream_t s = stream ? (hipStream_t)stream : t->stream;
    k_lookup<1><<<grid_for(q, BLOCK, 16384), BLOCK, 0, s>>>((const int2*)d_pairs, q, t->blk0, t->blk1, t->tb,
                                                           d_latency, d_reliability, d_ok);
    HIP_TRY(hipGetLastError());
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SPE_OK;
}

int spe_lookup_batch_host(const spe_table* t, const int32_t* pairs, int64_t q, double* latency, double* reliability,
                          uint8_t* ok) {
    if (!t || q < 0 || (q > 0 && (!pairs || !latency || !reliability || !ok))) return fail(SPE_EINVAL, "bad arguments");
    if (!t->built) return fail(SPE_ESTATE, "table not built");
    if (q == 0) return SPE_OK;
    int32_t dev = 0;
    if (int r = spe_table_replica_device(t, 0, &dev)) return r;
    spe_table::HostLookup* h = t->hlk;
    std::lock_guard<std::mutex> lock(h->mu);
    // chunks of up to 4M queries through pinned staging: H2D pairs, k_lookup on the
    // home replica, D2H answers, one synchronisation per chunk
    const int64_t chunk = std::min<int64_t>(q, (int64_t)1 << 22);
    if (int r = host_lookup_reserve(h, dev, chunk)) return r;
    for (int64_t i0 = 0; i0 < q; i0 += chunk) {
        const int64_t n = std::min(chunk, q - i0);
        std::memcpy(h->h_pairs, pairs + 2 * i0, (size_t)n * sizeof(int2));
        HIP_TRY(hipMemcpyAsync(h->d_pairs, h->h_pairs, (size_t)n * sizeof(int2), hipMemcpyHostToDevice, h->stream));
        if (int r = spe_lookup_batch_replica(t, 0, (const int32_t*)h->d_pairs, n, h->d_lat, h->d_rel, h->d_ok,
                                             h->stream))
            return r;
        HIP_TRY(hipMemcpyAsync(h->h_lat, h->d_lat, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(h->h_rel, h->d_rel, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(h->h_ok, h->d_ok, (size_t)n, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        std::memcpy(latency + i0, h->h_lat, (size_t)n * sizeof(double));
        std::memcpy(reliability + i0, h->h_rel, (size_t)n * sizeof(double));
        std::memcpy(ok + i0, h->h_ok, (size_t)n);
    }
    return SPE_OK;
}

int spe_table_check(const spe_table* t, spe_check_report* out) {
    if (!t || !out) return fail(SPE_EINVAL, "NULL argument");
    if (t->multi) return fail(SPE_EUNSUPPORTED, "spe_table_check runs on single-device tables");
    if (t->blk0 != 0 || t->blk1 != (t->A + WAVE - 1) / WAVE) return fail(SPE_EUNSUPPORTED, "spe_table_check needs every source row");
    if (!t->built) return fail(SPE_ESTATE, "table not built");
    HIP_TRY(hipSetDevice(t->g->device));
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc(&d, 10 * sizeof(unsigned long long)));
    unsigned long long h[10];
    std::memset(h, 0, sizeof(h));
    h[9] = ~0ull;
    hipError_t e = hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    // hop rule: per-source rows (no owner replay) of an undirected graph or a directed one alike
    const int32_t hop_rule = t->d_rank == nullptr;
    const int32_t undirected = !t->g->hg.directed && t->d_rank == nullptr;
    if (e == hipSuccess) {
        const int64_t total = (int64_t)((t->A + WAVE - 1) / WAVE) * t->A * WAVE;
        k_table_check<<<grid_for(total, BLOCK, 16384), BLOCK, 0, t->stream>>>(
            t->A, t->d_slot_vertex, t->d_vertex_slot, t->g->dev, undirected, hop_rule, t->tb, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(SPE_EHIP, std::string("spe_table_check: ") + hipGetErrorString(e));
    out->pairs = (int64_t)h[0];
    out->unroutable = (int64_t)h[1];
    out->bad_values = (int64_t)h[2];
    out->next_not_adjacent = (int64_t)h[3];
    out->hop_checked = (int64_t)h[4];
    out->hop_mismatch = (int64_t)h[5];
    out->sym_checked = (int64_t)h[6];
    out->sym_mismatch = (int64_t)h[7];
    double w;
    std::memcpy(&w, &h[8], sizeof(w));
    out->max_sym_rel_err = w;
    out->first_bad_s = h[9] == ~0ull ? -1 : (int32_t)(h[9] >> 32);
    out->first_bad_t = h[9] == ~0ull ? -1 : (int32_t)(h[9] & 0xFFFFFFFFu);
    return SPE_OK;
}

int spe_table_replica_device(const spe_table* t, int32_t replica, int32_t* device) {
    if (!t || !device) return fail(SPE_EINVAL, "NULL argument");
    if (t->multi) return spe::multi_replica_device(t->multi, replica, device);
    if (replica != 0) return fail(SPE_EINVAL, "a single-device table has one replica (0)");
    *device = t->g->device;
    return SPE_OK;
}

}  // extern "C"

int spe::lookup_on_replica(int32_t device, const void* latrel, int32_t A, int32_t nblk, const int32_t* d_pairs,
                           int64_t q, double* d_latency, double* d_reliability, uint8_t* d_ok, void* stream) {
    HIP_TRY(hipSetDevice(device));
    Table tb{};
    tb.lr = (double2*)latrel;
    tb.A = A;
    hipStream_t s = (hipStream_t)stream;
    k_lookup<1><<<grid_for(q, BLOCK, 16384), BLOCK, 0, s>>>((const int2*)d_pairs, q, 0, nblk, tb, d_latency,
                                                           d_reliability, d_ok);
    HIP_TRY(hipGetLastError());
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return SPE_OK;
}

extern "C" {

int spe_fw_apsp(spe_graph* g, double* d_dist, int64_t ld, int32_t* d_next, void* stream, double* seconds) {
    if (!g || !d_dist) return fail(SPE_EINVAL, "NULL argument");
    const int32_t n = g->hg.nc;
    const int32_t nb = (n + FWB - 1) / FWB;
    if (ld < (int64_t)nb * FWB) return fail(SPE_EINVAL, "ld must be >= the relaxation vertex count rounded up to 64");
    if (ld % FWB) return fail(SPE_EINVAL, "ld must be a multiple of 64");
    HIP_TRY(hipSetDevice(g->device));
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(hipEventRecord(a, s));
    k_fw_init<<<grid_for(ld * ld, 256, 16384), 256, 0, s>>>(n, ld, g->dev, d_dist);
    const int32_t nrel = (int32_t)g->hg.icol.size();
    if (nrel > 0) k_fw_edges<<<(nrel + 255) / 256, 256, 0, s>>>(nrel, ld, g->dev, d_dist);
    // padding rows / columns stay +inf off the diagonal: they never shorten a path
    for (int32_t kb = 0; kb < nb; ++kb) {
        k_fw_panel<<<1, 256, 0, s>>>(kb, nb, ld, d_dist, 0);
        if (nb > 1) k_fw_panel<<<2 * nb - 2, 256, 0, s>>>(kb, nb, ld, d_dist, 1);
        if (nb > 1) k_fw_rest<<<(nb - 1) * (nb - 1), 256, 0, s>>>(kb, nb, ld, d_dist);
    }
    HIP_TRY(hipEventRecord(b, s));
    if (d_next) k_fw_next<<<grid_for((int64_t)n * n, 256, 16384), 256, 0, s>>>(n, ld, g->dev, d_dist, d_next);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    if (seconds) *seconds = ms / 1e3;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return SPE_OK;
}

namespace {
__global__ __launch_bounds__(256) void k_fw3_first_hop(int64_t total, const int32_t* __restrict__ irow,
                                                       int32_t* __restrict__ nxt) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        const int32_t k = nxt[e];
        nxt[e] = k < 0 ? -1 : irow[k];
    }
}
}  // namespace

int spe_fw_closure(spe_graph* g, double* d_dist, double* d_rel, int32_t* d_next, int64_t ld, void* stream,
                   double* seconds) {
    if (!g || !d_dist || !d_rel || !d_next) return fail(SPE_EINVAL, "NULL argument");
    const int32_t n = g->hg.nc;
    if (ld < ((int64_t)n + FWB - 1) / FWB * FWB || ld % FWB) return fail(SPE_EINVAL, "ld must be a multiple of 64 >= n");
    HIP_TRY(hipSetDevice(g->device));
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    HIP_TRY(hipEventRecord(a, s));
    if (int r = fw3_closure(g, Fw3{d_dist, d_rel, d_next}, ld, s)) return r;
    HIP_TRY(hipEventRecord(b, s));
    k_fw3_first_hop<<<grid_for(ld * ld, 256, 16384), 256, 0, s>>>(ld * ld, g->dev.irow, d_next);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    if (seconds) *seconds = ms / 1e3;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return SPE_OK;
}

int spe_table_source_tree(spe_table* t, int32_t s_slot, int32_t* parent) {
    if (!t || !parent) return fail(SPE_EINVAL, "NULL argument");
    if (t->multi) return spe::multi_source_tree(t->multi, s_slot, parent);
    if (s_slot < 0 || s_slot >= t->A) return fail(SPE_EINVAL, "slot out of range");
    const int32_t b = s_slot / WAVE;
    if (b < t->blk0 || b >= t->blk1) return fail(SPE_EINVAL, "source block not owned by this table");
    if (t->md.complete) return fail(SPE_EUNSUPPORTED, "DIRECT table: every path is its one edge");
    // owner replay rewrites pairs across blocks (k_owner_replay): rebuilding one block would undo it
    if (t->d_rank) return fail(SPE_EUNSUPPORTED, "owner-replay table: its entries are not one source's tree");
    const spe::HostGraph& h = t->g->hg;
    const int32_t nc = h.nc, s = t->attached[(size_t)s_slot];
    // pk[v]: in-CSR entry of the relaxation vertex v's parent edge; -1 none (root or
    // unreached); -2 (batch / FW state) the pruned pendant source itself
    std::vector<int32_t> pk((size_t)std::max(1, nc), -1);
    HIP_TRY(hipSetDevice(t->g->device));
    // The source is re-run into scratch rows of one block, never into the table itself:
    // concurrent readers of a live table (the topology shim's queries) keep seeing its
    // finished rows (a prefer-direct row would otherwise lack the DIRECT overlay for a while).
    const size_t be = (size_t)t->A * WAVE;
    const bool scratch = !t->tb.prev && !t->tb.aux;   // aux tables (offline tool only) rebuild in place
    void* sbuf = nullptr;
    if (scratch) HIP_TRY(hipMalloc(&sbuf, be * (sizeof(double2) + sizeof(int32_t) + sizeof(uint16_t))));
    double2* s_lr = (double2*)sbuf;
    int32_t* s_next = (int32_t*)(s_lr + (scratch ? be : 0));
    uint16_t* s_hops = (uint16_t*)(s_next + (scratch ? be : 0));
    int rc = SPE_OK;
    if (t->engine == SPE_ENGINE_LDS) {
        // one workgroup re-runs this source; the parent entries stay in that workgroup's scratch
        Table tb = t->tb;
        int32_t blk0 = t->blk0;
        if (scratch) {
            tb.lr = s_lr;
            tb.next = s_next;
            tb.hops = s_hops;
            blk0 = b;   // the scratch holds block b only
        }
        k_sssp_lds<<<1, LDS_T, lds_bytes(nc), t->stream>>>(s_slot, s_slot + 1, t->d_slots, blk0, t->g->dev, t->md, tb,
                                                         t->lsc, nullptr);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(pk.data(), t->lsc.par, sizeof(int32_t) * (size_t)nc,
                                                hipMemcpyDeviceToHost, t->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
        if (e != hipSuccess) rc = fail(SPE_EHIP, hipGetErrorString(e));
        // in place (aux tables): the row just rewritten lacks the DIRECT overlay; rebuild the block
        if (!rc && !scratch && t->md.prefer) rc = spe_table_build_blocks(t, b, b + 1, nullptr);
    } else {
        // re-run the source's block, one lane per source (no shared anchor trees); its
        // state is left in the first buffer
        t->share_off = true;
        rc = scratch ? spe_table_build_blocks_into(t, b, b + 1, s_lr, s_next, s_hops, nullptr)
                     : spe_table_build_blocks(t, b, b + 1, nullptr);
        t->share_off = false;
        if (!rc) {
            const hipError_t e = hipStreamSynchronize(t->stream);
            if (e != hipSuccess) rc = fail(SPE_EHIP, hipGetErrorString(e));
        }
    }
    if (sbuf) (void)hipFree(sbuf);
    if (rc) return rc;
    if (t->engine != SPE_ENGINE_LDS && t->cx) {
        // the contracted graph: kept rows carry entries of the contracted CSR (a shortcut
        // entry's parent is its x); a removed vertex's parent is the best of its three
        // neighbours, the rows kernel's rule
        const spe::HostGraph::Contracted& cx = h.cx;
        const int32_t nk = cx.nk, L = t->lanes, j = s_slot % WAVE;
        const int32_t g = L <= WAVE ? j / L : 0, lane = L <= WAVE ? j % L : j;
        std::vector<int32_t> kp((size_t)std::max(1, nk));
        std::vector<double> kd((size_t)std::max(1, nk));
        const size_t off = ((size_t)g * nk) * (size_t)L + (size_t)lane;
        HIP_TRY(hipMemcpy2D(kp.data(), sizeof(int32_t), t->st_buf[0].P + off, sizeof(int32_t) * (size_t)L,
                            sizeof(int32_t), (size_t)nk, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy2D(kd.data(), sizeof(double), t->st_buf[0].D + off, sizeof(double) * (size_t)L,
                            sizeof(double), (size_t)nk, hipMemcpyDeviceToHost));
        std::fill(parent, parent + h.n, -1);
        auto orig = [&](int32_t kv) { return h.corev[(size_t)cx.kcore[(size_t)kv]]; };
        for (int32_t v = 0; v < nk; ++v) {
            const int32_t k = kp[(size_t)v];
            if (k >= 0) parent[orig(v)] = cx.via[(size_t)k] >= 0 ? cx.via[(size_t)k] : orig(cx.col[(size_t)k]);
            else if (k == -2) parent[orig(v)] = s;   // the source's first edge (pendant or contracted source)
        }
        for (size_t r = 0; r < cx.rcore.size(); ++r) {
            const int32_t x = h.corev[(size_t)cx.rcore[r]];
            if (x == s) continue;
            int32_t bq = -1;
            double bd = INF, bdu = INF;
            for (int q = 0; q < 3; ++q) {
                const double du = kd[(size_t)cx.rnb[3 * r + q]];
                if (!(du < INF)) continue;
                const double alt = du + cx.rw[3 * r + q];
                if (bq < 0 || alt < bd || (alt == bd && du < bdu)) {
                    bq = q;
                    bd = alt;
                    bdu = du;
                }
            }
            if (bq >= 0) parent[x] = orig(cx.rnb[3 * r + bq]);
        }
        if (h.pruned)
            for (int32_t v = 0; v < h.n; ++v) {
                if (h.core_id[(size_t)v] >= 0 || v == s) continue;
                const int32_t a = h.anchor_core[(size_t)v];   // (never a removed vertex)
                if (a >= 0 && kd[(size_t)cx.kid[(size_t)a]] < INF) parent[v] = h.corev[(size_t)a];
            }
        parent[s] = -1;
        return SPE_OK;
    }
    if (t->engine != SPE_ENGINE_LDS) {
        const int32_t L = t->lanes, j = s_slot % WAVE;
        const int32_t g = L <= WAVE ? j / L : 0, lane = L <= WAVE ? j % L : j;
        const int32_t* P = t->st_buf[0].P + ((size_t)g * nc) * (size_t)L + (size_t)lane;
        HIP_TRY(hipMemcpy2D(pk.data(), sizeof(int32_t), P, sizeof(int32_t) * (size_t)L, sizeof(int32_t), (size_t)nc,
                            hipMemcpyDeviceToHost));
    }
    std::fill(parent, parent + h.n, -1);
    const int32_t sc = h.core_id[(size_t)s];
    const int32_t root = sc >= 0 ? sc : h.anchor_core[(size_t)s];   // relaxation vertex the tree grows from
    std::vector<uint8_t> reach((size_t)std::max(1, nc), 0);
    for (int32_t v = 0; v < nc; ++v) {
        const int32_t k = pk[(size_t)v];
        if (k >= 0) {
            parent[h.corev[(size_t)v]] = h.corev[(size_t)h.icol[(size_t)k]];
            reach[(size_t)v] = 1;
        } else if (v == root) {
            if (sc < 0) parent[h.corev[(size_t)v]] = s;   // s -> anchor: the pendant source's edge
            reach[(size_t)v] = 1;
        }
    }
    if (h.pruned)
        for (int32_t v = 0; v < h.n; ++v) {
            if (h.core_id[(size_t)v] >= 0 || v == s) continue;
            const int32_t a = h.anchor_core[(size_t)v];
            if (a >= 0 && reach[(size_t)a]) parent[v] = h.corev[(size_t)a];
        }
    parent[s] = -1;
    return SPE_OK;
}

int spe_table_min_latency(const spe_table* t, double* out) {
    if (!t || !out) return fail(SPE_EINVAL, "NULL argument");
    if (!t->built) return fail(SPE_ESTATE, "table not built (every owned block)");
    if (t->multi) return spe::multi_min_latency(t->multi, out);
    HIP_TRY(hipSetDevice(t->g->device));
    const unsigned long long init = 0x7FF0000000000000ull;  // +inf
    HIP_TRY(hipMemcpyAsync(t->d_min, &init, sizeof(init), hipMemcpyHostToDevice, t->stream));
    const int64_t elems = (int64_t)(t->blk1 - t->blk0) * t->A * WAVE;
    k_min_latency<<<grid_for(elems, BLOCK, 4096), BLOCK, 0, t->stream>>>(t->tb.lr, elems, t->A, t->blk0,
                                                                        t->d_min);
    HIP_TRY(hipGetLastError());
    unsigned long long bits = 0;
    HIP_TRY(hipMemcpyAsync(&bits, t->d_min, sizeof(bits), hipMemcpyDeviceToHost, t->stream));
    HIP_TRY(hipStreamSynchronize(t->stream));
    double v;
    std::memcpy(&v, &bits, sizeof(v));
    *out = (v == INF) ? 0.0 : v;   // reference's "0 = unset" sentinel, shd-topology.c:1360
    return SPE_OK;
}

// ---------------------------------------------------------------- table cache
// File: 64-byte header, then the owned SB64 span of each field (latrel, next,
// hops), raw.  Written to "<path>.tmp" and renamed, so a reader never sees a
// partial file under the final name.
namespace {
struct CacheHeader {
    char magic[8];        // "SPETAB01"
    uint64_t key;
    int32_t A, blk0, blk1, pad;
    int64_t elems;
    int64_t bytes;        // payload bytes after the header
    char reserved[16];
};
static_assert(sizeof(CacheHeader) == 64, "cache header is 64 bytes");
const char kMagic[8] = {'S', 'P', 'E', 'T', 'A', 'B', '0', '1'};
constexpr size_t kChunk = 64u << 20;   // staging chunk

struct Field {
    void* dev;
    size_t bytes;
};

void fields_of(const spe_table* t, Field f[3], int64_t* elems) {
    const int64_t e = (int64_t)(t->blk1 - t->blk0) * t->A * WAVE;
    *elems = e;
    f[0] = {t->tb.lr, (size_t)e * sizeof(double2)};
    f[1] = {t->tb.next, (size_t)e * sizeof(int32_t)};
    f[2] = {t->tb.hops, (size_t)e * sizeof(uint16_t)};
}
}  // namespace

int spe_table_key(const spe_table* t, uint64_t* key) {
    if (!t || !key) return fail(SPE_EINVAL, "NULL argument");
    *key = t->key;
    return SPE_OK;
}

int spe_table_save(const spe_table* t, const char* path) {
    if (t && t->tb.aux) return fail(SPE_EUNSUPPORTED, "the table cache does not hold want_aux rows");
    if (t && t->multi) return fail(SPE_EUNSUPPORTED, "the table cache holds single-device tables");
    if (!t || !path) return fail(SPE_EINVAL, "NULL argument");
    if (!t->built) return fail(SPE_ESTATE, "table not built (every owned block)");
    HIP_TRY(hipSetDevice(t->g->device));
    HIP_TRY(hipStreamSynchronize(t->stream));
    Field f[3];
    int64_t elems = 0;
    fields_of(t, f, &elems);
    CacheHeader h{};
    std::memcpy(h.magic, kMagic, 8);
    h.key = t->key;
    h.A = t->A;
    h.blk0 = t->blk0;
    h.blk1 = t->blk1;
    h.elems = elems;
    h.bytes = (int64_t)(f[0].bytes + f[1].bytes + f[2].bytes);
    const std::string tmp = std::string(path) + ".tmp";
    FILE* fp = fopen(tmp.c_str(), "wb");
    if (!fp) return fail(SPE_EINVAL, "cannot create " + tmp);
    void* stage = nullptr;
    if (hipHostMalloc(&stage, kChunk) != hipSuccess) {
        fclose(fp);
        remove(tmp.c_str());
        return fail(SPE_ENOMEM, "cache staging buffer");
    }
    int rc = SPE_OK;
    if (fwrite(&h, sizeof(h), 1, fp) != 1) rc = fail(SPE_EINVAL, "short write " + tmp);
    for (int i = 0; i < 3 && rc == SPE_OK; ++i) {
        for (size_t off = 0; off < f[i].bytes && rc == SPE_OK; off += kChunk) {
            const size_t n = std::min(kChunk, f[i].bytes - off);
            const hipError_t e = hipMemcpy(stage, (const char*)f[i].dev + off, n, hipMemcpyDeviceToHost);
            if (e != hipSuccess) rc = fail(SPE_EHIP, std::string("hipMemcpy D2H: ") + hipGetErrorString(e));
            else if (fwrite(stage, 1, n, fp) != n) rc = fail(SPE_EINVAL, "short write " + tmp);
        }
    }
    (void)hipHostFree(stage);
    if (fclose(fp) != 0 && rc == SPE_OK) rc = fail(SPE_EINVAL, "close " + tmp);
    if (rc == SPE_OK && rename(tmp.c_str(), path) != 0) rc = fail(SPE_EINVAL, std::string("rename to ") + path);
    if (rc != SPE_OK) remove(tmp.c_str());
    return rc;
}

int spe_table_load(spe_table* t, const char* path) {
    if (t && t->tb.aux) return fail(SPE_EUNSUPPORTED, "the table cache does not hold want_aux rows");
    if (t && t->multi) return fail(SPE_EUNSUPPORTED, "the table cache holds single-device tables");
    if (!t || !path) return fail(SPE_EINVAL, "NULL argument");
    HIP_TRY(hipSetDevice(t->g->device));
    FILE* fp = fopen(path, "rb");
    if (!fp) return fail(SPE_EINVAL, std::string("no cache file ") + path);
    Field f[3];
    int64_t elems = 0;
    fields_of(t, f, &elems);
    CacheHeader h{};
    int rc = SPE_OK;
    if (fread(&h, sizeof(h), 1, fp) != 1 || std::memcmp(h.magic, kMagic, 8) != 0)
        rc = fail(SPE_EINVAL, std::string("not a path-table cache: ") + path);
    else if (h.key != t->key || h.A != t->A || h.blk0 != t->blk0 || h.blk1 != t->blk1 || h.elems != elems ||
             h.bytes != (int64_t)(f[0].bytes + f[1].bytes + f[2].bytes))
        rc = fail(SPE_EINVAL, std::string("cache file is for another graph / attached set / options: ") + path);
    void* stage = nullptr;
    if (rc == SPE_OK && hipHostMalloc(&stage, kChunk) != hipSuccess) rc = fail(SPE_ENOMEM, "cache staging buffer");
    for (int i = 0; i < 3 && rc == SPE_OK; ++i) {
        for (size_t off = 0; off < f[i].bytes && rc == SPE_OK; off += kChunk) {
            const size_t n = std::min(kChunk, f[i].bytes - off);
            if (fread(stage, 1, n, fp) != n) {
                rc = fail(SPE_EINVAL, std::string("truncated cache file ") + path);
                break;
            }
            const hipError_t e = hipMemcpy((char*)f[i].dev + off, stage, n, hipMemcpyHostToDevice);
            if (e != hipSuccess) rc = fail(SPE_EHIP, std::string("hipMemcpy H2D: ") + hipGetErrorString(e));
        }
    }
    if (stage) (void)hipHostFree(stage);
    fclose(fp);
    if (rc == SPE_OK) {
        t->built = true;
        std::fill(t->blk_built.begin(), t->blk_built.end(), (uint8_t)1);
    }
    return rc;
}

static void host_lookup_free(spe_table::HostLookup* h) {
    if (!h) return;
    if (h->device >= 0) {
        (void)hipSetDevice(h->device);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        for (void* p : {(void*)h->d_pairs, (void*)h->d_lat, (void*)h->d_rel, (void*)h->d_ok})
            if (p) (void)hipFree(p);
        for (void* p : {(void*)h->h_pairs, (void*)h->h_lat, (void*)h->h_rel, (void*)h->h_ok, (void*)h->h_entry})
            if (p) (void)hipHostFree(p);
        if (h->stream) (void)hipStreamDestroy(h->stream);
    }
    delete h;
}

void spe_table_free(spe_table* t) {
    if (!t) return;
    host_lookup_free(t->hlk);
    t->hlk = nullptr;
    if (t->multi) {
        spe::multi_free(t->multi);
        delete t;
        return;
    }
    (void)hipSetDevice(t->g->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    for (void* p : t->allocs) (void)hipFree(p);
    if (t->h_srcv) (void)hipHostFree(t->h_srcv);
    if (t->h_rows) (void)hipHostFree(t->h_rows);
    if (t->h_unsafe) (void)hipHostFree(t->h_unsafe);
    if (t->h_der) (void)hipHostFree(t->h_der);
    if (t->h_sunsafe) (void)hipHostFree(t->h_sunsafe);
    if (t->h_counts) (void)hipHostFree(t->h_counts);
    for (hipEvent_t e : t->ev_pool) (void)hipEventDestroy(e);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    if (t->rows_stream) (void)hipStreamDestroy(t->rows_stream);
    if (t->ev_relaxed) (void)hipEventDestroy(t->ev_relaxed);
    for (hipEvent_t e : t->ev_rows)
        if (e) (void)hipEventDestroy(e);
    delete t;
}

}  // extern "C"

