// spe_internal.h -- shared declarations of libspe (not part of the public ABI).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/spe.h"

namespace spe {

// Host copy of the device graph layout.
struct HostGraph {
    int32_t n = 0;
    int64_t m = 0;
    bool directed = false;
    bool prefer_direct = false;
    bool complete = false;
    bool multi_rep = false;        // some merged pair's get_eid latency != relaxation latency
    bool weight_floor_ok = true;

    // Pendant pruning (undirected graphs): a vertex whose only non-loop neighbour
    // is its anchor c (itself not pendant) never lies inside a shortest path, so
    // the relaxation runs on the remaining "core" and pendant rows/targets are
    // one edge away from their anchor.  nc = relaxation vertex count.
    bool pruned = false;
    int32_t nc = 0;
    std::vector<int32_t> core_id;      // [n] relaxation id, -1 for a pruned pendant
    std::vector<int32_t> corev;        // [nc] original id
    std::vector<int32_t> anchor_core;  // [n] relaxation id of a pendant's anchor, -1 otherwise
    // full in-CSR (original ids): DIRECT lookups and the pendant edges
    std::vector<int32_t> fiptr, ficol;
    std::vector<double> fiw, fia, fiwrep;
    std::vector<int64_t> fieid;        // get_eid edge id of each full in-CSR entry

    // relaxation in-CSR (relaxation ids): entries u -> v grouped by v, sorted by u
    std::vector<int32_t> iptr, icol;
    std::vector<double> iw;        // min latency over parallel u->v edges (what Dijkstra relaxes)
    std::vector<double> ia;        // 1 - loss of the get_eid edge
    std::vector<double> iwrep;     // latency of the get_eid edge
    std::vector<int64_t> ieid;     // id of the get_eid edge (per-edge auxiliary attributes)
    // out-CSR (directed only; undirected graphs reuse the in-CSR)
    std::vector<int32_t> optr, ocol;
    std::vector<int32_t> orev;     // out entry -> in-CSR index of the same (merged) edge
    std::vector<double> owrep, oarep, ow;
    // per vertex
    std::vector<double> vfac;      // 1 - vertex loss, NaN when absent
    std::vector<int64_t> loop_eid;
    std::vector<double> loop_w, loop_a;       // get_eid(v,v) self-loop, NaN when none
    std::vector<double> self_w2, self_a2;     // SELF rule: 2*min latency, r*r
    std::vector<int32_t> self_other;          // other endpoint of the SELF edge, -1 none
};

int prepare_graph(const spe_graph_desc* d, HostGraph* hg, std::string* err);
// Restrict the relaxation CSR to the core (no-op for directed graphs or when
// `enable` is false); keeps the full CSR in hg->f*.
void prune_pendants(HostGraph* hg, bool enable);

}  // namespace spe
