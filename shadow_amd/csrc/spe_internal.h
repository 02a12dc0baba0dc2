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

    // Degree-3 contraction for the batch engine (contract_degree3): an independent
    // set of relaxation vertices x with exactly three neighbours (no pendant anchored
    // at x) is taken out of the batch engine's relaxation graph; each x is replaced by
    // "shortcut" entries a -> b via x between its neighbours, offering the two-add
    // path fold fl(fl(d[a] + w(a,x)) + w(x,b)), and x's rows are derived from its
    // three neighbours' rows.  The kept vertices keep their relative (core) order.
    struct Contracted {
        bool active = false;
        int32_t nk = 0;                    // kept relaxation vertices
        std::vector<int32_t> kid;          // [nc] kept id of a core vertex, -1 = removed
        std::vector<int32_t> kcore;        // [nk] core id of a kept vertex
        std::vector<int32_t> rid;          // [nc] removed index of a core vertex, -1 = kept
        std::vector<int32_t> rcore;        // [nr] core id of a removed vertex
        std::vector<int32_t> rnb;          // [3 nr] kept ids of its neighbours (increasing)
        std::vector<double> rw, ra;        // [3 nr] relaxation latency / 1 - p of the edge (nb, x)
        // in-CSR over kept ids: entry k of v = a -> v, plain or via a removed x
        std::vector<int32_t> ptr, col, rev;
        std::vector<double> w1, w2, a1, a2;   // plain: (w, 0, a, 1); shortcut: (w(a,x), w(x,v), a(a,x), a(x,v))
        std::vector<int32_t> key;          // core id of the entry's parent (x for a shortcut, a for a plain edge)
        std::vector<int32_t> via;          // original id of x, -1 for a plain edge
        // Sources whose rows a shared table may derive from their neighbours' lanes
        // (k_rows_derived): every removed vertex, and an independent set
        // (in the contracted graph) of kept vertices with at most DER_LEGS_KEPT
        // contracted entries, at most one removed neighbour and no pendant anchored
        // (they stay relaxation vertices; only their own lane goes).  Each derived
        // source's row is the best of its LEGS: a first path prefix (one or two edges)
        // to a kept vertex whose lane is read, or a direct edge to one target.
        struct Leg {
            int32_t ref;                   // core id of the kept vertex whose lane the leg reads, -1: direct
            int32_t tc;                    // direct: the one target's relaxation code (kept id, or -2 - removed index)
            int32_t hop;                   // first hop (original id)
            int32_t inc;                   // edges of the prefix (1 or 2)
            double w;                      // prefix latency, summed in path order from the source
            double a;                      // prefix reliability factors, multiplied in path order
        };
        std::vector<uint8_t> der;          // [nc]
        std::vector<int32_t> dptr;         // [nc + 1] legs of core vertex c: dlegs[dptr[c] .. dptr[c + 1])
        std::vector<Leg> dlegs;
        int32_t nd4 = 0;                   // derived kept vertices
    } cx;

    // Shared anchor trees for the batch engine (share_prep): a pruned
    // pendant source s reaches every vertex through its anchor c, so its row is c's
    // row with the prefix s -> c folded in front -- exactly when c's parent decisions
    // hold for the offset o = w(s, c) too (integer-valued sums, or a margin check).
    struct Share {
        bool eligible = false;     // undirected, pruned, no vertex factor other than 1 / absent
        bool exact = false;        // every weight k / 2^q and every path sum below 2^53: fl sums exact
        bool prod_exact = false;   // every edge factor 1 - p is 1.0: every reliability product exact
        double wmin = 0.0;         // smallest relaxation weight (bounds a path's edge count)
        double omax = 0.0;         // largest pendant-edge weight (a source's offset)
    } share;
};

int prepare_graph(const spe_graph_desc* d, HostGraph* hg, std::string* err);
// spe_last_error's message for the calling thread; returns code
int set_error(int code, const std::string& msg);
// the prepared graph uploaded to another device (multi-device tables)
int graph_clone(const spe_graph* g, int32_t device, spe_graph** out);
// k_lookup over a caller-described SB64 {latency, reliability} span holding
// blocks [0, nblk) of an A-target table on `device`
int lookup_on_replica(int32_t device, const void* latrel, int32_t A, int32_t nblk, const int32_t* d_pairs,
                      int64_t q, double* d_latency, double* d_reliability, uint8_t* d_ok, void* stream);

// Multi-device tables (spe_multi.cpp): one part table per device over a
// contiguous share of the 64-source blocks; the {latency, reliability}
// records are then all-gathered so every device holds the whole table.
struct MultiDev;
int multi_create(spe_graph* g, const int32_t* attached, int32_t A, const spe_table_opts& o, MultiDev** out);
void multi_free(MultiDev* m);
int multi_build(MultiDev* m, spe_build_stats* stats);
bool multi_built(const MultiDev* m);
int multi_get(const MultiDev* m, int32_t s_slot, int32_t t_slot, spe_entry* out);
int multi_download(const MultiDev* m, int32_t row_begin, int32_t row_end, double* latency, double* reliability,
                   int32_t* next_hop, int32_t* hops);
int multi_lookup(const MultiDev* m, int32_t replica, const int32_t* d_pairs, int64_t q, double* d_latency,
                 double* d_reliability, uint8_t* d_ok, void* stream);
int multi_replica_device(const MultiDev* m, int32_t replica, int32_t* device);
// x* of the compute-versus-gather split
double multi_shared_fraction(int32_t n_dev, double t1_s, double span_bytes, double gather_bps);
int multi_min_latency(const MultiDev* m, double* out);
int multi_layout(const MultiDev* m, spe_table_layout* out);
int multi_profile_enable(MultiDev* m, int32_t enable);
int multi_profile_get(const MultiDev* m, spe_kernel_profile* out);
int multi_source_tree(MultiDev* m, int32_t s_slot, int32_t* parent);
// The FW engine's closure buffers of one (part) table, for the multi-device
// closure: pivot-row broadcast between devices, each device relaxing its own
// row blocks (spe.hip fw_*; driven by spe_multi.cpp).
struct FwPart {
    double* D = nullptr;
    double* R = nullptr;
    int32_t* N = nullptr;
    int64_t ld = 0;        // row stride; ld / 64 row blocks
    int32_t device = 0;
    void* stream = nullptr;
    bool* done = nullptr;  // set once the closure is complete on this device
};
int fw_part(spe_table* t, FwPart* out);
int fw_init(const spe_graph* g, const FwPart& p);
int fw_pivot_owner(const FwPart& p, int32_t kb);                         // diagonal tile + pivot row panel
int fw_pivot_rows(const FwPart& p, int32_t kb, int32_t rb0, int32_t rb1);  // column panel + rest, own rows

// Restrict the relaxation CSR to the core (no-op for directed graphs or when
// `enable` is false); keeps the full CSR in hg->f*.
void prune_pendants(HostGraph* hg, bool enable);
// Build hg->cx when the graph qualifies (undirected, no multigraph latency
// representatives, no vertex factor other than 1 / absent, some eligible vertex).
void contract_degree3(HostGraph* hg);
// Fill hg->share (after prune_pendants / contract_degree3).
void share_prep(HostGraph* hg);

}  // namespace spe
