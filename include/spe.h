/*
 * spe.h -- C ABI of the MI355X shortest-path engine (libspe.so).
 *
 * This is the library the C topology host code (include/shd_topology_spe.h)
 * calls in place of igraph + the per-pair path cache of the reference
 * (src/main/routing/shd-topology.c).  Plain C types only: no glib, no igraph,
 * no torch.  Device pointers appear only where the caller hands over its own
 * HBM buffers (external table storage, batched lookups); streams are passed as
 * `void*` holding a hipStream_t (NULL = the library's own stream).
 *
 * Which reference interface each entry point replaces:
 *   spe_graph_create     igraph_read_graph_graphml result + _topology_checkGraphProperties
 *                        + _topology_extractEdgeWeights   shd-topology.c:356-384, 709-794, 1197-1231
 *   spe_graph_info       top->isComplete / isDirected / prefersDirectPaths  shd-topology.c:39-52, 736-775
 *   spe_table_create     verticesWithAttachedHosts (the target set A)     shd-topology.c:1510-1528, 2366-2367
 *   spe_table_build      _topology_computeSourcePaths / _lookupDirectPath / _computeShortestPathToSelf
 *                        for every source row                              shd-topology.c:1530-1912
 *   spe_table_get        _topology_getPathEntry + path_getLatency/Reliability shd-topology.c:1952-2070
 *   spe_lookup_batch     3 x _topology_getPathEntry per packet (shd-worker.c:235,243,247), batched
 *   spe_lookup_batch_host  the same from host arrays (the shim's topology_getPathInfoBatch)
 *   spe_table_min_latency top->minimumPathLatency -> worker_updateMinTimeJump shd-topology.c:1359-1370
 *   spe_last_error       the critical()/warning() log lines of the reference
 *
 * Semantics of one table entry (s_slot, t_slot), s,t = attached vertices:
 *   DIRECT if the graph is complete, or prefers direct paths and has an s->t edge;
 *   else t == s: the Dijkstra row's [s] path (self-loop) under SPE_SELF_ROW,
 *                or 2 x min incident edge under SPE_SELF_RULE (and whenever s has no self-loop);
 *   else the shortest path of the source row of s (per-source rows: tree_s(s->t)).
 *   latency/reliability are bit-identical to the reference's f64 operation order;
 *   route (next hop, hops) follows the canonical tie-break
 *   parent(v) = argmin (dist[u], u) over {u : fl(dist[u] + w) == dist[v]},
 *   which equals igraph's choice whenever no two candidates share dist[u].
 *   Unroutable: latency = reliability = -1, hops = 0 (topology_getLatency's -1.0).
 */
#ifndef SPE_H_
#define SPE_H_

/* ABI guard: every struct the library reads or fills starts with struct_size,
 * which the caller sets to sizeof() of the struct as IT was compiled
 * (SPE_STRUCT_INIT).  The library refuses (SPE_EINVAL) a struct of another size,
 * so a caller built against an older spe.h -- whose structs lack trailing fields
 * this one has -- is rejected instead of having its stack read as options or
 * overwritten with statistics. */
#define SPE_STRUCT_INIT(T) {(uint32_t)sizeof(T)}

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* return codes */
#define SPE_OK 0
#define SPE_EINVAL (-1)      /* bad argument / graph fails the reference's validation */
#define SPE_EHIP (-2)        /* a HIP runtime call failed */
#define SPE_ENOMEM (-3)
#define SPE_EUNSUPPORTED (-4)
#define SPE_ESTATE (-5)      /* call order violated (e.g. get before build) */
#define SPE_ENODEV (-6)      /* no gfx950 device visible */

#define SPE_SELF_ROW 0       /* (s,s) from the Dijkstra row's [s] path (igraph 0.7-0.9) */
#define SPE_SELF_RULE 1      /* (s,s) = 2 x min incident edge (shd-topology.c:1530-1638) */

#define SPE_ENGINE_AUTO 0    /* LDS engine when the relaxation graph fits one CU's LDS, else BATCH */
#define SPE_ENGINE_BATCH 1   /* 64-source lane groups, HBM-resident state, frontier rounds */
#define SPE_ENGINE_LDS 2     /* one workgroup per source row, state resident in LDS (<= 10,240 relaxation vertices) */
#define SPE_ENGINE_FW 3      /* blocked min-plus Floyd-Warshall closure carrying (latency, reliability, first
                              * edge), then every row re-folded in path order along the first-edge walk
                              * (<= 32,768 relaxation vertices; never picked by AUTO: the LDS engine is
                              * faster on every graph it fits).  Bit-exact where shortest paths are unique
                              * (tie-free weights); equal-length paths resolve to the lowest pivot, not to
                              * the canonical (d[u], u) rule */

typedef struct spe_graph spe_graph;
typedef struct spe_table spe_table;

/* Edge list exactly as the GraphML file gives it: vertex i = i-th <node>,
 * edge e = e-th <edge>.  vertex_packetloss[v] = NaN when absent (or the
 * pointer is NULL: all absent).  Validation mirrors _topology_checkGraph:
 * latency > 0, 0 <= packetloss <= 1, endpoints in range. */
typedef struct spe_graph_desc {
    uint32_t struct_size;           /* sizeof(spe_graph_desc) as the caller compiled it */
    int32_t n_vertices;
    int64_t n_edges;
    const int32_t* edge_source;
    const int32_t* edge_target;
    const double* edge_latency;     /* ms */
    const double* edge_packetloss;
    const double* vertex_packetloss;
    int32_t directed;
    int32_t prefer_direct;          /* graph attribute preferdirectpaths */
    int32_t keep_pendants;          /* 1: relax over every vertex (no pendant pruning, so relaxation
                                     * ids = vertex ids, e.g. for spe_fw_apsp's matrix); 0 = prune */
} spe_graph_desc;

typedef struct spe_graph_info {
    uint32_t struct_size;           /* sizeof(spe_graph_info) as the caller compiled it */
    int32_t n_vertices;
    int64_t n_edges;
    int64_t n_relax_entries;        /* directed adjacency entries after merging parallel edges
                                     * (of the relaxation graph: pendants pruned) */
    int32_t directed;
    int32_t prefer_direct;
    int32_t complete;               /* _topology_isComplete */
    int32_t parallel_latency_differs; /* multigraph whose get_eid edge is not the lightest */
    int32_t weight_floor_ok;        /* every fl(d + w) > d is guaranteed (no absorbed edges) */
    int32_t device;
    int32_t n_relax_vertices;       /* vertices the relaxation runs on: undirected pendant
                                     * vertices (one neighbour) are one edge off their anchor
                                     * and need no relaxation state */
    int32_t sums_exact;             /* every latency is k / 2^q with every path sum below 2^53:
                                     * every f64 path sum is exact, so the LATENCIES of shared /
                                     * derived rows (spe_table_opts.exact_sources = 0) are the
                                     * path-order sums bit for bit (and no margin check is needed) */
    int32_t shared_rows_exact;      /* sums_exact and every edge factor 1 - p is 1.0: shared / derived
                                     * rows' reliabilities (a(s, c) r_c(t) instead of the path-order
                                     * product from the source, shd-topology.c:1415-1484) are exact
                                     * too, so the default build equals exact_sources = 1 bit for bit */
} spe_graph_info;

typedef struct spe_table_opts {
    uint32_t struct_size;           /* sizeof(spe_table_opts) as the caller compiled it */
    int32_t self_mode;              /* SPE_SELF_ROW | SPE_SELF_RULE */
    int32_t force_sssp;             /* 1: ignore complete/preferdirectpaths (diagnostic) */
    int32_t groups_per_launch;      /* 64-source groups relaxed together; 0 = auto (with shared
                                     * anchor trees: 64-lane blocks of roots the state holds) */
    int32_t block_begin;            /* first 64-row source block owned by this table */
    int32_t block_end;              /* one past the last; 0,0 = all blocks */
    /* optional caller-owned device storage for the owned blocks (all three or none),
     * each sized (block_end-block_begin) * n_attached * 64 elements */
    void* ext_latrel;               /* double[2] {latency, reliability} */
    void* ext_next_hop;             /* int32_t  */
    void* ext_hops;                 /* uint16_t */
    int32_t ext_filled;             /* 1: the external storage already holds the rows (e.g. an
                                     * RCCL all-gather of other tables' blocks): usable for
                                     * get / download / lookup without spe_table_build */
    const int32_t* owner_rank;      /* host array [n_attached] or NULL.  Non-NULL: compat mode that
                                     * replays the reference's first-writer-wins path cache
                                     * (shd-topology.c:1292-1321, 1952-2034) as if every source
                                     * slot had run its Dijkstra in increasing owner_rank order:
                                     * entry (s,t) then answers the path stored for {s,t} in
                                     * either direction.  Needs a table owning all blocks; applied
                                     * by spe_table_build (not spe_table_build_blocks). */
    int32_t engine;                 /* SPE_ENGINE_* */
    int32_t lanes_per_group;        /* sources sharing one relaxation frontier: 64 or 128 (each
                                     * thread carries 2 sources); 0 = default: 128 when
                                     * groups_per_launch is even (no padding lanes), else 64 */
    int32_t want_aux;               /* 1: also fold the graph's auxiliary edge attribute
                                     * (spe_graph_set_edge_aux) along every row's path, in path
                                     * order from 0.0 -- the offline completion tool's jitter sum
                                     * (compute-topology-paths.py:27-33).  SSSP rows on the batch
                                     * engine only (force_sssp for complete / preferdirect graphs);
                                     * (s,s) = 0, unroutable = -1. */
    /* Multi-device build in ONE process (Shadow is single-process, shd-master.c:390-394).
     * n_devices > 1: device i builds the contiguous share i of the 64-source blocks
     * (spe_device_shares) on its own host thread and stream, into a replica of the
     * {latency, reliability} records on that device; spe_table_build then all-gathers
     * the records (RCCL ncclAllGather over xGMI, communicators from ncclCommInitAll)
     * so that every device holds the whole table.  Next hop / hops stay with the
     * building device.  devices[0] is the table's home (lookups, layout).  Not
     * combinable with block ranges, external storage, owner replay or want_aux; the
     * on-disk cache and spe_table_build_blocks are single-device only. */
    const int32_t* devices;         /* n_devices device indices (NULL: the graph's device) */
    int32_t n_devices;              /* 0 or 1: single device */
    int32_t gather;                 /* SPE_GATHER_* */
    /* Batch-engine tuning of 128-lane rows (64-lane rows ignore the first three); 0 everywhere =
     * the measured defaults.  Tests and A/B experiments set these; the
     * library reads no environment variables. */
    int32_t relax_kernel;           /* SPE_RELAX_* (128-lane rows only) */
    int32_t rows_in_flight;         /* neighbour rows per memory round trip (0 = default) */
    int32_t waves_per_simd;         /* occupancy the relaxation kernel is held to (0 = the shape's
                                     * default, 1 = the compiler's choice) */
    int32_t no_overlap;             /* 1: batch i's rows do not overlap batch i+1's relaxation */
    double delta_ms;                /* > 0: Delta-stepping schedule (measured slower, MEASUREMENTS.md) */
    int32_t trace;                  /* 1: per-launch kernel times to stderr while profiling */
    /* Multi-device compute-versus-gather split: the first S source blocks
     * are sharded (contiguous shares, built in chunks whose records are broadcast to
     * every device while the next chunk builds), the remaining blocks are built by
     * every device itself.  S / nblk = shared_fraction when in (0, 1]; 0 = from the
     * model x* = T1 N / ((N - 1)(span / B + T1)) with T1 = build_seconds_hint (or the
     * library's estimate) and B = gather_gbps (or 300 GB/s). */
    double shared_fraction;
    double gather_gbps;
    double build_seconds_hint;      /* one-device whole-table build time, if the caller measured it */
    /* 1: the batch engine relaxes the graph itself instead of its degree-3 contraction
     * (same rows; the contraction is the default where it applies) */
    int32_t no_contract;
    /* 1: every pruned pendant source relaxes on its own lane, so its latencies are the
     * path-order sums bit for bit.  Default 0: pendant sources sharing an anchor take
     * the anchor's relaxation, their rows the anchor's with the pendant edge folded in
     * front -- routes (next hop, hops, routability) identical, latency / reliability
     * within a few ulps: measured over every entry against exact_sources = 1, at most
     * 8.3e-16 relative on C3 and 7.5e-16 on C4 (tests assert 1e-12; the north star
     * allows 1e-9), exact where every weight is k / 2^q.  A source whose
     * anchor's parent decisions are within rounding of a tie is rebuilt on its own lane. */
    int32_t exact_sources;
} spe_table_opts;

#define SPE_RELAX_AUTO 0            /* the default below */
#define SPE_RELAX_REGISTER 1        /* k_relax_m: neighbour rows staged in registers */
#define SPE_RELAX_LDS_RING 2        /* k_relax_s: neighbour rows gathered into a per-wave LDS ring by
                                     * LDS-DMA, in-CSR bounds prefetched with the frontier word */

#define SPE_GATHER_AUTO 0           /* RCCL when the devices are distinct and librccl loads, else PEER */
#define SPE_GATHER_RCCL 1           /* ncclAllGather, in place, one communicator per device */
#define SPE_GATHER_PEER 2           /* hipMemcpyPeerAsync from every share's owner to every other device */

/* The multi-device share of device i: 64-source blocks [block_begin[i], block_end[i])
 * of the ceil(n_attached / 64) blocks, contiguous, every share padded to the same
 * ceil(blocks / n_devices) (the all-gather's equal counts; a share past the end is
 * empty).  Host-only. */
int spe_device_shares(int32_t n_attached, int32_t n_devices, int32_t* block_begin, int32_t* block_end);
/* The multi-device split for shared_fraction x in [0, 1]: x = 1 is
 * spe_device_shares (every block sharded, local_begin = the block count); x < 1
 * gives every device an equal share of floor(x nblk / N) blocks of [0, S),
 * S = N floor(x nblk / N), and *local_begin = S: blocks [S, nblk) are built by
 * every device itself.  Host-only. */
int spe_device_split(int32_t n_attached, int32_t n_devices, double shared_fraction, int32_t* block_begin,
                     int32_t* block_end, int32_t* local_begin);

/* Where a table keeps its rows.  Element (s_slot, t_slot) of a field lives at
 *   ((s_slot / 64 - block_begin) * n_attached + t_slot) * 64 + s_slot % 64
 * ("SB64": 64 source rows interleaved per target, so one source block is one
 * contiguous span and a 64-source batch writes whole segments).  Latency and
 * reliability share one 16-byte record (the per-packet lookup reads both:
 * one HBM line per query instead of two). */
typedef struct spe_table_layout {
    uint32_t struct_size;           /* sizeof(spe_table_layout) as the caller compiled it */
    int32_t n_attached;
    int32_t block_begin;
    int32_t block_end;
    int64_t elems;                  /* per field */
    void* latrel;                   /* device pointers: double[2] {latency, reliability} */
    void* next_hop;
    void* hops;
    int32_t groups_per_launch;      /* 64-source blocks one build launch covers (shared anchor
                                     * trees: 64-lane blocks of roots one relaxation holds) */
    int32_t engine;                 /* the engine the table runs on (SPE_ENGINE_BATCH / _LDS) */
    int32_t n_devices;              /* > 1: a multi-device table; latrel is the home device's
                                     * replica of ALL blocks (padded to n_devices equal shares),
                                     * next_hop / hops are NULL (they stay with each share's device) */
    int32_t device;                 /* the device latrel lives on */
    int32_t lanes_per_group;        /* batch engine: sources per relaxation row (64 or 128 by default) */
    int32_t relax_kernel;           /* batch engine: the SPE_RELAX_* kernel it runs */
    int32_t contracted_vertices;    /* batch engine on the degree-3 contraction: its relaxation
                                     * vertices (0: the table relaxes the graph itself) */
    int32_t shared_sources;         /* 1: pendant sources take their anchor's relaxation
                                     * (spe_table_opts.exact_sources) */
    int32_t host_reads;             /* single entries (spe_table_get / _get_latrel): 1 = host
                                     * loads of the device memory, mapped into the process on a
                                     * large-BAR host; 0 = a device-to-host copy each; -1 = not
                                     * decided yet (decided at the first read of a built table;
                                     * SPE_HOST_READS=0 forces copies) */
    int32_t host_prefault;          /* host_reads = 1: the host mapping of the latrel field is
                                     * faulted in by a background thread from the first host read
                                     * on, so later reads take no page fault: 0 not started,
                                     * 1 running, 2 done, -1 off (SPE_HOST_PREFAULT=0; =N: N
                                     * threads, 1 by default) */
    int32_t reserved0;
    double host_prefault_s;         /* seconds the pre-fault took (2) or has taken so far (1) */
} spe_table_layout;

typedef struct spe_entry {
    double latency;                 /* ms, -1 if unroutable */
    double reliability;             /* -1 if unroutable */
    int32_t next_hop;               /* vertex index of the first hop, -1 if unroutable */
    int32_t hops;                   /* edges on the path, 0 if unroutable */
} spe_entry;

typedef struct spe_build_stats {
    uint32_t struct_size;           /* sizeof(spe_build_stats) as the caller compiled it */
    int64_t iterations;             /* relaxation rounds summed over launches */
    int64_t active_rounds;          /* relaxation rounds in which some distance/route changed */
    int64_t launches;
    double seconds;                 /* wall time of the last spe_table_build (incl. the gather) */
    double gather_seconds;          /* multi-device: the all-gather of the records */
    int32_t n_devices;
    int32_t gather;                 /* the SPE_GATHER_* mode used */
    int32_t shared_blocks;          /* multi-device: blocks sharded and gathered (the rest built on every device) */
    int32_t local_blocks;
    double build_wait_seconds;      /* multi-device: slowest device's build time (shares + local part) */
    int64_t relaxed_lanes;          /* batch engine: relaxation lanes (sources, or shared anchor
                                     * roots) the last build ran, padding excluded */
    int32_t fallback_blocks;        /* shared anchor trees: source blocks rebuilt lane per source */
    int64_t derived_sources;        /* contracted shared tables: sources whose rows came from their
                                     * neighbours' roots (three for a contracted vertex, four for a
                                     * degree-4 one), without a relaxation lane */
} spe_build_stats;

const char* spe_last_error(void);
int spe_device_count(int32_t* out);

int spe_graph_create(const spe_graph_desc* desc, int32_t device, spe_graph** out);
int spe_graph_info_get(const spe_graph* g, spe_graph_info* out);
/* A slot order for `attached` that clusters sources for the batch engine.
 * Sources are grouped into the Voronoi cells of ceil(A / 64) seeded-random
 * centres over the relaxation graph (then by distance to the centre, by
 * relaxation vertex, by id); a pruned pendant counts at its anchor, so sources
 * sharing an anchor are adjacent.  Lanes of one 64-source group then advance in
 * similar relaxation rounds (fewer row visits): C4 (100k stubs on 20k anchors)
 * +17 %, C3 +6 %.  The table semantics do not depend on slot order (the
 * reference's target set A is unordered, shd-topology.c:1510-1528), so a caller
 * that numbers slots itself (the topology shim, the bench) may use it.
 * order_out[i] = the vertex to put in slot i (a permutation of attached). */
int spe_order_sources(const spe_graph* g, const int32_t* attached, int32_t n_attached, int32_t* order_out);
/* Optional per-edge auxiliary attribute (e.g. GraphML "jitter"), edge_aux[e] for
 * every edge e of the description; a merged vertex pair takes its get_eid edge's
 * value.  Replaces nothing in shd-topology.c (which only validates jitter,
 * :1090-1100); it serves the offline completion tool (compute-topology-paths.py). */
int spe_graph_set_edge_aux(spe_graph* g, const double* edge_aux);
/* Host-side rule evaluation (no GPU work; thread-safe), for a caller that keeps
 * the reference's lazy path cache semantics (the topology shim):
 *   spe_graph_self_path  _topology_computeShortestPathToSelf  shd-topology.c:1530-1638:
 *                        the first minimum-latency edge of v's OUT incidence list,
 *                        taken twice: latency 2w, reliability r*r, no vertex loss,
 *                        next_hop = the edge's other endpoint, hops = 2; latency -1 /
 *                        hops 0 when v has no incident edge;
 *   spe_graph_adjacent   _topology_verticesAreAdjacent        shd-topology.c:1233-1249:
 *                        *out = 1 when an edge from -> to exists (either direction
 *                        for undirected graphs; a self-loop for from == to). */
int spe_graph_self_path(const spe_graph* g, int32_t v, spe_entry* out);
int spe_graph_adjacent(const spe_graph* g, int32_t from, int32_t to, int32_t* out);
/* The get_eid edge from -> to (shd-topology.c:387-429 _topology_getEdgeHelper, the
 * highest-id parallel edge as DESIGN §1 restates igraph): its latency and
 * reliability 1 - packetloss; SPE_EINVAL when there is no such edge.  Host-only. */
int spe_graph_edge(const spe_graph* g, int32_t from, int32_t to, double* latency, double* reliability);
void spe_graph_free(spe_graph* g);

/* attached[i] = vertex of source/target slot i (unique vertices). */
int spe_table_create(spe_graph* g, const int32_t* attached, int32_t n_attached,
                     const spe_table_opts* opts, spe_table** out);
/* Compute every owned source row (enqueued on `stream`, returns after completion). */
int spe_table_build(spe_table* t, void* stream);
/* Compute only source blocks [block_begin, block_end) (absolute block ids, a
 * sub-range of the owned ones): incremental / stepped builds. */
int spe_table_build_blocks(spe_table* t, int32_t block_begin, int32_t block_end, void* stream);
/* Build blocks [block_begin, block_end) of the owned range into caller device
 * buffers instead of the table's storage: latrel / next_hop / hops address block
 * block_begin's first element, in the SB64 layout of (block_end - block_begin)
 * blocks.  The table's own rows are untouched and not marked built.  For
 * schedules that place the records and the next hops / hop counts apart (a rank
 * keeping the next hops of its own blocks only, beside a replicated record
 * span).  Not for owner-replay or want_aux tables. */
int spe_table_build_blocks_into(spe_table* t, int32_t block_begin, int32_t block_end, void* latrel,
                                void* next_hop, void* hops, void* stream);

/* Per-kernel device time, from HIP events recorded around every launch on the
 * build stream while profiling is enabled (costs one event pair per launch). */
enum { SPE_K_INIT = 0, SPE_K_SEED, SPE_K_HEAVY, SPE_K_RELAX, SPE_K_ROWS, SPE_K_DIRECT, SPE_K_LDS, SPE_K_FW,
       SPE_K_ROUTES,   /* the route pass after an LDS-ring relaxation (k_routes_init, k_routes) */
       SPE_K_COUNT };
typedef struct spe_kernel_profile {
    double ms[SPE_K_COUNT];
    int64_t launches[SPE_K_COUNT];
} spe_kernel_profile;
int spe_table_profile_enable(spe_table* t, int32_t enable);   /* also resets the counters */
int spe_table_profile_get(const spe_table* t, spe_kernel_profile* out);
int spe_table_build_stats(const spe_table* t, spe_build_stats* out);
int spe_table_layout_get(const spe_table* t, spe_table_layout* out);
/* One entry, read back from HBM (synchronous). */
int spe_table_get(const spe_table* t, int32_t s_slot, int32_t t_slot, spe_entry* out);
/* Only the {latency, reliability} record of one entry (one 16-B read back): what
 * topology_getLatency / getReliability need (shd-topology.c:2036-2061). */
int spe_table_get_latrel(const spe_table* t, int32_t s_slot, int32_t t_slot, double* latency, double* reliability);
/* The {latency, reliability} records of one whole source row (n_attached each), read
 * back in one gather on the device (a host mirror of a row that is read repeatedly). */
int spe_table_get_row_latrel(const spe_table* t, int32_t s_slot, double* latency, double* reliability);
/* Copy owned rows [row_begin,row_end) x [0,n_attached) to host, row-major;
 * any output pointer may be NULL. */
int spe_table_download(const spe_table* t, int32_t row_begin, int32_t row_end, double* latency,
                       double* reliability, int32_t* next_hop, int32_t* hops);
/* Blocked min-plus Floyd-Warshall over the relaxation graph (vertex ids as in
 * spe_graph_info.n_relax_vertices: undirected pendants pruned), the north
 * star's dense-regime algorithm, kept as a measured comparison engine and an
 * independent distance check.  d_dist: caller device buffer of ld x ld doubles
 * (ld = a multiple of 64 >= n_relax_vertices); d_next (optional, n x n int32):
 * the first hop, argmin over out-neighbours u of w(i,u) + dist(u,j).  FW sums
 * path segments in its own association order, so distances agree with the
 * table's path-order folds only to rounding (the table is what is bit-exact).
 * `seconds`: device time of the closure (init + pivot steps). */
int spe_fw_apsp(spe_graph* g, double* d_dist, int64_t ld, int32_t* d_next, void* stream, double* seconds);
/* The same closure carrying the north star's triple (the FW engine's first
 * stage): d_dist / d_rel / d_next are caller device buffers of ld x ld elements;
 * d_rel(i,j) = the product of the edge factors (1 - p) of the chosen path,
 * multiplied in FW's association order (rel(i,k) * rel(k,j) at the pivot that
 * last improved the pair), d_next(i,j) = the first hop (relaxation vertex id,
 * -1 unreachable / i == j).  Replaces the all-pairs step of the offline tool
 * (compute-topology-paths.py:89-94) and, in the table, igraph's per-source
 * Dijkstra (shd-topology.c:1741).  d_rel may be NULL: the (latency, first hop)
 * pair only -- what the FW engine's table build runs, since its rows re-fold
 * latency and reliability in path order along the first hops (half the LDS
 * panels and registers of the triple). */
int spe_fw_closure(spe_graph* g, double* d_dist, double* d_rel, int32_t* d_next, int64_t ld, void* stream,
                   double* seconds);
/* The shortest-path tree the SSSP row of source slot s_slot follows:
 * parent[v] (n_vertices entries, original ids) = the vertex before v on the
 * row's path from s to v; -1 for s itself and unreachable v.  The row's path to
 * any v is the parent walk from v back to s -- what the reference's per-path log
 * line prints (shd-topology.c:1809-1829, the path string of :1413-1493).  The
 * source's block is recomputed (its rows are rewritten with the same values),
 * so this is for logging and diagnostics, not the query path.  Not for DIRECT
 * (complete-graph) tables nor owner-replay tables (SPE_EUNSUPPORTED). */
int spe_table_source_tree(spe_table* t, int32_t s_slot, int32_t* parent);
/* Owned rows [row_begin,row_end) of the want_aux field, row-major, to host. */
int spe_table_download_aux(const spe_table* t, int32_t row_begin, int32_t row_end, double* aux);
/* Batched per-packet lookups against the HBM-resident table.  d_pairs holds q
 * (s_slot, t_slot) int32 pairs; outputs are device arrays of q elements.
 * ok = 1 when routable (topology_isRoutable).  Pairs whose source row is not
 * owned by this table return ok = 0, latency = reliability = -1. */
int spe_lookup_batch(const spe_table* t, const int32_t* d_pairs, int64_t q, double* d_latency,
                     double* d_reliability, uint8_t* d_ok, void* stream);
/* The same against replica `replica` of a multi-device table (0 = the home
 * device; for a single-device table only 0): pairs and outputs live on that
 * replica's device (spe_table_replica_device), so every device answers its own
 * batch from its own HBM (the C5 replicas; shd-worker.c:235-247 is
 * the per-packet lookup it batches).  The stream, if given, is on that device. */
int spe_lookup_batch_replica(const spe_table* t, int32_t replica, const int32_t* d_pairs, int64_t q,
                             double* d_latency, double* d_reliability, uint8_t* d_ok, void* stream);
int spe_table_replica_device(const spe_table* t, int32_t replica, int32_t* device);
/* spe_lookup_batch with HOST arrays (pairs: q (s_slot, t_slot) int32 pairs): the
 * batch is staged through pinned buffers to the home replica and answered there,
 * in chunks of 4M queries, synchronously.  For a host caller (the topology shim's
 * topology_getPathInfoBatch) that resolves a round of packets at once instead of
 * one device read per query.  Thread-safe (callers are serialised per table). */
int spe_lookup_batch_host(const spe_table* t, const int32_t* pairs, int64_t q, double* latency,
                          double* reliability, uint8_t* ok);

/* Whole-table self-check on the device (every (s, t) entry, s != t, of a built
 * single-device table owning every row): the consequences of the reference's
 * per-target path walk (shd-topology.c:1790-1849) that hold entry by entry --
 * routable entries have latency > 0, reliability in (0, 1] and hops >= 1; the
 * next hop is an out-neighbour of s (get_eid(s, next) exists, :1473-1480); where
 * the next hop is an attached vertex other than t, hops(s, t) = 1 + hops(next, t)
 * (unique shortest paths: the rest of s's path is next's path); and on an
 * undirected graph lat / rel of (s, t) and (t, s) agree within 1e-12 relative
 * (the same edges summed / multiplied in opposite orders).  Counts only: which
 * of them must be zero depends on the graph (unroutable pairs, ties). */
typedef struct spe_check_report {
    int64_t pairs;
    int64_t unroutable;
    int64_t bad_values;
    int64_t next_not_adjacent;
    int64_t hop_checked;
    int64_t hop_mismatch;
    int64_t sym_checked;
    int64_t sym_mismatch;
    double max_sym_rel_err;
    int32_t first_bad_s;            /* one offending (s, t) slot pair, -1 if none */
    int32_t first_bad_t;
} spe_check_report;
int spe_table_check(const spe_table* t, spe_check_report* out);
/* Entry-by-entry comparison of two built single-device tables over the same
 * attached slots, owned block range and device (e.g. the library default --
 * shared / derived rows -- against exact_sources = 1, which is what the topology
 * shim seals on non-dyadic latencies), on the device, every (s, t) entry:
 *   route_mismatch      routability, next hop or hop count differ (must be 0:
 *                       routes are exact in every mode);
 *   latency_differs / reliability_differs   bit differences of routable entries;
 *   beyond_tolerance    |a - b| > rel_tol |b| in latency or reliability;
 *   delivery_flips      ceil(latency * 1e6) differs: the packet delay in ns
 *                       Shadow's worker derives from getLatency (shd-worker.c:244,
 *                       SIMTIME_ONE_MILLISECOND = 1e6), i.e. simulated behaviour. */
typedef struct spe_compare_report {
    uint32_t struct_size;           /* sizeof(spe_compare_report) as the caller compiled it */
    int64_t pairs;
    int64_t routable;               /* routable in table b */
    int64_t route_mismatch;
    int64_t latency_differs;
    int64_t reliability_differs;
    int64_t beyond_tolerance;
    int64_t delivery_flips;
    double max_latency_rel_err;
    double max_reliability_rel_err;
    int32_t first_bad_s;            /* first route mismatch or out-of-tolerance pair (slots), -1 none */
    int32_t first_bad_t;
} spe_compare_report;
int spe_table_compare(const spe_table* a, const spe_table* b, double rel_tol, spe_compare_report* out);
/* Minimum latency over every owned routable entry (minimumPathLatency). */
/* On-disk path-table cache (the reference recomputes its paths
 * every run).  The key hashes everything that determines the rows: the graph
 * description, the attached set, self_mode, force_sssp, owner_rank and the block
 * range.  spe_table_save writes the owned rows of a built table (atomically:
 * "<path>.tmp" then rename); spe_table_load fills a created table from a file
 * saved under the same key and marks it built, or returns SPE_EINVAL (other key,
 * not a cache file, truncated) and leaves it unbuilt. */
int spe_table_key(const spe_table* t, uint64_t* key);
int spe_table_save(const spe_table* t, const char* path);
int spe_table_load(spe_table* t, const char* path);
int spe_table_min_latency(const spe_table* t, double* out);
void spe_table_free(spe_table* t);

#ifdef __cplusplus
}
#endif
#endif /* SPE_H_ */
