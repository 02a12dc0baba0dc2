/*
 * oracle.h -- CPU restatement of Shadow's topology path rules on top of an
 * igraph-0.7..0.9-faithful Dijkstra.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in shadow_amd/ links or calls this; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker / the timed CPU baseline.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   DIRECT regime  -- pinned by the reference's own fixtures (the shipped
 *                     resource/topology.graphml.xml.xz and the 1-vertex test
 *                     configs under src/test/), see tests/golden/.
 *   SSSP regime    -- the reference has no test that reaches Dijkstra and igraph
 *                     is absent from this image: distances are cross-checked
 *                     against scipy's Dijkstra; routes/ties are
 *                     "parity unpinned" beyond this restatement.
 */
#ifndef SPE_ORACLE_H_
#define SPE_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_graph orc_graph;

/* Row entry kinds (which reference rule produced the value). */
enum { ORC_FAIL = 0, ORC_DIRECT = 1, ORC_SSSP = 2, ORC_SELF = 3 };

/* self_mode: how (s,s) is answered when DIRECT does not apply.
 *   0 = ROW : the Dijkstra row's [s] path (self-loop edge, shd-topology.c:1456-1484);
 *             falls back to SELF when s has no self-loop (the row entry would fail).
 *   1 = SELF: 2 x min incident edge (_topology_computeShortestPathToSelf, :1530-1638). */
/* tie_mode: 0 = igraph 2wheap pop order (exact restatement);
 *           1 = canonical (dist[u] asc, u asc) -- the rule the HIP kernels implement. */
/* force_sssp: 1 = ignore completeness / preferdirectpaths (the diagnostic SSSP
 * table of SURVEY.md K4 on a complete graph). */
typedef struct orc_opts {
    int32_t self_mode;
    int32_t tie_mode;
    int32_t force_sssp;
} orc_opts;

/* Edge list in GraphML order: edge id e = e-th <edge>, vertices in <node> order.
 * vloss[v] = NaN when the vertex has no packetloss attribute. */
orc_graph* orc_graph_new(int32_t n, int64_t m, const int32_t* esrc, const int32_t* edst,
                         const double* elat, const double* eloss, const double* vloss,
                         int32_t directed, int32_t prefer_direct);
void orc_graph_free(orc_graph* g);

int32_t orc_is_complete(const orc_graph* g);                 /* shd-topology.c:435-537 */
int64_t orc_get_eid(const orc_graph* g, int32_t from, int32_t to); /* -1 when absent */

/* igraph_get_shortest_paths_dijkstra (mode OUT) restated; dist[v] = -1 if never
 * reached; parent_eid[v] = -1 for the source / unreached.  stop_early mirrors
 * igraph's to_reach early exit.  pop_rank (optional) = order of extraction. */
int32_t orc_dijkstra(const orc_graph* g, int32_t src, const int32_t* targets, int32_t ntargets,
                     int32_t stop_early, double* dist, int64_t* parent_eid, int32_t* pop_rank);

/* Build per-source rows.  Outputs are [nsrc][A] row-major.  kind[] as enum above.
 * double_ties (optional) accumulates vertices on reported paths whose igraph
 * parent differs from the canonical one or whose choice was a double tie.
 * dijkstra_seconds (optional) accumulates the time spent inside Dijkstra only
 * (the reference's own timer, shd-topology.c:1736-1773). nthreads>1 uses OpenMP. */
int32_t orc_rows(const orc_graph* g, const orc_opts* opts,
                 const int32_t* sources, int32_t nsrc, const int32_t* targets, int32_t A,
                 double* lat, double* rel, int32_t* next, int32_t* hops, uint8_t* kind,
                 int64_t* double_ties, double* dijkstra_seconds, int32_t nthreads);
/* orc_rows plus prev[] (optional): the vertex before the target on each path
 * (the source for one-edge and [s] paths, the other endpoint for SELF, -1 on failure). */
int32_t orc_rows2(const orc_graph* g, const orc_opts* opts,
                  const int32_t* sources, int32_t nsrc, const int32_t* targets, int32_t A,
                  double* lat, double* rel, int32_t* next, int32_t* hops, uint8_t* kind, int32_t* prev,
                  int64_t* double_ties, double* dijkstra_seconds, int32_t nthreads);

/* Per-packet lookup restatement (C5 CPU baseline): IP -> slot hash, then the
 * two-level path cache src -> (dst -> path), shd-topology.c:1952-2075. */
typedef struct orc_cache orc_cache;
orc_cache* orc_cache_new(int32_t A, const uint32_t* ips, int64_t npairs, const int32_t* pairs, const double* lat,
                         const double* rel);
void orc_cache_free(orc_cache* c);
int64_t orc_cache_lookup(const orc_cache* c, const uint32_t* sip, const uint32_t* dip, int64_t q, double* lat,
                         double* rel, uint8_t* ok, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
