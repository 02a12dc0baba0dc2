/*
 * oracle.c -- CPU restatement of the reference's topology path computation.
 *
 * TEST INFRASTRUCTURE ONLY (the checker and the timed CPU baseline).  The
 * product path (shadow_amd/) never links, loads or calls this file.
 *
 * What is restated, and from where:
 *   - igraph 0.7-0.9 graph storage (third-party, NOT vendored in the reference,
 *     no pinned version: cmake/FindIGRAPH.cmake:14-53; API use at
 *     src/main/routing/shd-topology.c:1741 bounds it to 0.7.x-0.9.x):
 *       * undirected edges stored as (from=max, to=min)           [igraph_add_edges]
 *       * oi/ii edge indices from the two-pass radix sort           [igraph_vector_order]
 *         -> (primary asc, secondary asc, edge id DESC within equal keys)
 *       * incidence lists: directed OUT = oi range of v; undirected = oi range
 *         then ii range (ascending neighbour id, self-loops twice) [igraph_incident]
 *       * get_eid = lower-bound binary search in the smaller list  [FIND_DIRECTED_EDGE]
 *       * indexed binary max-heap igraph_2wheap (shift_up on >=, sink left on
 *         ties, strict < swaps)                                     [indheap.c]
 *       * igraph_get_shortest_paths_dijkstra: dist=-1 unvisited, strict '<'
 *         relaxation, early exit when every target is popped, target==source
 *         yields the one-vertex path [src]
 *   - Shadow's rules, with the exact floating-point operation order:
 *       * _topology_isComplete                 shd-topology.c:435-537
 *       * _topology_getEdgeHelper              shd-topology.c:387-429 (rel = 1.0f - p)
 *       * _topology_computePathProperties      shd-topology.c:1392-1508
 *       * _topology_computeShortestPathToSelf  shd-topology.c:1530-1638
 *       * _topology_computeSourcePaths         shd-topology.c:1640-1860 (lat==0 -> 1)
 *       * _topology_lookupDirectPath           shd-topology.c:1862-1912
 *       * regime dispatch                      shd-topology.c:2002-2014
 *
 * Compile with -O2 -ffp-contract=off (no fused multiply-add, no fast-math): the
 * reference's additions and multiplications are separately rounded IEEE f64.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

struct orc_graph {
    int32_t n;
    int64_t m;
    int32_t directed;
    int32_t prefer_direct;
    int32_t complete;
    int32_t* from;   /* igraph-normalised endpoints */
    int32_t* to;
    double* lat;
    double* loss;
    double* vloss;   /* NaN = attribute absent */
    int64_t* oi;     /* edges ordered by (from, to, eid desc) */
    int64_t* ii;     /* edges ordered by (to, from, eid desc) */
    int64_t* os;     /* n+1 offsets into oi */
    int64_t* is;     /* n+1 offsets into ii */
};

/* ---------------------------------------------------------------- storage */

/* igraph_vector_order(v, v2, res, nodes): two bucket passes.  The first pass
 * buckets by v2 pushing at the head of each bucket list (so equal v2 come out in
 * DESCENDING edge id); the second walks that result backwards and buckets by v
 * (so it is stable with respect to the first pass). */
static void orc_vector_order(const int32_t* v, const int32_t* v2, int64_t m, int32_t n, int64_t* res) {
    int64_t* ptr = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t* rad = (int64_t*)calloc((size_t)(m > 0 ? m : 1), sizeof(int64_t));
    int64_t i, j;
    for (i = 0; i < m; i++) {
        int64_t radix = v2[i];
        if (ptr[radix] != 0) rad[i] = ptr[radix];
        ptr[radix] = i + 1;
    }
    j = 0;
    for (i = 0; i < (int64_t)n + 1; i++) {
        if (ptr[i] != 0) {
            int64_t next = ptr[i] - 1;
            res[j++] = next;
            while (rad[next] != 0) {
                next = rad[next] - 1;
                res[j++] = next;
            }
        }
    }
    memset(ptr, 0, ((size_t)n + 1) * sizeof(int64_t));
    memset(rad, 0, (size_t)(m > 0 ? m : 1) * sizeof(int64_t));
    for (i = 0; i < m; i++) {
        int64_t edge = res[m - i - 1];
        int64_t radix = v[edge];
        if (ptr[radix] != 0) rad[edge] = ptr[radix];
        ptr[radix] = edge + 1;
    }
    j = 0;
    for (i = 0; i < (int64_t)n + 1; i++) {
        if (ptr[i] != 0) {
            int64_t next = ptr[i] - 1;
            res[j++] = next;
            while (rad[next] != 0) {
                next = rad[next] - 1;
                res[j++] = next;
            }
        }
    }
    free(ptr);
    free(rad);
}

static void orc_offsets(const int32_t* key, const int64_t* order, int64_t m, int32_t n, int64_t* off) {
    int64_t i;
    int32_t v = 0;
    off[0] = 0;
    for (i = 0; i < m; i++) {
        int32_t k = key[order[i]];
        while (v < k) off[++v] = i;
    }
    while (v < n) off[++v] = m;
}

static int32_t orc_other(const orc_graph* g, int64_t e, int32_t v) {
    return g->to[e] == v ? g->from[e] : g->to[e];
}

/* number of incident edges and the edge at position k of incident(v, OUT) */
static int64_t orc_inc_len(const orc_graph* g, int32_t v) {
    int64_t len = g->os[v + 1] - g->os[v];
    if (!g->directed) len += g->is[v + 1] - g->is[v];
    return len;
}
static int64_t orc_inc_at(const orc_graph* g, int32_t v, int64_t k) {
    int64_t no = g->os[v + 1] - g->os[v];
    if (k < no) return g->oi[g->os[v] + k];
    return g->ii[g->is[v] + (k - no)];
}

/* BINSEARCH: first position in [start,end) whose key >= value, then equality test */
static int64_t orc_binsearch(int64_t start, int64_t end, int32_t value, const int64_t* iindex,
                             const int32_t* keys) {
    int64_t N = end;
    while (start < end) {
        int64_t mid = start + (end - start) / 2;
        int64_t e = iindex[mid];
        if (keys[e] < value) start = mid + 1;
        else end = mid;
    }
    if (start < N) {
        int64_t e = iindex[start];
        if (keys[e] == value) return e;
    }
    return -1;
}

int64_t orc_get_eid(const orc_graph* g, int32_t from, int32_t to) {
    if (from < 0 || to < 0 || from >= g->n || to >= g->n) return -1;
    int32_t xfrom = from, xto = to;
    if (!g->directed) {
        xfrom = from > to ? from : to;
        xto = from > to ? to : from;
    }
    int64_t start = g->os[xfrom], end = g->os[xfrom + 1];
    int64_t start2 = g->is[xto], end2 = g->is[xto + 1];
    if (end - start < end2 - start2) return orc_binsearch(start, end, xto, g->oi, g->to);
    return orc_binsearch(start2, end2, xfrom, g->ii, g->from);
}

orc_graph* orc_graph_new(int32_t n, int64_t m, const int32_t* esrc, const int32_t* edst,
                         const double* elat, const double* eloss, const double* vloss,
                         int32_t directed, int32_t prefer_direct) {
    orc_graph* g = (orc_graph*)calloc(1, sizeof(orc_graph));
    int64_t e;
    g->n = n;
    g->m = m;
    g->directed = directed ? 1 : 0;
    g->prefer_direct = prefer_direct ? 1 : 0;
    size_t mm = (size_t)(m > 0 ? m : 1);
    g->from = (int32_t*)malloc(mm * sizeof(int32_t));
    g->to = (int32_t*)malloc(mm * sizeof(int32_t));
    g->lat = (double*)malloc(mm * sizeof(double));
    g->loss = (double*)malloc(mm * sizeof(double));
    g->vloss = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    g->oi = (int64_t*)malloc(mm * sizeof(int64_t));
    g->ii = (int64_t*)malloc(mm * sizeof(int64_t));
    g->os = (int64_t*)malloc(((size_t)n + 1) * sizeof(int64_t));
    g->is = (int64_t*)malloc(((size_t)n + 1) * sizeof(int64_t));
    for (e = 0; e < m; e++) {
        if (directed || esrc[e] > edst[e]) {
            g->from[e] = esrc[e];
            g->to[e] = edst[e];
        } else {
            g->from[e] = edst[e];
            g->to[e] = esrc[e];
        }
        g->lat[e] = elat[e];
        g->loss[e] = eloss[e];
    }
    memcpy(g->vloss, vloss, (size_t)n * sizeof(double));
    orc_vector_order(g->from, g->to, m, n, g->oi);
    orc_vector_order(g->to, g->from, m, n, g->ii);
    orc_offsets(g->from, g->oi, m, n, g->os);
    orc_offsets(g->to, g->ii, m, n, g->is);
    g->complete = orc_is_complete(g);
    return g;
}

void orc_graph_free(orc_graph* g) {
    if (!g) return;
    free(g->from); free(g->to); free(g->lat); free(g->loss); free(g->vloss);
    free(g->oi); free(g->ii); free(g->os); free(g->is);
    free(g);
}

/* _topology_isComplete, shd-topology.c:435-537 */
int32_t orc_is_complete(const orc_graph* g) {
    int32_t v;
    for (v = 0; v < g->n; v++) {
        int64_t ecount = orc_inc_len(g, v);
        if (!g->directed && orc_get_eid(g, v, v) >= 0) ecount -= 1;
        if (ecount < g->n) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------- 2wheap */

typedef struct {
    double* data;     /* heap keys (-dist) */
    int64_t* index;   /* heap position -> vertex */
    int64_t* index2;  /* vertex -> position + 2, 0 = not in heap */
    int64_t size;
} orc_heap;

#define H_PARENT(x) ((((x) + 1) / 2) - 1)
#define H_LEFT(x) (((x) + 1) * 2 - 1)
#define H_RIGHT(x) (((x) + 1) * 2)

static void heap_switch(orc_heap* h, int64_t e1, int64_t e2) {
    if (e1 != e2) {
        double tmp3 = h->data[e1];
        h->data[e1] = h->data[e2];
        h->data[e2] = tmp3;
        int64_t tmp1 = h->index[e1];
        int64_t tmp2 = h->index[e2];
        h->index2[tmp1] = e2 + 2;
        h->index2[tmp2] = e1 + 2;
        h->index[e1] = tmp2;
        h->index[e2] = tmp1;
    }
}

static void heap_shift_up(orc_heap* h, int64_t elem) {
    while (!(elem == 0 || h->data[elem] < h->data[H_PARENT(elem)])) {
        heap_switch(h, elem, H_PARENT(elem));
        elem = H_PARENT(elem);
    }
}

static void heap_sink(orc_heap* h, int64_t head) {
    for (;;) {
        int64_t size = h->size;
        if (H_LEFT(head) >= size) {
            return;
        } else if (H_RIGHT(head) == size || h->data[H_LEFT(head)] >= h->data[H_RIGHT(head)]) {
            if (h->data[head] < h->data[H_LEFT(head)]) {
                heap_switch(h, head, H_LEFT(head));
                head = H_LEFT(head);
            } else {
                return;
            }
        } else {
            if (h->data[head] < h->data[H_RIGHT(head)]) {
                heap_switch(h, head, H_RIGHT(head));
                head = H_RIGHT(head);
            } else {
                return;
            }
        }
    }
}

static void heap_push(orc_heap* h, int64_t idx, double elem) {
    int64_t size = h->size;
    h->data[size] = elem;
    h->index[size] = idx;
    h->size++;
    h->index2[idx] = size + 2;
    heap_shift_up(h, size);
}

static double heap_delete_max(orc_heap* h, int64_t* idx_out) {
    double tmp = h->data[0];
    int64_t tmpidx = h->index[0];
    heap_switch(h, 0, h->size - 1);
    h->size--;
    h->index2[tmpidx] = 0;
    heap_sink(h, 0);
    *idx_out = tmpidx;
    return tmp;
}

static void heap_modify(orc_heap* h, int64_t idx, double elem) {
    int64_t pos = h->index2[idx] - 2;
    h->data[pos] = elem;
    heap_sink(h, pos);
    heap_shift_up(h, pos);
}

/* ------------------------------------------------------------ Dijkstra */

typedef struct {
    orc_heap heap;
    uint8_t* is_target;
} orc_ws;

static void ws_init(orc_ws* w, int32_t n) {
    w->heap.data = (double*)malloc(((size_t)n + 1) * sizeof(double));
    w->heap.index = (int64_t*)malloc(((size_t)n + 1) * sizeof(int64_t));
    w->heap.index2 = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    w->heap.size = 0;
    w->is_target = (uint8_t*)calloc((size_t)n + 1, 1);
}
static void ws_free(orc_ws* w) {
    free(w->heap.data); free(w->heap.index); free(w->heap.index2); free(w->is_target);
}

static int32_t dijkstra_ws(const orc_graph* g, orc_ws* w, int32_t src, const int32_t* targets,
                           int32_t ntargets, int32_t stop_early, double* dist, int64_t* parent_eid,
                           int32_t* pop_rank) {
    int32_t n = g->n, v;
    int64_t to_reach, i, rank = 0;
    if (src < 0 || src >= n) return -1;
    for (v = 0; v < n; v++) {
        dist[v] = -1.0;
        parent_eid[v] = -1;   /* igraph: parent_eids[v] = 0 (1-based edge ids) */
        w->is_target[v] = 0;
        w->heap.index2[v] = 0;
        if (pop_rank) pop_rank[v] = -1;
    }
    w->heap.size = 0;
    to_reach = ntargets;
    for (i = 0; i < ntargets; i++) {
        if (!w->is_target[targets[i]]) w->is_target[targets[i]] = 1;
        else to_reach--;
    }
    if (!stop_early) to_reach = INT64_MAX;
    dist[src] = 0.0;
    heap_push(&w->heap, src, 0);
    while (w->heap.size > 0 && to_reach > 0) {
        int64_t minnei;
        double mindist = -heap_delete_max(&w->heap, &minnei);
        if (pop_rank) pop_rank[minnei] = (int32_t)rank;
        rank++;
        if (w->is_target[minnei]) {
            w->is_target[minnei] = 0;
            to_reach--;
        }
        int64_t nlen = orc_inc_len(g, (int32_t)minnei);
        for (i = 0; i < nlen; i++) {
            int64_t edge = orc_inc_at(g, (int32_t)minnei, i);
            int32_t tto = orc_other(g, edge, (int32_t)minnei);
            double altdist = mindist + g->lat[edge];
            double curdist = dist[tto];
            if (curdist < 0) {
                dist[tto] = altdist;
                parent_eid[tto] = edge;
                heap_push(&w->heap, tto, -altdist);
            } else if (altdist < curdist) {
                dist[tto] = altdist;
                parent_eid[tto] = edge;
                heap_modify(&w->heap, tto, -altdist);
            }
        }
    }
    return 0;
}

int32_t orc_dijkstra(const orc_graph* g, int32_t src, const int32_t* targets, int32_t ntargets,
                     int32_t stop_early, double* dist, int64_t* parent_eid, int32_t* pop_rank) {
    orc_ws w;
    ws_init(&w, g->n);
    int32_t r = dijkstra_ws(g, &w, src, targets, ntargets, stop_early, dist, parent_eid, pop_rank);
    ws_free(&w);
    return r;
}

/* Incoming edges of v as Dijkstra sees them: for mode OUT, u->v edges (undirected:
 * every incident edge). */
static int64_t orc_in_len(const orc_graph* g, int32_t v) {
    if (g->directed) return g->is[v + 1] - g->is[v];
    return orc_inc_len(g, v);
}
static int64_t orc_in_at(const orc_graph* g, int32_t v, int64_t k) {
    if (g->directed) return g->ii[g->is[v] + k];
    return orc_inc_at(g, v, k);
}

/* Canonical parent: argmin (dist[u], u) over candidates u != v with
 * fl(dist[u]+w) == dist[v] and fl(dist[u]+w) > dist[u].  Returns -1 if none.
 * *tie is set when two different u share the minimal dist[u]. */
static int32_t canonical_parent(const orc_graph* g, const double* dist, int32_t v, int* tie) {
    int64_t k, len = orc_in_len(g, v);
    int32_t best = -1;
    double bestd = 0.0;
    *tie = 0;
    for (k = 0; k < len; k++) {
        int64_t e = orc_in_at(g, v, k);
        int32_t u = orc_other(g, e, v);
        if (u == v) continue;
        double du = dist[u];
        if (du < 0) continue;
        double alt = du + g->lat[e];
        if (!(alt > du) || alt != dist[v]) continue;
        if (best < 0 || du < bestd || (du == bestd && u < best)) {
            best = u;
            bestd = du;
        }
    }
    if (best < 0) return best;
    for (k = 0; k < len; k++) {   /* a second candidate with the same dist[u]? */
        int64_t e = orc_in_at(g, v, k);
        int32_t u = orc_other(g, e, v);
        if (u == v || u == best) continue;
        double du = dist[u];
        if (du != bestd) continue;
        double alt = du + g->lat[e];
        if (alt > du && alt == dist[v]) *tie = 1;
    }
    return best;
}

/* ----------------------------------------------------------- row rules */

static int has_attr(double x) { return isnan(x) == 0; }

/* _topology_lookupDirectPath, shd-topology.c:1862-1912 */
static uint8_t rule_direct(const orc_graph* g, int32_t s, int32_t t, double* lat, double* rel,
                           int32_t* next, int32_t* hops) {
    double totalLatency = 0.0, totalReliability = 1.0;
    if (has_attr(g->vloss[s])) totalReliability *= (1.0 - g->vloss[s]);
    if (has_attr(g->vloss[t])) totalReliability *= (1.0 - g->vloss[t]);
    int64_t e = orc_get_eid(g, s, t);
    if (e < 0) return ORC_FAIL;
    double edgeLatency = g->lat[e];
    double edgeReliability = 1.0 - g->loss[e];
    totalLatency += edgeLatency;
    totalReliability *= edgeReliability;
    *lat = totalLatency;
    *rel = totalReliability;
    *next = t;
    *hops = 1;
    return ORC_DIRECT;
}

/* _topology_computeShortestPathToSelf, shd-topology.c:1530-1638 */
static uint8_t rule_self(const orc_graph* g, int32_t s, double* lat, double* rel, int32_t* next,
                         int32_t* hops) {
    double minLatency = 0.0, reliabilityOfMinLatencyEdge = 0.0;
    int64_t idx = -1, k, len = orc_inc_len(g, s);
    for (k = 0; k < len; k++) {
        int64_t e = orc_inc_at(g, s, k);
        double edgeLatency = g->lat[e];
        if (minLatency == 0 || edgeLatency < minLatency) {
            minLatency = edgeLatency;
            reliabilityOfMinLatencyEdge = 1.0 - g->loss[e];
            idx = e;
        }
    }
    if (idx < 0) return ORC_FAIL;
    *lat = 2.0 * minLatency;
    *rel = reliabilityOfMinLatencyEdge * reliabilityOfMinLatencyEdge;
    *next = (g->from[idx] == s) ? g->to[idx] : g->from[idx];
    *hops = 2;
    return ORC_SELF;
}

/* _topology_computePathProperties, shd-topology.c:1392-1508, plus the
 * lat==0 -> 1 substitution of :1833-1837.  path[0..np) as igraph returns it. */
static uint8_t rule_path(const orc_graph* g, int32_t s, const int32_t* path, int64_t np, double* lat,
                         double* rel, int32_t* next, int32_t* hops) {
    double totalLatency = 0.0, totalReliability = 1.0;
    if (np <= 0) return ORC_FAIL;
    if (has_attr(g->vloss[s])) totalReliability *= (1.0 - g->vloss[s]);
    int32_t tgt = path[np - 1];
    if ((s != tgt) || (s == tgt && np > 2)) {
        if (has_attr(g->vloss[tgt])) totalReliability *= (1.0 - g->vloss[tgt]);
    }
    int64_t start = np == 1 ? 0 : 1, i;
    int32_t from = s;
    for (i = start; i < np; i++) {
        int32_t to = path[i];
        int64_t e = orc_get_eid(g, from, to);
        if (e < 0) return ORC_FAIL;
        double edgeLatency = g->lat[e];
        double edgeReliability = 1.0 - g->loss[e];
        totalLatency += edgeLatency;
        totalReliability *= edgeReliability;
        from = to;
    }
    if (totalLatency == 0) totalLatency = 1;
    *lat = totalLatency;
    *rel = totalReliability;
    *next = np == 1 ? s : path[1];
    *hops = np == 1 ? 1 : (int32_t)(np - 1);
    return ORC_SSSP;
}

typedef struct {
    orc_ws ws;
    double* dist;
    int64_t* peid;
    int32_t* cpar;
    int32_t* path;
} orc_rowws;

static void rowws_init(orc_rowws* r, int32_t n) {
    ws_init(&r->ws, n);
    r->dist = (double*)malloc(((size_t)n + 1) * sizeof(double));
    r->peid = (int64_t*)malloc(((size_t)n + 1) * sizeof(int64_t));
    r->cpar = (int32_t*)malloc(((size_t)n + 1) * sizeof(int32_t));
    r->path = (int32_t*)malloc(((size_t)n + 1) * sizeof(int32_t));
}
static void rowws_free(orc_rowws* r) {
    ws_free(&r->ws);
    free(r->dist); free(r->peid); free(r->cpar); free(r->path);
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* Reconstruct the vertex path src -> t (igraph order: path[0] = src unless the
 * path is the single vertex t). tie_mode 0 follows igraph parent edges, 1 the
 * canonical parent vertices. Returns the length. */
static int64_t build_path(const orc_graph* g, const orc_rowws* r, int32_t tie_mode, int32_t t) {
    int64_t size = 0;
    int32_t act = t;
    if (tie_mode == 0) {
        while (r->peid[act] >= 0) {
            size++;
            act = orc_other(g, r->peid[act], act);
        }
    } else {
        while (r->cpar[act] >= 0) {
            size++;
            act = r->cpar[act];
        }
    }
    r->path[size] = t;
    act = t;
    int64_t k = size;
    while (k > 0) {
        act = tie_mode == 0 ? orc_other(g, r->peid[act], act) : r->cpar[act];
        k--;
        r->path[k] = act;
    }
    return size + 1;
}

static void row_one(const orc_graph* g, const orc_opts* opts, orc_rowws* r, int32_t s,
                    const int32_t* targets, int32_t A, double* lat, double* rel, int32_t* next,
                    int32_t* hops, uint8_t* kind, int32_t* prev, int64_t* ties, double* dj_seconds) {
    int32_t j, v;
    int need_sssp = 0;
    int tie_mode = opts ? opts->tie_mode : 0;
    int self_mode = opts ? opts->self_mode : 0;
    int force = opts ? opts->force_sssp : 0;
    int complete = g->complete && !force, prefer = g->prefer_direct && !force;
    for (j = 0; j < A && !need_sssp; j++) {
        int32_t t = targets[j];
        if (complete || (prefer && orc_get_eid(g, s, t) >= 0)) continue;
        if (t == s) continue;
        need_sssp = 1;
    }
    if (need_sssp) {
        double t0 = now_s();
        /* early exit only when nothing needs the full tree (results are identical) */
        dijkstra_ws(g, &r->ws, s, targets, A, tie_mode == 0 && !ties, r->dist, r->peid, NULL);
        if (dj_seconds) *dj_seconds += now_s() - t0;
        if (tie_mode == 1 || ties) {
            for (v = 0; v < g->n; v++) {
                int tie = 0;
                if (v == s || r->dist[v] < 0) {
                    r->cpar[v] = -1;
                    continue;
                }
                r->cpar[v] = canonical_parent(g, r->dist, v, &tie);
                if (ties && tie) (*ties)++;
            }
        }
    }
    for (j = 0; j < A; j++) {
        int32_t t = targets[j];
        uint8_t k;
        double L = -1.0, R = -1.0;
        int32_t N = -1, H = 0, PV = s;   /* PV: vertex before the target on the path */
        if (complete || (prefer && orc_get_eid(g, s, t) >= 0)) {
            k = rule_direct(g, s, t, &L, &R, &N, &H);
        } else if (t == s) {
            if (self_mode == 0 && orc_get_eid(g, s, s) >= 0) {
                r->path[0] = s;
                k = rule_path(g, s, r->path, 1, &L, &R, &N, &H);
            } else {
                k = rule_self(g, s, &L, &R, &N, &H);
                PV = N;
            }
        } else if (r->dist[t] < 0) {
            k = ORC_FAIL;
        } else {
            int64_t np = build_path(g, r, tie_mode, t);
            k = rule_path(g, s, r->path, np, &L, &R, &N, &H);
            if (np >= 2) PV = r->path[np - 2];
        }
        if (k == ORC_FAIL) {
            L = -1.0; R = -1.0; N = -1; H = 0; PV = -1;
        }
        if (prev) prev[j] = PV;
        lat[j] = L;
        rel[j] = R;
        next[j] = N;
        hops[j] = H;
        kind[j] = k;
    }
}

int32_t orc_rows2(const orc_graph* g, const orc_opts* opts, const int32_t* sources, int32_t nsrc,
                  const int32_t* targets, int32_t A, double* lat, double* rel, int32_t* next,
                  int32_t* hops, uint8_t* kind, int32_t* prev, int64_t* double_ties,
                  double* dijkstra_seconds, int32_t nthreads) {
    int64_t ties = 0;
    double djs = 0.0;
    int32_t i;
    if (nthreads <= 1) {
        orc_rowws r;
        rowws_init(&r, g->n);
        for (i = 0; i < nsrc; i++) {
            size_t off = (size_t)i * (size_t)A;
            row_one(g, opts, &r, sources[i], targets, A, lat + off, rel + off, next + off, hops + off,
                    kind + off, prev ? prev + off : NULL, double_ties ? &ties : NULL,
                    dijkstra_seconds ? &djs : NULL);
        }
        rowws_free(&r);
    } else {
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads) reduction(+ : ties, djs)
        {
            orc_rowws r;
            rowws_init(&r, g->n);
#pragma omp for schedule(dynamic, 1)
            for (i = 0; i < nsrc; i++) {
                size_t off = (size_t)i * (size_t)A;
                row_one(g, opts, &r, sources[i], targets, A, lat + off, rel + off, next + off,
                        hops + off, kind + off, prev ? prev + off : NULL, double_ties ? &ties : NULL,
                        dijkstra_seconds ? &djs : NULL);
            }
            rowws_free(&r);
        }
#else
        return -2;
#endif
    }
    if (double_ties) *double_ties += ties;
    if (dijkstra_seconds) *dijkstra_seconds += djs;
    return 0;
}

int32_t orc_rows(const orc_graph* g, const orc_opts* opts, const int32_t* sources, int32_t nsrc,
                 const int32_t* targets, int32_t A, double* lat, double* rel, int32_t* next,
                 int32_t* hops, uint8_t* kind, int64_t* double_ties, double* dijkstra_seconds,
                 int32_t nthreads) {
    return orc_rows2(g, opts, sources, nsrc, targets, A, lat, rel, next, hops, kind, NULL, double_ties,
                     dijkstra_seconds, nthreads);
}

/* ---------------------------------------------------------------------------
 * CPU restatement of the per-packet path lookup, for the C5 CPU baseline:
 * topology_getLatency / getReliability / isRoutable -> _topology_getPathEntry
 * (shd-topology.c:1952-2075): the source and destination IPs resolve to
 * vertices through a hash table (top->virtualIP, :1958-1961), then the
 * two-level path cache src -> (dst -> Path*) is probed (:1975-1990).  Here:
 * open-addressing hash tables (linear probing) in place of GHashTable, holding
 * the pairs of the measured sample.  Test / baseline infrastructure only. */
typedef struct { uint64_t* key; int32_t* val; uint64_t mask; } orc_hmap;

static uint64_t orc_mix(uint64_t x) {   /* splitmix64 finaliser */
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull; return x ^ (x >> 31);
}
static int orc_hmap_init(orc_hmap* h, int64_t n) {
    uint64_t cap = 16;
    while (cap < (uint64_t)n * 2) cap <<= 1;
    h->key = malloc(cap * sizeof(uint64_t));
    h->val = malloc(cap * sizeof(int32_t));
    if (!h->key || !h->val) return -1;
    memset(h->key, 0xff, cap * sizeof(uint64_t));   /* empty = all ones */
    h->mask = cap - 1;
    return 0;
}
static void orc_hmap_put(orc_hmap* h, uint64_t k, int32_t v) {
    uint64_t i = orc_mix(k) & h->mask;
    while (h->key[i] != ~0ull && h->key[i] != k) i = (i + 1) & h->mask;
    h->key[i] = k;
    h->val[i] = v;
}
static int32_t orc_hmap_get(const orc_hmap* h, uint64_t k) {
    uint64_t i = orc_mix(k) & h->mask;
    for (;;) {
        if (h->key[i] == k) return h->val[i];
        if (h->key[i] == ~0ull) return -1;
        i = (i + 1) & h->mask;
    }
}

struct orc_cache {
    orc_hmap ip, src, pair;   /* ip -> slot; src slot -> cache id; (cache id, dst slot) -> path */
    double* lat;
    double* rel;
};

orc_cache* orc_cache_new(int32_t A, const uint32_t* ips, int64_t npairs, const int32_t* pairs, const double* lat,
                         const double* rel) {
    orc_cache* c = calloc(1, sizeof(*c));
    if (!c || orc_hmap_init(&c->ip, A) || orc_hmap_init(&c->src, A) || orc_hmap_init(&c->pair, npairs)) return NULL;
    c->lat = malloc(sizeof(double) * (size_t)(npairs > 0 ? npairs : 1));
    c->rel = malloc(sizeof(double) * (size_t)(npairs > 0 ? npairs : 1));
    for (int32_t s = 0; s < A; ++s) orc_hmap_put(&c->ip, ips[s], s);
    int32_t nsrc = 0;
    for (int64_t i = 0; i < npairs; ++i) {
        const int32_t s = pairs[2 * i], t = pairs[2 * i + 1];
        int32_t id = orc_hmap_get(&c->src, (uint64_t)s);
        if (id < 0) orc_hmap_put(&c->src, (uint64_t)s, id = nsrc++);
        orc_hmap_put(&c->pair, ((uint64_t)id << 32) | (uint32_t)t, (int32_t)i);
        c->lat[i] = lat[i];
        c->rel[i] = rel[i];
    }
    return c;
}

void orc_cache_free(orc_cache* c) {
    if (!c) return;
    free(c->ip.key); free(c->ip.val); free(c->src.key); free(c->src.val); free(c->pair.key); free(c->pair.val);
    free(c->lat); free(c->rel); free(c);
}

/* q queries (src ip, dst ip) -> latency, reliability, routable; returns hits. */
int64_t orc_cache_lookup(const orc_cache* c, const uint32_t* sip, const uint32_t* dip, int64_t q, double* lat,
                         double* rel, uint8_t* ok, int32_t nthreads) {
    int64_t hits = 0;
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : hits) schedule(static)
    for (int64_t i = 0; i < q; ++i) {
        double L = -1.0, R = -1.0;
        const int32_t s = orc_hmap_get(&c->ip, sip[i]), t = orc_hmap_get(&c->ip, dip[i]);
        if (s >= 0 && t >= 0) {
            const int32_t id = orc_hmap_get(&c->src, (uint64_t)s);
            const int32_t p = id >= 0 ? orc_hmap_get(&c->pair, ((uint64_t)id << 32) | (uint32_t)t) : -1;
            if (p >= 0) {
                L = c->lat[p];
                R = c->rel[p];
                hits++;
            }
        }
        lat[i] = L;
        rel[i] = R;
        ok[i] = L > -1.0;
    }
    return hits;
}
