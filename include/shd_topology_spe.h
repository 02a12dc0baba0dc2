/*
 * shd_topology_spe.h -- drop-in for src/main/routing/shd-topology.h:12-25 of the
 * reference, implemented over the gfx950 path engine (spe.h) instead of igraph
 * + the per-pair GHashTable path cache.
 *
 * The reference signatures take glib / Shadow types (gchar*, Address*,
 * Random*).  This header keeps every entry point, argument meaning and error
 * convention but with plain C types, so it builds without glib (absent here):
 *   Address* -> in_addr_t (address_toNetworkIP(address), the key the reference
 *               hashes on, shd-topology.c:1378)
 *   Random*  -> a next-double callback (random_nextDouble, shd-random.c:37-41)
 * A Shadow tree maps its types onto these in a 20-line adapter.
 *
 * Reference entry point                         -> here
 *   topology_new              shd-topology.c:2469   topology_new
 *   topology_free             shd-topology.c:2424   topology_free
 *   topology_attach           shd-topology.c:2354   topology_attach
 *   topology_detach           shd-topology.c:2415   topology_detach
 *   topology_isRoutable       shd-topology.c:2072   topology_isRoutable
 *   topology_getLatency       shd-topology.c:2048   topology_getLatency
 *   topology_getReliability   shd-topology.c:2060   topology_getReliability
 *   topology_incrementPathPacketCounter :2036       topology_incrementPathPacketCounter
 * plus engine hooks the reference had inline:
 *   worker_updateMinTimeJump (shd-topology.c:1369) -> topology_set_min_latency_callback
 *   logging (message/info/critical)                -> topology_set_log_callback
 */
#ifndef SHD_TOPOLOGY_SPE_H_
#define SHD_TOPOLOGY_SPE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Inside a Shadow tree the reference's own shd-topology.h declares the
 * topology_* names with Shadow's types; build this library (and include this
 * header in the adapter) with -DSHD_TOPOLOGY_SPE_PREFIXED and every entry point
 * below is spe_topology_* instead. */
#ifdef SHD_TOPOLOGY_SPE_PREFIXED
#define SHD_TOPO(name) spe_##name
#else
#define SHD_TOPO(name) name
#endif

typedef uint32_t spe_in_addr_t;          /* network byte order, like in_addr_t */
typedef struct _Topology Topology;

typedef double (*topology_random_fn)(void* ctx);                 /* in [0,1] */
typedef void (*topology_min_latency_fn)(double min_latency_ms, void* ctx);
/* level: 0 error, 1 critical, 2 warning, 3 message, 4 info, 5 debug (shd-options.c:89) */
typedef void (*topology_log_fn)(int level, const char* text, void* ctx);

/* GraphML file -> validated topology on `device`; NULL on any validation
 * failure (shd-topology.c:2485-2490).  The file is read synchronously.
 * topology_new builds on device SHADOW_SPE_DEVICE (default 0). */
Topology* SHD_TOPO(topology_new)(const char* graphPath);
Topology* SHD_TOPO(topology_new_on_device)(const char* graphPath, int32_t device);
/* The ingest and validation of topology_new alone (no device work): 1 when the
 * reference would accept the file, else 0. */
int32_t SHD_TOPO(topology_check_graphml)(const char* graphPath);
void SHD_TOPO(topology_free)(Topology* top);

/* Hint-matched attachment (shd-topology.c:2077-2413).  Hints may be NULL. */
void SHD_TOPO(topology_attach)(Topology* top, spe_in_addr_t address, topology_random_fn random, void* random_ctx,
                     const char* ipHint, const char* citycodeHint, const char* countrycodeHint,
                     const char* geocodeHint, const char* typeHint, uint64_t* bwDownOut, uint64_t* bwUpOut);
void SHD_TOPO(topology_detach)(Topology* top, spe_in_addr_t address);

int32_t SHD_TOPO(topology_isRoutable)(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
double SHD_TOPO(topology_getLatency)(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
double SHD_TOPO(topology_getReliability)(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
void SHD_TOPO(topology_incrementPathPacketCounter)(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
/* worker_sendPacket's three per-packet calls (isRoutable, getReliability,
 * getLatency, shd-worker.c:235-247) answered by one slot resolution and one
 * table read: returns routable; *latency / *reliability as the two getters
 * (-1.0 when unroutable).  Either output pointer may be NULL. */
int32_t SHD_TOPO(topology_getPathInfo)(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress, double* latency,
                             double* reliability);

/* A whole round of packets at once (no reference counterpart: Shadow's workers
 * ask per packet, shd-worker.c:235-247).  For i < n: routable[i], latency[i] and
 * reliability[i] exactly as topology_getPathInfo(src[i], dst[i]) would answer,
 * with the same path-cache bookkeeping per query, in order; the table reads of a
 * batch of n >= 256 (n >= 4096 when the whole table is mirrored on the host) go to
 * ONE device lookup launch (spe_lookup_batch_host), smaller ones to the host
 * mirror / single reads.  Returns the number of
 * routable pairs; -1 on bad arguments, or when no table covering the queried
 * hosts could be sealed (device or memory failure) -- then every output is
 * filled as unroutable (latency = reliability = -1, routable = 0). */
int64_t SHD_TOPO(topology_getPathInfoBatch)(Topology* top, int64_t n, const spe_in_addr_t* srcAddress,
                                  const spe_in_addr_t* dstAddress, double* latency, double* reliability,
                                  uint8_t* routable);
/* topology_incrementPathPacketCounter for n (src, dst) pairs (e.g. the delivered
 * packets of a round), each counted on the Path its query hits. */
void SHD_TOPO(topology_incrementPathPacketCounterBatch)(Topology* top, int64_t n, const spe_in_addr_t* srcAddress,
                                              const spe_in_addr_t* dstAddress);

/* engine hooks (callbacks run on the calling thread, some inside the topology's
 * locks: they must not call back into the topology) */
void SHD_TOPO(topology_set_log_callback)(Topology* top, topology_log_fn fn, void* ctx);
/* levels above `level` are not formatted (default 3, message; 4 enables the
 * per-path info lines of a source's first query and the cached-path dump at
 * topology_free, 5 the per-target debug lines) */
void SHD_TOPO(topology_set_log_level)(Topology* top, int32_t level);
void SHD_TOPO(topology_set_min_latency_callback)(Topology* top, topology_min_latency_fn fn, void* ctx);

/* What a query answers.  The reference lazily caches one Path per vertex pair,
 * first writer wins, and answers (s, t) with the cached (t, s) path when t's
 * Dijkstra ran first (shd-topology.c:1292-1321, 1952-2034), so its answers
 * depend on query order.  Both modes keep that cache's bookkeeping (which Path
 * each query hits, its packetCount, the dump at topology_free):
 *   TOPOLOGY_ANSWER_ROWS       (default) the source row of s: tree_s(s -> t),
 *                              independent of query order;
 *   TOPOLOGY_ANSWER_REFERENCE  the cached Path's values, exactly as the
 *                              reference would return them for this query
 *                              order (also: -1 for a query whose Dijkstra row
 *                              fails, quirk B5; minimumPathLatency over stored
 *                              Paths, reported to the callback as it changes).
 * The environment variable SHADOW_SPE_PATH_CACHE=reference selects the second
 * at topology_new. */
#define TOPOLOGY_ANSWER_ROWS 0
#define TOPOLOGY_ANSWER_REFERENCE 1
int32_t SHD_TOPO(topology_set_answer_mode)(Topology* top, int32_t mode);

/* Build the path table now (otherwise done on the first query).  Hosts may
 * attach after sealing: the published table keeps answering the pairs it holds
 * while the first query that needs a new vertex builds a replacement, which is
 * swapped in atomically (readers never see a freed or half-built table; packet
 * counts and cache state are per vertex pair and carry over). */
int32_t SHD_TOPO(topology_seal)(Topology* top);
/* introspection used by tests */
int32_t SHD_TOPO(topology_vertex_count)(const Topology* top);
int32_t SHD_TOPO(topology_attached_vertex)(const Topology* top, spe_in_addr_t address);   /* -1 if unknown */
/* packetCount of the cached Path the query (src, dst) hits (exact, every pair) */
uint64_t SHD_TOPO(topology_path_packet_count)(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
double SHD_TOPO(topology_min_path_latency)(Topology* top);
/* number of Paths the reference's cache would hold now (the lines the dump at
 * topology_free prints at log level 4) */
int64_t SHD_TOPO(topology_cached_path_count)(Topology* top);

#ifdef __cplusplus
}
#endif
#endif /* SHD_TOPOLOGY_SPE_H_ */
