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

typedef uint32_t spe_in_addr_t;          /* network byte order, like in_addr_t */
typedef struct _Topology Topology;

typedef double (*topology_random_fn)(void* ctx);                 /* in [0,1] */
typedef void (*topology_min_latency_fn)(double min_latency_ms, void* ctx);
/* level: 0 error, 1 critical, 2 warning, 3 message, 4 info, 5 debug (shd-options.c:89) */
typedef void (*topology_log_fn)(int level, const char* text, void* ctx);

/* GraphML file -> validated topology on `device`; NULL on any validation
 * failure (shd-topology.c:2485-2490).  The file is read synchronously. */
Topology* topology_new(const char* graphPath);
Topology* topology_new_on_device(const char* graphPath, int32_t device);
void topology_free(Topology* top);

/* Hint-matched attachment (shd-topology.c:2077-2413).  Hints may be NULL. */
void topology_attach(Topology* top, spe_in_addr_t address, topology_random_fn random, void* random_ctx,
                     const char* ipHint, const char* citycodeHint, const char* countrycodeHint,
                     const char* geocodeHint, const char* typeHint, uint64_t* bwDownOut, uint64_t* bwUpOut);
void topology_detach(Topology* top, spe_in_addr_t address);

int32_t topology_isRoutable(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
double topology_getLatency(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
double topology_getReliability(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
void topology_incrementPathPacketCounter(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
/* worker_sendPacket's three per-packet calls (isRoutable, getReliability,
 * getLatency, shd-worker.c:235-247) answered by one slot resolution and one
 * table read: returns routable; *latency / *reliability as the two getters
 * (-1.0 when unroutable).  Either output pointer may be NULL. */
int32_t topology_getPathInfo(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress, double* latency,
                             double* reliability);

/* engine hooks */
void topology_set_log_callback(Topology* top, topology_log_fn fn, void* ctx);
void topology_set_min_latency_callback(Topology* top, topology_min_latency_fn fn, void* ctx);
/* Build the path table now (otherwise done once, on the first query). */
int32_t topology_seal(Topology* top);
/* introspection used by tests */
int32_t topology_vertex_count(const Topology* top);
int32_t topology_attached_vertex(const Topology* top, spe_in_addr_t address);   /* -1 if unknown */
uint64_t topology_path_packet_count(Topology* top, spe_in_addr_t srcAddress, spe_in_addr_t dstAddress);
double topology_min_path_latency(Topology* top);

#ifdef __cplusplus
}
#endif
#endif /* SHD_TOPOLOGY_SPE_H_ */
