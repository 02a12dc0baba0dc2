/* A Shadow-worker-shaped user of the drop-in topology API
 * (include/shd_topology_spe.h, which re-hosts src/main/routing/shd-topology.h).
 *
 * What Shadow does with a topology, in order:
 *   master:  topology_new(graphml)                       shd-master.c:209
 *   hosts:   topology_attach(addr, random, hints...)     shd-host.c:140
 *   workers: per packet isRoutable / getReliability / getLatency
 *            (shd-worker.c:235-247) + incrementPathPacketCounter,
 *            concurrently from --workers pthreads
 *   master:  topology_free                               shd-master.c:100
 * Here the three per-packet calls are topology_getPathInfo (one table read);
 * every 64th packet is re-asked through the three separate getters, which must
 * agree bit for bit.  With batch > 0 a worker instead collects rounds of `batch`
 * packets and answers each round with one topology_getPathInfoBatch call (and
 * counts the routable ones with one topology_incrementPathPacketCounterBatch),
 * every 64th packet of a round re-asked through topology_getPathInfo.  With late_hosts > 0 the main thread attaches that many
 * more hosts AFTER the table is sealed while the workers are querying (a
 * replacement table is built and swapped in under them), and the workers also
 * address the late hosts once attached.  At the end the packet counters of
 * every cached path must add up to the number of counted packets exactly.
 *
 *   shd_topology_demo <graph.graphml> <hosts> <packets> [threads] [seed] [late_hosts] [batch]
 * prints one JSON line; exit 0 ok, 1 disagreement, 2 setup failure. */
#include <arpa/inet.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "shd_topology_spe.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* host attachment draws, like Shadow's per-host Random (rand_r based) */
static double next_double(void* ctx) { return (double)rand_r((unsigned*)ctx) / (double)RAND_MAX; }

static spe_in_addr_t host_addr(int32_t i) { return htonl((11u << 24) | (uint32_t)(i + 1)); }

typedef struct {
    Topology* top;
    int32_t hosts;         /* hosts addressed: the first ones plus the late ones */
    int64_t packets;
    int64_t batch;         /* packets per round through the batch calls (0: per packet) */
    unsigned seed;
    int64_t routable, mismatches, skipped;
    double latency_sum;
} Worker;

static void worker_batches(Worker* w) {
    spe_in_addr_t* src = (spe_in_addr_t*)malloc((size_t)w->batch * sizeof(spe_in_addr_t));
    spe_in_addr_t* dst = (spe_in_addr_t*)malloc((size_t)w->batch * sizeof(spe_in_addr_t));
    spe_in_addr_t* csrc = (spe_in_addr_t*)malloc((size_t)w->batch * sizeof(spe_in_addr_t));
    spe_in_addr_t* cdst = (spe_in_addr_t*)malloc((size_t)w->batch * sizeof(spe_in_addr_t));
    double* lat = (double*)malloc((size_t)w->batch * sizeof(double));
    double* rel = (double*)malloc((size_t)w->batch * sizeof(double));
    uint8_t* ok = (uint8_t*)malloc((size_t)w->batch);
    for (int64_t p0 = 0; p0 < w->packets; p0 += w->batch) {
        int64_t n = 0;
        for (int64_t p = p0; p < p0 + w->batch && p < w->packets; ++p) {
            const spe_in_addr_t s = host_addr(rand_r(&w->seed) % w->hosts);
            const spe_in_addr_t d = host_addr(rand_r(&w->seed) % w->hosts);
            if (topology_attached_vertex(w->top, s) < 0 || topology_attached_vertex(w->top, d) < 0) {
                ++w->skipped;
                continue;
            }
            src[n] = s;
            dst[n] = d;
            ++n;
        }
        topology_getPathInfoBatch(w->top, n, src, dst, lat, rel, ok);
        int64_t nc = 0;
        for (int64_t i = 0; i < n; ++i) {
            if (ok[i]) {
                ++w->routable;
                w->latency_sum += lat[i];
                csrc[nc] = src[i];
                cdst[nc] = dst[i];
                ++nc;
            }
            if ((i & 63) == 0) {
                double l1 = 0.0, r1 = 0.0;
                const int32_t ok1 = topology_getPathInfo(w->top, src[i], dst[i], &l1, &r1);
                if (ok1 != (ok[i] != 0) || (ok1 && (l1 != lat[i] || r1 != rel[i]))) ++w->mismatches;
            }
        }
        topology_incrementPathPacketCounterBatch(w->top, nc, csrc, cdst);
    }
    free(src); free(dst); free(csrc); free(cdst); free(lat); free(rel); free(ok);
}

static void* worker_run(void* arg) {
    Worker* w = (Worker*)arg;
    if (w->batch > 0) {
        worker_batches(w);
        return NULL;
    }
    for (int64_t p = 0; p < w->packets; ++p) {
        const spe_in_addr_t s = host_addr(rand_r(&w->seed) % w->hosts);
        const spe_in_addr_t d = host_addr(rand_r(&w->seed) % w->hosts);
        if (topology_attached_vertex(w->top, s) < 0 || topology_attached_vertex(w->top, d) < 0) {
            ++w->skipped;   /* a late host not attached yet */
            continue;
        }
        double lat = 0.0, rel = 0.0;
        const int32_t ok = topology_getPathInfo(w->top, s, d, &lat, &rel);
        if (ok) {
            ++w->routable;
            w->latency_sum += lat;
            topology_incrementPathPacketCounter(w->top, s, d);
        }
        if ((p & 63) == 0) {   /* worker_sendPacket's original three calls */
            const int32_t ok3 = topology_isRoutable(w->top, s, d);
            const double rel3 = topology_getReliability(w->top, s, d);
            const double lat3 = topology_getLatency(w->top, s, d);
            if (ok3 != ok || rel3 != rel || lat3 != lat) ++w->mismatches;
        }
    }
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <graph.graphml> <hosts> <packets> [threads] [seed] [late_hosts] [batch]\n",
                argv[0]);
        return 2;
    }
    const int32_t hosts = atoi(argv[2]);
    const int64_t packets = atoll(argv[3]);
    const int32_t threads = argc > 4 ? atoi(argv[4]) : 4;
    unsigned seed = argc > 5 ? (unsigned)atoi(argv[5]) : 1u;
    const int32_t late = argc > 6 ? atoi(argv[6]) : 0;
    const int64_t batch = argc > 7 ? atoll(argv[7]) : 0;
    if (hosts < 1 || packets < 0 || threads < 1 || late < 0 || batch < 0) return 2;

    const double t0 = now_s();
    Topology* top = topology_new(argv[1]);
    if (!top) {
        fprintf(stderr, "topology_new failed for %s\n", argv[1]);
        return 2;
    }
    const double t1 = now_s();
    for (int32_t i = 0; i < hosts; ++i) {
        uint64_t bw_down = 0, bw_up = 0;
        topology_attach(top, host_addr(i), next_double, &seed, NULL, NULL, NULL, NULL, NULL, &bw_down, &bw_up);
    }
    int32_t distinct = 0;
    {   /* attached vertices (a host maps to one vertex; several hosts may share it) */
        const int32_t n = topology_vertex_count(top);
        uint8_t* seen = (uint8_t*)calloc((size_t)n, 1);
        for (int32_t i = 0; i < hosts; ++i) {
            const int32_t v = topology_attached_vertex(top, host_addr(i));
            if (v >= 0 && v < n && !seen[v]) {
                seen[v] = 1;
                ++distinct;
            }
        }
        free(seen);
    }
    const double t2 = now_s();
    if (topology_seal(top) != 0) {
        fprintf(stderr, "topology_seal failed\n");
        topology_free(top);
        return 2;
    }
    const double t3 = now_s();

    Worker* ws = (Worker*)calloc((size_t)threads, sizeof(Worker));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int32_t k = 0; k < threads; ++k) {
        ws[k].top = top;
        ws[k].hosts = hosts + late;
        ws[k].packets = packets / threads + (k < packets % threads ? 1 : 0);
        ws[k].batch = batch;
        ws[k].seed = seed + 7919u * (unsigned)(k + 1);
        pthread_create(&th[k], NULL, worker_run, &ws[k]);
    }
    for (int32_t i = 0; i < late; ++i) {   /* attach after seal, under concurrent readers */
        uint64_t bw_down = 0, bw_up = 0;
        topology_attach(top, host_addr(hosts + i), next_double, &seed, NULL, NULL, NULL, NULL, NULL, &bw_down,
                        &bw_up);
    }
    int64_t routable = 0, mismatches = 0, skipped = 0;
    double latency_sum = 0.0;
    for (int32_t k = 0; k < threads; ++k) {
        pthread_join(th[k], NULL);
        routable += ws[k].routable;
        mismatches += ws[k].mismatches;
        skipped += ws[k].skipped;
        latency_sum += ws[k].latency_sum;
    }
    const double t4 = now_s();
    /* every counted packet sits on exactly one cached path: one per unordered
     * vertex pair (undirected graphs), asked through one representative host each */
    const int32_t nh = hosts + late, nv = topology_vertex_count(top);
    int32_t* rep = (int32_t*)malloc((size_t)nv * sizeof(int32_t));
    for (int32_t v = 0; v < nv; ++v) rep[v] = -1;
    for (int32_t i = 0; i < nh; ++i) {
        const int32_t v = topology_attached_vertex(top, host_addr(i));
        if (v >= 0 && rep[v] < 0) rep[v] = i;
    }
    uint64_t counted = 0;
    for (int32_t a = 0; a < nv; ++a)
        for (int32_t b = a; b < nv && rep[a] >= 0; ++b)
            if (rep[b] >= 0) counted += topology_path_packet_count(top, host_addr(rep[a]), host_addr(rep[b]));
    free(rep);
    /* the counters are per (src, dst) pair and atomic: re-count one pair */
    const uint64_t c00 = topology_path_packet_count(top, host_addr(0), host_addr(0));
    const double min_lat = topology_min_path_latency(top);
    printf("{\"graph\": \"%s\", \"vertices\": %d, \"hosts\": %d, \"attached_vertices\": %d, "
           "\"load_s\": %.4f, \"attach_s\": %.4f, \"seal_s\": %.4f, \"packets\": %lld, \"threads\": %d, "
           "\"packets_per_s\": %.1f, \"routable\": %lld, \"latency_sum\": %.6f, \"min_path_latency\": %.6f, "
           "\"count_pair_0_0\": %llu, \"late_hosts\": %d, \"skipped\": %lld, \"counted\": %llu, "
           "\"mismatches\": %lld, \"batch\": %lld}\n",
           argv[1], topology_vertex_count(top), hosts, distinct, t1 - t0, t2 - t1, t3 - t2, (long long)packets,
           threads, packets > 0 ? (double)packets / (t4 - t3) : 0.0, (long long)routable, latency_sum, min_lat,
           (unsigned long long)c00, late, (long long)skipped, (unsigned long long)counted, (long long)mismatches,
           (long long)batch);
    free(th);
    free(ws);
    topology_free(top);
    return (mismatches == 0 && counted == (uint64_t)routable) ? 0 : 1;
}
