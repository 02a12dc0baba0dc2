/* Per-packet single calls through the drop-in, timed in C (no Python in the loop):
 * what Shadow's workers pay per topology_getPathInfo (shd-worker.c:235-247 asks
 * isRoutable / getReliability / getLatency for every packet).
 *
 *   shd_topology_single_calls <graph.graphml> <hints.txt> <calls> [threads] [seed] [settle_s]
 *
 * hints.txt: one IP hint per line; host i (address 11.x.y.z = i) attaches by the
 * exact-IP hint of line i (shd-topology.c:2354-2413), as bench.py's shim lines do.
 * After topology_seal, `threads` workers each make calls/threads calls on seeded
 * uniform (src, dst) host pairs.  Prints one JSON line: calls per second for one
 * worker alone, then for all workers at once.  settle_s > 0: both again after that many
 * more seconds, when the library's background pre-fault of the table's host mapping
 * (spe_table_layout.host_prefault) has had time to finish: the rates a long simulation
 * runs at. */
#include <arpa/inet.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "shd_topology_spe.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static double next_double(void* ctx) { return (double)rand_r((unsigned*)ctx) / (double)RAND_MAX; }

static spe_in_addr_t host_addr(int32_t i) { return htonl((11u << 24) | (uint32_t)i); }

typedef struct {
    Topology* top;
    int32_t hosts;
    int64_t calls;
    unsigned seed;
    int64_t routable;
    double latency_sum;
} Worker;

static void* run(void* arg) {
    Worker* w = (Worker*)arg;
    for (int64_t p = 0; p < w->calls; ++p) {
        const spe_in_addr_t s = host_addr(rand_r(&w->seed) % w->hosts);
        const spe_in_addr_t d = host_addr(rand_r(&w->seed) % w->hosts);
        double lat = 0.0, rel = 0.0;
        if (topology_getPathInfo(w->top, s, d, &lat, &rel)) {
            ++w->routable;
            w->latency_sum += lat;
        }
    }
    return NULL;
}

static double timed(Topology* top, int32_t hosts, int64_t calls, int32_t threads, unsigned seed, int64_t* routable) {
    Worker* ws = (Worker*)calloc((size_t)threads, sizeof(Worker));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    const double t0 = now_s();
    for (int32_t k = 0; k < threads; ++k) {
        ws[k] = (Worker){top, hosts, calls / threads, seed + 7919u * (unsigned)(k + 1), 0, 0.0};
        pthread_create(&th[k], NULL, run, &ws[k]);
    }
    *routable = 0;
    for (int32_t k = 0; k < threads; ++k) {
        pthread_join(th[k], NULL);
        *routable += ws[k].routable;
    }
    const double el = now_s() - t0;
    free(th);
    free(ws);
    return (double)(calls / threads * threads) / el;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <graph.graphml> <hints.txt> <calls> [threads] [seed] [settle_s]\n", argv[0]);
        return 2;
    }
    const int64_t calls = atoll(argv[3]);
    const int32_t threads = argc > 4 ? atoi(argv[4]) : 16;
    const unsigned seed = argc > 5 ? (unsigned)atoi(argv[5]) : 5u;
    const double settle = argc > 6 ? atof(argv[6]) : 0.0;
    FILE* f = fopen(argv[2], "r");
    if (!f || calls < 1 || threads < 1) return 2;
    int32_t cap = 1024, hosts = 0;
    char** hint = (char**)malloc((size_t)cap * sizeof(char*));
    char line[64];
    while (fgets(line, sizeof line, f)) {
        line[strcspn(line, "\r\n")] = 0;
        if (hosts == cap) hint = (char**)realloc(hint, (size_t)(cap *= 2) * sizeof(char*));
        hint[hosts++] = strdup(line);
    }
    fclose(f);
    const double t0 = now_s();
    Topology* top = topology_new(argv[1]);
    if (!top) return 2;
    const double t1 = now_s();
    unsigned rs = seed;
    for (int32_t i = 0; i < hosts; ++i) {
        uint64_t bw_down = 0, bw_up = 0;
        topology_attach(top, host_addr(i), next_double, &rs, hint[i], NULL, NULL, NULL, NULL, &bw_down, &bw_up);
    }
    const double t2 = now_s();
    if (topology_seal(top) != 0) return 2;
    const double t3 = now_s();
    int64_t r1 = 0, rn = 0;
    timed(top, hosts, calls / 4 + 1, 1, seed + 1, &r1);   /* warm: code, the path-cache model's first stores */
    const double one = timed(top, hosts, calls, 1, seed, &r1);
    const double all = timed(top, hosts, calls, threads, seed + 99, &rn);
    double one_s = 0.0, all_s = 0.0;
    int64_t r1s = calls, rns = calls / threads * threads;
    if (settle > 0.0) {
        const double until = now_s() + settle;
        while (now_s() < until) usleep(10000);
        one_s = timed(top, hosts, calls, 1, seed + 3, &r1s);
        all_s = timed(top, hosts, calls, threads, seed + 199, &rns);
    }
    printf("{\"hosts\": %d, \"load_s\": %.3f, \"attach_s\": %.3f, \"seal_s\": %.3f, \"calls\": %lld, "
           "\"single_calls_per_s_1_thread\": %.1f, \"threads\": %d, \"single_calls_per_s_all_threads\": %.1f, "
           "\"settle_s\": %.1f, \"settled_calls_per_s_1_thread\": %.1f, \"settled_calls_per_s_all_threads\": %.1f, "
           "\"routable\": %lld}\n",
           hosts, t1 - t0, t2 - t1, t3 - t2, (long long)calls, one, threads, all, settle, one_s, all_s,
           (long long)(r1 + rn));
    topology_free(top);
    for (int32_t i = 0; i < hosts; ++i) free(hint[i]);
    free(hint);
    return (r1 == calls && rn == calls / threads * threads && r1s == calls && rns == calls / threads * threads) ? 0 : 1;
}
