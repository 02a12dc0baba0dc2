/* Round-6 diagnostic (not product code): spe_table_get_latrel from `threads` pthreads
 * at once on a built table, uniform random (s, t); returns calls per second in all.
 * build: gcc -O2 -shared -fPIC -o build_ab/libmtreads.so tools/mt_reads.c -I include -L shadow_amd -lspe -lpthread */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

#include "spe.h"

typedef struct {
    const spe_table* t;
    int32_t A;
    int64_t per;
    unsigned seed;
    double sum;
} Job;

static void* run(void* p) {
    Job* j = (Job*)p;
    for (int64_t i = 0; i < j->per; ++i) {
        const int32_t s = (int32_t)(rand_r(&j->seed) % (unsigned)j->A), u = (int32_t)(rand_r(&j->seed) % (unsigned)j->A);
        double lat = 0.0, rel = 0.0;
        if (spe_table_get_latrel(j->t, s, u, &lat, &rel) == SPE_OK) j->sum += lat;
    }
    return NULL;
}

double mt_reads(const spe_table* t, int32_t A, int32_t threads, int64_t per) {
    pthread_t th[256];
    Job jb[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int k = 0; k < threads && k < 256; ++k) {
        jb[k] = (Job){t, A, per, 17u + 7919u * (unsigned)k, 0.0};
        pthread_create(&th[k], NULL, run, &jb[k]);
    }
    for (int k = 0; k < threads && k < 256; ++k) pthread_join(th[k], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    const double el = (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
    return (double)threads * (double)per / el;
}

/* touch one double every `stride` bytes of [p, p + bytes) from `threads` threads; seconds */
typedef struct {
    const volatile double* p;
    size_t n, stride_d;
    double acc;
} Touch;

static void* touch(void* a) {
    Touch* t = (Touch*)a;
    double acc = 0.0;
    for (size_t i = 0; i < t->n; ++i) acc += t->p[i * t->stride_d];
    t->acc = acc;
    return NULL;
}

double prefault(const void* p, size_t bytes, size_t stride, int32_t threads) {
    pthread_t th[256];
    Touch tj[256];
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    const size_t total = bytes / stride, sd = stride / sizeof(double);
    for (int k = 0; k < threads && k < 256; ++k) {
        const size_t i0 = total * (size_t)k / (size_t)threads, i1 = total * (size_t)(k + 1) / (size_t)threads;
        tj[k] = (Touch){(const volatile double*)p + i0 * sd, i1 - i0, sd, 0.0};
        pthread_create(&th[k], NULL, touch, &tj[k]);
    }
    for (int k = 0; k < threads && k < 256; ++k) pthread_join(th[k], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
