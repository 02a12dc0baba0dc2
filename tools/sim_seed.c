/* sim_seed.c -- CPU model (design tool, not product code) of the multi-source
 * relaxation schedule when lanes start from upper-bound seeds instead of +inf.
 * Same synchronous pull model as sim_relax.c; a candidate only propagates when
 * it beats the lane's current value, so a tight seed prunes every non-final
 * update.  Seeds: a row per lane, given by the caller (INFINITY = no bound).
 *
 * build: gcc -O2 -shared -fPIC -o tools/_sim_seed.so tools/sim_seed.c
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t rounds, visits, lane_updates, nbr_rows;
    int64_t hist[65];        /* changed lanes per changing row visit */
    int64_t nbr_bytes_list;  /* neighbour reads priced as a 128-B change list when <= cap lanes changed, else 512 B */
    int64_t list_cap;
} sim_out;

/* plain binary-heap Dijkstra (distances only) */
int sim_dijkstra(int32_t n, const int32_t* ptr, const int32_t* col, const double* w, int32_t s, double* d) {
    int32_t* heap = malloc(sizeof(int32_t) * (size_t)n);
    int32_t* pos = malloc(sizeof(int32_t) * (size_t)n);
    int hn = 0;
    for (int i = 0; i < n; ++i) {
        d[i] = INFINITY;
        pos[i] = -1;
    }
    d[s] = 0.0;
    heap[hn] = s;
    pos[s] = hn++;
#define SWAP(a, b)                     \
    do {                               \
        int32_t t_ = heap[a];          \
        heap[a] = heap[b];             \
        heap[b] = t_;                  \
        pos[heap[a]] = a;              \
        pos[heap[b]] = b;              \
    } while (0)
    while (hn) {
        int32_t u = heap[0];
        pos[u] = -2;
        heap[0] = heap[--hn];
        if (hn) {
            pos[heap[0]] = 0;
            int i = 0;
            for (;;) {
                int l = 2 * i + 1, r = l + 1, b = i;
                if (l < hn && d[heap[l]] < d[heap[b]]) b = l;
                if (r < hn && d[heap[r]] < d[heap[b]]) b = r;
                if (b == i) break;
                SWAP(i, b);
                i = b;
            }
        }
        for (int k = ptr[u]; k < ptr[u + 1]; ++k) {
            int v = col[k];
            if (pos[v] == -2) continue;
            double a = d[u] + w[k];
            if (a < d[v]) {
                d[v] = a;
                int i = pos[v];
                if (i < 0) {
                    i = hn++;
                    heap[i] = v;
                    pos[v] = i;
                }
                while (i > 0 && d[heap[(i - 1) / 2]] > d[heap[i]]) {
                    SWAP(i, (i - 1) / 2);
                    i = (i - 1) / 2;
                }
            }
        }
    }
#undef SWAP
    free(heap);
    free(pos);
    return 0;
}

/* seed: L rows of n (row l = bounds for lane l), or NULL. */
int sim_seeded(int32_t n, const int32_t* ptr, const int32_t* col, const double* w, int32_t L, const int32_t* src,
               const double* seed, sim_out* out) {
    double* d = malloc(sizeof(double) * (size_t)n * 64);
    uint64_t* pend = calloc((size_t)n, 8);
    uint64_t* nxt = calloc((size_t)n, 8);
    const int64_t cap = out->list_cap;
    memset(out, 0, sizeof(*out));
    out->list_cap = cap;
    for (int v = 0; v < n; ++v)
        for (int l = 0; l < 64; ++l) d[(size_t)v * 64 + l] = (seed && l < L) ? seed[(size_t)l * n + v] : INFINITY;
    for (int l = 0; l < L; ++l) {
        d[(size_t)src[l] * 64 + l] = 0.0;
        pend[src[l]] |= 1ull << l;
    }
    for (;;) {
        int any = 0;
        for (int v = 0; v < n && !any; ++v) any = pend[v] != 0;
        if (!any) break;
        out->rounds++;
        memset(nxt, 0, (size_t)n * 8);
        for (int v = 0; v < n; ++v) {
            uint64_t cand = 0;
            int64_t rows = 0;
            for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
                if (!pend[col[k]]) continue;
                cand |= pend[col[k]];
                rows++;
                out->nbr_bytes_list += __builtin_popcountll(pend[col[k]]) <= cap ? 128 : 512;
            }
            if (!cand) continue;
            out->visits++;
            out->nbr_rows += rows;
            uint64_t ch = 0;
            for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
                const int u = col[k];
                uint64_t e = pend[u];
                while (e) {
                    int l = __builtin_ctzll(e);
                    e &= e - 1;
                    const double a = d[(size_t)u * 64 + l] + w[k];
                    if (a < d[(size_t)v * 64 + l]) {
                        d[(size_t)v * 64 + l] = a;
                        ch |= 1ull << l;
                    }
                }
            }
            nxt[v] = ch;
            out->lane_updates += __builtin_popcountll(ch);
            if (ch) out->hist[__builtin_popcountll(ch)]++;
        }
        memcpy(pend, nxt, (size_t)n * 8);
    }
    free(d);
    free(pend);
    free(nxt);
    return 0;
}
