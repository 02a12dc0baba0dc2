/* sim_relax.c -- CPU model of the multi-source relaxation schedule (design tool,
 * not product code).  Synchronous rounds over one group of L <= 64 lanes
 * (lane = source) on an undirected CSR.  Reports rounds, vertex visits, lane
 * updates and a byte model for (a) whole 512-B rows and (b) 64-B sectors
 * (8 lanes) touched, under optional per-lane delta gating.
 *
 * build: gcc -O2 -shared -fPIC -o tools/_sim_relax.so tools/sim_relax.c
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t rounds, visits, lane_updates, nbr_rows, nbr_sectors, own_sectors, write_sectors;
} sim_out;

static int popc(uint64_t x) { return __builtin_popcountll(x); }
static uint64_t sector_mask(uint64_t lanes) {   /* 8-lane sectors with any lane set -> bit per sector */
    uint64_t s = 0;
    for (int q = 0; q < 8; ++q)
        if ((lanes >> (8 * q)) & 0xFF) s |= 1ull << q;
    return s;
}

/* delta <= 0: no gating. */
int sim_run(int32_t n, const int32_t* ptr, const int32_t* col, const double* w, int32_t L, const int32_t* src,
            double delta, sim_out* out) {
    double* d = malloc(sizeof(double) * (size_t)n * 64);
    uint64_t* pend = calloc((size_t)n, 8);
    uint64_t* nxt = calloc((size_t)n, 8);
    uint64_t* elig = calloc((size_t)n, 8);
    memset(out, 0, sizeof(*out));
    for (size_t i = 0; i < (size_t)n * 64; ++i) d[i] = INFINITY;
    for (int l = 0; l < L; ++l) {
        d[(size_t)src[l] * 64 + l] = 0.0;
        pend[src[l]] |= 1ull << l;
    }
    for (;;) {
        /* thresholds */
        double T[64];
        for (int l = 0; l < 64; ++l) T[l] = INFINITY;
        int any = 0;
        if (delta > 0) {
            double mn[64];
            for (int l = 0; l < 64; ++l) mn[l] = INFINITY;
            for (int v = 0; v < n; ++v) {
                uint64_t m = pend[v];
                while (m) {
                    int l = __builtin_ctzll(m);
                    m &= m - 1;
                    if (d[(size_t)v * 64 + l] < mn[l]) mn[l] = d[(size_t)v * 64 + l];
                }
            }
            for (int l = 0; l < 64; ++l) T[l] = mn[l] + delta;
        }
        for (int v = 0; v < n; ++v) {
            uint64_t m = pend[v], e = 0;
            while (m) {
                int l = __builtin_ctzll(m);
                m &= m - 1;
                if (d[(size_t)v * 64 + l] <= T[l]) e |= 1ull << l;
            }
            elig[v] = e;
            if (e) any = 1;
        }
        if (!any) break;
        out->rounds++;
        memset(nxt, 0, (size_t)n * 8);
        /* pull: v reads eligible changed lanes of in-neighbours (values of this round's start) */
        for (int v = 0; v < n; ++v) {
            uint64_t cand = 0;
            int64_t rows = 0, secs = 0;
            for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
                const uint64_t e = elig[col[k]];
                if (!e) continue;
                cand |= e;
                rows++;
                secs += popc(sector_mask(e));
            }
            if (!cand) continue;
            out->visits++;
            out->nbr_rows += rows;
            out->nbr_sectors += secs;
            out->own_sectors += popc(sector_mask(cand));
            uint64_t ch = 0;
            for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
                const int u = col[k];
                uint64_t e = elig[u];
                while (e) {
                    int l = __builtin_ctzll(e);
                    e &= e - 1;
                    const double a = d[(size_t)u * 64 + l] + w[k];
                    if (a < d[(size_t)v * 64 + l]) {   /* synchronous: write to d directly is a Gauss-Seidel */
                        d[(size_t)v * 64 + l] = a;     /* effect; acceptable for the model */
                        ch |= 1ull << l;
                    }
                }
            }
            nxt[v] = ch;
            out->lane_updates += popc(ch);
            out->write_sectors += popc(sector_mask(ch));
        }
        for (int v = 0; v < n; ++v) pend[v] = (pend[v] & ~elig[v]) | nxt[v];
    }
    free(d);
    free(pend);
    free(nxt);
    free(elig);
    return 0;
}
