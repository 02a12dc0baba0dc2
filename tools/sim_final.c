/* sim_final.c -- CPU model (design tool, not product code) of k_relax_s's schedule on
 * one 128-lane group: Gauss-Seidel rounds in vertex order, in-edge flags carrying the
 * neighbour's changed 16-lane segments (SPE_SEG_FLAGS), and the settle bound
 *
 *     lane l of row v is final once D[v][l] < fl(F_l + w_min),
 *
 * F_l = the smallest value lane l took in any change of the previous round (every
 * offer still to come is >= F_l + w_min, so a value strictly below cannot be
 * beaten or tied again; fl() is monotone).  Reports per round: rows visited, lane
 * updates, own-row lines and neighbour lines read without and with the bound
 * (a 128-B line = 16 lanes; a line is skipped when every lane of it that the flag
 * names is final at v).
 *
 * build: gcc -O2 -shared -fPIC -o tools/_sim_final.so tools/sim_final.c
 * driver: tools/sim_final.py */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define L 128
#define SEG 16
#define NSEG (L / SEG)

typedef struct {
    int64_t visits, lane_updates, own_lines, own_lines_final, nbr_lines, nbr_lines_final, rows_all_final;
} round_out;

/* returns the number of rounds (<= max_rounds); per-round stats in out[] */
int sim_final(int32_t n, const int32_t* ptr, const int32_t* col, const double* w, const int32_t* src,
              double w_min, int32_t max_rounds, round_out* out, int per_item, int order) {
    double* d = malloc(sizeof(double) * (size_t)n * L);
    double* dprev = malloc(sizeof(double) * (size_t)n * L);
    uint8_t* cur = calloc((size_t)ptr[n], 1);   /* in-edge flag: changed segments of col[k] */
    uint8_t* nxt = calloc((size_t)ptr[n], 1);
    uint8_t* fin = calloc((size_t)n, 1);        /* segments whose every lane is final */
    int32_t* rev = malloc(sizeof(int32_t) * (size_t)ptr[n]);
    for (size_t i = 0; i < (size_t)n * L; ++i) d[i] = INFINITY;
    /* reverse entry of every in-entry (undirected: the out-list is the in-list) */
    for (int32_t v = 0; v < n; ++v)
        for (int32_t k = ptr[v]; k < ptr[v + 1]; ++k) {
            const int32_t u = col[k];
            int32_t r = -1;
            for (int32_t q = ptr[u]; q < ptr[u + 1]; ++q)
                if (col[q] == v) { r = q; break; }
            rev[k] = r;
        }
    double F[L], Fn[L];
    for (int l = 0; l < L; ++l) {
        F[l] = 0.0;
        Fn[l] = INFINITY;
        if (src[l] < 0) continue;
        const int32_t s = src[l];
        d[(size_t)s * L + l] = 0.0;
        for (int32_t k = ptr[s]; k < ptr[s + 1]; ++k) nxt[rev[k]] |= 1u << (l / SEG);
    }
    int rounds = 0;
    for (; rounds < max_rounds; ++rounds) {
        uint8_t* t = cur; cur = nxt; nxt = t;
        memset(nxt, 0, (size_t)ptr[n]);
        round_out* o = &out[rounds];
        memset(o, 0, sizeof(*o));
        int any = 0;
        for (int l = 0; l < L; ++l) Fn[l] = INFINITY;
        if (order == 2) memcpy(dprev, d, sizeof(double) * (size_t)n * L);
        for (int32_t vi = 0; vi < n; ++vi) {
            const int32_t v = (order == 1 && (rounds & 1)) ? n - 1 - vi : vi;
            uint8_t segs = 0;
            for (int32_t k = ptr[v]; k < ptr[v + 1]; ++k) segs |= cur[k];
            if (!segs) continue;
            any = 1;
            o->visits++;
            double* dv = d + (size_t)v * L;
            double wv = INFINITY;   /* the vertex's lightest in-entry */
            for (int32_t k = ptr[v]; k < ptr[v + 1]; ++k) wv = w[k] < wv ? w[k] : wv;
            /* lanes final at v under this round's bound */
            uint8_t fseg = fin[v];
            for (int q = 0; q < NSEG; ++q) {
                if (fseg >> q & 1) continue;
                int all = 1;
                for (int l = q * SEG; l < (q + 1) * SEG && all; ++l)
                    if (src[l] >= 0 && !(dv[l] < F[l] + w_min)) all = 0;
                if (all) fseg |= 1u << q;
            }
            fin[v] = fseg;
            if (fseg == (1u << NSEG) - 1) o->rows_all_final++;
            o->own_lines += NSEG;
            o->own_lines_final += NSEG - __builtin_popcount(fseg);
            uint8_t chg = 0;
            for (int32_t k = ptr[v]; k < ptr[v + 1]; ++k) {
                const uint8_t f = cur[k];
                if (!f) continue;
                cur[k] = 0;
                const int32_t u = col[k];
                const double* du = (order == 2 ? dprev : d) + (size_t)u * L;
                o->nbr_lines += __builtin_popcount(f);
                for (int q = 0; q < NSEG; ++q) {
                    if (!(f >> q & 1)) continue;
                    /* a line whose lanes are all final at v (under this edge's weight) is skipped */
                    int need = 0;
                    for (int l = q * SEG; l < (q + 1) * SEG; ++l)
                        if (src[l] >= 0 && !(dv[l] < F[l] + (per_item ? wv : w[k]))) { need = 1; break; }
                    if (need) o->nbr_lines_final++;
                    for (int l = q * SEG; l < (q + 1) * SEG; ++l) {
                        if (src[l] < 0 || src[l] == v) continue;
                        const double a = du[l] + w[k];
                        if (a < dv[l]) {
                            dv[l] = a;
                            chg |= 1u << q;
                            o->lane_updates++;
                            if (a < Fn[l]) Fn[l] = a;
                        }
                    }
                }
            }
            if (chg)
                for (int32_t k = ptr[v]; k < ptr[v + 1]; ++k) nxt[rev[k]] |= chg;
        }
        /* changes made in this round bound the next one (GS changes in the next round are larger) */
        for (int l = 0; l < L; ++l) F[l] = Fn[l];
        if (!any) break;
    }
    free(d); free(dprev); free(cur); free(nxt); free(fin); free(rev);
    return rounds;
}
