/* sim_records.c -- CPU model (design tool, not product code) comparing two
 * relaxation schedules for one 128-lane row group on an undirected CSR:
 *
 *   GS   the shipped k_relax_m: live neighbour rows (Gauss-Seidel reads), the
 *        route record (r, h, f) gathered from the parent's row per change;
 *   REC  distance-only relaxation where a row that changes publishes a packed
 *        record {128-bit lane mask, the changed lanes' distances} for the next
 *        round (stale by one round), followed by a parent pass and a
 *        level-synchronous tree pass for (r, h, f);
 *   DIST distance-only relaxation with live rows (GS, no route records), then
 *        the same parent pass and tree pass.
 *
 * Byte model: 128-B lines, per row visit; a 128-lane f64 row is 8 lines, i32
 * 4, u16 2.  Gathers count distinct (row, line) pairs.
 *
 * build: gcc -O2 -shared -fPIC -o tools/_sim_records.so tools/sim_records.c
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifndef L
#define L 128
#endif

typedef struct {
    int64_t rounds, visits, lane_updates;
    int64_t rd_lines, wr_lines;       /* relaxation */
    int64_t nbr_lines, own_lines, route_lines;
    int64_t par_rd, par_wr;           /* REC: parent pass */
    int64_t tree_visits, tree_rounds, tree_rd, tree_wr;
    int64_t max_hops;
    int64_t prune_row, prune_line16, prune_line32, nbr_reads;   /* GS: min/max summary tests */
} sim_out;

typedef struct {
    uint64_t m[L / 64];
} mask128;

static int popc128(const mask128* a) {
    int c = 0;
    for (int i = 0; i < L / 64; ++i) c += __builtin_popcountll(a->m[i]);
    return c;
}
static int lines_of(const mask128* a, int per_line) { /* lines of a row touched by the lanes in a */
    int c = 0;
    for (int l0 = 0; l0 < L; l0 += per_line) {
        int any = 0;
        for (int l = l0; l < l0 + per_line; ++l)
            if ((a->m[l >> 6] >> (l & 63)) & 1) any = 1;
        c += any;
    }
    return c;
}
static inline int bit(const mask128* a, int l) { return (a->m[l >> 6] >> (l & 63)) & 1; }
static inline void setb(mask128* a, int l) { a->m[l >> 6] |= 1ull << (l & 63); }

/* distinct (row, line) pairs among lanes with rows[l] >= 0 */
static int gather_lines(const int32_t* rows, const mask128* lanes, int per_line) {
    int c = 0;
    for (int l0 = 0; l0 < L; l0 += per_line) {
        int seen[L];
        int ns = 0;
        for (int l = l0; l < l0 + per_line; ++l) {
            if (!bit(lanes, l)) continue;
            int r = rows[l], dup = 0;
            for (int q = 0; q < ns; ++q)
                if (seen[q] == r) dup = 1;
            if (!dup) seen[ns++] = r;
        }
        c += ns;
    }
    return c;
}

/* mode 0 = GS, 1 = REC, 2 = DIST */
int sim_run(int32_t n, const int32_t* ptr, const int32_t* col, const double* w, const int32_t* src, int mode,
            sim_out* out) {
    memset(out, 0, sizeof(*out));
    double* d = malloc(sizeof(double) * (size_t)n * L);
    int32_t* par = malloc(sizeof(int32_t) * (size_t)n * L);
    uint8_t* mark[2] = {calloc(n, 1), calloc(n, 1)};
    const int32_t m = ptr[n];
    uint8_t* fl[2] = {calloc(m, 1), calloc(m, 1)};
    mask128* rec[2] = {calloc(n, sizeof(mask128)), calloc(n, sizeof(mask128))};
    double* recv[2] = {malloc(sizeof(double) * (size_t)n * L), malloc(sizeof(double) * (size_t)n * L)};
    /* reverse entry: for entry k (u = col[k] -> v), index of (v) in u's list */
    int32_t* rev = malloc(sizeof(int32_t) * m);
    for (int v = 0; v < n; ++v)
        for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
            int u = col[k];
            for (int q = ptr[u]; q < ptr[u + 1]; ++q)
                if (col[q] == v) {
                    rev[k] = q;
                    break;
                }
        }
    for (size_t i = 0; i < (size_t)n * L; ++i) {
        d[i] = INFINITY;
        par[i] = -1;
    }
    int cur = 0;
    for (int l = 0; l < L; ++l) {
        int s = src[l];
        d[(size_t)s * L + l] = 0.0;
        recv[1][(size_t)s * L + l] = 0.0;
        setb(&rec[1][s], l);
    }
    for (int l = 0; l < L; ++l) {   /* seed: out-edges of the sources flagged for round 1 */
        int s = src[l];
        for (int k = ptr[s]; k < ptr[s + 1]; ++k) {
            mark[0][col[k]] = 1;
            fl[0][rev[k]] = 1;
        }
    }
    for (;;) {
        const int nx = cur ^ 1;
        int any = 0;
        for (int v = 0; v < n; ++v) {
            if (!mark[cur][v]) continue;
            mark[cur][v] = 0;
            out->visits++;
            mask128 ch = {{0}}, offered = {{0}};
            int32_t prow[L];
            for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
                if (!fl[cur][k]) continue;
                fl[cur][k] = 0;
                const int u = col[k];
                if (mode != 1) {
                    out->nbr_lines += L / 16;
                    out->nbr_reads++;
                    {   /* summary tests (conservative): line j of u can be skipped when
                         * fl(min over the line's lanes of d_u + w) > max over them of d_v */
                        double mn16[L / 16], mx16[L / 16];
                        for (int j = 0; j < L / 16; ++j) {
                            mn16[j] = INFINITY;
                            mx16[j] = -INFINITY;
                        }
                        for (int l = 0; l < L; ++l) {
                            const double du = d[(size_t)u * L + l], dv = d[(size_t)v * L + l];
                            if (du < mn16[l / 16]) mn16[l / 16] = du;
                            if (src[l] != v && dv > mx16[l / 16]) mx16[l / 16] = dv;
                        }
                        int all = 1;
                        for (int j = 0; j < L / 16; ++j) {
                            const int sk = mn16[j] + w[k] > mx16[j];
                            out->prune_line16 += sk;
                            all &= sk;
                        }
                        for (int j = 0; j < L / 32; ++j) {
                            const double mn = fmin(mn16[2 * j], mn16[2 * j + 1]);
                            const double mx = fmax(mx16[2 * j], mx16[2 * j + 1]);
                            out->prune_line32 += 2 * (mn + w[k] > mx);
                        }
                        out->prune_row += (L / 16) * all;
                    }
                    for (int l = 0; l < L; ++l) {
                        if (src[l] == v) continue;
                        double a = d[(size_t)u * L + l] + w[k];
                        if (a < d[(size_t)v * L + l]) {
                            d[(size_t)v * L + l] = a;
                            par[(size_t)v * L + l] = u;
                            setb(&ch, l);
                        }
                    }
                } else {
                    /* the record u published last round (its buffer is [nx] this round) */
                    const mask128* rm = &rec[nx][u];
                    const int c = popc128(rm);
                    out->nbr_lines += 1 + (c * 8 + 127) / 128;
                    for (int l = 0; l < L; ++l) {
                        if (!bit(rm, l) || src[l] == v) continue;
                        setb(&offered, l);
                        double a = recv[nx][(size_t)u * L + l] + w[k];
                        if (a < d[(size_t)v * L + l]) {
                            d[(size_t)v * L + l] = a;
                            par[(size_t)v * L + l] = u;
                            setb(&ch, l);
                        }
                    }
                }
            }
            out->own_lines += (mode != 1) ? L / 16 : lines_of(&offered, 16);
            const int c = popc128(&ch);
            out->lane_updates += c;
            if (mode == 0) {
                for (int l = 0; l < L; ++l) prow[l] = par[(size_t)v * L + l];
                out->route_lines += gather_lines(prow, &ch, 8);               /* parent RT (16 B) */
                out->wr_lines += lines_of(&ch, 16) + lines_of(&ch, 32) + lines_of(&ch, 8);   /* D, P, RT */
            } else if (mode == 2) {
                out->wr_lines += lines_of(&ch, 16);   /* D only */
            } else {
                out->wr_lines += lines_of(&ch, 16) + (c ? 1 + (c * 8 + 127) / 128 : 0);   /* D + record */
                rec[cur][v] = ch;
                for (int l = 0; l < L; ++l)
                    if (bit(&ch, l)) recv[cur][(size_t)v * L + l] = d[(size_t)v * L + l];
            }
            if (c) {
                any = 1;
                for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
                    mark[nx][col[k]] = 1;
                    fl[nx][rev[k]] = 1;
                }
            }
        }
        if (mode == 1)   /* records of the round before last are dead: clear for reuse */
            for (int v = 0; v < n; ++v) memset(&rec[nx][v], 0, sizeof(mask128));
        out->rounds++;
        cur ^= 1;
        if (!any) break;
    }
    out->rd_lines = out->nbr_lines + out->own_lines + out->route_lines + out->visits * 2;   /* +2: CSR, flags */
    if (mode != 0) {
        /* parent pass: every row reads all in-neighbour rows + own, writes P (i32) */
        for (int v = 0; v < n; ++v) {
            out->par_rd += 8 + 8 * (ptr[v + 1] - ptr[v]) + 2;
            out->par_wr += 4;
        }
        /* hop levels (BFS on the parent trees) */
        int32_t* h = malloc(sizeof(int32_t) * (size_t)n * L);
        for (size_t i = 0; i < (size_t)n * L; ++i) h[i] = -1;
        int maxh = 0;
        for (int l = 0; l < L; ++l) {
            h[(size_t)src[l] * L + l] = 0;
        }
        /* repeated sweeps (model only) */
        for (int changed = 1; changed;) {
            changed = 0;
            for (int v = 0; v < n; ++v)
                for (int l = 0; l < L; ++l) {
                    size_t i = (size_t)v * L + l;
                    if (h[i] >= 0 || par[i] < 0) continue;
                    int hp = h[(size_t)par[i] * L + l];
                    if (hp >= 0) {
                        h[i] = hp + 1;
                        if (h[i] > maxh) maxh = h[i];
                        changed = 1;
                    }
                }
        }
        out->max_hops = maxh;
        /* level-synchronous tree pass with discovery: round k visits rows with an
         * in-neighbour that finished lanes at level k-1 (marks on out-edges);
         * a visit reads its pending mask (2 lines, u16 hops), P for pending lanes,
         * the parents' hops (u16) for pending lanes, and (r, f) of the parents of
         * lanes that finish (level k); writes r, h, f of finishing lanes. */
        uint8_t* tm = calloc(n, 1);
        uint8_t* fin = calloc(n, 1);   /* row finished lanes at level k-1 */
        for (int l = 0; l < L; ++l) fin[src[l]] = 1;
        for (int k = 1; k <= maxh; ++k) {
            memset(tm, 0, n);
            for (int u = 0; u < n; ++u)
                if (fin[u])
                    for (int q = ptr[u]; q < ptr[u + 1]; ++q) tm[col[q]] = 1;
            memset(fin, 0, n);
            out->tree_rounds++;
            for (int v = 0; v < n; ++v) {
                if (!tm[v]) continue;
                mask128 pend = {{0}}, now = {{0}};
                int32_t prow[L];
                for (int l = 0; l < L; ++l) {
                    size_t i = (size_t)v * L + l;
                    prow[l] = par[i];
                    if (h[i] >= k) setb(&pend, l);
                    if (h[i] == k) setb(&now, l);
                }
                if (!popc128(&pend)) continue;   /* a row with nothing pending exits after its mask */
                out->tree_visits++;
                out->tree_rd += 2 + lines_of(&pend, 32) + gather_lines(prow, &pend, 64) + gather_lines(prow, &now, 16) +
                                gather_lines(prow, &now, 32);
                out->tree_wr += lines_of(&now, 16) + lines_of(&now, 64) + lines_of(&now, 32);
                if (popc128(&now)) fin[v] = 1;
            }
        }
        free(tm);
        free(fin);
        free(h);
    }
    free(d);
    free(par);
    free(mark[0]);
    free(mark[1]);
    free(fl[0]);
    free(fl[1]);
    free(rec[0]);
    free(rec[1]);
    free(recv[0]);
    free(recv[1]);
    free(rev);
    return 0;
}
