/* sim_delta.c -- CPU model (design tool, not product code) of 64-lane row relaxation
 * with firing gated by a distance threshold (Delta-stepping buckets): mode 0 = no gate
 * (the shipped Gauss-Seidel rounds), 1 = one bucket bound per group, 2 = per lane.
 * build: gcc -O2 -shared -fPIC -o tools/_sim_delta.so tools/sim_delta.c
 * driver: tools/sim_schedules.py */
/* GS relaxation of 64 lanes with firing gated by a threshold.
 * mode 0: no gating; 1: group threshold T = min pending + delta (all lanes);
 * 2: per-lane threshold T_l = min pending_l + delta.  Pull model: v reads every in-neighbour u that fires this round. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
typedef struct { int64_t rounds, visits, lane_updates, nbr_rows, nbr_lines, fires; } so;
int simd(int32_t n, const int32_t* ptr, const int32_t* col, const double* w, const int32_t* src, int mode, double delta, so* out) {
    double* d = malloc(sizeof(double)*(size_t)n*64);
    uint64_t* pend = calloc(n,8); uint64_t* fire = calloc(n,8);
    memset(out,0,sizeof(*out));
    for (size_t i=0;i<(size_t)n*64;++i) d[i]=INFINITY;
    for (int l=0;l<64;++l){ d[(size_t)src[l]*64+l]=0; pend[src[l]]|=1ull<<l; }
    for(;;){
        double T[64]; for(int l=0;l<64;++l) T[l]=INFINITY;
        if(mode){
            double mn[64]; for(int l=0;l<64;++l) mn[l]=INFINITY;
            for(int v=0;v<n;++v){ uint64_t m=pend[v]; while(m){int l=__builtin_ctzll(m); m&=m-1; if(d[(size_t)v*64+l]<mn[l]) mn[l]=d[(size_t)v*64+l];}}
            double g=INFINITY; for(int l=0;l<64;++l) if(mn[l]<g) g=mn[l];
            for(int l=0;l<64;++l) T[l]= mode==1 ? g+delta : mn[l]+delta;
        }
        int any=0;
        for(int v=0;v<n;++v){ uint64_t m=pend[v], e=0; while(m){int l=__builtin_ctzll(m); m&=m-1; if(d[(size_t)v*64+l]<=T[l]) e|=1ull<<l;} fire[v]=e; pend[v]&=~e; if(e){any=1; out->fires++;} }
        if(!any) break;
        out->rounds++;
        for(int v=0;v<n;++v){
            int vis=0;
            for(int k=ptr[v];k<ptr[v+1];++k){ uint64_t e=fire[col[k]]; if(!e) continue; vis=1; out->nbr_rows++;
                for(int q=0;q<4;++q) if((e>>(16*q))&0xFFFF) out->nbr_lines++;
                int u=col[k];
                while(e){int l=__builtin_ctzll(e); e&=e-1; double a=d[(size_t)u*64+l]+w[k]; if(a<d[(size_t)v*64+l]){d[(size_t)v*64+l]=a; pend[v]|=1ull<<l; out->lane_updates++;}}
            }
            if(vis) out->visits++;
        }
    }
    free(d); free(pend); free(fire);
    return 0;
}
