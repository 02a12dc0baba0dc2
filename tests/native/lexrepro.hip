// lexrepro.hip -- test-only reproducer of a gfx950 code-generation fault (ROCm 7.2)
// behind wrong route tie-breaks at hubs (MEASUREMENTS.md, round 4).  Not part of
// libspe: tests/test_gpu_lexrepro.py loads it as a checker of the compiler.
//
// The heavy partial kept a running lexicographic best (alt, d[u], u) over
// candidates whose vertex u is wave-uniform (readlane of a packed in-list entry).
// Written with the short-circuit compare
//     if (alt < ba || (alt == ba && (du < bdu || (du == bdu && u < bu)))) { ba = alt; bdu = du; bu = u; bk = kk; }
// the compiler produced code whose tie-winning lanes took the new (ba, bdu) but
// kept the OLD (bk, bu).  libspe writes every such compare branch-free
// (lex_less3: bitwise & / | on bools, then selects); form 1 below.  Both forms are
// built here in the same shape so the test can run them on the same inputs.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr double INF = __builtin_inf();

template <int FORM>
__global__ __launch_bounds__(256) void k_lexmin(const int4* __restrict__ pack, const double* __restrict__ D,
                                                int32_t cnt, int32_t nitems, double* __restrict__ out_a,
                                                double* __restrict__ out_d, int2* __restrict__ out_uk) {
    const int32_t lane = threadIdx.x & 63;
    const int32_t item = (int32_t)((blockIdx.x * 256 + threadIdx.x) >> 6);   // wave-uniform
    if (item >= nitems) return;
    // one 64-entry in-list per item: lane k holds entry k (u, w), as G.ipack does
    const int4 pk = pack[(size_t)item * 64 + lane];
    const int32_t u_j = pk.x;
    const double w_j = __hiloint2double(pk.w, pk.z);
    double ba = INF, bdu = INF;
    int32_t bu = -1, bk = -1;
    for (int32_t kk = 0; kk < cnt; ++kk) {
        const int32_t u = __builtin_amdgcn_readlane(u_j, kk);   // wave-uniform vertex
        const int32_t lo = __builtin_amdgcn_readlane((int32_t)pk.z, kk), hi = __builtin_amdgcn_readlane((int32_t)pk.w, kk);
        const double w = __hiloint2double(hi, lo);
        const double du = D[((size_t)item * 64 + u) * 64 + lane];   // the neighbour's row, this lane's source
        if (!(du < INF)) continue;
        const double alt = du + w;
        if constexpr (FORM == 0) {
            if (alt < ba || (alt == ba && (du < bdu || (du == bdu && u < bu)))) {
                ba = alt;
                bdu = du;
                bu = u;
                bk = kk;
            }
        } else {
            const bool better = (alt < ba) | ((alt == ba) & ((du < bdu) | ((du == bdu) & (u < bu))));
            ba = better ? alt : ba;
            bdu = better ? du : bdu;
            bu = better ? u : bu;
            bk = better ? kk : bk;
        }
    }
    (void)w_j;
    const size_t o = (size_t)item * 64 + lane;
    out_a[o] = ba;
    out_d[o] = bdu;
    out_uk[o] = make_int2(bu, bk);
}

}  // namespace

extern "C" int lexrepro_run(int form, const int32_t* pack, const double* D, int32_t cnt, int32_t nitems, double* a,
                            double* d, int32_t* uk) {
    const size_t ne = (size_t)nitems * 64;
    int4* dp = nullptr;
    double *dD = nullptr, *da = nullptr, *dd = nullptr;
    int2* duk = nullptr;
    hipError_t e = hipMalloc(&dp, ne * sizeof(int4));
    if (e == hipSuccess) e = hipMalloc(&dD, ne * 64 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&da, ne * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&dd, ne * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&duk, ne * sizeof(int2));
    if (e == hipSuccess) e = hipMemcpy(dp, pack, ne * sizeof(int4), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dD, D, ne * 64 * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess && (cnt < 0 || cnt > 64)) e = hipErrorInvalidValue;
    if (e == hipSuccess) {
        const unsigned grid = (unsigned)((ne + 255) / 256);
        if (form == 0) k_lexmin<0><<<grid, 256>>>(dp, dD, cnt, nitems, da, dd, duk);
        else k_lexmin<1><<<grid, 256>>>(dp, dD, cnt, nitems, da, dd, duk);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(a, da, ne * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(d, dd, ne * sizeof(double), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(uk, duk, ne * sizeof(int2), hipMemcpyDeviceToHost);
    (void)hipFree(dp);
    (void)hipFree(dD);
    (void)hipFree(da);
    (void)hipFree(dd);
    (void)hipFree(duk);
    return e == hipSuccess ? 0 : (int)e;
}
