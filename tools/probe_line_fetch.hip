// Round-6 calibration probe: what does a uniformly random 16-B record read cost on
// MI355X HBM, and what does FETCH_SIZE report for it?  (MI355X_MICROARCH.md: the
// x2 correction of FETCH_SIZE is calibrated for wide coalesced streaming reads only;
// C5's k_lookup reads one random 16-B record per query.)
//
// Three kernels read the same number of random 128-B-aligned LOCATIONS of a 16-GiB
// buffer of 16-B records, one result (8 B) stored per location:
//   r16  : one lane per location, 16 B read           (k_lookup's access)
//   r64  : 4 lanes per location, the 64-B half line    (one 64-B sector)
//   r128 : 8 lanes per location, the whole 128-B line
// Time per location says which granularity the memory system moves for r16; a
// separate `rocprofv3 --pmc FETCH_SIZE` pass of this binary gives the counter's view.
//
//   hipcc --offload-arch=gfx950 -O3 -o build_ab/probe_line_fetch tools/probe_line_fetch.hip
//   build_ab/probe_line_fetch [locations_millions=128]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

typedef double dvec2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}

// LANES lanes per location read LANES consecutive 16-B records of it
template <int LANES>
__global__ __launch_bounds__(256) void k_read(const dvec2* __restrict__ rec, uint64_t nlines, uint64_t locs,
                                              double* __restrict__ out, uint64_t salt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < locs * LANES; i += stride) {
        const uint64_t loc = i / LANES;
        const uint64_t line = mix(loc + salt) % nlines;
        const dvec2 v = __builtin_nontemporal_load(rec + line * 8 + (i % LANES));
        if (i % LANES == 0) out[loc] = v.x + v.y;
        else if (v.x == -1.0) out[loc] = v.y;   // (never: keeps the other lanes' loads)
    }
}

__global__ void k_fill(dvec2* rec, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        rec[i] = dvec2{(double)(i & 1023), 0.5};
}

template <int LANES>
static float run(const dvec2* rec, uint64_t nlines, uint64_t locs, double* out, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    k_read<LANES><<<8192, 256>>>(rec, nlines, locs, out, 99);   // warm-up
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) k_read<LANES><<<8192, 256>>>(rec, nlines, locs, out, (uint64_t)r * 7919u);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const uint64_t locs = (uint64_t)(argc > 1 ? atof(argv[1]) : 128.0) * 1000000ull;
    const uint64_t bytes = 16ull << 30;   // 16 GiB: far beyond the 256-MiB Infinity Cache
    const uint64_t nrec = bytes / 16, nlines = bytes / 128;
    dvec2* rec = nullptr;
    double* out = nullptr;
    CHECK(hipMalloc(&rec, bytes));
    CHECK(hipMalloc(&out, locs * sizeof(double)));
    k_fill<<<8192, 256>>>(rec, nrec);
    CHECK(hipDeviceSynchronize());
    const int reps = 5;
    const float t16 = run<1>(rec, nlines, locs, out, reps);
    const float t64 = run<4>(rec, nlines, locs, out, reps);
    const float t128 = run<8>(rec, nlines, locs, out, reps);
    printf("{\"locations\": %llu, \"buffer_GiB\": 16, \"ms\": {\"r16\": %.3f, \"r64\": %.3f, \"r128\": %.3f}, "
           "\"G_locations_per_s\": {\"r16\": %.2f, \"r64\": %.2f, \"r128\": %.2f}, "
           "\"GB_per_s_if_line_128\": {\"r16\": %.0f, \"r64\": %.0f, \"r128\": %.0f}}\n",
           (unsigned long long)locs, t16, t64, t128, locs / t16 / 1e6, locs / t64 / 1e6, locs / t128 / 1e6,
           locs * 136.0 / t16 / 1e6, locs * 136.0 / t64 / 1e6, locs * 136.0 / t128 / 1e6);
    CHECK(hipFree(rec));
    CHECK(hipFree(out));
    return 0;
}
