// probe_single_call.hip -- design probe (not product code) for the drop-in's
// per-packet single reads on a table that lives only in HBM (C4: 160 GB of
// records): what one 16-B record read round trip costs on this box by
//   (a) hipMemcpyAsync + hipStreamSynchronize (the round-5 path),
//   (b) a one-wave kernel writing the record into pinned host memory + sync,
//   (c) a resident service wave polling request slots in pinned host memory and
//       answering into them (one round trip per call, no launch),
//   (d) the same service wave polling request slots in device memory the host
//       writes through a host mapping (when the box maps fine-grained VRAM).
// build: hipcc -O3 --offload-arch=gfx950 -o build_ab/probe_single_call tools/probe_single_call.hip
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <csetjmp>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

struct alignas(64) Slot {
    unsigned long long req;   // request sequence number (written last by the host)
    int32_t s, t;             // the pair (here: a record index)
    unsigned long long done;  // answered sequence number (written last by the device)
    double lat, rel;
    int32_t next, hops;
};

__global__ void k_one(const double2* lr, int64_t o, double* out) {
    if (threadIdx.x == 0) {
        const double2 v = lr[o];
        out[0] = v.x;
        out[1] = v.y;
    }
}

// one wave; lane i serves slot i; exits on *stop or after `limit` ticks of the
// 100-MHz wall clock with no request (every lane reaches the same decision)
__global__ void k_service(Slot* slots, int32_t nslots, const double2* lr, const int* stop, long long limit) {
    const int lane = threadIdx.x;
    unsigned long long last = 0;
    long long idle0 = wall_clock64();
    for (;;) {
        bool work = false;
        if (lane < nslots) {
            const unsigned long long r = __hip_atomic_load(&slots[lane].req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            if (r != last) {
                const int32_t s = __hip_atomic_load(&slots[lane].s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const double2 v = lr[s];
                __hip_atomic_store(&slots[lane].lat, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&slots[lane].rel, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&slots[lane].done, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                last = r;
                work = true;
            }
        }
        const long long now = wall_clock64();
        if (__ballot(work)) idle0 = now;
        const int st = __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (__ballot(st != 0 || now - idle0 > limit)) break;
    }
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void service_round_trips(const char* label, Slot* host_view, Slot* dev_view, const double2* lr, int* stop_h,
                                int* stop_d, int64_t nrec, int iters) {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    memset((void*)host_view, 0, sizeof(Slot) * 64);
    *stop_h = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, st, dev_view, 64, lr, stop_d, 200000000LL /* 2 s */);
    CK(hipGetLastError());
    // wait for the first answer (launch latency excluded)
    std::vector<double> lat(iters);
    uint64_t x = 88172645463325252ull;
    double sum = 0.0;
    for (int i = 0; i < iters; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const int32_t s = (int32_t)(x % (uint64_t)nrec);
        Slot* sl = &host_view[0];
        const unsigned long long seq = (unsigned long long)i + 1;
        const double t0 = now_s();
        __atomic_store_n(&sl->s, s, __ATOMIC_RELAXED);
        __atomic_store_n(&sl->req, seq, __ATOMIC_RELEASE);
        const double tl = t0 + 1.0;
        while (__atomic_load_n(&sl->done, __ATOMIC_ACQUIRE) != seq)
            if (now_s() > tl) {
                fprintf(stderr, "%s: no answer within 1 s at call %d\n", label, i);
                __atomic_store_n(stop_h, 1, __ATOMIC_SEQ_CST);
                CK(hipStreamSynchronize(st));
                return;
            }
        lat[i] = now_s() - t0;
        double v;
        memcpy(&v, (const void*)&sl->lat, sizeof v);
        sum += v;
    }
    __atomic_store_n(stop_h, 1, __ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(st));
    CK(hipStreamDestroy(st));
    std::vector<double> s2 = lat;
    std::sort(s2.begin(), s2.end());
    double tot = 0.0;
    for (double v : lat) tot += v;
    printf("%s: %d calls, mean %.2f us, median %.2f us, p99 %.2f us -> %.0f calls/s (checksum %.3f)\n", label, iters,
           1e6 * tot / iters, 1e6 * s2[iters / 2], 1e6 * s2[iters * 99 / 100], iters / tot, sum);
}

int main() {
    const int64_t nrec = (int64_t)1 << 28;   // 4 GB of 16-B records: random reads miss every cache
    double2* lr = nullptr;
    CK(hipMalloc(&lr, sizeof(double2) * nrec));
    CK(hipMemset(lr, 0, sizeof(double2) * nrec));
    CK(hipDeviceSynchronize());
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int iters = 20000;
    // (a) memcpy + sync
    {
        double* h = nullptr;
        CK(hipHostMalloc((void**)&h, 64, hipHostMallocDefault));
        uint64_t x = 1;
        const double t0 = now_s();
        for (int i = 0; i < iters; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            CK(hipMemcpyAsync(h, lr + (x >> 36) % nrec, 16, hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
        }
        const double el = now_s() - t0;
        printf("(a) hipMemcpyAsync 16 B + sync: %.2f us/call -> %.0f calls/s\n", 1e6 * el / iters, iters / el);
        CK(hipHostFree(h));
    }
    // (b) kernel into pinned host memory + sync
    {
        double* h = nullptr;
        CK(hipHostMalloc((void**)&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
        double* hd = nullptr;
        CK(hipHostGetDevicePointer((void**)&hd, h, 0));
        uint64_t x = 1;
        const double t0 = now_s();
        for (int i = 0; i < iters; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, st, lr, (int64_t)((x >> 36) % nrec), hd);
            CK(hipStreamSynchronize(st));
        }
        const double el = now_s() - t0;
        printf("(b) one-wave kernel into pinned memory + sync: %.2f us/call -> %.0f calls/s\n", 1e6 * el / iters,
               iters / el);
        CK(hipHostFree(h));
    }
    // (c) service wave polling pinned host memory
    {
        Slot* h = nullptr;
        int* stop = nullptr;
        CK(hipHostMalloc((void**)&h, sizeof(Slot) * 64, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostMalloc((void**)&stop, 64, hipHostMallocMapped | hipHostMallocCoherent));
        Slot* hd = nullptr;
        int* sd = nullptr;
        CK(hipHostGetDevicePointer((void**)&hd, h, 0));
        CK(hipHostGetDevicePointer((void**)&sd, stop, 0));
        service_round_trips("(c) service wave, request slots in pinned host memory", h, hd, lr, stop, sd, nrec, iters);
        CK(hipHostFree(h));
        CK(hipHostFree(stop));
    }
    // (d) fine-grained VRAM slots written by the host through a host mapping
    for (unsigned flag : {(unsigned)hipDeviceMallocFinegrained, (unsigned)hipDeviceMallocUncached}) {
        Slot* d = nullptr;
        hipError_t e = hipExtMallocWithFlags((void**)&d, sizeof(Slot) * 64, flag);
        if (e != hipSuccess) {
            printf("(d) hipExtMallocWithFlags(%u): %s\n", flag, hipGetErrorString(e));
            continue;
        }
        struct sigaction sa{}, old{};
        sa.sa_handler = on_segv;
        sigaction(SIGSEGV, &sa, &old);
        bool ok = false;
        if (sigsetjmp(g_jb, 1) == 0) {
            volatile unsigned long long* p = &d->req;
            *p = 7;
            ok = *p == 7;
        }
        sigaction(SIGSEGV, &old, nullptr);
        printf("(d) flag %u VRAM: host store/load through the device pointer %s\n", flag, ok ? "works" : "faults");
        if (ok) {
            int* stop = nullptr;
            CK(hipHostMalloc((void**)&stop, 64, hipHostMallocMapped | hipHostMallocCoherent));
            int* sd = nullptr;
            CK(hipHostGetDevicePointer((void**)&sd, stop, 0));
            service_round_trips(flag == hipDeviceMallocFinegrained ? "(d) service wave, slots in fine-grained VRAM"
                                                                   : "(d) service wave, slots in uncached VRAM",
                                d, d, lr, stop, sd, nrec, iters);
            CK(hipHostFree(stop));
        }
        CK(hipFree(d));
    }
    CK(hipFree(lr));
    return 0;
}
