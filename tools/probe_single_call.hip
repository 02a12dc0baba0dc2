// probe_single_call.hip -- design probe (not product code) for the drop-in's
// per-packet single reads on a table that lives only in HBM (C4: 160 GB of
// records): what one 16-B record read round trip costs on this box by
//   (a) hipMemcpyAsync + hipStreamSynchronize (the round-5 path),
//   (b) a one-wave kernel writing the record into pinned host memory + sync,
//   (c) a resident service wave polling request slots in pinned host memory and
//       answering into them (one round trip per call, no launch),
//   (d) the same service wave polling request slots in device memory the host
//       writes through a host mapping (when the box maps fine-grained VRAM),
//   (e) a plain host load of the record from fine-grained VRAM (no device work),
//   (f) whether plain hipMalloc memory is host-mapped at all,
//   (g) what fine-grained placement costs device kernels: streaming nontemporal
//       record writes and random record reads, coarse vs fine-grained,
//   (h) the pointer attributes of plain hipMalloc memory, and (i) one 16-B host
//       load of a record in plain hipMalloc memory: latency and the values read
//       (written by a kernel, then synchronised) against the expected pattern,
//   (j) bulk device-to-host copies for a host mirror: 8 GB into touched anonymous
//       memory registered with hipHostRegister (time to register, DMA rate) against
//       pinned staging + memcpy on 8 threads,
//   (k) host loads from 1 / 4 / 16 threads at once (do uncached BAR reads overlap?),
//   (l) the service wave with 1 / 4 / 16 threads, each on its own request slot.
// build: hipcc -O3 --offload-arch=gfx950 -o build_ab/probe_single_call tools/probe_single_call.hip
#include <hip/hip_runtime.h>

#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <sys/mman.h>
#include <thread>
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

typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ void k_write(double2* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        dv2 v;
        v.x = (double)i;
        v.y = 1.0;
        __builtin_nontemporal_store(v, reinterpret_cast<dv2*>(p + i));
    }
}
__global__ void k_gather(const double2* p, int64_t n, int64_t q, double* out) {
    double acc = 0.0;
    uint64_t x = 0x9E3779B97F4A7C15ull * (blockIdx.x * blockDim.x + threadIdx.x + 1);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < q; i += (int64_t)gridDim.x * blockDim.x) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const double2 v = p[x % (uint64_t)n];
        acc += v.x + v.y;
    }
    if (acc == -1.0) out[0] = acc;
}

static void device_rates(const char* label, double2* p, int64_t n) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    double* sink = nullptr;
    CK(hipMalloc(&sink, 64));
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, p, n);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        const int64_t q = (int64_t)1 << 27;
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_gather, dim3(16384), dim3(256), 0, 0, p, n, q, sink);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms2 = 0.f;
        CK(hipEventElapsedTime(&ms2, a, b));
        if (rep == 1)
            printf("(g) %s: nontemporal record writes %.0f GB/s, random 16-B record reads %.2f G/s\n", label,
                   16.0 * n / (ms * 1e-3) / 1e9, q / (ms2 * 1e-3) / 1e9);
    }
    CK(hipFree(sink));
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
    // (e) host loads of records in fine-grained VRAM, (g) device rates on it
    {
        double2* f = nullptr;
        CK(hipExtMallocWithFlags((void**)&f, sizeof(double2) * nrec, hipDeviceMallocFinegrained));
        hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, f, nrec);
        CK(hipDeviceSynchronize());
        uint64_t x = 3;
        double acc = 0.0;
        const int n = 200000;
        const double t0 = now_s();
        for (int i = 0; i < n; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            const volatile double2* r = f + (x >> 36) % nrec;
            acc += r->x + r->y;
        }
        const double el = now_s() - t0;
        printf("(e) host load of a 16-B record in fine-grained VRAM: %.2f us/read -> %.0f reads/s (checksum %.1f)\n",
               1e6 * el / n, n / el, acc);
        device_rates("fine-grained VRAM", f, nrec);
        CK(hipFree(f));
    }
    device_rates("coarse-grained VRAM (hipMalloc)", lr, nrec);
    // (f) plain hipMalloc memory through its pointer on the host
    {
        struct sigaction sa{}, old{};
        sa.sa_handler = on_segv;
        sigaction(SIGSEGV, &sa, &old);
        bool ok = false;
        if (sigsetjmp(g_jb, 1) == 0) {
            volatile double* p = &lr[5].x;
            ok = *p == *p;
        }
        sigaction(SIGSEGV, &old, nullptr);
        printf("(f) hipMalloc VRAM: host load through the device pointer %s\n", ok ? "works" : "faults");
        hipPointerAttribute_t at{};
        CK(hipPointerGetAttributes(&at, lr));
        printf("(h) hipMalloc attributes: type %d device %d devicePointer %p hostPointer %p isManaged %d allocationFlags %u\n",
               (int)at.type, at.device, at.devicePointer, at.hostPointer, at.isManaged, at.allocationFlags);
        if (ok) {   // (i)
            hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, lr, nrec);
            CK(hipDeviceSynchronize());
            uint64_t x = 5;
            int64_t bad = 0;
            const int n = 200000;
            const double t0 = now_s();
            for (int i = 0; i < n; ++i) {
                x = x * 6364136223846793005ull + 1442695040888963407ull;
                const int64_t k = (int64_t)((x >> 36) % (uint64_t)nrec);
                const __m128d v = _mm_load_pd(reinterpret_cast<const double*>(lr + k));
                double o[2];
                _mm_storeu_pd(o, v);
                bad += (o[0] != (double)k) || (o[1] != 1.0);
            }
            const double el = now_s() - t0;
            printf("(i) host 16-B load of a hipMalloc record: %.2f us/read -> %.0f reads/s, %lld of %d values wrong\n",
                   1e6 * el / n, n / el, (long long)bad, n);
        }
    }
    // (k) concurrent host loads
    for (int nt : {1, 4, 16}) {
        const int per = 50000;
        std::vector<std::thread> th;
        const double t0 = now_s();
        for (int k = 0; k < nt; ++k)
            th.emplace_back([=] {
                uint64_t x = 77 + k;
                double acc = 0.0;
                for (int i = 0; i < per; ++i) {
                    x = x * 6364136223846793005ull + 1442695040888963407ull;
                    const __m128d v = _mm_load_pd(reinterpret_cast<const double*>(lr + (int64_t)((x >> 36) % (uint64_t)nrec)));
                    double o[2];
                    _mm_storeu_pd(o, v);
                    acc += o[0];
                }
                if (acc == -1.0) printf("x");
            });
        for (auto& x : th) x.join();
        const double el = now_s() - t0;
        printf("(k) host loads, %2d threads: %.0f reads/s in all\n", nt, nt * per / el);
    }
    // (l) service wave, several callers
    {
        Slot* h = nullptr;
        int* stop = nullptr;
        CK(hipHostMalloc((void**)&h, sizeof(Slot) * 64, hipHostMallocMapped | hipHostMallocCoherent));
        CK(hipHostMalloc((void**)&stop, 64, hipHostMallocMapped | hipHostMallocCoherent));
        Slot* hd = nullptr;
        int* sd = nullptr;
        CK(hipHostGetDevicePointer((void**)&hd, h, 0));
        CK(hipHostGetDevicePointer((void**)&sd, stop, 0));
        for (int nt : {1, 4, 16}) {
            memset((void*)h, 0, sizeof(Slot) * 64);
            *stop = 0;
            std::atomic_thread_fence(std::memory_order_seq_cst);
            hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, st, hd, 64, lr, sd, 200000000LL);
            const int per = 20000;
            std::vector<std::thread> th;
            std::atomic<int> late{0};
            const double t0 = now_s();
            for (int k = 0; k < nt; ++k)
                th.emplace_back([&, k] {
                    Slot* sl = &h[k];
                    uint64_t x = 99 + k;
                    for (int i = 0; i < per; ++i) {
                        x = x * 6364136223846793005ull + 1442695040888963407ull;
                        const unsigned long long seq = (unsigned long long)i + 1;
                        __atomic_store_n(&sl->s, (int32_t)((x >> 36) % (uint64_t)nrec), __ATOMIC_RELAXED);
                        __atomic_store_n(&sl->req, seq, __ATOMIC_RELEASE);
                        const double tl = now_s() + 1.0;
                        while (__atomic_load_n(&sl->done, __ATOMIC_ACQUIRE) != seq)
                            if (now_s() > tl) {
                                late++;
                                return;
                            }
                    }
                });
            for (auto& x : th) x.join();
            const double el = now_s() - t0;
            __atomic_store_n(stop, 1, __ATOMIC_SEQ_CST);
            CK(hipStreamSynchronize(st));
            printf("(l) service wave, %2d callers: %.0f calls/s in all%s\n", nt, nt * per / el, late ? " (some timed out)" : "");
        }
        CK(hipHostFree(h));
        CK(hipHostFree(stop));
    }
    // (j) mirror copies
    {
        const size_t bytes = (size_t)8 << 30;
        char* dsrc = nullptr;
        CK(hipMalloc(&dsrc, bytes));
        CK(hipMemset(dsrc, 1, bytes));
        char* m = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        madvise(m, bytes, MADV_HUGEPAGE);
        {
            std::vector<std::thread> th;
            for (int k = 0; k < 16; ++k)
                th.emplace_back([=] { for (size_t i = bytes * k / 16; i < bytes * (k + 1) / 16; i += 4096) m[i] = 0; });
            for (auto& x : th) x.join();
        }
        double t0 = now_s();
        CK(hipHostRegister(m, bytes, hipHostRegisterDefault));
        const double reg = now_s() - t0;
        CK(hipDeviceSynchronize());
        t0 = now_s();
        const size_t chunk = (size_t)256 << 20;
        for (size_t o = 0; o < bytes; o += chunk) CK(hipMemcpyAsync(m + o, dsrc + o, chunk, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        const double dma = now_s() - t0;
        t0 = now_s();
        CK(hipHostUnregister(m));
        const double unreg = now_s() - t0;
        printf("(j) hipHostRegister 8 GB %.3f s, DMA into it %.3f s (%.1f GB/s), unregister %.3f s, first byte %d\n", reg,
               dma, bytes / dma / 1e9, unreg, (int)m[12345]);
        // pinned staging (two 256-MB slots) + memcpy on 8 threads
        char* pin[2];
        CK(hipHostMalloc((void**)&pin[0], chunk, hipHostMallocDefault));
        CK(hipHostMalloc((void**)&pin[1], chunk, hipHostMallocDefault));
        hipStream_t s2[2];
        CK(hipStreamCreateWithFlags(&s2[0], hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s2[1], hipStreamNonBlocking));
        t0 = now_s();
        const size_t nch = bytes / chunk;
        for (size_t k = 0; k < nch + 1; ++k) {
            if (k < nch) CK(hipMemcpyAsync(pin[k & 1], dsrc + k * chunk, chunk, hipMemcpyDeviceToHost, s2[k & 1]));
            if (k >= 1) {
                const size_t j = k - 1;
                CK(hipStreamSynchronize(s2[j & 1]));
                std::vector<std::thread> th;
                for (int q = 0; q < 8; ++q)
                    th.emplace_back([=] { memcpy(m + j * chunk + chunk * q / 8, pin[j & 1] + chunk * q / 8, chunk / 8); });
                for (auto& x : th) x.join();
            }
        }
        const double stg = now_s() - t0;
        printf("(j) pinned staging + memcpy on 8 threads: %.3f s (%.1f GB/s)\n", stg, bytes / stg / 1e9);
        munmap(m, bytes);
        CK(hipFree(dsrc));
    }
    CK(hipFree(lr));
    return 0;
}
