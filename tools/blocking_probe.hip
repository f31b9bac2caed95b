// blocking_probe.hip -- what a BLOCKING accumulate can reach on one MI355X, with no
// library around it (the bench's blocking_api line).
//
// The headline patch (f64, 2048 x 4096 elements, ld 8192, dst += a*src, 3 x 64 MiB of
// algorithmic traffic) as one minimal kernel of one-wave blocks (16 B per lane), issued
// and completed one call at a time the ways a blocking call can be completed:
//   stream  calls back to back, one synchronize at the end (the streamed reference)
//   sync    launch + hipStreamSynchronize per call
//   flag    launch + a one-lane kernel storing a sequence number into pinned host
//           memory (system-scope release), the host spinning on it (the library's
//           blocking wait, sched.cpp sched_wait_flag)
//   fused   the accumulate kernel itself publishes completion: each workgroup adds
//           one to a counter of its XCD (blockIdx % 8), the last of an XCD adds one
//           to a top counter, and the last of those stores the sequence number into
//           pinned host memory -- no second dispatch; each count a release at agent
//           scope (every workgroup's stores visible first)
//   fused_relaxed  the same with relaxed counts (loads done, stores maybe in flight)
//   event   launch + hipEventRecord, the host spinning on hipEventQuery
//   flag_relaxed  as flag with a relaxed system-scope store (no L2 write-back)
// argv[2] = "spin": hipSetDeviceFlags(hipDeviceScheduleSpin) first (the runtime's own
// waits spin instead of yielding / sleeping on an interrupt)
// Three buffer sets rotate (MALL defeat).  Prints per-call medians and the fraction
// of the 8 TB/s HBM peak.
//
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/blocking_probe tools/blocking_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("%s -> %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);           \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef double V2 __attribute__((ext_vector_type(2)));
constexpr int kCols = 2048, kRows = 4096, kLd = 8192;
constexpr int kChunks = kCols / 128;   // 64 lanes x 2 doubles per block

template <int FUSED>
__global__ __launch_bounds__(64) void k_acc(const double *src, double *dst, double a, uint32_t *ctr,
                                            uint64_t *flag, uint64_t seq) {
    const uint32_t b = blockIdx.x, row = b / kChunks, ch = b % kChunks;
    const V2 *s = reinterpret_cast<const V2 *>(src + (size_t)row * kLd) + ch * 64 + threadIdx.x;
    V2 *d = reinterpret_cast<V2 *>(dst + (size_t)row * kLd) + ch * 64 + threadIdx.x;
    const V2 x = __builtin_nontemporal_load(s);
    V2 y = __builtin_nontemporal_load(d);
    y.x = y.x + a * x.x;
    y.y = y.y + a * x.y;
    __builtin_nontemporal_store(y, d);
    if constexpr (FUSED) {
        if (threadIdx.x == 0) {
            const uint32_t x8 = b & 7u;
            const uint32_t per = gridDim.x / 8u + (x8 < gridDim.x % 8u ? 1u : 0u);
            // release: this workgroup's stores are visible before its count
            const uint32_t t = FUSED == 1
                ? __hip_atomic_fetch_add(ctr + 16u * x8, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT)
                : __hip_atomic_fetch_add(ctr + 16u * x8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t == per - 1u) {
                __hip_atomic_store(ctr + 16u * x8, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t u = __hip_atomic_fetch_add(ctr + 128u, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                if (u == 7u) {
                    __hip_atomic_store(ctr + 128u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_flag(uint64_t *flag, uint64_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(64) void k_flag_relaxed(uint64_t *flag, uint64_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 200;
    if (argc > 2 && !strcmp(argv[2], "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    hipEvent_t ev;
    const size_t bytes = (size_t)kRows * kLd * 8;
    double *src[3], *dst[3];
    for (int k = 0; k < 3; ++k) {
        CK(hipMalloc(&src[k], bytes));
        CK(hipMalloc(&dst[k], bytes));
        CK(hipMemset(src[k], 0, bytes));
        CK(hipMemset(dst[k], 0, bytes));
    }
    uint32_t *ctr;
    CK(hipMalloc(&ctr, 256 * sizeof(uint32_t)));
    CK(hipMemset(ctr, 0, 256 * sizeof(uint32_t)));
    uint64_t *flag_h, *flag_d;
    CK(hipHostMalloc((void **)&flag_h, 64, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void **)&flag_d, flag_h, 0));
    *flag_h = 0;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const dim3 grid(kRows * kChunks), blk(64);
    const double alg = 3.0 * kRows * kCols * 8;
    uint64_t seq = 0;
    auto spin = [&](uint64_t v) {
        while (__atomic_load_n((volatile uint64_t *)flag_h, __ATOMIC_ACQUIRE) < v) __builtin_ia32_pause();
    };
    const char *modes[] = {"stream", "sync", "flag", "fused", "fused_relaxed", "event", "flag_relaxed"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int m = 0; m < 7; ++m) {
            if (m == 3 || m == 4) continue;   // the fused forms: measured once, 164-1660 us per call
            std::vector<double> t;
            // warm-up
            for (int i = 0; i < 5; ++i)
                hipLaunchKernelGGL(k_acc<0>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, 0);
            CK(hipStreamSynchronize(st));
            if (m == 0) {
                const double t0 = now_us();
                for (int i = 0; i < calls; ++i)
                    hipLaunchKernelGGL(k_acc<0>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, 0);
                CK(hipStreamSynchronize(st));
                t.push_back((now_us() - t0) / calls);
            } else {
                for (int i = 0; i < calls; ++i) {
                    const double t0 = now_us();
                    if (m == 1) {
                        hipLaunchKernelGGL(k_acc<0>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, 0);
                        CK(hipStreamSynchronize(st));
                    } else if (m == 2) {
                        hipLaunchKernelGGL(k_acc<0>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, 0);
                        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, flag_d, ++seq);
                        spin(seq);
                    } else if (m == 3) {
                        hipLaunchKernelGGL(k_acc<1>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, ++seq);
                        spin(seq);
                    } else if (m == 4) {
                        hipLaunchKernelGGL(k_acc<2>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, ++seq);
                        spin(seq);
                    } else if (m == 6) {
                        hipLaunchKernelGGL(k_acc<0>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, 0);
                        hipLaunchKernelGGL(k_flag_relaxed, dim3(1), dim3(64), 0, st, flag_d, ++seq);
                        spin(seq);
                    } else {
                        hipLaunchKernelGGL(k_acc<0>, grid, blk, 0, st, src[i % 3], dst[i % 3], 1.5, ctr, flag_d, 0);
                        CK(hipEventRecord(ev, st));
                        while (hipEventQuery(ev) == hipErrorNotReady) __builtin_ia32_pause();
                    }
                    t.push_back(now_us() - t0);
                }
            }
            CK(hipStreamSynchronize(st));
            std::sort(t.begin(), t.end());
            const double med = t[t.size() / 2], p10 = t[t.size() / 10], p90 = t[t.size() * 9 / 10];
            printf("{\"mode\": \"%s\", \"spin_flag\": %d, \"rep\": %d, \"us_median\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f, "
                   "\"frac_of_8TBs\": %.4f}\n", modes[m], argc > 2 && !strcmp(argv[2], "spin"), rep, med, p10, p90, alg / (med * 1e-6) / 8e12);
            fflush(stdout);
        }
    }
    return 0;
}
