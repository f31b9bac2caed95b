// alloc_probe.hip -- does the rate of a streaming accumulate over a large block depend on
// the allocation (not the kernel)?  C5 at N = 1 (an 8 GiB block) read 0.845 of peak on one
// box and 0.787 on another with the same kernel and grid, and on one box a 4 GiB block
// read 0.787 where 2 and 8 GiB read 0.85 (tools/size_probe.py).  Here: the same
// 16-byte-per-lane axpy (2 reads + 1 write, one-wave blocks, non-temporal) over blocks of
// 1..8 GiB, each size allocated 3 times, with hipMalloc and with hipExtMallocWithFlags(
// hipDeviceMallocContiguous).  One JSON line per (mode, size, try): GB/s of 3 x bytes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(64) void k_axpy(const char *s, char *d, double a) {
    const size_t off = ((size_t)blockIdx.x * 64 + threadIdx.x) * 16;
    const d2 x = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(s + off));
    d2 y = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(d + off));
    y.x = y.x + x.x * a;
    y.y = y.y + x.y * a;
    __builtin_nontemporal_store(y, reinterpret_cast<d2 *>(d + off));
}

int main() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 2; ++mode) {
        for (size_t gib : {1, 2, 4, 8}) {
            const size_t bytes = gib << 30;
            for (int t = 0; t < 3; ++t) {
                char *a = nullptr, *b = nullptr;
                if (mode == 0) {
                    CK(hipMalloc(&a, bytes));
                    CK(hipMalloc(&b, bytes));
                } else {
                    if (hipExtMallocWithFlags((void **)&a, bytes, hipDeviceMallocContiguous) != hipSuccess ||
                        hipExtMallocWithFlags((void **)&b, bytes, hipDeviceMallocContiguous) != hipSuccess) {
                        (void)hipGetLastError();
                        printf("{\"mode\": \"contiguous\", \"GiB\": %zu, \"try\": %d, \"error\": \"allocation refused\"}\n", gib, t);
                        if (a) CK(hipFree(a));
                        if (b) CK(hipFree(b));
                        continue;
                    }
                }
                CK(hipMemset(a, 0, bytes));
                CK(hipMemset(b, 0, bytes));
                const unsigned blocks = (unsigned)(bytes / 1024);
                std::vector<float> ms;
                for (int r = 0; r < 8; ++r) {
                    CK(hipEventRecord(e0, 0));
                    hipLaunchKernelGGL(k_axpy, dim3(blocks), dim3(64), 0, 0, a, b, 0.5);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float m = 0;
                    CK(hipEventElapsedTime(&m, e0, e1));
                    if (r >= 2) ms.push_back(m);
                }
                std::sort(ms.begin(), ms.end());
                const double med = ms[ms.size() / 2] * 1e-3;
                printf("{\"mode\": \"%s\", \"GiB\": %zu, \"try\": %d, \"a_mod_1G\": %zu, \"b_minus_a\": %lld, "
                       "\"ms\": %.3f, \"GBps\": %.1f, \"frac\": %.4f}\n",
                       mode ? "contiguous" : "hipMalloc", gib, t, (size_t)((uintptr_t)a % (1ull << 30)),
                       (long long)((intptr_t)b - (intptr_t)a), med * 1e3, 3.0 * bytes / med / 1e9,
                       3.0 * bytes / med / 8e12);
                fflush(stdout);
                CK(hipFree(a));
                CK(hipFree(b));
            }
        }
    }
    return 0;
}
