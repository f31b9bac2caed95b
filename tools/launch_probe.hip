// launch_probe.hip -- host cost of one kernel launch on this runtime, with no library:
// an empty kernel launched back to back on one stream, with an 8-byte argument and with
// a 256-byte descriptor (the size of the library's strided descriptor), through
// hipLaunchKernelGGL and through hipModuleLaunchKernel on the function handle
// (hipGetFuncBySymbol, no per-launch lookup of the host stub).  Sets the library's
// per-call issue cost (3.5-4.5 us, tools/small_call_probe.cpp) against the runtime's.
// Build: hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <chrono>
#include <vector>

struct Big {
    unsigned long long w[32];
};

__global__ void k_small(unsigned long long *p) {
    if (p && threadIdx.x == 1u << 20) p[0] = 1;
}
__global__ void k_big(Big b) {
    if (threadIdx.x == 1u << 20) ((unsigned long long *)b.w[0])[0] = b.w[31];
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamDefault));
    hipFunction_t fs, fb;
    CK(hipGetFuncBySymbol(&fs, (const void *)k_small));
    CK(hipGetFuncBySymbol(&fb, (const void *)k_big));
    unsigned long long *nul = nullptr;
    Big b = {};
    // N = 48: the queue never fills, so the host cost alone; N = 4000: the queue fills
    // and the launch rate is what the GPU retires
    for (int N : {48, 4000})
    for (int mode = 0; mode < 4; ++mode) {
        std::vector<double> per;
        for (int rep = 0; rep < (N < 100 ? 200 : 7); ++rep) {
            CK(hipStreamSynchronize(st));
            const double t0 = now_us();
            for (int i = 0; i < N; ++i) {
                if (mode == 0) {
                    hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, st, nul);
                } else if (mode == 1) {
                    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, st, b);
                } else if (mode == 2) {
                    void *args[] = {&nul};
                    CK(hipModuleLaunchKernel(fs, 1, 1, 1, 64, 1, 1, 0, st, args, nullptr));
                } else {
                    void *args[] = {&b};
                    CK(hipModuleLaunchKernel(fb, 1, 1, 1, 64, 1, 1, 0, st, args, nullptr));
                }
            }
            const double t1 = now_us();
            if (rep >= 2) per.push_back((t1 - t0) / N);
        }
        CK(hipStreamSynchronize(st));
        CK(hipGetLastError());
        std::sort(per.begin(), per.end());
        static const char *names[] = {"GGL_8B", "GGL_256B", "module_8B", "module_256B"};
        printf("{\"launch\": \"%s\", \"batch\": %d, \"us_per_launch\": %.2f}\n", names[mode], N,
               per[per.size() / 2]);
    }
    return 0;
}
