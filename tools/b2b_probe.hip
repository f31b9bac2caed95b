// b2b_probe.hip -- are back-to-back read-modify-write kernels on ONE stream
// ordered and coherent?  The owner's progress thread lost whole io-vector
// accumulates (a request's contribution missing, never an extra one) with
// COMEX_AMD_STREAMS=1 and no other writer in the process; this probe isolates
// the pattern: K tiny one-block kernels, each dst[i] += src[i] (i < n), on one
// stream, launched as fast as the host can; the result must be exactly K.
//
// variants (argv[1]):
//   plain    : hipMalloc'd dst
//   ipc      : dst exported with hipIpcGetMemHandle first (as comex_malloc segments are)
//   events   : an event recorded after every launch, polled by the launching thread
//   thread   : launches from a second host thread, the first polls events
//   fence    : plain, with a system-scope acquire at the start of each kernel
//   nt       : plain, dst loads/stores non-temporal
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/b2b_probe tools/b2b_probe.hip -lpthread
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                                         \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
            exit(2);                                                                                  \
        }                                                                                             \
    } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void k_rmw(double *dst, const double *src, int n) {
    if constexpr (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const int i = threadIdx.x;
    if (i < n) {
        if constexpr (MODE == 2) {
            const double v = __builtin_nontemporal_load(dst + i) + __builtin_nontemporal_load(src + i);
            __builtin_nontemporal_store(v, dst + i);
        } else {
            dst[i] = dst[i] + src[i];
        }
    }
}

int main(int argc, char **argv) {
    const std::string v = argc > 1 ? argv[1] : "plain";
    const int K = argc > 2 ? atoi(argv[2]) : 20000;
    const int trials = argc > 3 ? atoi(argv[3]) : 5;
    const int n = 100;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamDefault));
    double *dst, *src;
    CK(hipMalloc(&dst, 1 << 20));
    CK(hipMalloc(&src, 1 << 20));
    if (v == "ipc") {
        hipIpcMemHandle_t h;
        CK(hipIpcGetMemHandle(&h, dst));
    }
    std::vector<double> ones(n, 1.0), out(n);
    CK(hipMemcpy(src, ones.data(), n * 8, hipMemcpyHostToDevice));
    int bad_trials = 0;
    for (int t = 0; t < trials; ++t) {
        CK(hipMemset(dst, 0, n * 8));
        CK(hipDeviceSynchronize());
        auto launch = [&](int k) {
            if (v == "fence") hipLaunchKernelGGL(k_rmw<1>, dim3(1), dim3(256), 0, st, dst, src, n);
            else if (v == "nt") hipLaunchKernelGGL(k_rmw<2>, dim3(1), dim3(256), 0, st, dst, src, n);
            else hipLaunchKernelGGL(k_rmw<0>, dim3(1), dim3(256), 0, st, dst, src, n);
            (void)k;
        };
        if (v == "events" || v == "thread") {
            std::vector<hipEvent_t> pool;
            std::deque<hipEvent_t> inflight;
            std::atomic<int> launched{0};
            auto poll = [&] {
                while (!inflight.empty()) {
                    hipError_t e = hipEventQuery(inflight.front());
                    if (e == hipErrorNotReady) break;
                    CK(e);
                    pool.push_back(inflight.front());
                    inflight.pop_front();
                }
            };
            if (v == "events") {
                for (int k = 0; k < K; ++k) {
                    launch(k);
                    hipEvent_t ev;
                    if (pool.empty()) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                    else { ev = pool.back(); pool.pop_back(); }
                    CK(hipEventRecord(ev, st));
                    inflight.push_back(ev);
                    poll();
                }
            } else {
                // a second thread launches; this one polls a stream query meanwhile
                std::thread th([&] {
                    for (int k = 0; k < K; ++k) {
                        launch(k);
                        launched.store(k + 1, std::memory_order_release);
                    }
                });
                while (launched.load(std::memory_order_acquire) < K) (void)hipStreamQuery(st);
                th.join();
            }
            CK(hipStreamSynchronize(st));
            poll();
        } else {
            for (int k = 0; k < K; ++k) launch(k);
        }
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(out.data(), dst, n * 8, hipMemcpyDeviceToHost));
        int bad = 0;
        double mn = 1e300;
        for (int i = 0; i < n; ++i) {
            if (out[i] != (double)K) ++bad;
            mn = std::min(mn, out[i]);
        }
        if (bad) ++bad_trials;
        printf("{\"variant\": \"%s\", \"K\": %d, \"trial\": %d, \"bad_elems\": %d, \"min\": %.0f}\n", v.c_str(), K,
               t, bad, mn);
        fflush(stdout);
    }
    printf("{\"variant\": \"%s\", \"bad_trials\": %d, \"trials\": %d}\n", v.c_str(), bad_trials, trials);
    return 0;
}
