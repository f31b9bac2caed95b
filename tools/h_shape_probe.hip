// h_shape_probe.hip -- launch-shape probe for the headline shape (tuning
// evidence, not product code): 2-D f64 accumulate, 4096 rows x 16 KiB, src and
// dst leading dimension 64 KiB, 8 rotating buffer sets (4 GiB), nt loads and
// stores, one block per chunk.  Variants: threads per block (64..1024), vectors
// per thread, 1 or 2 HIP streams.  Every variant runs interleaved rounds of
// `reps` launches between one event pair; GB/s of algorithmic traffic (24 B per
// element).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/h_shape_probe.hip -o tools/h_shape_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#pragma clang fp contract(off)

typedef double v2d __attribute__((ext_vector_type(2)));

#ifndef LD_BYTES
#define LD_BYTES 65536
#endif
constexpr int64_t kLd = LD_BYTES, kRow = 16384, kRows = 4096;

template <int BS, int U, int POL = 3>   // POL bit0: nt loads, bit1: nt stores
__global__ __launch_bounds__(BS) void k_h(const char *src, char *dst, double s) {
    constexpr uint32_t chunk_bytes = BS * U * 16;
    constexpr uint32_t cpr = kRow / chunk_bytes;   // chunks per row (power of two)
    const uint32_t b = blockIdx.x;
    const int64_t r = b / cpr, c = b % cpr;
    const int64_t off = r * kLd + c * chunk_bytes + threadIdx.x * 16;
    const v2d *sp = (const v2d *)(src + off);
    v2d *dp = (v2d *)(dst + off);
    v2d x[U], y[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        if constexpr (POL & 1) {
            x[k] = __builtin_nontemporal_load(sp + k * BS);
            y[k] = __builtin_nontemporal_load(dp + k * BS);
        } else {
            x[k] = sp[k * BS];
            y[k] = dp[k * BS];
        }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        v2d p = x[k] * s;
        if constexpr (POL & 2) __builtin_nontemporal_store(y[k] + p, dp + k * BS);
        else dp[k * BS] = y[k] + p;
    }
}

typedef void (*Launch)(const char *, char *, hipStream_t);
template <int BS, int U, int POL = 3>
static void launch(const char *s, char *d, hipStream_t st) {
    const uint32_t blocks = (uint32_t)(kRows * kRow / (BS * U * 16));
    hipLaunchKernelGGL((k_h<BS, U, POL>), dim3(blocks), dim3(BS), 0, st, s, d, 0.7071067811865476);
}

struct Variant { std::string name; Launch fn; int nstreams; std::vector<double> gbs; };

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const size_t span = (size_t)(kRows - 1) * kLd + kRow;
    std::vector<char *> S, D;
    for (int i = 0; i < 8; ++i) {
        char *a, *b;
        CK(hipMalloc(&a, span));
        CK(hipMalloc(&b, span));
        CK(hipMemset(a, 0, span));
        CK(hipMemset(b, 0, span));
        S.push_back(a);
        D.push_back(b);
    }
    hipStream_t st[2];
    CK(hipStreamCreate(&st[0]));
    CK(hipStreamCreate(&st[1]));
    std::vector<Variant> V = {
        {"bs256_u1", launch<256, 1>, 1, {}}, {"bs64_u1", launch<64, 1>, 1, {}},
        {"bs128_u1", launch<128, 1>, 1, {}}, {"bs512_u1", launch<512, 1>, 1, {}},
        {"bs1024_u1", launch<1024, 1>, 1, {}}, {"bs256_u2", launch<256, 2>, 1, {}},
        {"bs64_u4", launch<64, 4>, 1, {}}, {"bs128_u2", launch<128, 2>, 1, {}},
        {"bs256_u1_2streams", launch<256, 1>, 2, {}}, {"bs512_u1_2streams", launch<512, 1>, 2, {}},
        {"bs1024_u1_2streams", launch<1024, 1>, 2, {}},
        {"bs64_u1_2streams", launch<64, 1>, 2, {}},
        {"bs64_u1_2streams_plainloads", launch<64, 1, 2>, 2, {}},
        {"bs64_u1_2streams_plainstores", launch<64, 1, 1>, 2, {}},
        {"bs64_u1_2streams_plain", launch<64, 1, 0>, 2, {}},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double alg = 3.0 * kRows * kRow;
    for (int r = 0; r <= rounds; ++r) {
        for (auto &v : V) {
            CK(hipEventRecord(e0, st[0]));
            if (v.nstreams == 2) CK(hipStreamWaitEvent(st[1], e0, 0));
            for (int i = 0; i < reps; ++i) v.fn(S[i % 8], D[i % 8], st[i % v.nstreams]);
            if (v.nstreams == 2) {
                hipEvent_t j;
                CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
                CK(hipEventRecord(j, st[1]));
                CK(hipStreamWaitEvent(st[0], j, 0));
                CK(hipEventDestroy(j));
            }
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) v.gbs.push_back(alg * reps / (ms * 1e-3) / 1e9);
        }
    }
    for (auto &v : V) {
        std::sort(v.gbs.begin(), v.gbs.end());
        printf("{\"variant\": \"%s\", \"reps\": %d, \"GBps_median\": %.1f, \"GBps_min\": %.1f, \"GBps_max\": %.1f}\n",
               v.name.c_str(), reps, v.gbs[v.gbs.size() / 2], v.gbs.front(), v.gbs.back());
    }
    return 0;
}
