// persist_probe.hip -- software-pipelined persistent grids for the headline shape
// (tuning evidence, not product code).  2-D f64 accumulate, 4096 rows x 16 KiB,
// src and dst leading dimension 64 KiB, 8 rotating buffer sets, nt loads/stores.
//   base   : one 1 KiB chunk per one-wave block (the library's k_rows2d shape)
//   pers   : G blocks of BS threads loop over the chunks (chunk = block + k*G);
//            the loads of the next D chunks are issued before the current chunk's
//            store, so a wave always has D+1 chunks of loads in flight and no
//            block relaunch gap
// Variants run interleaved, `reps` launches between one event pair per round;
// GB/s of algorithmic traffic (24 B per element).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/persist_probe.hip -o tools/persist_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#pragma clang fp contract(off)

typedef double v2d __attribute__((ext_vector_type(2)));

constexpr int64_t kLd = 65536, kRow = 16384, kRows = 4096;

template <int BS>
__global__ __launch_bounds__(BS) void k_base(const char *src, char *dst, double s) {
    constexpr uint32_t cpr = kRow / (BS * 16);
    const uint32_t b = blockIdx.x;
    const int64_t off = (int64_t)(b / cpr) * kLd + (b % cpr) * (BS * 16) + threadIdx.x * 16;
    const v2d x = __builtin_nontemporal_load((const v2d *)(src + off));
    const v2d y = __builtin_nontemporal_load((const v2d *)(dst + off));
    __builtin_nontemporal_store(y + x * s, (v2d *)(dst + off));
}

template <int BS>
__device__ __forceinline__ int64_t chunk_off(uint32_t c) {
    constexpr uint32_t cpr = kRow / (BS * 16);
    return (int64_t)(c / cpr) * kLd + (c % cpr) * (BS * 16) + threadIdx.x * 16;
}

// D = prefetch depth (chunks in flight beyond the current one)
template <int BS, int D>
__global__ __launch_bounds__(BS) void k_pers(const char *src, char *dst, double s, uint32_t nchunks) {
    const uint32_t G = gridDim.x;
    uint32_t c = blockIdx.x;
    v2d x[D + 1], y[D + 1];
    int64_t off[D + 1];
#pragma unroll
    for (int k = 0; k <= D; ++k) {
        const uint32_t ck = c + k * G;
        off[k] = chunk_off<BS>(ck < nchunks ? ck : c);
        if (ck < nchunks) {
            x[k] = __builtin_nontemporal_load((const v2d *)(src + off[k]));
            y[k] = __builtin_nontemporal_load((const v2d *)(dst + off[k]));
        }
    }
    // ring of D+1 register slots, fully unrolled per step so indices are static
    while (c < nchunks) {
#pragma unroll
        for (int k = 0; k <= D; ++k) {
            if (c >= nchunks) break;
            __builtin_nontemporal_store(y[k] + x[k] * s, (v2d *)(dst + off[k]));
            const uint32_t cn = c + (D + 1) * G;
            if (cn < nchunks) {
                off[k] = chunk_off<BS>(cn);
                x[k] = __builtin_nontemporal_load((const v2d *)(src + off[k]));
                y[k] = __builtin_nontemporal_load((const v2d *)(dst + off[k]));
            }
            c += G;
        }
    }
}

typedef void (*Launch)(const char *, char *, hipStream_t, uint32_t);
// base with `lds` bytes of dynamic LDS per block: caps resident one-wave blocks per CU at 160 KiB / lds
template <int BS>
static void launch_base_lds(const char *s, char *d, hipStream_t st, uint32_t lds) {
    const uint32_t blocks = (uint32_t)(kRows * kRow / (BS * 16));
    hipLaunchKernelGGL((k_base<BS>), dim3(blocks), dim3(BS), lds, st, s, d, 0.7071067811865476);
}
template <int BS>
static void launch_base(const char *s, char *d, hipStream_t st, uint32_t) {
    const uint32_t blocks = (uint32_t)(kRows * kRow / (BS * 16));
    hipLaunchKernelGGL((k_base<BS>), dim3(blocks), dim3(BS), 0, st, s, d, 0.7071067811865476);
}
template <int BS, int D>
static void launch_pers(const char *s, char *d, hipStream_t st, uint32_t G) {
    const uint32_t n = (uint32_t)(kRows * kRow / (BS * 16));
    hipLaunchKernelGGL((k_pers<BS, D>), dim3(G), dim3(BS), 0, st, s, d, 0.7071067811865476, n);
}

struct Variant { std::string name; Launch fn; uint32_t grid; int nstreams; std::vector<double> gbs; };

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
    // correctness: one pers launch vs one base launch from identical inputs
    {
        std::vector<double> h(span / 8);
        for (size_t i = 0; i < h.size(); ++i) h[i] = (double)(i % 1000) * 0.25 - 7.0;
        CK(hipMemcpy(S[0], h.data(), span, hipMemcpyHostToDevice));
        CK(hipMemcpy(D[0], h.data(), span, hipMemcpyHostToDevice));
        CK(hipMemcpy(D[1], h.data(), span, hipMemcpyHostToDevice));
        launch_base<64>(S[0], D[0], 0, 0);
        launch_pers<64, 2>(S[0], D[1], 0, 3000);
        CK(hipDeviceSynchronize());
        std::vector<double> a(span / 8), b(span / 8);
        CK(hipMemcpy(a.data(), D[0], span, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), D[1], span, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < a.size(); ++i) bad += a[i] != b[i];
        fprintf(stderr, "check: %zu mismatches\n", bad);
        if (bad) return 2;
    }
    hipStream_t st[2];
    CK(hipStreamCreate(&st[0]));
    CK(hipStreamCreate(&st[1]));
    std::vector<Variant> V = {
        {"base_bs64_2streams", launch_base<64>, 0, 2, {}},
        {"base_bs64_cap28_lds5632_2streams", launch_base_lds<64>, 5632, 2, {}},
        {"base_bs64_cap24_lds6656_2streams", launch_base_lds<64>, 6656, 2, {}},
        {"base_bs64_cap20_lds8192_2streams", launch_base_lds<64>, 8192, 2, {}},
        {"base_bs64_cap18_lds8960_2streams", launch_base_lds<64>, 8960, 2, {}},
        {"base_bs64_cap16_lds10240_2streams", launch_base_lds<64>, 10240, 2, {}},
        {"base_bs64_cap15_lds10752_2streams", launch_base_lds<64>, 10752, 2, {}},
        {"base_bs64_cap14_lds11520_2streams", launch_base_lds<64>, 11520, 2, {}},
        {"base_bs64_cap13_lds12544_2streams", launch_base_lds<64>, 12544, 2, {}},
        {"base_bs64_cap12_lds13568_2streams", launch_base_lds<64>, 13568, 2, {}},
        {"base_bs64_cap11_lds14848_2streams", launch_base_lds<64>, 14848, 2, {}},
        {"base_bs64_cap10_lds16384_2streams", launch_base_lds<64>, 16384, 2, {}},
        {"base_bs64_cap9_lds18176_2streams", launch_base_lds<64>, 18176, 2, {}},
        {"base_bs64_cap24_lds6656_1stream", launch_base_lds<64>, 6656, 1, {}},
        {"base_bs64_cap16_lds10240_1stream", launch_base_lds<64>, 10240, 1, {}},
        {"base_bs64_cap12_lds13568_1stream", launch_base_lds<64>, 13568, 1, {}},
        {"base_bs128_cap12_lds13568_2streams", launch_base_lds<128>, 13568, 2, {}},
        {"base_bs128_cap8_lds20480_2streams", launch_base_lds<128>, 20480, 2, {}},
        {"base_bs128_cap6_lds27136_2streams", launch_base_lds<128>, 27136, 2, {}},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double alg = 3.0 * kRows * kRow;
    for (int r = 0; r <= rounds; ++r) {
        for (auto &v : V) {
            CK(hipEventRecord(e0, st[0]));
            if (v.nstreams == 2) CK(hipStreamWaitEvent(st[1], e0, 0));
            for (int i = 0; i < reps; ++i) v.fn(S[i % 8], D[i % 8], st[i % v.nstreams], v.grid);
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
