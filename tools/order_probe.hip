// order_probe.hip -- block->work order for the headline shape at several leading
// dimensions (tuning evidence, not product code).  2-D f64 accumulate, 4096 rows
// x 16 KiB, one-wave blocks of one 16-byte vector per lane (1 KiB chunks), nt
// loads/stores, 8 rotating buffer sets, 2 HIP streams.  Orders (block b):
//   rowmajor : row = b / 16, chunk = b % 16 (the library's k_rows2d)
//   colmajor : chunk = b / rows, row = b % rows
//   bandT    : bands of T rows; inside a band chunk-major (chunk = i / T, row = band*T + i % T)
//   xcd      : XCD x (= b % 8) takes the contiguous item range [x*items/8, (x+1)*items/8)
// GB/s of algorithmic traffic (24 B per element).  Usage: order_probe LD_ELEMS...
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/order_probe.hip -o tools/order_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#pragma clang fp contract(off)

typedef double v2d __attribute__((ext_vector_type(2)));
constexpr int64_t kRow = 16384, kRows = 4096, kCpr = kRow / 1024;
constexpr uint32_t kItems = (uint32_t)(kRows * kCpr);

template <int ORDER>
__global__ __launch_bounds__(64) void k_ord(const char *src, char *dst, int64_t ld, double s, uint32_t T) {
    const uint32_t b = blockIdx.x;
    uint32_t row, chunk;
    if constexpr (ORDER == 0) {
        row = b / kCpr;
        chunk = b % kCpr;
    } else if constexpr (ORDER == 1) {
        chunk = b / kRows;
        row = b % kRows;
    } else if constexpr (ORDER == 2) {
        const uint32_t per = T * kCpr, band = b / per, i = b % per;
        chunk = i / T;
        row = band * T + i % T;
    } else {
        const uint32_t it = (b & 7u) * (kItems / 8) + (b >> 3);
        row = it / kCpr;
        chunk = it % kCpr;
    }
    const int64_t off = (int64_t)row * ld + chunk * 1024 + threadIdx.x * 16;
    const v2d x = __builtin_nontemporal_load((const v2d *)(src + off));
    const v2d y = __builtin_nontemporal_load((const v2d *)(dst + off));
    __builtin_nontemporal_store(y + x * s, (v2d *)(dst + off));
}

typedef void (*Launch)(const char *, char *, int64_t, hipStream_t, uint32_t);
template <int ORDER>
static void launch(const char *s, char *d, int64_t ld, hipStream_t st, uint32_t T) {
    hipLaunchKernelGGL((k_ord<ORDER>), dim3(kItems), dim3(64), 0, st, s, d, ld, 0.7071067811865476, T);
}

struct Variant { std::string name; Launch fn; uint32_t T; std::vector<double> gbs; };

int main(int argc, char **argv) {
    std::vector<int64_t> lds;
    for (int i = 1; i < argc; ++i) lds.push_back(atoll(argv[i]) * 8);
    if (lds.empty()) lds = {65536};
    const int reps = 120, rounds = 5;
    const int64_t maxld = *std::max_element(lds.begin(), lds.end());
    const size_t span = (size_t)(kRows - 1) * maxld + kRow;
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
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double alg = 3.0 * kRows * kRow;
    for (int64_t ld : lds) {
        std::vector<Variant> V = {
            {"rowmajor", launch<0>, 0, {}}, {"colmajor", launch<1>, 0, {}}, {"band8", launch<2>, 8, {}},
            {"band32", launch<2>, 32, {}},  {"band128", launch<2>, 128, {}}, {"xcd", launch<3>, 0, {}},
        };
        for (int r = 0; r <= rounds; ++r) {
            for (auto &v : V) {
                CK(hipEventRecord(e0, st[0]));
                CK(hipStreamWaitEvent(st[1], e0, 0));
                for (int i = 0; i < reps; ++i) v.fn(S[i % 8], D[i % 8], ld, st[i % 2], v.T);
                hipEvent_t j;
                CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
                CK(hipEventRecord(j, st[1]));
                CK(hipStreamWaitEvent(st[0], j, 0));
                CK(hipEventDestroy(j));
                CK(hipEventRecord(e1, st[0]));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) v.gbs.push_back(alg * reps / (ms * 1e-3) / 1e9);
            }
        }
        for (auto &v : V) {
            std::sort(v.gbs.begin(), v.gbs.end());
            printf("{\"ld_elems\": %lld, \"order\": \"%s\", \"GBps_median\": %.1f, \"GBps_min\": %.1f, \"GBps_max\": %.1f}\n",
                   (long long)(ld / 8), v.name.c_str(), v.gbs[v.gbs.size() / 2], v.gbs.front(), v.gbs.back());
        }
        fflush(stdout);
    }
    return 0;
}
