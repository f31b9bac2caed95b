// granule_probe.hip -- what the HBM side moves when a kernel touches only part of
// every 128-byte line (rows <= 64 B read 0.34 of peak with
// FETCH_SIZE ~2x algorithmic, but FETCH_SIZE counts every read request as 64 B on
// gfx950, so the counter alone cannot say whether half-line reads fetch 64 or 128 B).
// Timing decides it: the same number of touched bytes spread as the first G bytes of
// every P-byte piece, over 4 GiB (beyond the 256 MiB MALL), 16 B per lane,
// non-temporal.  If a 64-of-128 read takes as long as reading the whole span, the
// fetch is line-granular.
//   modes: r  = read only (one value per wave stored to keep the loads)
//          w  = write only
//          a  = accumulate (read src + read dst + write dst: the strided _acc pattern)
// Output: one JSON line per (mode, G, P): touched GB/s and span GB/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

// piece k covers bytes [k*P, k*P + G); lane i of the grid handles one 16-byte vector
__global__ __launch_bounds__(256) void k_read(const char *p, uint64_t nvec, uint32_t vpp, uint32_t P, uint32_t *sink) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    const uint64_t piece = i / vpp, v = i % vpp;
    const v4 x = __builtin_nontemporal_load(reinterpret_cast<const v4 *>(p + piece * P + v * 16));
    const uint32_t s = x.x ^ x.y ^ x.z ^ x.w;
    if (s == 0x9e3779b9u) sink[0] = s;   // practically never: keeps the load alive
}

__global__ __launch_bounds__(256) void k_write(char *p, uint64_t nvec, uint32_t vpp, uint32_t P) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    const uint64_t piece = i / vpp, v = i % vpp;
    v4 x = {(uint32_t)i, 1u, 2u, 3u};
    __builtin_nontemporal_store(x, reinterpret_cast<v4 *>(p + piece * P + v * 16));
}

__global__ __launch_bounds__(256) void k_acc(const char *s, char *d, uint64_t nvec, uint32_t vpp, uint32_t P,
                                             double a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    const uint64_t off = (i / vpp) * P + (i % vpp) * 16;
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 x = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(s + off));
    d2 y = __builtin_nontemporal_load(reinterpret_cast<const d2 *>(d + off));
    y.x = y.x + x.x * a;
    y.y = y.y + x.y * a;
    __builtin_nontemporal_store(y, reinterpret_cast<d2 *>(d + off));
}

int main(int argc, char **argv) {
    const size_t span = (size_t)4 << 30;   // per buffer, beyond the MALL
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    char *a = nullptr, *b = nullptr;
    uint32_t *sink = nullptr;
    CK(hipMalloc(&a, span));
    CK(hipMalloc(&b, span));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, span));
    CK(hipMemset(b, 2, span));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg { char mode; uint32_t G, P; };
    std::vector<Cfg> cfgs;
    for (char m : {'r', 'w', 'a'}) {
        cfgs.push_back({m, 128, 128});   // whole lines
        cfgs.push_back({m, 64, 128});    // half lines (a 64-B row at a 128-B pitch)
        cfgs.push_back({m, 32, 128});
        cfgs.push_back({m, 64, 256});
        cfgs.push_back({m, 128, 256});
    }
    for (int round = 0; round < 2; ++round) {   // round 0: warm-up, not printed
        for (const Cfg &c : cfgs) {
            // the same TOUCHED bytes for every configuration: 1 GiB per buffer
            const uint64_t touched = 1ull << 30;
            const uint64_t pieces = touched / c.G;
            if (pieces * c.P > span) continue;
            const uint32_t vpp = c.G / 16;
            const uint64_t nvec = pieces * vpp;
            const dim3 grid((unsigned)((nvec + 255) / 256)), block(256);
            std::vector<float> ms;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                if (c.mode == 'r') hipLaunchKernelGGL(k_read, grid, block, 0, 0, a, nvec, vpp, c.P, sink);
                else if (c.mode == 'w') hipLaunchKernelGGL(k_write, grid, block, 0, 0, a, nvec, vpp, c.P);
                else hipLaunchKernelGGL(k_acc, grid, block, 0, 0, a, b, nvec, vpp, c.P, 0.5);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t = 0;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const double t = ms[ms.size() / 2] * 1e-3;
            const double streams = c.mode == 'a' ? 3.0 : 1.0;   // acc: src read, dst read, dst write
            if (round)
                printf("{\"mode\": \"%c\", \"G\": %u, \"P\": %u, \"ms\": %.3f, \"touched_GBps\": %.1f, "
                       "\"span_GBps\": %.1f}\n",
                       c.mode, c.G, c.P, t * 1e3, streams * touched / t / 1e9,
                       streams * (double)(pieces * c.P) / t / 1e9);
        }
    }
    return 0;
}
