// lds_mark_probe.hip -- where the one-workgroup ordering of k_iov_lds spends its time
// (VERDICT r5 item 3): one 1024-thread workgroup loads n keys into LDS, builds the hash
// table and the repeat marks (iov_lds_mark, the library's own code, included), then
// lists the repeated pairs; lane 0 stamps the wall clock (100 MHz) between the phases.
// n = 1 Ki .. 16 Ki random keys (27-bit), and the same with every key distinct and
// sequential (no probing beyond the first slot).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I ga_amd/csrc \
//        tools/lds_mark_probe.hip -L ga_amd -lga_amd -Wl,-rpath,'$ORIGIN/../ga_amd' -o tools/lds_mark_probe
#include "gaamd_iov.hip"
#include <stdio.h>
#include <random>
#include <vector>

using namespace gaamd;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(1024) void k_mark_probe(const uint32_t *keys_g, uint32_t n, uint64_t *stamps, uint32_t *out) {
    __shared__ uint32_t keys[kIovLdsMax];
    __shared__ uint32_t tab[(1u << kIovLdsLog) / 2];
    __shared__ uint32_t rep[kIovLdsMax / 32];
    const uint32_t t = threadIdx.x;
    if (t == 0) stamps[0] = wall_clock64();
    for (uint32_t w = t; w < (1u << kIovLdsLog) / 2; w += 1024) tab[w] = 0xffffffffu;
    for (uint32_t w = t; w < kIovLdsMax / 32; w += 1024) rep[w] = 0;
    for (uint32_t i = t; i < n; i += 1024) keys[i] = keys_g[i];
    __syncthreads();
    if (t == 0) stamps[1] = wall_clock64();
    iov_lds_mark(keys, tab, rep, n);
    if (t == 0) stamps[2] = wall_clock64();
    uint32_t c = 0;
    for (uint32_t w = t; w < (n + 31) / 32; w += 1024) c += __builtin_popcount(rep[w]);
    atomicAdd(out, c);
    __syncthreads();
    if (t == 0) stamps[3] = wall_clock64();
}

int main() {
    uint32_t *kd, *out;
    uint64_t *st;
    CK(hipMalloc(&kd, 4 * kIovLdsMax));
    CK(hipMalloc(&out, 4));
    CK(hipMalloc(&st, 64));
    std::mt19937 rng(5);
    for (int mode = 0; mode < 2; ++mode) {
        for (uint32_t n : {1024u, 2048u, 4096u, 8192u, 16384u}) {
            std::vector<uint32_t> k(n);
            for (uint32_t i = 0; i < n; ++i) k[i] = mode == 0 ? (rng() & ((1u << 27) - 1)) : i;
            CK(hipMemcpy(kd, k.data(), 4 * n, hipMemcpyHostToDevice));
            uint64_t best[3] = {~0ull, ~0ull, ~0ull};
            uint32_t reps = 0;
            for (int r = 0; r < 5; ++r) {
                CK(hipMemset(out, 0, 4));
                hipLaunchKernelGGL(k_mark_probe, dim3(1), dim3(1024), 0, 0, kd, n, st, out);
                CK(hipDeviceSynchronize());
                uint64_t s[4];
                CK(hipMemcpy(s, st, 32, hipMemcpyDeviceToHost));
                CK(hipMemcpy(&reps, out, 4, hipMemcpyDeviceToHost));
                for (int p = 0; p < 3; ++p) best[p] = std::min(best[p], s[p + 1] - s[p]);
            }
            printf("{\"probe\": \"lds_mark\", \"keys\": \"%s\", \"n\": %u, \"load_us\": %.2f, \"mark_us\": %.2f, "
                   "\"list_us\": %.2f, \"repeated\": %u}\n", mode ? "sequential" : "random", n, best[0] / 100.0,
                   best[1] / 100.0, best[2] / 100.0, reps);
            fflush(stdout);
        }
    }
    return 0;
}
