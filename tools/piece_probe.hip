// piece_probe.hip -- the read roofline of a column reduction's access pattern:
// 2048 rows of 64 KiB (128 MiB, three rotating copies = 384 MiB, beyond the MALL),
// each workgroup reading PIECE contiguous bytes of every row of a slice of rows
// (16 B per lane, 256 lanes, 16 loads in flight per lane), summing into registers.
// Sweeps the piece size (256 B .. 4 KiB) and the rows per workgroup.  What the column
// kernels can reach is bounded by the row this gives for their piece size
// (k_ordered_cols_lds reads 256-byte pieces, k_cols_sum 4 KiB).
// hipcc --offload-arch=gfx950 -O3 -o tools/piece_probe tools/piece_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            printf("%s -> %s\n", #x, hipGetErrorString(e_));                           \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef uint32_t V4 __attribute__((ext_vector_type(4)));
constexpr int kRows = 2048, kRowBytes = 65536;

__global__ __launch_bounds__(256) void k_pieces(const char *src, uint32_t piece, uint32_t R, uint32_t *out) {
    const uint32_t lanes_per_row = piece / 16u, rows_per_instr = 256u / lanes_per_row;
    const uint32_t pl = threadIdx.x % lanes_per_row, ri = threadIdx.x / lanes_per_row;
    const uint64_t xo = (uint64_t)blockIdx.x * piece + pl * 16u;
    const uint32_t rb = blockIdx.y * R, re = min(rb + R, (uint32_t)kRows);
    V4 acc = {0, 0, 0, 0};
    for (uint32_t r0 = rb; r0 < re; r0 += 16u * rows_per_instr) {
        V4 x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t r = min(r0 + (uint32_t)k * rows_per_instr + ri, re - 1u);
            x[k] = __builtin_nontemporal_load(reinterpret_cast<const V4 *>(src + (uint64_t)r * kRowBytes + xo));
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) acc += x[k];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) out[threadIdx.x] = acc.x;   // keeps the loads alive
}

int main() {
    const size_t bytes = (size_t)kRows * kRowBytes;
    char *src[3];
    for (int k = 0; k < 3; ++k) {
        CK(hipMalloc(&src[k], bytes));
        CK(hipMemset(src[k], k + 1, bytes));
    }
    uint32_t *out;
    CK(hipMalloc(&out, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t pieces[] = {64, 128, 256, 512, 1024, 2048, 4096};
    const uint32_t rows_per_wg[] = {2048, 1024, 512, 256, 128, 64, 32};
    for (uint32_t piece : pieces) {
        for (uint32_t R : rows_per_wg) {
            if (R < 16u * (256u / (piece / 16u))) continue;   // a slice shorter than one round of loads
            const dim3 grid(kRowBytes / piece, kRows / R);
            for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_pieces, grid, dim3(256), 0, 0, src[i % 3], piece, R, out);
            CK(hipEventRecord(e0, 0));
            const int n = 12;
            for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_pieces, grid, dim3(256), 0, 0, src[i % 3], piece, R, out);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / n;
            printf("{\"piece\": %u, \"rows_per_wg\": %u, \"workgroups\": %u, \"us\": %.1f, \"GBps\": %.0f}\n", piece, R,
                   grid.x * grid.y, us, bytes / (us * 1e-6) / 1e9);
            fflush(stdout);
        }
    }
    return 0;
}
