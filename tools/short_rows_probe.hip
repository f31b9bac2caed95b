// short_rows_probe.hip -- VERDICT r5 item 4: variants of the flat accumulate kernel on
// short rows (f64, rows of R bytes at a pitch of 2R, 64 MiB of payload, 4 rotating
// buffer sets), to find what raises 64-byte and 128-byte rows toward their
// line-granular bound.  Every variant writes only the patch's bytes and applies the
// library's AccDbl (no FMA).  Per variant: vectors per lane U, block size BS,
// non-temporal loads / stores, and the lane -> vector mapping:
//   MAP 0  consecutive lanes take consecutive vectors (the library's k_flat);
//   MAP 1  a lane takes U vectors of ONE row back to back (U = row vectors);
//   MAP 2  the grid walks the rows in XCD-blocked order: block b's rows come from
//          chunk (b % 8) of the patch, so each XCD's L2 sees one contiguous region.
// Prints one JSON line per (R, variant): us per launch, algorithmic TB/s and the
// fraction of the 8 TB/s peak, and a check that the result is exact against a
// reference computed by the MAP 0 / U 1 variant on a copy.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I ga_amd/csrc \
//        tools/short_rows_probe.hip -o tools/short_rows_probe
#include "gaamd_device.hpp"
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

using namespace gaamd;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int U, int BS, bool NTL, bool NTS, int MAP>
__global__ __launch_bounds__(BS) void k_probe(const char *src, char *dst, int64_t pitch, uint32_t lg_nvec,
                                              uint64_t items, AccDbl op) {
    typedef typename Vec<16>::T V;
    V a[U], b[U];
    char *dps[U];
    uint64_t blk = blockIdx.x;
    if constexpr (MAP == 2) {
        // XCD-blocked: launch order round-robins blocks over the 8 XCDs; give XCD x the
        // x-th eighth of the patch, in order
        const uint64_t nb = gridDim.x, per = nb / 8;
        if (per) blk = (blk % 8) * per + blk / 8;
        if (blk >= nb) blk = blockIdx.x;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        uint64_t g;
        if constexpr (MAP == 1) g = (blk * BS + threadIdx.x) * U + k;
        else g = blk * (uint64_t)(BS * U) + (uint64_t)k * BS + threadIdx.x;
        dps[k] = nullptr;
        if (g < items) {
            const uint64_t row = g >> lg_nvec, v = g & ((1u << lg_nvec) - 1);
            const char *sp = src + row * pitch + v * 16;
            dps[k] = dst + row * pitch + v * 16;
            a[k] = vload<16, NTL>(sp);
            b[k] = vload<16, NTL>(dps[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < U; ++k)
        if (dps[k]) vstore<16, NTS>(dps[k], op.template apply<16>(b[k], a[k]));
}

struct Var {
    const char *name;
    int U, BS;
    void (*launch)(const char *, char *, int64_t, uint32_t, uint64_t, AccDbl, hipStream_t);
};

template <int U, int BS, bool NTL, bool NTS, int MAP>
static void launch_v(const char *s, char *d, int64_t pitch, uint32_t lg, uint64_t items, AccDbl op, hipStream_t st) {
    const uint64_t blocks = (items + BS * U - 1) / (BS * U);
    hipLaunchKernelGGL((k_probe<U, BS, NTL, NTS, MAP>), dim3((uint32_t)blocks), dim3(BS), 0, st, s, d, pitch, lg,
                       items, op);
}

int main(int argc, char **argv) {
    const uint64_t payload = 64ull << 20;
    const int steps = argc > 1 ? atoi(argv[1]) : 40;
    // (row bytes, pitch): short rows at 2 x row, and the headline's 16 KiB rows at ld 8192 f64
    std::vector<std::pair<int, int64_t>> rows_list = {{32, 64}, {64, 128}, {128, 256}, {256, 512}, {512, 1024},
                                                      {1024, 2048}, {2048, 4096}, {16384, 65536}};
    if (argc > 2) {   // "R:P,R:P,..."
        rows_list.clear();
        for (char *tok = strtok(argv[2], ","); tok; tok = strtok(nullptr, ",")) {
            int R = 0;
            long long P = 0;
            if (sscanf(tok, "%d:%lld", &R, &P) == 2) rows_list.push_back({R, (int64_t)P});
        }
    }
    Var vars[] = {
        {"flat_u1_bs64_nt", 1, 64, launch_v<1, 64, true, true, 0>},          // the library's k_flat
        {"flat_u2_bs64_nt", 2, 64, launch_v<2, 64, true, true, 0>},
        {"flat_u4_bs64_nt", 4, 64, launch_v<4, 64, true, true, 0>},
        {"flat_u1_bs256_nt", 1, 256, launch_v<1, 256, true, true, 0>},
        {"flat_u2_bs256_nt", 2, 256, launch_v<2, 256, true, true, 0>},
        {"flat_u1_bs64_ntload", 1, 64, launch_v<1, 64, true, false, 0>},
        {"flat_u1_bs64_ntstore", 1, 64, launch_v<1, 64, false, true, 0>},
        {"flat_u1_bs64_plain", 1, 64, launch_v<1, 64, false, false, 0>},
        {"flat_u2_bs64_ntload", 2, 64, launch_v<2, 64, true, false, 0>},
        {"flat_u1_bs128_ntload", 1, 128, launch_v<1, 128, true, false, 0>},
        {"flat_u1_bs256_ntload", 1, 256, launch_v<1, 256, true, false, 0>},
        {"lane_row_u4_bs64_nt", 4, 64, launch_v<4, 64, true, true, 1>},
        {"lane_row_u8_bs64_nt", 8, 64, launch_v<8, 64, true, true, 1>},
        {"xcd_u1_bs64_nt", 1, 64, launch_v<1, 64, true, true, 2>},
        {"xcd_u2_bs64_nt", 2, 64, launch_v<2, 64, true, true, 2>},
        {"xcd_u2_bs256_nt", 2, 256, launch_v<2, 256, true, true, 2>},
    };
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    AccDbl op;
    op.s = 0.7071067811865476;
    for (auto rp : rows_list) {
        const int R = rp.first;
        const int64_t pitch = rp.second;
        const uint64_t rows = payload / R, span = pitch * (rows - 1) + R;
        const uint32_t lg = __builtin_ctz(R / 16);
        const uint64_t items = rows * (R / 16);
        const int nsets = 4;
        std::vector<char *> S(nsets), D(nsets);
        for (int i = 0; i < nsets; ++i) {
            CK(hipMalloc(&S[i], span));
            CK(hipMalloc(&D[i], span));
            CK(hipMemset(S[i], 0x3f, span));
            CK(hipMemset(D[i], 0x40, span));
        }
        // exactness: each variant once on a copy of set 0's pristine dst, compared with variant 0
        std::vector<unsigned char> ref(span), got(span);
        char *d0, *pristine;
        CK(hipMalloc(&d0, span));
        CK(hipMalloc(&pristine, span));
        CK(hipMemcpy(pristine, D[0], span, hipMemcpyDeviceToDevice));
        int vi = 0;
        for (const Var &v : vars) {
            if (R / 16 < 1 || (strncmp(v.name, "lane_row", 8) == 0 && v.U != R / 16)) { ++vi; continue; }
            CK(hipMemcpy(d0, pristine, span, hipMemcpyDeviceToDevice));
            v.launch(S[0], d0, pitch, lg, items, op, st);
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(vi == 0 ? ref.data() : got.data(), d0, span, hipMemcpyDeviceToHost));
            const bool exact = vi == 0 || memcmp(ref.data(), got.data(), span) == 0;
            for (int i = 0; i < 4; ++i) v.launch(S[i % nsets], D[i % nsets], pitch, lg, items, op, st);
            CK(hipStreamSynchronize(st));
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(e0, st));
                for (int i = 0; i < steps; ++i) v.launch(S[i % nsets], D[i % nsets], pitch, lg, items, op, st);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            const double us = best * 1e3 / steps, tbs = 3.0 * payload / (us * 1e-6) / 1e12;
            printf("{\"probe\": \"short_rows\", \"row_bytes\": %d, \"pitch\": %lld, \"variant\": \"%s\", \"us_per_launch\": %.2f, "
                   "\"alg_TBps\": %.3f, \"frac\": %.4f, \"exact_vs_flat_u1\": %s}\n",
                   R, (long long)pitch, v.name, us, tbs, tbs / 8.0, exact ? "true" : "false");
            fflush(stdout);
            ++vi;
        }
        CK(hipFree(d0));
        CK(hipFree(pristine));
        for (int i = 0; i < nsets; ++i) {
            CK(hipFree(S[i]));
            CK(hipFree(D[i]));
        }
    }
    return 0;
}
