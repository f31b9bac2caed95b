// hbm_ceiling.hip -- standalone HBM streaming ceilings on MI355X for the access
// mixes of this path (tuning evidence, not product code):
//   read2  : two read streams (src + dst of an accumulate, no store)
//   write1 : one write stream
//   copy   : one read + one write stream (pack/unpack)
//   axpy   : two reads + one write (the accumulate, f64, 16 B per lane)
// each at 64 MiB per stream (the headline patch, launch edges included) and
// 512 MiB per stream (steady state), one and two HIP streams.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/hbm_ceiling.hip -o tools/hbm_ceiling
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#ifndef BS
#define BS 256   // threads per block (-DBS=64 for the library's one-wave blocks)
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

template <int U>
__global__ __launch_bounds__(BS) void k_read2(const v4u *a, const v4u *b, v4u *sink, uint32_t magic) {
    const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
    v4u x[U], y[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        x[k] = __builtin_nontemporal_load(a + base + k * BS);
        y[k] = __builtin_nontemporal_load(b + base + k * BS);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= x[k].x ^ y[k].y ^ x[k].z ^ y[k].w;
    if (acc == magic) sink[threadIdx.x] = x[0];
}

template <int U>
__global__ __launch_bounds__(BS) void k_write1(v4u *b, uint32_t v) {
    const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
#pragma unroll
    for (int k = 0; k < U; ++k) __builtin_nontemporal_store((v4u){v, v, v, (uint32_t)k}, b + base + k * BS);
}

template <int U>
__global__ __launch_bounds__(BS) void k_copy(const v4u *a, v4u *b) {
    const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
    v4u x[U];
#pragma unroll
    for (int k = 0; k < U; ++k) x[k] = __builtin_nontemporal_load(a + base + k * BS);
#pragma unroll
    for (int k = 0; k < U; ++k) __builtin_nontemporal_store(x[k], b + base + k * BS);
}

#pragma clang fp contract(off)
template <int U>
__global__ __launch_bounds__(BS) void k_axpy(const v2d *a, v2d *b, double s) {
    const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
    v2d x[U], y[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        x[k] = __builtin_nontemporal_load(a + base + k * BS);
        y[k] = __builtin_nontemporal_load(b + base + k * BS);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        v2d p = x[k] * s;
        __builtin_nontemporal_store(y[k] + p, b + base + k * BS);
    }
}

struct Bufs { std::vector<char *> a, b; };

enum Kind { READ2, WRITE1, COPY, AXPY };
static const char *kname[] = {"read2", "write1", "copy", "axpy"};
static const int streams_per_elem[] = {2, 1, 2, 3};

template <int U>
static void launch(Kind k, char *a, char *b, size_t bytes, hipStream_t st, v4u *sink) {
    const uint32_t blocks = (uint32_t)(bytes / 16 / BS / U);
    switch (k) {
    case READ2: hipLaunchKernelGGL(k_read2<U>, dim3(blocks), dim3(BS), 0, st, (const v4u *)a, (const v4u *)b, sink, 0x9e3779b9u); break;
    case WRITE1: hipLaunchKernelGGL(k_write1<U>, dim3(blocks), dim3(BS), 0, st, (v4u *)b, 7u); break;
    case COPY: hipLaunchKernelGGL(k_copy<U>, dim3(blocks), dim3(BS), 0, st, (const v4u *)a, (v4u *)b); break;
    case AXPY: hipLaunchKernelGGL(k_axpy<U>, dim3(blocks), dim3(BS), 0, st, (const v2d *)a, (v2d *)b, 0.7071067811865476); break;
    }
}

static void run(Kind k, int U, size_t bytes, int nstreams, const Bufs &B, hipStream_t *st, v4u *sink, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nsets = (int)B.a.size();
    auto one = [&](int i) {
        hipStream_t s = st[i % nstreams];
        char *a = B.a[i % nsets], *b = B.b[i % nsets];
        if (U == 1) launch<1>(k, a, b, bytes, s, sink);
        else if (U == 2) launch<2>(k, a, b, bytes, s, sink);
        else launch<4>(k, a, b, bytes, s, sink);
    };
    for (int i = 0; i < 2 * nsets; ++i) one(i);
    CK(hipDeviceSynchronize());
    double best = 0, sum = 0;
    const int rounds = 5;
    for (int r = 0; r < rounds; ++r) {
        CK(hipEventRecord(e0, st[0]));
        for (int s = 1; s < nstreams; ++s) CK(hipStreamWaitEvent(st[s], e0, 0));
        for (int i = 0; i < reps; ++i) one(i);
        for (int s = 1; s < nstreams; ++s) {
            hipEvent_t j;
            CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
            CK(hipEventRecord(j, st[s]));
            CK(hipStreamWaitEvent(st[0], j, 0));
            CK(hipEventDestroy(j));
        }
        CK(hipEventRecord(e1, st[0]));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double gbs = (double)bytes * streams_per_elem[k] * reps / (ms * 1e-3) / 1e9;
        sum += gbs;
        if (gbs > best) best = gbs;
    }
    printf("{\"kernel\": \"%s\", \"BS\": %d, \"U\": %d, \"MiB_per_stream\": %zu, \"hip_streams\": %d, \"launches\": %d, "
           "\"GBps_mean\": %.1f, \"GBps_best\": %.1f, \"us_per_launch\": %.2f}\n",
           kname[k], BS, U, bytes >> 20, nstreams, reps, sum / rounds, best,
           (double)bytes * streams_per_elem[k] / (sum / rounds * 1e9) * 1e6);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main() {
    hipStream_t st[2];
    CK(hipStreamCreate(&st[0]));
    CK(hipStreamCreate(&st[1]));
    v4u *sink;
    CK(hipMalloc(&sink, 4096));
    // 64 MiB per stream, 8 rotating sets (1 GiB: beyond the 256 MiB MALL)
    Bufs small, big;
    for (int i = 0; i < 8; ++i) {
        char *a, *b;
        CK(hipMalloc(&a, 64 << 20));
        CK(hipMalloc(&b, 64 << 20));
        CK(hipMemset(a, 0, 64 << 20));
        CK(hipMemset(b, 0, 64 << 20));
        small.a.push_back(a);
        small.b.push_back(b);
    }
    for (int i = 0; i < 2; ++i) {
        char *a, *b;
        CK(hipMalloc(&a, 512ull << 20));
        CK(hipMalloc(&b, 512ull << 20));
        CK(hipMemset(a, 0, 512ull << 20));
        CK(hipMemset(b, 0, 512ull << 20));
        big.a.push_back(a);
        big.b.push_back(b);
    }
    CK(hipDeviceSynchronize());
    for (int k = 0; k < 4; ++k) {
        for (int U : {1, 2, 4}) {
            run((Kind)k, U, 64 << 20, 1, small, st, sink, 64);
            run((Kind)k, U, 512ull << 20, 1, big, st, sink, 8);
        }
        run((Kind)k, 1, 64 << 20, 2, small, st, sink, 64);
    }
    return 0;
}
