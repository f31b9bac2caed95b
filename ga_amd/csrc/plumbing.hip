// plumbing.hip -- kernel-level C ABI (ga_amd.h section 2) and the device
// plumbing used by tests and bench.py (section 3).
#include "gaamd_kernels.h"
#include "runtime.hpp"
#include <string.h>
#include <stdlib.h>
#include <dlfcn.h>

namespace gaamd {

LaunchInfo g_last;
LaunchInfo *last_launch_info() { return &g_last; }

static hipStream_t stream_of(void *s) {
    if (s) return (hipStream_t)s;
    Runtime &r = rt();
    if (r.stream) return r.stream;
    return nullptr;   // legacy default stream before comex_init
}

// splitmix64 element i (state after i+1 increments); must match
// oracle/comex_oracle.c splitmix64_at bit for bit.
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill(void *dst, long n, int type, uint64_t seed) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const uint64_t x = splitmix64_at(seed, (uint64_t)i);
        switch (type) {
        case 0: ((double *)dst)[i] = ((double)(x >> 11) * 0x1.0p-53) * 2.0 - 1.0; break;
        case 1: ((float *)dst)[i] = ((float)(x >> 40) * 0x1.0p-24f) * 2.0f - 1.0f; break;
        case 2: ((int32_t *)dst)[i] = (int32_t)(x >> 43) - (1 << 20); break;
        default: ((int64_t *)dst)[i] = (int64_t)(x >> 43) - (1 << 20); break;
        }
    }
}

// n 8-byte words of the same bit pattern (test and bench data: 2^rank constants)
__global__ __launch_bounds__(256) void k_fill_word(uint64_t *dst, long n, uint64_t word) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) dst[i] = word;
}

}  // namespace gaamd

using namespace gaamd;

extern "C" {

int gaamd_strided(int op, const void *scale, const void *src, const int *src_stride, void *dst,
                  const int *dst_stride, const int *count, int stride_levels, void *stream) {
    return launch_strided(op, scale, src, src_stride, dst, dst_stride, count, stride_levels, stream_of(stream),
                          &g_last);
}

int gaamd_plan_strided(int op, const void *src, const int *src_stride, const void *dst, const int *dst_stride,
                       const int *count, int stride_levels, unsigned long long row_begin,
                       unsigned long long row_end, long long plan[8]) {
    LaunchInfo li;
    const double one[2] = {1.0, 0.0};
    const int rc = launch_strided(op, one, src, src_stride, (void *)dst, dst_stride, count, stride_levels, nullptr,
                                  &li, row_begin, row_end, true);
    plan[0] = li.kind;
    plan[1] = li.width;
    plan[2] = li.unroll;
    plan[3] = li.block;
    plan[4] = li.launches;
    plan[5] = (long long)li.blocks;
    plan[6] = li.levels;
    plan[7] = li.aligned;
    return rc;
}

long gaamd_packed_size(const int *count, int stride_levels) {
    long n = count[0];
    for (int j = 1; j <= stride_levels; ++j) n *= count[j];
    return n;
}

static void packed_strides(const int *count, int levels, int *ps) {
    long acc = count[0];
    for (int j = 0; j < levels; ++j) {
        ps[j] = (int)acc;
        acc *= count[j + 1];
    }
}

int gaamd_pack(const void *src, const int *src_stride, const int *count, int stride_levels, void *packed,
               void *stream) {
    int ps[kMaxLevels + 1];
    if (stride_levels < 0 || stride_levels > kMaxLevels) return -2;
    packed_strides(count, stride_levels, ps);
    return launch_strided(kOpCopy, nullptr, src, src_stride, packed, ps, count, stride_levels, stream_of(stream),
                          &g_last);
}

int gaamd_unpack(const void *packed, void *dst, const int *dst_stride, const int *count, int stride_levels,
                 void *stream) {
    int ps[kMaxLevels + 1];
    if (stride_levels < 0 || stride_levels > kMaxLevels) return -2;
    packed_strides(count, stride_levels, ps);
    return launch_strided(kOpCopy, nullptr, packed, ps, dst, dst_stride, count, stride_levels, stream_of(stream),
                          &g_last);
}

int gaamd_unpack_acc(int op, const void *scale, const void *packed, void *dst, const int *dst_stride,
                     const int *count, int stride_levels, void *stream) {
    int ps[kMaxLevels + 1];
    if (stride_levels < 0 || stride_levels > kMaxLevels) return -2;
    if (op == kOpCopy) return -4;
    packed_strides(count, stride_levels, ps);
    return launch_strided(op, scale, packed, ps, dst, dst_stride, count, stride_levels, stream_of(stream),
                          &g_last);
}

int gaamd_last_launch(int *kind, int *width, int *unroll, int *launches, unsigned long long *blocks) {
    if (kind) *kind = g_last.kind;
    if (width) *width = g_last.width;
    if (unroll) *unroll = g_last.unroll;
    if (launches) *launches = g_last.launches;
    if (blocks) *blocks = g_last.blocks;
    return 0;
}

int gaamd_kernel_counts(unsigned long long counts[5]) {
    for (int k = 0; k < kKinds; ++k) counts[k] = kernel_count(k);
    return 0;
}

static int *tuning_field(const char *key) {
    Tuning &t = tuning();
    if (!strcmp(key, "kind")) return &t.kind;
    if (!strcmp(key, "flat_max_nvec")) return &t.flat_max_nvec;
    if (!strcmp(key, "block")) return &t.block;
    if (!strcmp(key, "align")) return &t.align;
    if (!strcmp(key, "flat_line_min")) return &t.flat_line_min;
    if (!strcmp(key, "ordered_cols")) return &t.ordered_cols;
    if (!strcmp(key, "iov_lds")) return &t.iov_lds;
    return nullptr;
}

int gaamd_set_tuning(const char *key, int value) {
    if (!strcmp(key, "streams")) {   // library streams used by the scheduler (sched.cpp)
        Runtime &r = rt();
        if (!r.initialized || value < 1 || value > 8) return -1;
        std::lock_guard<std::mutex> g(r.launch_mu);
        const int old = (int)r.streams.size();
        sched_resize(value);
        return old;
    }
    int *f = tuning_field(key);
    if (!f) return -1;
    if (!strcmp(key, "block") && value != 0 && value != 64 && value != 128) return -1;
    const int old = *f;
    *f = value;
    return old;
}

int gaamd_get_tuning(const char *key) {
    if (!strcmp(key, "streams")) return (int)rt().streams.size();
    int *f = tuning_field(key);
    return f ? *f : -1;
}

int gaamd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int gaamd_set_device(int dev) { return hipSetDevice(dev) == hipSuccess ? 0 : -1; }
void *gaamd_stream(void) { return rt().stream; }
void *gaamd_stream_at(int i) {
    Runtime &r = rt();
    return (i >= 0 && i < (int)r.streams.size()) ? (void *)r.streams[i] : nullptr;
}

void *gaamd_dev_malloc(size_t bytes) {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        segment_cache_flush();   // freed segments kept for reuse go back first
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    }
    addr_event('a', p, bytes, -1);
    return p;
}
int gaamd_dev_free(void *p) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess) addr_event('f', p, size, -1);
    else (void)hipGetLastError();
    return hipFree(p) == hipSuccess ? 0 : -1;
}

void *gaamd_host_malloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return nullptr;
    return p;
}
int gaamd_host_free(void *p) { return hipHostFree(p) == hipSuccess ? 0 : -1; }

int gaamd_memcpy(void *dst, const void *src, size_t bytes) {
    return hipMemcpy(dst, src, bytes, hipMemcpyDefault) == hipSuccess ? 0 : -1;
}
// a 2-D patch: `height` rows of `width` bytes, rows `spitch` / `dpitch` bytes
// apart (hipMemcpy2D; host or device on either side; returns when done)
int gaamd_memcpy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height) {
    return hipMemcpy2D(dst, dpitch, src, spitch, width, height, hipMemcpyDefault) == hipSuccess ? 0 : -1;
}
int gaamd_memset(void *dst, int value, size_t bytes) {
    return hipMemset(dst, value, bytes) == hipSuccess ? 0 : -1;
}
int gaamd_sync(void *stream) {
    Runtime &r = rt();
    if (!stream && r.initialized) {   // every library stream
        std::lock_guard<std::mutex> g(r.launch_mu);
        sched_sync_all();
        return 0;
    }
    hipStream_t s = stream_of(stream);
    hipError_t e = s ? hipStreamSynchronize(s) : hipDeviceSynchronize();
    return e == hipSuccess ? 0 : -(int)e;
}

int gaamd_join(void) {
    Runtime &r = rt();
    if (!r.initialized) return -1;
    std::lock_guard<std::mutex> g(r.launch_mu);
    sched_join();
    return 0;
}

int gaamd_num_streams(void) { return (int)rt().streams.size(); }

int gaamd_fill_word(void *dst, long n, unsigned long long word, void *stream) {
    if (n <= 0) return 0;
    if ((uintptr_t)dst & 7) return -2;
    long blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_fill_word, dim3((unsigned)blocks), dim3(256), 0, stream_of(stream), (uint64_t *)dst, n,
                       (uint64_t)word);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int gaamd_fill(void *dst, long n, int type, unsigned long long seed, void *stream) {
    if (n <= 0) return 0;
    if (type < 0 || type > 3) return -2;
    long blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_fill, dim3((unsigned)blocks), dim3(256), 0, stream_of(stream), dst, n, type,
                       (uint64_t)seed);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

void *gaamd_stream_create(void) {
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamDefault) != hipSuccess) return nullptr;
    return (void *)s;
}
int gaamd_stream_destroy(void *s) { return hipStreamDestroy((hipStream_t)s) == hipSuccess ? 0 : -1; }

void *gaamd_event_create(void) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return (void *)e;
}
int gaamd_event_destroy(void *ev) { return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? 0 : -1; }
int gaamd_event_record(void *ev, void *stream) {
    return hipEventRecord((hipEvent_t)ev, stream_of(stream)) == hipSuccess ? 0 : -1;
}
int gaamd_event_sync(void *ev) { return hipEventSynchronize((hipEvent_t)ev) == hipSuccess ? 0 : -1; }
float gaamd_event_elapsed_ms(void *start, void *stop) {
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, (hipEvent_t)start, (hipEvent_t)stop) != hipSuccess) return -1.f;
    return ms;
}

const char *gaamd_version(void) { return "ga_amd 0.1 (gfx950)"; }

// the file of the HIP runtime this library's calls resolve to: /opt/rocm's, or
// a copy with the same SONAME that another library (a torch wheel) loaded first
const char *gaamd_hip_runtime(void) {
    Dl_info info;
    hipError_t (*fn)(void **, size_t) = &hipMalloc;
    if (dladdr(reinterpret_cast<void *>(fn), &info) && info.dli_fname) return info.dli_fname;
    return "unknown";
}

}  // extern "C"
