// perf_strided.cpp -- message-size sweep of the device-resident strided
// accumulate through the C ABI, in the manner of the reference's
// comex/testing/perf_strided.c (accs of 16 B ... 64 MiB, bandwidth per size):
//   latency   : comex_accs + comex_fence_all per operation (blocking round trip)
//   pipelined : `iters` comex_accs back to back, one fence at the end
//   host      : CPU time of one comex_accs call (enqueue cost)
// for 1 and 2 library streams.  Shape per size: rows of min(size, 16 KiB),
// leading dimension 2 x row (strided), f64.  Tuning evidence, not product code.
// Build: g++ -O2 -std=c++17 tools/perf_strided.cpp -Iinclude -Lga_amd -lga_amd -Wl,-rpath,$PWD/ga_amd -o tools/perf_strided
#include <stdio.h>
#include <stdlib.h>
#include <chrono>
#include <vector>
#include <algorithm>
#include "comex.h"
#include "ga_amd.h"

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    if (comex_init() != COMEX_SUCCESS) return 1;
    const size_t cap = (size_t)256 << 20;
    char *src = (char *)gaamd_dev_malloc(cap), *dst = (char *)gaamd_dev_malloc(cap);
    if (!src || !dst) return 2;
    gaamd_memset(src, 0, cap);
    gaamd_memset(dst, 0, cap);
    double alpha = 0.5;
    for (int streams : {1, 2}) {
        gaamd_set_tuning("streams", streams);
        for (long size = 16; size <= (64l << 20); size *= 4) {
            const int row = (int)std::min<long>(size, 16384);
            const int rows = (int)(size / row);
            int count[2] = {row, rows};
            int stride[1] = {2 * row};
            const int levels = rows > 1 ? 1 : 0;
            const long span = (long)stride[0] * (rows - 1) + row;
            // 4 disjoint dst slots so back-to-back ops are independent
            const int slots = (int)std::min<long>(4, (long)(cap / (size_t)span));
            const int iters = size <= (1 << 20) ? 400 : (size <= (16 << 20) ? 60 : 20);
            for (int i = 0; i < 10; ++i) comex_accs(COMEX_ACC_DBL, &alpha, src, stride, dst, stride, count, levels, 0, 0);
            comex_fence_all(0);
            // latency
            std::vector<double> lat;
            for (int i = 0; i < iters; ++i) {
                const double t0 = now();
                comex_accs(COMEX_ACC_DBL, &alpha, src, stride, dst + (i % slots) * span, stride, count, levels, 0, 0);
                comex_fence_all(0);
                lat.push_back(now() - t0);
            }
            std::sort(lat.begin(), lat.end());
            // pipelined
            const double t0 = now();
            double host = 0;
            for (int i = 0; i < iters; ++i) {
                const double h0 = now();
                comex_accs(COMEX_ACC_DBL, &alpha, src, stride, dst + (i % slots) * span, stride, count, levels, 0, 0);
                host += now() - h0;
            }
            comex_fence_all(0);
            const double tp = (now() - t0) / iters;
            printf("{\"streams\": %d, \"bytes\": %ld, \"row\": %d, \"rows\": %d, \"latency_us_median\": %.2f, "
                   "\"latency_us_min\": %.2f, \"pipelined_us_per_op\": %.2f, \"host_us_per_call\": %.2f, "
                   "\"pipelined_GBps_alg\": %.1f}\n",
                   streams, size, row, rows, lat[lat.size() / 2] * 1e6, lat[0] * 1e6, tp * 1e6, host / iters * 1e6,
                   3.0 * size / tp / 1e9);
            fflush(stdout);
        }
    }
    gaamd_dev_free(src);
    gaamd_dev_free(dst);
    comex_finalize();
    return 0;
}
