// blocking_lib_probe.cpp -- the library's blocking comex_accs on the headline patch
// (f64 2048 x 4096, ld 8192, three rotating buffer sets), called from C: per-call
// medians and where the host time of a call goes, from the library's own stamps
// (comex.cpp stamp(): 0 entry, 1 launch lock taken, 2 stream picked, 3 kernel
// launched, 4 return).  Set against tools/blocking_probe.hip (the same kernel shape
// with no library) it shows what the library adds to a blocking call.
// Build: g++ -O2 -std=c++17 tools/blocking_lib_probe.cpp -Iinclude -Lga_amd -lga_amd \
//          -Wl,-rpath,$PWD/ga_amd -o tools/blocking_lib_probe
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>
#include "comex.h"
#include "ga_amd.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int calls = argc > 1 ? atoi(argv[1]) : 200;
    if (comex_init() != COMEX_SUCCESS) return 1;
    const int cols = 2048, rows = 4096, ld = 8192;
    const size_t bytes = (size_t)rows * ld * 8;
    char *src[3], *dst[3];
    for (int k = 0; k < 3; ++k) {
        src[k] = (char *)gaamd_dev_malloc(bytes);
        dst[k] = (char *)gaamd_dev_malloc(bytes);
        if (!src[k] || !dst[k]) return 2;
        gaamd_memset(src[k], 0, bytes);
        gaamd_memset(dst[k], 0, bytes);
    }
    int count[2] = {cols * 8, rows}, stride[1] = {ld * 8};
    double alpha = 1.5;
    for (int i = 0; i < 10; ++i) comex_accs(COMEX_ACC_DBL, &alpha, src[i % 3], stride, dst[i % 3], stride, count, 1, 0, 0);
    comex_fence_all(0);
    const double alg = 3.0 * rows * cols * 8;
    for (int rep = 0; rep < 2; ++rep) {
        std::vector<double> t, d01, d12, d23, d34, tail;
        unsigned long long st[8];
        for (int i = 0; i < calls; ++i) {
            gaamd_diag("stamps", 1, nullptr, 0);
            const double t0 = now_us();
            comex_accs(COMEX_ACC_DBL, &alpha, src[i % 3], stride, dst[i % 3], stride, count, 1, 0, 0);
            const double t1 = now_us();
            gaamd_diag("stamps", 0, st, 8);
            t.push_back(t1 - t0);
            d01.push_back((st[1] - st[0]) * 1e-3);
            d12.push_back((st[2] - st[1]) * 1e-3);
            d23.push_back((st[3] - st[2]) * 1e-3);
            d34.push_back((st[4] - st[3]) * 1e-3);
        }
        auto med = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            return v[v.size() / 2];
        };
        const double m = med(t);
        printf("{\"rep\": %d, \"us_median\": %.2f, \"frac_of_8TBs\": %.4f, \"entry_to_lock_us\": %.2f, "
               "\"pick_us\": %.2f, \"launch_us\": %.2f, \"wait_us\": %.2f}\n",
               rep, m, alg / (m * 1e-6) / 8e12, med(d01), med(d12), med(d23), med(d34));
        fflush(stdout);
    }
    gaamd_diag("stamps", 0, nullptr, 0);
    comex_finalize();
    return 0;
}
