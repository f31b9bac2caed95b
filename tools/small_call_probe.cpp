// small_call_probe.cpp -- small ComEx calls from C (no Python in the timing): the blocking
// comex_accs / comex_acc per call, and the issue rate of many non-blocking comex_nbaccs
// (K calls to distinct destinations, then comex_wait_all), from HBM, pinned and pageable
// sources.  GA codes that accumulate many small patches (NGA_NbAcc, task-parallel Fock
// builds) pay the per-call issue cost, not the blocking latency.  Diagnostic evidence.
// Build: g++ -O2 -std=c++17 tools/small_call_probe.cpp -Iinclude -Lga_amd -lga_amd
//          -Wl,-rpath,'$ORIGIN/../ga_amd' -o tools/small_call_probe
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>
#include "comex.h"
#include "ga_amd.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    // non-blocking calls per batch: 48 leaves the queue unfilled (the host's issue cost),
    // 1024 fills it (the rate the GPU retires them)
    const int K = argc > 1 ? atoi(argv[1]) : 48;
    if (comex_init() != COMEX_SUCCESS) return 1;
    const size_t span = (size_t)64 << 20;
    char *dev = (char *)gaamd_dev_malloc(span), *dst = (char *)gaamd_dev_malloc(span);
    char *pin = (char *)gaamd_host_malloc(1 << 20);
    std::vector<double> host_vec(1 << 17, 1.0);
    char *host = (char *)host_vec.data();
    if (!dev || !dst || !pin) return 2;
    gaamd_memset(dev, 0, span);
    gaamd_memset(dst, 0, span);
    memset(pin, 0, 1 << 20);
    double alpha = 0.5;
    struct Src { const char *name; char *p; } srcs[3] = {{"dev", dev}, {"pinned", pin}, {"pageable", host}};
    for (int bytes : {64, 512, 4096}) {
        int count[1] = {bytes}, stride[1] = {bytes};
        for (const Src &s : srcs) {
            // blocking, one destination
            std::vector<double> t;
            for (int i = 0; i < 220; ++i) {
                const double t0 = now_us();
                comex_accs(COMEX_ACC_DBL, &alpha, s.p, stride, dst, stride, count, 0, 0, COMEX_GROUP_WORLD);
                if (i >= 20) t.push_back(now_us() - t0);
            }
            printf("{\"call\": \"accs_blocking\", \"src\": \"%s\", \"bytes\": %d, \"median_us\": %.2f}\n",
                   s.name, bytes, median(t));
            // non-blocking: K calls to distinct destinations (a 4 KiB pitch), then wait_all
            std::vector<double> issue, total;
            for (int rep = 0; rep < (K < 100 ? 100 : 12); ++rep) {
                const double t0 = now_us();
                for (int k = 0; k < K; ++k) {
                    comex_request_t h;
                    comex_nbaccs(COMEX_ACC_DBL, &alpha, s.p, stride, dst + (size_t)k * 4096, stride, count, 0, 0,
                                 COMEX_GROUP_WORLD, &h);
                }
                const double t1 = now_us();
                comex_wait_all(COMEX_GROUP_WORLD);
                const double t2 = now_us();
                if (rep >= 2) {
                    issue.push_back((t1 - t0) / K);
                    total.push_back((t2 - t0) / K);
                }
            }
            printf("{\"call\": \"nbaccs_x%d_wait_all\", \"src\": \"%s\", \"bytes\": %d, \"issue_us_per_call\": %.2f, "
                   "\"total_us_per_call\": %.2f}\n", K, s.name, bytes, median(issue), median(total));
        }
    }
    // where one non-blocking call's host time goes: the library's stamps of each call
    // (0 entry, 1 launch lock taken, 2 stream picked, 3 kernel launched, 4 return)
    for (const Src &s : srcs) {
        int count[1] = {64}, stride[1] = {64};
        unsigned long long st[8];
        std::vector<double> d[4];
        gaamd_diag("stamps", 1, nullptr, 0);
        for (int i = 0; i < 600; ++i) {
            comex_request_t h;
            comex_nbaccs(COMEX_ACC_DBL, &alpha, s.p, stride, dst + (size_t)(i % 200) * 4096, stride, count, 0, 0,
                         COMEX_GROUP_WORLD, &h);
            gaamd_diag("stamps", -1, st, 8);
            if (i >= 100)
                for (int k = 0; k < 4; ++k) d[k].push_back((double)(st[k + 1] - st[k]) / 1e3);
            if (i % 200 == 199) comex_wait_all(COMEX_GROUP_WORLD);
        }
        gaamd_diag("stamps", 0, nullptr, 0);
        printf("{\"call\": \"nbaccs_stamps\", \"src\": \"%s\", \"bytes\": 64, \"entry_to_lock_us\": %.2f, "
               "\"lock_to_pick_us\": %.2f, \"pick_to_launched_us\": %.2f, \"launched_to_return_us\": %.2f}\n",
               s.name, median(d[0]), median(d[1]), median(d[2]), median(d[3]));
    }
    comex_finalize();
    return 0;
}
