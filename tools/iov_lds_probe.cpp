// iov_lds_probe.cpp -- kernel-only timing of the io-vector ordering paths (VERDICT r5
// item 3), linked against libga_amd.so's internal launchers: n single-f64 pairs with
// random destinations in 1 GiB, contiguous sources, lists in HBM or in mapped pinned
// memory; per n the one-launch LDS path (one workgroup reads the lists from HBM; up to
// 16 Ki pairs), the path as the library routes it (lists in mapped pinned memory: below
// 1 Ki pairs that one launch, from 1 Ki the keys + partitioned launches) and the hashed
// three-launch path, HIP events
// around 50 back-to-back calls on one stream.  Checks each path's result (one call)
// against the pairs applied one by one in input order on the host (bit-exact); the
// hashed path alone leaves heavy repeats (> 8192 conflicting pairs) to its caller's
// radix fallback, so it reports "partial" there.
// Build: hipcc -O2 -std=c++17 -ffp-contract=off -D__HIP_PLATFORM_AMD__ -I ga_amd/csrc tools/iov_lds_probe.cpp \
//        -L ga_amd -lga_amd -Wl,-rpath,'$ORIGIN/../ga_amd' -o tools/iov_lds_probe
#include "gaamd_kernels.h"
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <random>
#include <vector>

using namespace gaamd;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int steps = 50;
    const uint64_t region = 1ull << 30;
    char *dst;
    CK(hipMalloc(&dst, region));
    CK(hipMemset(dst, 0, region));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    IovHash *h = iov_hash_create();
    uint32_t *flag_host, *flag_dev;
    CK(hipHostMalloc((void **)&flag_host, 64, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void **)&flag_dev, flag_host, 0));
    const double alpha = 0.7071067811865476;
    std::mt19937_64 rng(7);
    int slots_arg = argc > 1 ? atoi(argv[1]) : 0;   // destinations from this many slots (0: all of 1 GiB)
    for (uint32_t n : {1024u, 2048u, 4096u, 8192u, 16384u, 32768u, 65536u, 262144u, 1048576u}) {
        std::vector<uint64_t> dl(n);
        const uint64_t slots = slots_arg ? (uint64_t)slots_arg : region / 8;
        for (uint32_t i = 0; i < n; ++i) dl[i] = (uint64_t)(uintptr_t)dst + 8 * (rng() % slots);
        uint64_t dlo = ~0ull, dhi = 0;
        for (uint64_t a : dl) { dlo = a < dlo ? a : dlo; dhi = a > dhi ? a : dhi; }
        const uint64_t units = (dhi - dlo) / 8 + 1;
        double *src;
        CK(hipMalloc(&src, 8 * n));
        std::vector<double> sv(n);
        for (uint32_t i = 0; i < n; ++i) sv[i] = (double)(i % 97) - 48;
        CK(hipMemcpy(src, sv.data(), 8 * n, hipMemcpyHostToDevice));
        uint64_t *dl_dev, *dl_pin, *dl_pin_dev;
        CK(hipMalloc(&dl_dev, 8 * n));
        CK(hipMemcpy(dl_dev, dl.data(), 8 * n, hipMemcpyHostToDevice));
        CK(hipHostMalloc(&dl_pin, 8 * n, hipHostMallocMapped));
        memcpy(dl_pin, dl.data(), 8 * n);
        CK(hipHostGetDevicePointer((void **)&dl_pin_dev, dl_pin, 0));
        char *scratch;
        const size_t scratch_bytes = std::max(iov_lds_scratch_bytes(n), iov_runs_work_bytes(n)) + 256;
        CK(hipMalloc(&scratch, scratch_bytes));
        int deferred = 0;
        IovDesc d;
        memset(&d, 0, sizeof(d));
        d.src_base = (const char *)src;
        d.bytes = 8;
        d.n = n;
        uint64_t align_or = 0;
        for (uint64_t a : dl) align_or |= a;
        auto run = [&](int mode) {
            IovDesc z = d;
            int rc = 0;
            if (mode == 0) {          // LDS, lists in HBM, one workgroup
                if (n > kIovLdsMax) return;
                z.dst_list = dl_dev;
                rc = launch_iov_lds(38, &alpha, z, align_or, dlo, units, st);
            } else if (mode == 1) {   // LDS, lists in mapped pinned memory (the local call's case):
                z.dst_list = dl_pin_dev;  // from 1 Ki pairs the partitioned form (keys + partitions)
                if (n <= kIovPartWindowMax) {
                    rc = launch_iov_lds(38, &alpha, z, align_or, dlo, units, st, false, scratch);
                } else {              // as iov.cpp: overflowed partitions deferred to the radix path
                    IovPartState ps;
                    *flag_host = 0;
                    ps.flag_dev = flag_dev;
                    rc = launch_iov_lds(38, &alpha, z, align_or, dlo, units, st, false, scratch, &ps);
                    CK(hipStreamSynchronize(st));
                    if (!rc && *(volatile uint32_t *)flag_host) {
                        IovDesc h = d;
                        h.dst_list = dl_dev;
                        rc = launch_iov_runs(38, &alpha, h, align_or, dlo, units, scratch, scratch_bytes, st, false,
                                             nullptr, &ps);
                        ++deferred;
                    }
                }
            } else {                  // hashed, lists in HBM
                z.dst_list = dl_dev;
                rc = launch_iov_hashed(h, 38, &alpha, z, align_or, dlo, units, st);
            }
            if (rc) { fprintf(stderr, "mode %d rc %d\n", mode, rc); exit(1); }
        };
        const char *names[3] = {"lds_hbm_lists_1wg", "lds_pinned_lists_as_routed", "hashed_3_launches"};
        std::vector<double> res[3];
        std::vector<double> want(n);   // the pairs one by one, in order (acc: dst + alpha * src)
        {
            std::vector<std::pair<uint64_t, double>> acc;
            std::vector<uint64_t> ord(dl);
            std::sort(ord.begin(), ord.end());
            ord.erase(std::unique(ord.begin(), ord.end()), ord.end());
            std::vector<double> val(ord.size(), 0.0);
            for (uint32_t i = 0; i < n; ++i) {
                double &y = val[std::lower_bound(ord.begin(), ord.end(), dl[i]) - ord.begin()];
                volatile double prod = sv[i] * alpha;
                y = y + prod;
            }
            for (uint32_t i = 0; i < n; ++i) want[i] = val[std::lower_bound(ord.begin(), ord.end(), dl[i]) - ord.begin()];
        }
        for (int mode = 0; mode < 3; ++mode) {
            if (mode == 0 && n > kIovLdsMax) { res[0] = std::vector<double>(n, 0.0); continue; }
            if (mode == 2 && n > (1u << 19)) continue;   // the hashed path's limit (radix above)
            CK(hipMemset(dst, 0, region));
            run(mode);
            CK(hipStreamSynchronize(st));
            // every destination up to 64 Ki pairs, above a sample of 4096 of them
            std::vector<uint32_t> chk;
            for (uint32_t i = 0; i < n; i += (n > 65536 ? n / 4096 : 1)) chk.push_back(i);
            std::vector<double> got(chk.size()), wk(chk.size());
            for (size_t c = 0; c < chk.size(); ++c) {
                CK(hipMemcpy(&got[c], (void *)dl[chk[c]], 8, hipMemcpyDeviceToHost));
                wk[c] = want[chk[c]];
            }
            res[mode] = got;
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(e0, st));
                for (int s = 0; s < steps; ++s) run(mode);
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            const bool exact = memcmp(got.data(), wk.data(), 8 * got.size()) == 0;
            printf("{\"probe\": \"iov_lds\", \"pairs\": %u, \"slots\": %llu, \"path\": \"%s\", \"us_per_call\": %.2f, "
                   "\"exact\": %s, \"deferred_calls\": %d}\n",
                   n, (unsigned long long)slots, names[mode], best * 1e3 / steps,
                   exact ? "true" : (mode == 2 ? "\"partial\"" : "false"), mode == 1 ? deferred : 0);
            fflush(stdout);
        }
        CK(hipFree(src));
        CK(hipFree(dl_dev));
        CK(hipHostFree(dl_pin));
        CK(hipFree(scratch));
    }
    return 0;
}
