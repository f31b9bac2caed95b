// completion_probe.hip -- how much of the headline region's closing edge is the
// runtime's completion path?  The bench region ends when
// hipStreamSynchronize returns on both library streams after the last of K
// accumulate kernels; profiled, that return comes 23-35 us after the last kernel
// ends.  Here the same shape (K = 20 launches of a 64 MiB f64 axpy, 1 KiB per
// one-wave block, 65536 blocks, two streams alternating) runs with a completion
// counter: every block, after its stores, bumps a per-launch device counter
// (agent-scope release first); the block that completes the launch stores the
// launch number into pinned host memory (system-scope release).  The host spins
// on that word, stamps when the last launch's number appears, then calls
// hipStreamSynchronize on both streams and stamps again.  Reported per region:
//   flag_us  -- region start to the host seeing the last launch's flag
//   sync_us  -- region start to both synchronizations returning (the bench's end)
//   gap_us   -- sync_us - flag_us: what a flag-polling wait would save
// and the same region without the counter (plain_us), the counter's own cost.
// argv: K rounds [h]: with a third argument 1, instead the bare-HIP region of the
// headline H shape (2-D, ld 8192): what a program with no library around the
// kernel reads on the bench's clock.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/completion_probe.hip -o tools/completion_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <algorithm>
#include <array>
#include <vector>

#define CK(x)                                                                                         \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
            exit(1);                                                                                  \
        }                                                                                             \
    } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

#pragma clang fp contract(off)
template <bool FLAG>
__global__ __launch_bounds__(64) void k_axpy(const v2d *a, v2d *b, double s, unsigned long long *count,
                                             unsigned long long target, unsigned int *host_flag, unsigned int tag) {
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    const v2d x = __builtin_nontemporal_load(a + i);
    const v2d y = __builtin_nontemporal_load(b + i);
    v2d r;
    r.x = y.x + s * x.x;
    r.y = y.y + s * x.y;
    __builtin_nontemporal_store(r, b + i);
    if (FLAG) {
        __syncthreads();   // every lane's store issued and complete (vmcnt) before the count
        if (threadIdx.x == 0) {
            __atomic_thread_fence(__ATOMIC_RELEASE);   // agent scope by default: the block's stores first
            const unsigned long long old = atomicAdd(count, 1ull);
            if (host_flag && old + 1 == target) {
                __atomic_thread_fence(__ATOMIC_SEQ_CST);
                __hip_atomic_store(host_flag, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// the headline H shape: 2048 rows of 32 KiB (f64), row pitch 64 KiB on both sides,
// one 1 KiB chunk per one-wave block (32 blocks per row), as the library's k_rows2d
__global__ __launch_bounds__(64) void k_axpy2d(const v2d *a, v2d *b, double s) {
    const size_t row = blockIdx.x >> 5, chunk = blockIdx.x & 31;
    const size_t i = row * 4096 + chunk * 64 + threadIdx.x;   // 4096 v2d = 64 KiB pitch
    const v2d x = __builtin_nontemporal_load(a + i);
    const v2d y = __builtin_nontemporal_load(b + i);
    v2d r;
    r.x = y.x + s * x.x;
    r.y = y.y + s * x.y;
    __builtin_nontemporal_store(r, b + i);
}

// the same kernel with a chosen store policy (mode 2): does the end-of-launch release
// (which writes back the dirty L2 lines before the completion signal) shorten when the
// stores leave nothing dirty in L2?  0 = nt (the library's), 1 = sc0 sc1 (system scope:
// written through), 2 = sc0 sc1 nt, 3 = plain, 4 = sc1 (agent scope: written through,
// the line dropped from L2), 5 = sc1 nt
template <int POL>
__global__ __launch_bounds__(64) void k_axpy2d_pol(const v2d *a, v2d *b, double s) {
    const size_t row = blockIdx.x >> 5, chunk = blockIdx.x & 31;
    const size_t i = row * 4096 + chunk * 64 + threadIdx.x;
    const v2d x = __builtin_nontemporal_load(a + i);
    const v2d y = __builtin_nontemporal_load(b + i);
    v2d r;
    r.x = y.x + s * x.x;
    r.y = y.y + s * x.y;
    if (POL == 0) __builtin_nontemporal_store(r, b + i);
    else if (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(b + i), "v"(r) : "memory");
    else if (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(b + i), "v"(r) : "memory");
    else if (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(b + i), "v"(r) : "memory");
    else if (POL == 5) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(b + i), "v"(r) : "memory");
    else b[i] = r;
}

// mode 3: a one-lane tail kernel that stores a tag into pinned host memory with a
// system-scope release; stream order starts it only after the kernel before it ended
__global__ void k_tail_flag(unsigned int *flag, unsigned int tag) {
    __hip_atomic_store(flag, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static void launch_pol(int pol, int blocks, hipStream_t st, const v2d *a, v2d *b) {
    switch (pol) {
    case 1: k_axpy2d_pol<1><<<blocks, 64, 0, st>>>(a, b, 0.5); break;
    case 2: k_axpy2d_pol<2><<<blocks, 64, 0, st>>>(a, b, 0.5); break;
    case 3: k_axpy2d_pol<3><<<blocks, 64, 0, st>>>(a, b, 0.5); break;
    case 4: k_axpy2d_pol<4><<<blocks, 64, 0, st>>>(a, b, 0.5); break;
    case 5: k_axpy2d_pol<5><<<blocks, 64, 0, st>>>(a, b, 0.5); break;
    default: k_axpy2d_pol<0><<<blocks, 64, 0, st>>>(a, b, 0.5); break;
    }
}

static double now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 20;
    const int rounds = argc > 2 ? atoi(argv[2]) : 40;
    const size_t n2 = (64ull << 20) / 16;   // v2d per 64 MiB
    const int blocks = (int)(n2 / 64);
    const int sets = 8;                     // rotate buffers as the bench does (MALL cannot hold them)
    std::vector<v2d *> A(sets), B(sets);
    for (int k = 0; k < sets; ++k) {
        CK(hipMalloc((void **)&A[k], n2 * 16));
        CK(hipMalloc((void **)&B[k], n2 * 16));
        CK(hipMemset(A[k], 0, n2 * 16));
        CK(hipMemset(B[k], 0, n2 * 16));
    }
    unsigned long long *cnt;
    CK(hipMalloc((void **)&cnt, 8));
    CK(hipMemset(cnt, 0, 8));
    unsigned int *flag_h, *flag_d;
    CK(hipHostMalloc((void **)&flag_h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void **)&flag_d, flag_h, 0));
    *(volatile unsigned int *)flag_h = 0;
    hipStream_t st[2];
    CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
    unsigned long long launched = 0;   // launches with the counter so far (the counter's target)
    unsigned int tag = 0;
    int it = 0;
    auto region = [&](bool flag, double *flag_us, double *sync_us) {
        CK(hipStreamSynchronize(st[0]));
        CK(hipStreamSynchronize(st[1]));
        const double t0 = now_us();
        unsigned int last = 0;
        for (int k = 0; k < K; ++k, ++it) {
            const int s = it % sets;
            if (flag) {
                ++launched;
                last = ++tag;
                // one counter shared by all launches: launch number m completes when the
                // count reaches m * blocks (launches on two streams can overlap, so the
                // count only says "m launches' worth of blocks finished"; the flag of
                // the K-th launch of a region is written once all K are done; only the
                // region's last launch writes it)
                k_axpy<true><<<blocks, 64, 0, st[k & 1]>>>(A[s], B[s], 0.5, cnt, launched * (unsigned long long)blocks,
                                                          k == K - 1 ? flag_d : nullptr, last);
            } else {
                k_axpy<false><<<blocks, 64, 0, st[k & 1]>>>(A[s], B[s], 0.5, nullptr, 0, nullptr, 0);
            }
        }
        if (flag) {
            const double give_up = now_us() + 1e6;
            while (__atomic_load_n((volatile unsigned int *)flag_h, __ATOMIC_ACQUIRE) != last) {
                if (now_us() > give_up) {
                    fprintf(stderr, "flag %u never arrived (saw %u)\n", last, *(volatile unsigned int *)flag_h);
                    exit(2);
                }
            }
            *flag_us = now_us() - t0;
        }
        CK(hipStreamSynchronize(st[0]));
        CK(hipStreamSynchronize(st[1]));
        *sync_us = now_us() - t0;
    };
    // the bare-HIP region of the headline shape: K launches of the 2-D kernel over 8
    // buffer sets of 2 x 128 MiB (H: src and dst both ld 8192 f64), two streams,
    // barrier-free: host clock from the first launch to both synchronizations
    const int reg2d = argc > 3 ? atoi(argv[3]) : 0;
    if (reg2d == 3) {
        // blocking-call completion: K launches of the H-shape kernel on one stream, then
        // (a) hipStreamSynchronize, or (b) a tail flag kernel and a host spin on the flag
        // (then hipStreamSynchronize, outside the time).  K = 1 is a blocking comex_accs;
        // K = 20 the value region's close.  Interleaved, `rounds` each.
        std::vector<v2d *> A2(sets), B2(sets);
        for (int k = 0; k < sets; ++k) {
            CK(hipMalloc((void **)&A2[k], 128ull << 20));
            CK(hipMalloc((void **)&B2[k], 128ull << 20));
            CK(hipMemset(A2[k], 0, 128ull << 20));
            CK(hipMemset(B2[k], 0, 128ull << 20));
        }
        int j = 0;
        auto reg = [&](int k_launches, bool tail, double *flag_us) {
            CK(hipStreamSynchronize(st[0]));
            const double t0 = now_us();
            for (int k = 0; k < k_launches; ++k, ++j) launch_pol(0, 65536, st[0], A2[j % sets], B2[j % sets]);
            if (tail) {
                const unsigned int want = ++tag;
                k_tail_flag<<<1, 1, 0, st[0]>>>(flag_d, want);
                const double give_up = now_us() + 1e6;
                while (__atomic_load_n((volatile unsigned int *)flag_h, __ATOMIC_ACQUIRE) != want)
                    if (now_us() > give_up) { fprintf(stderr, "tail flag never arrived\n"); exit(2); }
                *flag_us = now_us() - t0;
                CK(hipStreamSynchronize(st[0]));
                return now_us() - t0;
            }
            CK(hipStreamSynchronize(st[0]));
            return now_us() - t0;
        };
        double f = 0;
        const double warm_until = now_us() + 500e3;
        while (now_us() < warm_until) { reg(1, false, &f); reg(1, true, &f); }
        for (int kl : {1, 20}) {
            std::vector<double> vs, vf, vfs;
            for (int r = 0; r < rounds; ++r) {
                vs.push_back(reg(kl, false, &f));
                vfs.push_back(reg(kl, true, &f));
                vf.push_back(f);
            }
            auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
            printf("{\"probe\": \"tail_flag\", \"launches\": %d, \"rounds\": %d, \"sync_us\": %.2f, "
                   "\"tail_flag_seen_us\": %.2f, \"tail_then_sync_us\": %.2f}\n",
                   kl, rounds, med(vs), med(vf), med(vfs));
        }
        return 0;
    }
    if (reg2d == 2) {
        // store-policy sweep, interleaved: configs (policy of every launch, policy of the
        // region's last launch); regions of K and 2K launches, so that per config the
        // slope is the per-launch time and the intercept the region's two edges
        std::vector<v2d *> A2(sets), B2(sets);
        for (int k = 0; k < sets; ++k) {
            CK(hipMalloc((void **)&A2[k], 128ull << 20));
            CK(hipMalloc((void **)&B2[k], 128ull << 20));
            CK(hipMemset(A2[k], 0, 128ull << 20));
            CK(hipMemset(B2[k], 0, 128ull << 20));
        }
        // configs "all:last,all:last,..." (argv[4]); default every policy once plus the
        // library's nt with a write-through last launch
        std::vector<std::array<int, 2>> cfg;
        const char *spec = argc > 4 ? argv[4] : "0:0,1:1,2:2,3:3,4:4,5:5,0:4";
        for (const char *p = spec; *p;) {
            int a = 0, b = 0, used = 0;
            if (sscanf(p, "%d:%d%n", &a, &b, &used) != 2) break;
            cfg.push_back({a, b});
            p += used;
            if (*p == ',') ++p;
        }
        const int ncfg = (int)cfg.size();
        int j = 0;
        auto reg = [&](int c, int k_launches) {
            CK(hipStreamSynchronize(st[0]));
            CK(hipStreamSynchronize(st[1]));
            const double t0 = now_us();
            for (int k = 0; k < k_launches; ++k, ++j)
                launch_pol(k == k_launches - 1 ? cfg[c][1] : cfg[c][0], 65536, st[k & 1], A2[j % sets], B2[j % sets]);
            CK(hipStreamSynchronize(st[0]));
            CK(hipStreamSynchronize(st[1]));
            return now_us() - t0;
        };
        const double warm_until = now_us() + 500e3;
        while (now_us() < warm_until)
            for (int c = 0; c < ncfg; ++c) reg(c, K);
        std::vector<std::vector<double>> v1(ncfg), v2(ncfg);
        for (int r = 0; r < rounds; ++r)
            for (int q = 0; q < ncfg; ++q) {   // the order rotates every round: no config always follows another
                const int c = (q + r) % ncfg;
                if (r & 1) {
                    v2[c].push_back(reg(c, 2 * K));
                    v1[c].push_back(reg(c, K));
                } else {
                    v1[c].push_back(reg(c, K));
                    v2[c].push_back(reg(c, 2 * K));
                }
            }
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        for (int c = 0; c < ncfg; ++c) {
            const double m1 = med(v1[c]), m2 = med(v2[c]);
            const double per = (m2 - m1) / K, edges = m1 - K * per;
            const double bytes = 3.0 * 64 * (1 << 20) * K;
            printf("{\"probe\": \"store_policy\", \"policy_all\": %d, \"policy_last\": %d, \"launches\": %d, "
                   "\"rounds\": %d, \"median_us\": %.2f, \"median_2k_us\": %.2f, \"per_launch_us\": %.3f, "
                   "\"edges_us\": %.2f, \"frac_median\": %.4f}\n",
                   cfg[c][0], cfg[c][1], K, rounds, m1, m2, per, edges, bytes / (m1 * 1e-6) / 8e12);
        }
        return 0;
    }
    if (reg2d) {
        std::vector<v2d *> A2(sets), B2(sets);
        for (int k = 0; k < sets; ++k) {
            CK(hipMalloc((void **)&A2[k], 128ull << 20));
            CK(hipMalloc((void **)&B2[k], 128ull << 20));
            CK(hipMemset(A2[k], 0, 128ull << 20));
            CK(hipMemset(B2[k], 0, 128ull << 20));
        }
        int j = 0;
        auto reg = [&]() {
            CK(hipStreamSynchronize(st[0]));
            CK(hipStreamSynchronize(st[1]));
            const double t0 = now_us();
            for (int k = 0; k < K; ++k, ++j)
                k_axpy2d<<<65536, 64, 0, st[k & 1]>>>(A2[j % sets], B2[j % sets], 0.5);
            CK(hipStreamSynchronize(st[0]));
            CK(hipStreamSynchronize(st[1]));
            return now_us() - t0;
        };
        const double warm_until = now_us() + 500e3;   // the bench's time-based warm-up
        while (now_us() < warm_until) reg();
        std::vector<double> v;
        for (int r = 0; r < rounds; ++r) v.push_back(reg());
        std::sort(v.begin(), v.end());
        const double bytes = 3.0 * 64 * (1 << 20) * K;
        printf("{\"probe\": \"bare_region_H\", \"launches\": %d, \"rounds\": %d, \"min_us\": %.2f, \"median_us\": %.2f, "
               "\"max_us\": %.2f, \"frac_median\": %.4f, \"frac_best\": %.4f}\n",
               K, rounds, v[0], v[v.size() / 2], v.back(), bytes / (v[v.size() / 2] * 1e-6) / 8e12,
               bytes / (v[0] * 1e-6) / 8e12);
        return 0;
    }
    double f, s;
    for (int w = 0; w < 10; ++w) { region(true, &f, &s); region(false, &f, &s); }
    std::vector<double> fl, sy, pl;
    for (int r = 0; r < rounds; ++r) {
        region(true, &f, &s);
        fl.push_back(f);
        sy.push_back(s);
        region(false, &f, &s);
        pl.push_back(s);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    std::vector<double> gap(fl.size());
    for (size_t k = 0; k < fl.size(); ++k) gap[k] = sy[k] - fl[k];
    const double bytes = 3.0 * 64 * (1 << 20) * K;
    printf("{\"probe\": \"completion\", \"launches\": %d, \"rounds\": %d, \"flag_us\": %.2f, \"sync_us\": %.2f, "
           "\"gap_us\": %.2f, \"gap_min_us\": %.2f, \"plain_us\": %.2f, \"frac_at_flag\": %.4f, \"frac_at_sync\": %.4f, "
           "\"frac_plain\": %.4f}\n",
           K, rounds, med(fl), med(sy), med(gap), *std::min_element(gap.begin(), gap.end()), med(pl),
           bytes / (med(fl) * 1e-6) / 8e12, bytes / (med(sy) * 1e-6) / 8e12, bytes / (med(pl) * 1e-6) / 8e12);
    return 0;
}
