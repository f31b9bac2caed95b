/*
 * mt_split.h -- P host workers, each on its own partition of one strided patch.
 * TEST INFRASTRUCTURE ONLY (the CPU baseline of bench.py, SURVEY.md §8(d):
 * "P workers concurrently on their own partitions").
 *
 * The patch is cut along its outermost level (count[L] for L > 0, whole
 * elements of count[0] for L == 0) into P contiguous slabs; worker w runs the
 * single-threaded strided accumulate `ACCS_FN` on slab w.  Slabs never share a
 * destination byte unless the patch itself overlaps, so for non-overlapping
 * patches the result equals the single-worker result bit for bit.
 */
#include <pthread.h>

typedef int (*mt_accs_fn)(int, const void *, const char *, const int *, char *, const int *,
                          const int *, int);

struct mt_job {
    mt_accs_fn fn;
    int op, levels;
    const void *scale;
    const char *src;
    char *dst;
    int src_stride[8], dst_stride[8], count[8];
};

static void *mt_worker(void *arg)
{
    struct mt_job *j = (struct mt_job *)arg;
    if (j->count[j->levels] > 0)
        j->fn(j->op, j->scale, j->src, j->src_stride, j->dst, j->dst_stride, j->count, j->levels);
    return 0;
}

static int mt_accs(mt_accs_fn fn, int esize, int op, const void *scale, const char *src,
                   const int *src_stride, char *dst, const int *dst_stride, const int *count,
                   int levels, int nthreads)
{
    struct mt_job job[64];
    pthread_t tid[64];
    int L = levels, w, i;
    long total, per, lo = 0;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    total = L ? count[L] : count[0] / esize;
    per = (total + nthreads - 1) / nthreads;
    for (w = 0; w < nthreads; ++w) {
        long hi = lo + per < total ? lo + per : total;
        struct mt_job *j = &job[w];
        j->fn = fn; j->op = op; j->levels = L; j->scale = scale;
        for (i = 0; i < L; ++i) { j->src_stride[i] = src_stride[i]; j->dst_stride[i] = dst_stride[i]; }
        for (i = 0; i <= L; ++i) j->count[i] = count[i];
        if (L) {
            j->src = src + lo * (long)src_stride[L - 1];
            j->dst = dst + lo * (long)dst_stride[L - 1];
            j->count[L] = (int)(hi - lo);
        } else {
            j->src = src + lo * esize;
            j->dst = dst + lo * esize;
            j->count[0] = (int)((hi - lo) * esize);
            if (w == nthreads - 1) j->count[0] += count[0] - (int)(total * esize);   /* partial tail */
        }
        lo = hi;
    }
    for (w = 1; w < nthreads; ++w)
        if (pthread_create(&tid[w], 0, mt_worker, &job[w])) return -1;
    mt_worker(&job[0]);
    for (w = 1; w < nthreads; ++w) pthread_join(tid[w], 0);
    return 0;
}
