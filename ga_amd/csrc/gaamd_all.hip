// gaamd_all.hip -- the library's device code as ONE translation unit, hence one code
// object: HIP loads a module onto the GPU at the first launch of one of its kernels,
// so kernels split over several modules would make the first blocking call (k_flag),
// the first comex_malloc (k_seg_tags) and the first io-vector call each pay a module
// load of their own (≈ 0.5-16 ms, seen in profiles/r05/final and s1 before this).
// The sources stay separate files for reading; they are compiled together here.
#include "gaamd_kernels.hip"
#include "gaamd_iov.hip"
#include "gaamd_misc.hip"
