/*
 * ga.h -- the Global Arrays C API subset on the one-sided accumulate path,
 * exported by libga_amd_ga.so (the caller row a15 of SURVEY.md §8(a)), a
 * library of its own over libga_amd.so's public ABI.  libga_amd.so -- the
 * drop-in beneath global/src -- defines none of these names, so a real GA that
 * defines them itself (global/src/capi.c) links against it unchanged.
 *
 * Same names, argument order and index conventions as the reference C API
 * (global/src/capi.c, global/src/ga.h): C (row-major, 0-based) subscripts at
 * the API, converted to GA's Fortran order (column-major, 1-based) inside, as
 * capi.c:54-61 does.  Arrays use the REGULAR block distribution: the process
 * grid of ddb/ddb_h2 (global/src/decomp.c) and the block map of pnga_allocate
 * (base.c:2550-2630), or an explicit map with NGA_Create_irreg.  Each rank's
 * block lives in its GPU's HBM (one comex_malloc segment per array).
 */
#ifndef GA_AMD_GA_H
#define GA_AMD_GA_H

#if defined(__cplusplus)
extern "C" {
#endif

/* global/src/gacommon.h:14-22 (MT_BASE 1000, ma/macommon.h:11-20) */
#define C_INT 1001
#define C_LONG 1002
#define C_FLOAT 1003
#define C_DBL 1004
#define C_SCPL 1006
#define C_DCPL 1007
#define GA_MAX_DIM 7

/* complex scalars (comex/src-common/acc.h:6-15) */
#ifndef GA_AMD_COMPLEX_TYPES
#define GA_AMD_COMPLEX_TYPES
typedef struct { double real; double imag; } DoubleComplex;
typedef struct { float real; float imag; } SingleComplex;
#endif

int GA_Initialize(void);
void GA_Terminate(void);
int GA_Nodeid(void);
int GA_Nnodes(void);
void GA_Sync(void);
void GA_Error(char *msg, int code);

int NGA_Create(int type, int ndim, int dims[], char *name, int chunk[]);
int NGA_Create_irreg(int type, int ndim, int dims[], char *name, int block[], int map[]);
void GA_Destroy(int g_a);
void GA_Zero(int g_a);
void NGA_Distribution(int g_a, int iproc, int lo[], int hi[]);
int NGA_Locate_num_blocks(int g_a, int lo[], int hi[]);

/* one-sided patch operations (capi.c:2079-2089, onesided.c:1334-1471) */
void NGA_Acc(int g_a, int lo[], int hi[], void *buf, int ld[], void *alpha);
void NGA_Put(int g_a, int lo[], int hi[], void *buf, int ld[]);
void NGA_Get(int g_a, int lo[], int hi[], void *buf, int ld[]);

/* non-blocking patch operations (capi.c:2103-2190 -> pnga_nbacc/nbput/nbget,
   onesided.c:685, 1300, 1481) and their wait (pnga_nbwait, onesided.c:368);
   ga_nbhdl_t is GA's Integer (ga.h:18) */
typedef long ga_nbhdl_t;
void NGA_NbAcc(int g_a, int lo[], int hi[], void *buf, int ld[], void *alpha, ga_nbhdl_t *nbhandle);
void NGA_NbPut(int g_a, int lo[], int hi[], void *buf, int ld[], ga_nbhdl_t *nbhandle);
void NGA_NbGet(int g_a, int lo[], int hi[], void *buf, int ld[], ga_nbhdl_t *nbhandle);
void NGA_NbWait(ga_nbhdl_t *nbhandle);
/* every skip[d]-th element of the patch; buf holds only the selected elements
   (capi.c:1990-2060 -> pnga_strided_acc/put/get, onesided.c:4225-4470) */
void NGA_Strided_acc(int g_a, int lo[], int hi[], int skip[], void *buf, int ld[], void *alpha);
void NGA_Strided_put(int g_a, int lo[], int hi[], int skip[], void *buf, int ld[]);
void NGA_Strided_get(int g_a, int lo[], int hi[], int skip[], void *buf, int ld[]);
/* direct access to the local block (an HBM address) */
/* gather / scatter / scatter-accumulate of single elements: capi.c:3026-3160 ->
   gai_gatscat onesided.c:2747 (one ARMCI_GetV/PutV/AccV per owner).  subsArray[k]
   points at the ndim C subscripts of element k; *_flat takes them as one array. */
void NGA_Scatter(int g_a, void *v, int *subsArray[], int n);
void NGA_Scatter_flat(int g_a, void *v, int subsArray[], int n);
void NGA_Scatter_acc(int g_a, void *v, int *subsArray[], int n, void *alpha);
void NGA_Scatter_acc_flat(int g_a, void *v, int subsArray[], int n, void *alpha);
void NGA_Gather(int g_a, void *v, int *subsArray[], int n);
void NGA_Gather_flat(int g_a, void *v, int subsArray[], int n);

void NGA_Access(int g_a, int lo[], int hi[], void *ptr, int ld[]);
void NGA_Release(int g_a, int lo[], int hi[]);
void NGA_Release_update(int g_a, int lo[], int hi[]);

/* process grid the REGULAR distribution chose, C order (ga.h GA_Get_proc_grid) */
void GA_Get_proc_grid(int g_a, int dims[]);
/* process grid (C order) that NGA_Create picks for npes ranks (restated
 * ddb/ddb_h2 of global/src/decomp.c); host-only, no GPU */
int gaamd_ga_proc_grid(int ndim, const int *dims, const int *chunk, int npes, int *grid);
/* statistics of global/src/onesided.c:1372-1419 (GAstat.numacc, GAbytes.acctot/accloc) */
void GA_Print_stats(void);

#if defined(__cplusplus)
}
#endif

#endif /* GA_AMD_GA_H */
