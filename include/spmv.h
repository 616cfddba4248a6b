/*
 * spmv.h — C-ABI of the MI355X (gfx950) fp64 SpMV kernels: y = A·x.
 *
 * This is the drop-in boundary that replaces the reference's
 * "clSetKernelArg ×k → clEnqueueNDRangeKernel" call sites
 * (reference coo.c:163-194, csr.c:170-201, ell.c:242-273,
 *  sigma_c.c:280-311, cmrs.c:195-232) and the five OpenCL kernels
 * (reference kernels/{Coo,Csr,Ell,Sigma_C,Cmrs}.cl).  Everything here is
 * plain C: device pointers, sizes, a hipStream_t passed as `void *`.
 *
 * A caller uses it in two steps:
 *   1. spmv_plan_<fmt>(dims, the format's device arrays, options) looks at
 *      the matrix once and builds everything the measured-best kernel path
 *      for it needs (x windows, head copies, tile plans, workspace);
 *   2. spmv_plan_run(plan, x, y, stream) launches that path.
 * ./bin/{coo,csr,ell,sigma_c,cmrs} (drivers/driver.c) and the Python
 * binding (spmv_amd.to_device) both go through the plans, so the programs
 * run the kernels bench.py measures.  The five spmv_<fmt>_run entry points
 * below are the reference kernels' one-call equivalents (no build step,
 * global x gathers); the individual kernel variants the plans choose
 * between, the compressed formats and the device builders are in
 * spmv_ext.h.
 *
 * Conventions (all entry points):
 *   - Every array argument is a DEVICE pointer on `d.device`, owned by the
 *     caller; a plan keeps pointers to them (they must outlive the plan)
 *     and owns only what it builds.  The library's own scratch
 *     (spmv_flush_cache's buffer) is freed by spmv_release().
 *   - y is FULLY overwritten (rows without entries get 0.0).  The reference
 *     COO relied on fresh device memory being zero (reference coo.c:120);
 *     here no pre-zeroing is required.
 *   - Runs are asynchronous on the given stream (NULL = the device's
 *     default stream).  No hidden device-wide synchronisation and no
 *     allocation inside a run, so a caller may capture runs into a
 *     hipGraph.  Plan creation synchronises d.stream (build time).
 *   - Return value: 0 on success, otherwise a code of spmv_rc.h with the
 *     reference's numeric meaning (reference inc/enums.h:4-11):
 *     1 device error, 2 launch/copy error, 4 bad arguments.
 *     spmv_last_error() returns a human readable message for the last
 *     failure on the calling thread.
 *   - Indices are 0-based.  Column indices are int32 (as the reference);
 *     offsets into the value arrays are int64 (the reference's int32
 *     offsets overflow past 2^31 entries).
 */
#ifndef SPMV_H
#define SPMV_H

#include <stddef.h>
#include <stdint.h>

#include "spmv_rc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spmv_dims {
    int64_t n_rows; /* N: rows of A, length of y            */
    int64_t n_cols; /* M: columns of A, length of x         */
    int64_t nnz;    /* Z: stored entries that are multiplied */
    int device;     /* HIP device ordinal holding the arrays */
    void *stream;   /* hipStream_t (NULL: default stream)    */
} spmv_dims;

/* --------------------------------------------------------------- plans ---
 * One plan per matrix and format.  The arrays are the format's device
 * arrays as the host builders of spmv_host.h (or the device builders of
 * spmv_ext.h) produce them; the plan keeps pointers to them.
 *
 * Options (spmv_plan_opts_init sets the library defaults; every "-1" means
 * "the library's rule for this matrix"):
 *   lanes      CSR lanes per row (2..64, a power of two); 0 = rule
 *   variant    CSR: -1 rule (4 when the longest row exceeds 4,096 entries
 *              and 64x the mean, else the x-window kernel), 1 direct,
 *              2 staged, 3 staged persistent (x windows when xwin), 4
 *              entry-balanced tiles; CMRS: -1 rule, 1 strip runs, 2
 *              entry-balanced tiles
 *   xwin       x windows in LDS: -1 default (CSR, ELL, SELL, CMRS on; COO
 *              off), 0 off, 1 on
 *   xwin_rows  CSR rows per x window; 0 = 128
 *   head       SELL small matrices: the head copy of every wave's first
 *              slot groups; -1 default (on), 0 off
 *   index16    SELL: 1 = SELL16, 16-bit column offsets from each
 *              workgroup's window base (plan-owned copy; C = 64, refused
 *              when a window spans more than 65,536 columns)
 *   coo_pass   COO: -1 the single pass wherever every row ends within 80
 *              entries past its tile, else the carry pass; 0 carry pass;
 *              1 single pass or SPMV_OTHER_ERROR
 *   split      SELL wide slices: -1 rule (spmv_sell_split_auto), 0 off,
 *              T > 0 (a multiple of ki) slot columns per slice in the main
 *              kernel, the rest in chunks
 *   bigplan    tiled CSR: list the rows of tiles owning > 1,024 rows
 *              (runs of empty rows); -1 default (on), 0 off
 *   H          hot-column table for power-law columns (COO, tiled CSR,
 *              SELL, tiled CMRS): the plan renumbers the H most frequent
 *              columns into a compact x table gathered at the start of
 *              every run (spmv_hot_columns, spmv_host.h; plan-owned column
 *              copy); -1 the rule (2^19 columns when n_cols > 2^21 and they
 *              hold half the entries), 0 none (e.g. columns already
 *              relabelled by degree, spmv_column_relabel), > 0 that many  */
enum spmv_fmt { SPMV_FMT_COO = 0, SPMV_FMT_CSR = 1, SPMV_FMT_ELL = 2, SPMV_FMT_SELL = 3, SPMV_FMT_CMRS = 4 };

typedef struct spmv_plan_opts {
    int32_t lanes;
    int32_t variant;
    int32_t xwin;
    int32_t xwin_rows;
    int32_t head;
    int32_t index16;
    int32_t coo_pass;
    int32_t split;
    int32_t bigplan;
    int32_t reserved;
    int64_t H;
} spmv_plan_opts;

typedef struct spmv_plan spmv_plan;

/* What a plan runs (spmv_plan_get_info): kernel = the dominant kernel's
 * name as rocprofv3 reports it (without the namespace and template
 * arguments), desc = one line naming the path and its parameters.       */
typedef struct spmv_plan_info {
    int32_t format;      /* enum spmv_fmt */
    int32_t path;        /* internal path id (stable within a build) */
    int32_t lanes;       /* CSR lanes per row */
    int32_t variant;     /* CSR 1-4; CMRS 0 strip runs, 1 tiles */
    int32_t ki;          /* ELL / SELL k-interleave */
    int32_t xcap;        /* LDS x-window entries (0: no window fits / none) */
    int32_t xwin;        /* x windows built */
    int32_t head;        /* SELL head copy built */
    int32_t single_pass; /* COO without the carry kernel */
    int32_t index16;     /* SELL16 */
    int32_t split_T;     /* SELL split width (0: none) */
    int32_t reserved;
    int64_t n_chunks;    /* SELL split chunks */
    int64_t big_tiles;   /* tiled CSR tiles with a listed row plan */
    int64_t head_bytes;
    int64_t ws_bytes;
    int64_t owned_bytes; /* device bytes the plan allocated */
    int64_t H;
    char kernel[64];
    char desc[320];
} spmv_plan_info;

void spmv_plan_opts_init(spmv_plan_opts *o);
/* Replaces the COO launch (reference coo.c:47-48,68-73,163-168,194;
 * kernels/Coo.cl:24).  Entries sorted by row (any order inside a row:
 * spmv_coo_sort_by_row, spmv_host.h).  o = NULL: defaults.                */
int spmv_plan_coo(spmv_dims d, const int32_t *row, const int32_t *col, const double *val,
                  const spmv_plan_opts *o, spmv_plan **out);
/* Replaces the CSR launch (reference csr.c:47-48,170-175,201;
 * kernels/Csr.cl:1).  row_ptr[N+1] int64, col/val[Z].                     */
int spmv_plan_csr(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                  const spmv_plan_opts *o, spmv_plan **out);
/* Replaces the ELL launch (reference ell.c:47-48,242-248,273;
 * kernels/Ell.cl:1).  Layout of spmv_ell_run below.                       */
int spmv_plan_ell(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *col, const double *val,
                  const spmv_plan_opts *o, spmv_plan **out);
/* Replaces the SELL-C-sigma launch (reference sigma_c.c:50-51,71-72,
 * 280-285,311; kernels/Sigma_C.cl:1).  Layout of spmv_sell_run below.     */
int spmv_plan_sell(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices, const int64_t *slice_ptr,
                   const int32_t *perm, const int32_t *col, const double *val, const spmv_plan_opts *o,
                   spmv_plan **out);
/* Replaces the CMRS launch (reference cmrs.c:51-52,195-205,232;
 * kernels/Cmrs.cl:1).  Layout of spmv_cmrs_run below.                     */
int spmv_plan_cmrs(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr, const uint8_t *row_in_strip,
                   const int32_t *col, const double *val, const spmv_plan_opts *o, spmv_plan **out);
/* y = A x on `stream` (NULL = the default stream; the plan's d.stream is
 * used for building only).  x[n_cols], y[n_rows], device pointers.        */
int spmv_plan_run(const spmv_plan *p, const double *x, double *y, void *stream);
int spmv_plan_get_info(const spmv_plan *p, spmv_plan_info *info);
/* Frees what the plan allocated (never the caller's arrays). */
int spmv_plan_destroy(spmv_plan *p);

/* ------------------------------------------ the five reference kernels ---
 * One call each, no build step, x gathered from global memory: the
 * direct equivalents of the reference's five kernels.  Plans run these
 * or faster variants of them (spmv_ext.h).                               */

/* COO — kernel `coo(row,col,val,x,y,int Z)` (reference kernels/Coo.cl:24).
 * Entries MUST be sorted by row (any order inside a row).  Wave-level
 * segmented reduction over fixed tiles of entries; rows that straddle
 * tiles are finished by a second, deterministic carry pass — no atomics,
 * bitwise reproducible.  `ws` is device scratch of at least
 * spmv_coo_ws_bytes(nnz) bytes.                                          */
size_t spmv_coo_ws_bytes(int64_t nnz);
int spmv_coo_run(spmv_dims d, const int32_t *row, const int32_t *col,
                 const double *val, const double *x, double *y, void *ws,
                 size_t ws_bytes);

/* CSR — kernel `csr(ptr,col,val,x,y,int N)` (reference kernels/Csr.cl:1).
 * CSR-vector: a group of `lanes_per_row` lanes (2..64, power of two) works
 * on one row; the entry stream is staged in LDS; partial sums are reduced
 * with cross-lane moves.  lanes_per_row = 0 picks from the mean row length
 * (spmv_csr_auto_lanes).                                                 */
int spmv_csr_auto_lanes(int64_t n_rows, int64_t nnz);
int spmv_csr_run(spmv_dims d, const int64_t *row_ptr, const int32_t *col,
                 const double *val, const double *x, double *y,
                 int lanes_per_row);

/* ELL — kernel `ell(val,idx,x,y,int N,int K,__local)` (reference
 * kernels/Ell.cl:1).  Column-major, leading dimension `ld` (>= N, multiple
 * of 64), with a k-interleave `ki` in {1,2}: entry (row i, slot k) lives at
 *     (k / ki) * ld * ki + i * ki + (k % ki)
 * so one lane per row reads 8·ki contiguous bytes per step (ki = 2: 16-byte
 * dwordx4 value loads).  K (a multiple of ki) slots per row; padding slots
 * hold value 0.0 and a column already used by the row.                   */
int spmv_ell_run(spmv_dims d, int32_t K, int64_t ld, int32_t ki,
                 const int32_t *col, const double *val, const double *x,
                 double *y);

/* SELL-C-sigma — kernel `sigma_c(val,idx,x,y,slice_ptr,int C)` (reference
 * kernels/Sigma_C.cl:1).  Slices of C rows (C = 64 = one wave by default),
 * rows sorted by length inside windows of sigma rows (builder only), slice
 * s occupies [slice_ptr[s], slice_ptr[s+1]) with entry (slot r, k) at
 *     slice_ptr[s] + (k / ki) * C * ki + r * ki + (k % ki)
 * perm[s*C + r] is the original row of slot r of slice s (-1 = padding
 * slot); y[perm[.]] is written directly, no un-permute pass.  `sigma` is
 * the sorting window the builder used (1 = none; else a multiple of C):
 * one workgroup covers one window so its scattered y stores merge in one
 * L2.  spmv_sell_auto_ki: the k-interleave the SELL builders should use
 * for an n_rows matrix (2 for matrices small enough for the
 * waves-per-slice kernel, else 1), the default of ./bin/sigma_c and
 * spmv_amd.to_device.                                                     */
int spmv_sell_auto_ki(int64_t n_rows, int32_t C);
int spmv_sell_run(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                  const int64_t *slice_ptr, const int32_t *perm,
                  const int32_t *col, const double *val, const double *x,
                  double *y);

/* CMRS — kernel `cmrs(val,idx,strip_ptr,row_in_strip,x,y,N,h,__local)`
 * (reference kernels/Cmrs.cl:1).  Strips of h consecutive rows
 * (1 <= h <= 64); strip s holds entries [strip_ptr[s], strip_ptr[s+1]) in
 * row order and row_in_strip[j] in [0,h) (uint8, the reference used
 * int32).  The strip runs are staged in LDS, each row's slice summed by a
 * lane group; the tail strip is bounds-checked (reference Cmrs.cl:38-42
 * wrote past y).                                                          */
int spmv_cmrs_run(spmv_dims d, int32_t h, int64_t n_strips,
                  const int64_t *strip_ptr, const uint8_t *row_in_strip,
                  const int32_t *col, const double *val, const double *x,
                  double *y);

/* ------------------------------------------------------------ helpers ---
 * Device discovery (replaces reference inc/helper_functions.h:76-129),
 * memory (replaces clCreateBuffer / clEnqueueWriteBuffer /
 * clEnqueueReadBuffer, reference csr.c:123-127,183-186,220), timing.    */
int spmv_device_count(int *count);
int spmv_set_device(int device);
int spmv_device_name(int device, char *buf, size_t len);
int spmv_malloc(void **dptr, size_t bytes);
int spmv_free(void *dptr);
int spmv_memset(void *dptr, int value, size_t bytes, void *stream);
int spmv_upload(void *dptr, const void *host, size_t bytes, void *stream);
int spmv_download(void *host, const void *dptr, size_t bytes, void *stream);
int spmv_stream_create(void **stream);
int spmv_stream_destroy(void *stream);
int spmv_sync(void *stream);
/* Write `bytes` (0 = 512 MiB) of library-owned scratch on `stream` so the
 * 256 MiB Infinity Cache and the per-XCD L2s hold no SpMV operand.      */
int spmv_flush_cache(void *stream, size_t bytes);
/* The same eviction by READING the scratch (the caches then hold clean
 * lines, so the next kernel pays no write-back): bench.py's cold state. */
int spmv_flush_cache_read(void *stream, size_t bytes);
/* Timing events on a stream (hipEvent_t as void *). */
int spmv_event_create(void **ev);
int spmv_event_destroy(void *ev);
int spmv_event_record(void *ev, void *stream);
/* Milliseconds from `start` to `end`; waits for `end` to complete. */
int spmv_event_elapsed(void *start, void *end, double *ms);
/* Time one launch: record an event, call launch(arg), record an event,
 * synchronise, return elapsed milliseconds in *ms.                      */
typedef int (*spmv_launch_fn)(void *arg);
int spmv_time_launch(spmv_launch_fn launch, void *arg, void *stream,
                     double *ms);
/* Frees library-owned scratch on the current device. */
int spmv_release(void);
/* ---------------------------------------------------------- multi-GPU ---
 * Single-process row sharding over several GPUs: the
 * reference creates its OpenCL context over every GPU it finds but uses
 * device 0 only (reference csr.c:107,115; its device loop breaks after the
 * first, csr.c:30,279).  spmv_multi_init builds one RCCL communicator per
 * device with ncclCommInitAll and one non-blocking stream each; the caller
 * cuts contiguous row ranges (spmv_partition_rows), runs every shard's
 * spmv_<fmt>_run on its device's stream writing y_full_d + bounds[d], and
 * spmv_multi_allgatherv completes every device's y_full in place: one
 * ncclBroadcast of each shard's REAL row count from its owner, all in one
 * ncclGroupStart/End (an allgatherv; no padding to the largest shard).  */
typedef struct spmv_multi spmv_multi;
int spmv_multi_init(int n_gpus, const int *devices /* NULL: 0..n_gpus-1 */, spmv_multi **out);
int spmv_multi_free(spmv_multi *m);
int spmv_multi_size(const spmv_multi *m);
int spmv_multi_device(const spmv_multi *m, int i);
void *spmv_multi_stream(const spmv_multi *m, int i);
/* y_full[i]: device i's n-row y (device pointer); bounds[n_gpus + 1]      */
int spmv_multi_allgatherv(spmv_multi *m, double *const *y_full, const int64_t *bounds);
int spmv_multi_sync(spmv_multi *m);
/* Time one launch on every device together: optional flush on each, an
 * event pair around launch(arg, i) on each device's stream, all devices
 * synchronised; ms[i] = device i's elapsed time.                        */
typedef int (*spmv_multi_launch_fn)(void *arg, int i);
int spmv_multi_time(spmv_multi *m, spmv_multi_launch_fn launch, void *arg, int flush, double *ms);

const char *spmv_strerror(int rc);
const char *spmv_last_error(void);
/* Version string of the library build, e.g. "spmv-hip 0.2 gfx950". */
const char *spmv_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SPMV_H */
