/*
 * spmv_host.h — host side of the MI355X SpMV suite (libspmv_host.so).
 *
 * Replaces the reference's host layers L1-L3:
 *   - Matrix Market reading with the reference's acceptance semantics
 *     (reference inc/helper_functions.h:134-165, mmio/mmio.c:96-217,
 *      entry lines "%d %d %lg", csr.c:81);
 *   - the per-format builders that the reference interleaves with fscanf
 *     (reference coo.c:79-84, csr.c:68-91, ell.c:68-164,
 *      sigma_c.c:71-202, cmrs.c:72-117), re-designed for wave64 layouts
 *     and without the reference's empty-row / last-row assumptions;
 *   - the OpenMP CPU loops (reference coo.c:280-300, csr.c:285-309,
 *     ell.c:357-383, cmrs.c:319-345; the reference has none for SELL);
 *   - the run-time result check (reference inc/helper_functions.h:184-236);
 *   - synthetic generators for the configs in BASELINE.json.
 *
 * All functions take caller-allocated arrays ("plan" functions return the
 * sizes to allocate) so the same calls serve the C drivers and ctypes.
 * Return values are spmv_rc.h codes unless stated otherwise.
 */
#ifndef SPMV_HOST_H
#define SPMV_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "spmv_rc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------ Matrix Market ---*/
typedef struct spmv_mtx_info {
    int64_t n_rows;
    int64_t n_cols;
    int64_t nnz;   /* entries listed in the file (= entries multiplied)   */
    int symmetric; /* symmetric / skew / hermitian banner: entries are    */
                   /* taken literally, never mirrored (reference A12)     */
    int pattern;   /* pattern banner: every entry's value is 1.0          */
    int integer;   /* integer banner: values parsed as numbers            */
} spmv_mtx_info;

/* Banner + size line only.  SPMV_FILE_ERROR if the file is missing, the
 * banner is malformed, or the matrix is complex or dense (array).       */
int spmv_mtx_read_info(const char *path, spmv_mtx_info *info);
/* Banner + size + exactly info->nnz entries in FILE ORDER, converted to
 * 0-based.  row/col/val must hold info->nnz elements (read_info first).
 * Out-of-range indices or a short file give SPMV_FILE_ERROR.            */
int spmv_mtx_read(const char *path, spmv_mtx_info *info, int32_t *row,
                  int32_t *col, double *val);
/* Writes a coordinate real file with %.17g values (exact round trip).   */
int spmv_mtx_write(const char *path, int64_t n_rows, int64_t n_cols,
                   int64_t nnz, const int32_t *row, const int32_t *col,
                   const double *val, int symmetric);

/* Binary cache of a parsed file: header + row, col,
 * val arrays in file order.  The drivers' --cache option keeps PATH.bin
 * next to PATH and reads it instead of the text when it is newer.       */
int spmv_bin_write(const char *path, const spmv_mtx_info *info,
                   const int32_t *row, const int32_t *col, const double *val);
int spmv_bin_read_info(const char *path, spmv_mtx_info *info);
int spmv_bin_read(const char *path, spmv_mtx_info *info, int32_t *row,
                  int32_t *col, double *val);

/* ------------------------------------------------------------ formats ---*/
/* COO sorted by row, stable (file order kept inside a row).             */
int spmv_coo_sort_by_row(int64_t n_rows, int64_t nnz, const int32_t *row,
                         const int32_t *col, const double *val,
                         int32_t *row_out, int32_t *col_out, double *val_out);
/* CSR from COO in any order: stable counting sort by row; empty rows ok.
 * row_ptr[n_rows+1], col_out[nnz], val_out[nnz].                        */
int spmv_csr_from_coo(int64_t n_rows, int64_t nnz, const int32_t *row,
                      const int32_t *col, const double *val,
                      int64_t *row_ptr, int32_t *col_out, double *val_out);
/* Entries of every CSR row reordered by increasing column (stable).  With
 * degree-relabelled columns (spmv_column_relabel) a long row then reads x
 * from its dense hot prefix in address order.  Changes each row's
 * summation order (not the products): y within the parity rule.          */
int spmv_csr_sort_rows(int64_t n_rows, const int64_t *row_ptr, int32_t *col, double *val);
/* Row-length statistics of a CSR matrix. */
int spmv_csr_row_stats(int64_t n_rows, const int64_t *row_ptr,
                       int64_t *min_len, int64_t *max_len, double *mean_len);
/* CSR kernel variant for this matrix (include/spmv.h): 4 = entry-balanced
 * tiled (spmv_csr_run_tiled) when the longest row exceeds both 4,096
 * entries and 64x the mean (a row-per-group kernel would then wait on one
 * group), else 0 (the library's row-group default).                    */
int spmv_csr_pick_variant(int64_t n_rows, const int64_t *row_ptr);
/* The rule itself, from the longest row (max_len) and the entry count:
 * shared with the CSR plan of spmv.h, which finds max_len on the device. */
int spmv_csr_variant_rule(int64_t n_rows, int64_t nnz, int64_t max_len);

/* Hot columns for spmv_csr_run_tiled_hot: the H most frequent columns in
 * decreasing count (ties: lower column first) into hot[], and col_out
 * (may alias col) = col with every hot column c renumbered n_cols +
 * rank(c).  H_req > 0 takes min(H_req, non-empty columns); H_req = 0 is
 * the rule: 2^19 columns (4 MiB of x, one XCD's L2; halved down to 2^16
 * while above nnz / 32) when n_cols > 2^21,
 * they hold at least half of the entries and at least 8 entries each on
 * average (the table fill re-reads each once), else none (col_out = col).
 * hot[] holds max(H_req, 2^19) entries.  Returns H, -1 on bad input.    */
int64_t spmv_hot_columns(int64_t n_cols, int64_t nnz, const int32_t *col, int64_t H_req, int32_t *hot,
                         int32_t *col_out);
/* 0 when spmv_hot_columns(n_cols, ..., H_req, ...) returns 0 whatever the
 * columns (the rule never tables a matrix of <= 2^21 columns): lets a
 * caller skip fetching the columns.                                      */
int spmv_hot_columns_possible(int64_t n_cols, int64_t H_req);

/* Big-tile plan of the entry-balanced CSR (spmv_csr_run_tiled_plan):
 * with tiles of `tile` entries (spmv_csr_tiled_tile), every tile owning
 * more than `cap` rows (the rows whose first offset lies in it; the last
 * tile also the trailing rows) and at most 65,536 gets the list of its
 * owned rows that have entries in it, as int32 pairs {row - first owned
 * row, a | b << 16} with [a, b) relative to the tile start.  Layout
 * (int32): idx[tiles] (-1 or the big tile's number k), start[nbig + 1]
 * (absolute, even positions), then the pairs.  plan = NULL returns the
 * length only.  Returns the int32 length, -1 on bad input.                */
int64_t spmv_csr_tiled_bigplan(int64_t n_rows, const int64_t *row_ptr, int64_t tile, int32_t cap,
                               int32_t *plan);

/* Degree-ordered column relabel (power-law columns, x replicated): the
 * columns ranked by decreasing entry count (ties: lower column first;
 * columns without entries last, in id order).  order[rank] = column,
 * newid[column] = rank, and col_out (may alias col) = newid[col].  The
 * relabelled matrix A' = A·Pᵀ takes x' = P·x (x'[k] = x[order[k]]) and
 * gives the same y in the same row order, bit for bit with any kernel
 * whose per-row summation order does not depend on column ids: the hot
 * columns are x'[0..H) (no per-run hot-table fill) and the touched part of
 * x is one dense prefix.  Returns the number of non-empty columns, -1 on
 * bad input.                                                             */
int64_t spmv_column_relabel(int64_t n_cols, int64_t nnz, const int32_t *col, int32_t *order, int32_t *newid,
                            int32_t *col_out);
/* The same with a choice of tie order among equal counts: ties = 0 lower
 * column first (spmv_column_relabel), 1 first appearance in col (for a
 * row-major CSR col: the first row that uses the column, so the low-degree
 * columns of neighbouring rows share x' lines).  -1 on bad input.        */
int64_t spmv_column_relabel_ex(int64_t n_cols, int64_t nnz, const int32_t *col, int32_t *order, int32_t *newid,
                               int32_t *col_out, int32_t ties);

/* ELL, column-major with leading dimension ld = round_up(N, 64) and
 * k-interleave ki (spmv.h).  K = round_up(max row length, ki).
 * spmv_ell_plan gives K and ld; arrays are ld*K elements.               */
int spmv_ell_plan(int64_t n_rows, const int64_t *row_ptr, int32_t ki,
                  int32_t *K, int64_t *ld);
int spmv_ell_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col,
                  const double *val, int32_t K, int64_t ld, int32_t ki,
                  int32_t *col_out, double *val_out);

/* SELL-C-sigma: rows sorted by decreasing length inside windows of sigma
 * rows (sigma = 1: no sorting, the reference's sigma_c.c:48 behaviour;
 * sigma must be 1 or a multiple of C), slices of C rows, slice width =
 * round_up(longest row of the slice, ki).  Plan returns n_slices and the
 * stored element count; perm has n_slices*C entries.                    */
int spmv_sell_plan(int64_t n_rows, const int64_t *row_ptr, int32_t C,
                   int32_t sigma, int32_t ki, int64_t *n_slices,
                   int64_t *stored);
int spmv_sell_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col,
                   const double *val, int32_t C, int32_t sigma, int32_t ki,
                   int64_t n_slices, int64_t *slice_ptr, int32_t *perm,
                   int32_t *col_out, double *val_out);

/* CMRS: strips of h rows (1..64), n_strips = ceil(N/h).  The CSR arrays
 * are reused unchanged; this builds strip_ptr[n_strips+1] and
 * row_in_strip[nnz].                                                    */
int spmv_cmrs_build(int64_t n_rows, const int64_t *row_ptr, int32_t h,
                    int64_t *strip_ptr, uint8_t *row_in_strip);
/* 1 = entry-balanced (spmv_cmrs_run_tiled) when the longest strip exceeds
 * both 4,096 entries and 64x the mean strip, else 0 (spmv_cmrs_run).    */
int spmv_cmrs_pick_variant(int64_t n_strips, const int64_t *strip_ptr);
/* The rule from the longest strip and the entry count (the CMRS plan).  */
int spmv_cmrs_variant_rule(int64_t n_strips, int64_t nnz, int64_t max_len);

/* SELL split plan for wide slices (spmv_sell_run_split).  _auto gives T
 * (slot columns kept by the main kernel, a multiple of ki) or 0 when no
 * slice is wider than both 1,024 and 16x the mean width.  _plan lists the
 * chunks [k0, k0+T) beyond the first T columns of every slice (T = 256), in slice
 * order, and returns their count (arrays may be NULL: count only); -1 on
 * bad arguments.                                                        */
int32_t spmv_sell_split_auto(int64_t n_slices, const int64_t *slice_ptr, int32_t C, int32_t ki);
int64_t spmv_sell_split_plan(int64_t n_slices, const int64_t *slice_ptr, int32_t C, int32_t T,
                             int32_t *chunk_slice, int32_t *chunk_k0);

/* HYB = ELL + COO tail: the first K entries of every
 * row in the column-major ELL layout of spmv_ell_fill (ld, ki), the rest
 * as a row-sorted COO tail.  K_req > 0 forces K (rounded up to ki); 0
 * picks the K that minimises stored bytes (12 per ELL slot, 16 per tail
 * entry) plus 32 MB when both parts are non-empty (the second kernel's
 * fixed cost): K = 0 (all tail) or the longest row (no tail) where the
 * split does not save more.  Fill: ell_col/ell_val[K*ld],
 * tail_row/col/val[tail_nnz].                                            */
int spmv_hyb_plan(int64_t n_rows, const int64_t *row_ptr, int32_t ki, int32_t K_req, int32_t *K,
                  int64_t *ld, int64_t *tail_nnz);
int spmv_hyb_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col, const double *val,
                  int32_t K, int64_t ld, int32_t ki, int32_t *ell_col, double *ell_val,
                  int32_t *tail_row, int32_t *tail_col, double *tail_val);

/* CSR with compressed 16-bit column indices: the
 * CSR entries are cut into 64-entry blocks (entry p in block p/64).  A
 * block whose columns span < 65536 stores blk_base = its smallest column
 * and col_off[p] = col[p] - blk_base; any other block stores its columns
 * whole in col_esc[slot*64 .. +64) and blk_base = -1 - slot.  row_ptr and
 * val are CSR's.  Plan: n_blocks = ceil(nnz/64), n_esc escaped blocks.
 * Fill: blk_base[n_blocks], col_off[nnz], col_esc[n_esc*64].            */
int spmv_csr16_plan(int64_t nnz, const int32_t *col, int64_t *n_blocks, int64_t *n_esc);
int spmv_csr16_fill(int64_t nnz, const int32_t *col, int32_t *blk_base, uint16_t *col_off,
                    int32_t *col_esc);

/* Column-grouped CSR (CSRG) for gather-bound power-law matrices (R-MAT,
 * BASELINE.json configs[3]).  x is cut into `groups` (1..64) groups of
 * whole 128-byte lines (16 columns): the line c/16 belongs to group
 * spmv_csrg_group(c, groups), a hash, so hot and cold lines spread evenly.
 * The entries are stored group after group; inside a group, as a CSR over
 * the PAIRS (row, group) that hold entries, rows ascending, each pair's
 * entries in CSR order.  A run sums every pair (the groups one after
 * another, so the x lines being gathered stay in the L2s) and then adds
 * each row's pair sums in group order, block by block of
 * SPMV_CSRG_ROWS rows: blk_off[g*(nb+1) + b] is the first pair of group g
 * whose row is >= b*SPMV_CSRG_ROWS (nb = ceil(n_rows / SPMV_CSRG_ROWS)),
 * pair_row[p] the pair's row modulo SPMV_CSRG_ROWS.  Plan: n_pairs.
 * Fill: pair_ptr[n_pairs+1], col_g/val_g[nnz], blk_off[groups*(nb+1)],
 * pair_row[n_pairs].                                                    */
/* fixed (no -D override): the host fill, the device reduce and the Python
 * binding (spmv_csrg_block_rows) must agree on it */
#define SPMV_CSRG_ROWS 4096 /* also in spmv.h */
int32_t spmv_csrg_block_rows(void); /* SPMV_CSRG_ROWS as built into libspmv_host */
int32_t spmv_csrg_group(int32_t col, int32_t groups);
int spmv_csrg_plan(int64_t n_rows, const int64_t *row_ptr, const int32_t *col, int32_t groups,
                   int64_t *n_pairs);
int spmv_csrg_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col, const double *val,
                   int32_t groups, int64_t *pair_ptr, int32_t *col_g, double *val_g,
                   int32_t *blk_off, uint16_t *pair_row);

/* ----------------------------------------------------- multi-GPU shard ---
 * Row-range partition for one process per GPU: `parts`
 * contiguous ranges [bounds[p], bounds[p+1]) holding about nnz/parts
 * entries each; every inner boundary is a multiple of `align` (use the
 * SELL sigma, 1024, so sorting windows never straddle two GPUs).
 * bounds has parts+1 entries, bounds[0] = 0, bounds[parts] = n_rows.    */
int spmv_partition_rows(int64_t n_rows, const int64_t *row_ptr, int parts,
                        int64_t align, int64_t *bounds);
/* The entries of rows [lo, hi) in FILE ORDER with rows renumbered to the
 * shard (row - lo), for a device that owns those rows; returns the count
 * (output arrays NULL: count only), -1 on bad arguments.  Every entry
 * lands in exactly one shard of a partition, so the shards' y slices,
 * written at y + lo, reassemble y.                                      */
int64_t spmv_coo_row_shard(int64_t nnz, const int32_t *row, const int32_t *col, const double *val,
                           int64_t lo, int64_t hi, int32_t *row_out, int32_t *col_out, double *val_out);
/* Same cut, balancing entries + row_weight per row (a row costs the
 * kernels about as much as row_weight entries: its offset, its y store and
 * its reduction; 0 = spmv_partition_rows).                              */
int spmv_partition_rows_weighted(int64_t n_rows, const int64_t *row_ptr, int parts, int64_t align,
                                 double row_weight, int64_t *bounds);
/* Profile-guided re-cut: old_bounds (old_parts + 1) with the measured time
 * of each old shard (old_ms) give every row the cost rate_g * (entries +
 * row_weight) of the old shard g holding it (rate_g = ms_g / that shard's
 * entries + row_weight * rows); the new `parts` ranges hold equal shares
 * of that cost, aligned as spmv_partition_rows.  For shards whose cost per
 * entry differs (R-MAT hub shards against shards of short rows).         */
int spmv_partition_rows_calibrated(int64_t n_rows, const int64_t *row_ptr, int parts, int64_t align,
                                   double row_weight, int old_parts, const int64_t *old_bounds,
                                   const double *old_ms, int64_t *bounds);

/* ---------------------------------------------------------- CPU loops ---
 * OpenMP restatements of the reference's compute_using_cpu loops, with
 * zero-initialised output (the reference accumulated into malloc'd
 * memory, reference csr.c:102).  `threads` <= 0 uses omp_get_max_threads.
 * They are the CPU baseline the drivers print, never a device fallback. */
int spmv_cpu_coo(int64_t n_rows, int64_t nnz, const int32_t *row,
                 const int32_t *col, const double *val, const double *x,
                 double *y, int threads);
int spmv_cpu_csr(int64_t n_rows, const int64_t *row_ptr, const int32_t *col,
                 const double *val, const double *x, double *y, int threads);
int spmv_cpu_ell(int64_t n_rows, int32_t K, int64_t ld, int32_t ki,
                 const int32_t *col, const double *val, const double *x,
                 double *y, int threads);
int spmv_cpu_sell(int64_t n_rows, int32_t C, int32_t ki, int64_t n_slices,
                  const int64_t *slice_ptr, const int32_t *perm,
                  const int32_t *col, const double *val, const double *x,
                  double *y, int threads);
int spmv_cpu_cmrs(int64_t n_rows, int32_t h, int64_t n_strips,
                  const int64_t *strip_ptr, const uint8_t *row_in_strip,
                  const int32_t *col, const double *val, const double *x,
                  double *y, int threads);
int spmv_cpu_threads(void);

/* ------------------------------------------------------ result check ---
 * The reference's check_result (inc/helper_functions.h:184-236): y_ref
 * is accumulated sequentially in FILE ORDER.  Returns the number of rows
 * that fail; *first_bad gets the first failing row (-1 if none).
 * abs_tol > 0: the reference's |y - y_ref| <= 1e-6 rule;
 * rel_tol > 0: |y - y_ref| <= rel_tol * max(|y_ref|, sum_j |a_ij x_j|).  */
int64_t spmv_check(int64_t n_rows, int64_t nnz, const int32_t *row,
                   const int32_t *col, const double *val, const double *x,
                   const double *y, double abs_tol, double rel_tol,
                   int64_t *first_bad, double *y_ref_at_bad);

/* --------------------------------------------------------- generators ---
 * Deterministic (splitmix64 counter-based), identical on every host.
 *
 * cant-like stand-in for SuiteSparse cant (N = M = 62,451 = 3 dof x
 * 9x9x257 nodes, 27-node neighbourhood).  The pattern is thinned
 * symmetrically to exactly 4,007,383 entries (2,034,917 in the lower
 * triangle incl. diagonal) — the real cant's counts.  mode:
 *   0 = full pattern, row-major order          ("cant-sorted" shape)
 *   1 = full pattern, column-major order       ("cant" shape)
 *   2 = lower triangle only, column-major order (SuiteSparse storage;
 *       banner symmetric — the reference multiplies it literally)
 * `copies` > 1 stacks that many independent copies block-diagonally.
 * Call with row == NULL to get *nnz only.                              */
int spmv_gen_cantlike(int mode, int64_t copies, int64_t *n_rows,
                      int64_t *nnz, int32_t *row, int32_t *col, double *val);
/* R-MAT (a,b,c,d) = (0.57,0.19,0.19,0.05) on 2^scale ids, rejection to
 * [0,n); exactly nnz entries, duplicates kept; values uniform [-1,1).
 * Entries in generation order.                                         */
int spmv_gen_rmat(int64_t n, int64_t nnz, int scale, uint64_t seed,
                  int32_t *row, int32_t *col, double *val);
/* Banded: row i has 16 entries at columns (i + o) mod n, o in -8..7,
 * directly in CSR form (row_ptr[n+1], col[16n], val[16n]).             */
int spmv_gen_banded_csr(int64_t n, uint64_t seed, int64_t row_begin,
                        int64_t row_end, int64_t *row_ptr, int32_t *col,
                        double *val);
/* Uniformly random sparse matrix with row lengths in [min_len,max_len]
 * (test helper for ragged inputs), CSR order.                          */
int spmv_gen_random(int64_t n_rows, int64_t n_cols, int64_t min_len,
                    int64_t max_len, uint64_t seed, int64_t *nnz,
                    int32_t *row, int32_t *col, double *val);
/* splitmix64 of (seed, index), exported for tests. */
uint64_t spmv_splitmix64(uint64_t seed, uint64_t index);

#ifdef __cplusplus
}
#endif

#endif /* SPMV_HOST_H */
