/*
 * spmv_ext.h — the extended C-ABI of libspmv_hip.so (beyond the drop-in
 * boundary of spmv.h):
 *   - the kernel variants the plans of spmv.h choose between (x windows in
 *     LDS, head copies, the single-pass COO, entry-balanced tiles with
 *     their tile and big-tile plans, the SELL split, hot-column tables),
 *     each callable on its own: the A/B tools and the tests that pin each
 *     variant's bits use them;
 *   - the SURVEY.md §8f row-4 formats (CSR16, CSR with fp32 values, HYB,
 *     SELL16, column-grouped CSR), the device format builders (§8f row 2),
 *     the banded generator of configs[4] and the vector kernels of the
 *     iterated SpMV (§8f row 3);
 *   - the library's A/B switches (placement and load policy; never a
 *     result bit).
 * The conventions of spmv.h hold for every entry point here.  A drop-in
 * caller needs none of this: spmv_plan_<fmt> + spmv_plan_run select and
 * prepare these paths themselves.
 */
#ifndef SPMV_EXT_H
#define SPMV_EXT_H

#include "spmv.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- COO ---
 * (spmv_coo_run / spmv_coo_ws_bytes: spmv.h) */
/* Single-pass COO (no carry pass): every workgroup also loads the entries of
 * its last row that lie past its 1,536-entry tile and finishes that row; a
 * row begun in an earlier tile is left to that tile.  Build once:
 * spmv_coo_tail_build counts those entries per tile into `tails`
 * (spmv_coo_tail_bytes bytes) and returns SPMV_OTHER_ERROR when a row runs
 * more than 80 entries past a tile end (use spmv_coo_run).  Deterministic;
 * rows that span tiles are summed in one pass, so y agrees with
 * spmv_coo_run to the parity rule.  (reference kernels/Coo.cl, coo.c:194) */
size_t spmv_coo_tail_bytes(int64_t nnz);
int spmv_coo_tail_build(spmv_dims d, const int32_t *row, void *tails, size_t tails_bytes);
int spmv_coo_run_tail(spmv_dims d, const int32_t *row, const int32_t *col, const double *val,
                      const double *x, double *y, const void *tails);

/* ---------------------------------------------------------------- CSR ---
 * (spmv_csr_run / spmv_csr_auto_lanes: spmv.h) */
/* spmv_csr_run, with the kernel variant explicit: 0 = library default,
 * 1 = direct (each lane group streams its own row's entries),
 * 2 = staged (all 256 lanes of a workgroup stream the workgroup's entry
 *     range through LDS, then each lane group reduces its row from LDS),
 * 3 = staged, persistent workgroups with row-offset prefetch.
 * Variants 2 and 3 give bit-identical y (and so does spmv_csr_run_xwin);
 * any other value is refused (the entry-balanced kernel for skewed rows is
 * spmv_csr_run_tiled).                                                    */
int spmv_csr_run_variant(spmv_dims d, const int64_t *row_ptr,
                         const int32_t *col, const double *val,
                         const double *x, double *y, int lanes_per_row,
                         int variant);
/* CSR with each row group's x window staged in LDS (the default staged
 * kernel, variant 3, whose gathers read LDS instead of global memory).
 * Build once: spmv_csr_xwin_build scans col (device) for the column range
 * of every window of rows_per_window rows (0 = library default, 128;
 * rounded up to whole groups of 256/L rows, L = lanes_per_row, 0 = auto)
 * into `win` (spmv_csr_xwin_bytes bytes) and returns in *xcap the LDS
 * entries the run stages (0: no window fits).  The run must pass the same
 * lanes_per_row and rows_per_window.  y is bit-identical to
 * spmv_csr_run_variant(..., L, 3).                                       */
size_t spmv_csr_xwin_bytes(int64_t n_rows, int64_t nnz, int lanes_per_row, int32_t rows_per_window);
int spmv_csr_xwin_build(spmv_dims d, const int64_t *row_ptr, const int32_t *col, int lanes_per_row,
                        int32_t rows_per_window, void *win, size_t win_bytes, int32_t *xcap);
int spmv_csr_run_xwin(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                      const double *x, double *y, int lanes_per_row, int32_t rows_per_window,
                      const void *win, int32_t xcap);
/* CSR with compressed 16-bit column indices (arrays
 * from spmv_csr16_plan/fill in spmv_host.h): 10.06 instead of 12 bytes per
 * entry when 64-entry blocks of columns span < 65536 (banded / FEM
 * matrices).  Same kernel as CSR variant 3 with the column source swapped,
 * so y is bit-identical to spmv_csr_run_variant(..., 3).                 */
int spmv_csr16_run(spmv_dims d, const int64_t *row_ptr, const int32_t *blk_base,
                   const uint16_t *col_off, const int32_t *col_esc, const double *val,
                   const double *x, double *y, int lanes_per_row);
/* CSR16 on the x-window pipeline of spmv_csr_run_xwin (same chunks, same
 * order: y bit-identical to it).  win/xcap from spmv_csr_xwin_build over
 * the matrix's int32 columns with the same lanes_per_row/rows_per_window. */
int spmv_csr16_run_xwin(spmv_dims d, const int64_t *row_ptr, const int32_t *blk_base,
                        const uint16_t *col_off, const int32_t *col_esc, const double *val,
                        const double *x, double *y, int lanes_per_row, int32_t rows_per_window,
                        const void *win, int32_t xcap);
/* CSR with fp32 values (§8f row 4): 8 bytes per entry instead of 12.  The
 * x-window kernel widens each value to fp64 and sums in fp64, so y equals
 * spmv_csr_run_xwin on the fp32-rounded values bit for bit (|y - y64| <=
 * 2^-24 * sum_j |a_ij x_j|, inside the 1e-6 parity criterion).  win/xcap
 * from spmv_csr_xwin_build (same row_ptr, col, lanes, rows_per_window).  */
int spmv_csr_f32v_run_xwin(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const float *val,
                           const double *x, double *y, int lanes_per_row, int32_t rows_per_window,
                           const void *win, int32_t xcap);
/* fp32 values on the entry-balanced CSR (skewed rows), with the hot-column
 * table and tile plan of spmv_csr_run_tiled_hot (H = 0: no table).     */
int spmv_csr_f32v_run_tiled_hot(spmv_dims d, const int64_t *row_ptr, const int32_t *col_hot,
                                const float *val, const double *x, double *y, int64_t H,
                                const int32_t *hot, const int32_t *own_lo_plan, void *ws,
                                size_t ws_bytes);
/* Entry-balanced CSR for skewed row lengths (power-law / R-MAT hubs):
 * every workgroup takes the same number of ENTRIES, whatever the rows; a
 * row that spans workgroups is finished by a deterministic carry pass (as
 * COO).  `ws` is device scratch of spmv_csr_tiled_ws_bytes() bytes.      */
size_t spmv_csr_tiled_ws_bytes(int64_t n_rows, int64_t nnz);
int spmv_csr_run_tiled(spmv_dims d, const int64_t *row_ptr, const int32_t *col,
                       const double *val, const double *x, double *y, void *ws,
                       size_t ws_bytes);

/* Hot-column CSR for power-law columns (R-MAT: the 2^19 most frequent of
 * 1e7 columns hold ~84 % of the entries): col_hot from spmv_hot_columns
 * (spmv_host.h) names the H hottest columns n_cols + rank; the run gathers
 * xh[rank] = x[hot[rank]] into the workspace and the tiled kernel reads
 * those x values from the compact table, which stays in L2, instead of
 * from one 128-B line each spread over the whole vector.  y is
 * bit-identical to spmv_csr_run_tiled.  `ws` holds
 * spmv_csr_hot_ws_bytes() bytes; H = 0 is spmv_csr_run_tiled.           */
size_t spmv_csr_hot_ws_bytes(int64_t n_rows, int64_t nnz, int64_t H);
int spmv_csr_run_tiled_hot(spmv_dims d, const int64_t *row_ptr, const int32_t *col_hot,
                           const double *val, const double *x, double *y, int64_t H,
                           const int32_t *hot, const int32_t *own_lo_plan, void *ws,
                           size_t ws_bytes);
/* The tile -> first owned row table of the entry-balanced CSR (int32,
 * spmv_csr_tiled_plan_len(nnz) entries) built once from row_ptr; passed as
 * own_lo_plan it saves every run its pre-pass (NULL: built per run).     */
int64_t spmv_csr_tiled_plan_len(int64_t nnz);
int spmv_csr_tiled_plan(spmv_dims d, const int64_t *row_ptr, int32_t *own_lo);
/* Entries per tile of the entry-balanced CSR for this matrix (the `tile`
 * of spmv_csr_tiled_bigplan, spmv_host.h). */
int64_t spmv_csr_tiled_tile(int64_t n_rows, int64_t nnz);
/* spmv_csr_run_tiled_hot with the big-tile plan (spmv_csr_tiled_bigplan,
 * uploaded; own_lo_plan required): a tile owning more than 1,024 rows (long
 * runs of empty rows) writes its rows without entries as zeros and sums
 * only the listed ones.  big_len = the plan's int32 length, big_tile = the
 * tile it was built for; the call refuses a plan built for another tile
 * (spmv_csr_tiled_tile) or shorter than its tile index, and the kernel
 * bounds-checks every plan read against big_len.  big = NULL is
 * spmv_csr_run_tiled_hot.  Same products; rows of a big tile are summed in
 * entry order by one lane. */
int spmv_csr_run_tiled_plan(spmv_dims d, const int64_t *row_ptr, const int32_t *col_hot,
                            const double *val, const double *x, double *y, int64_t H,
                            const int32_t *hot, const int32_t *own_lo_plan, const int32_t *big,
                            int64_t big_len, int64_t big_tile, void *ws, size_t ws_bytes);
/* Column-grouped CSR (CSRG, spmv_csrg_plan/fill in spmv_host.h) for
 * gather-bound power-law matrices; replaces the same reference kernel
 * (kernels/Csr.cl) on that input.  The entry-balanced kernel runs the
 * n_pairs (row, column-group) pairs group after group, so the x lines the
 * tiles in flight gather from are one group's and stay in L2; each pair's
 * sum goes to the workspace, then one workgroup per SPMV_CSRG_ROWS rows adds
 * its rows' pair sums in group order in LDS (blk_off / pair_row) and writes
 * y.  own_lo_plan: spmv_csr_tiled_plan over (pair_ptr, n_rows = n_pairs),
 * or NULL.  `ws` holds spmv_csrg_ws_bytes(n_pairs, nnz) bytes.
 * Deterministic; agrees with spmv_csr_run to the parity rule (the row sums
 * are grouped by column group).                                          */
/* fixed (no -D override): the host fill, the device reduce and the Python
 * binding (spmv_csrg_block_rows) must agree on it */
#define SPMV_CSRG_ROWS 4096 /* also in spmv_host.h */
size_t spmv_csrg_ws_bytes(int64_t n_pairs, int64_t nnz);
int spmv_csrg_run(spmv_dims d, int32_t groups, int64_t n_pairs, const int64_t *pair_ptr,
                  const int32_t *col_g, const double *val_g, const int32_t *own_lo_plan,
                  const int32_t *blk_off, const uint16_t *pair_row, const double *x, double *y,
                  void *ws, size_t ws_bytes);

/* ---------------------------------------------------------------- ELL ---
 * (spmv_ell_run and the layout: spmv.h) */
/* ELL with each 256-row workgroup's x window staged in LDS (see
 * spmv_sell_xwin_build for the protocol); y bit-identical to spmv_ell_run. */
size_t spmv_ell_xwin_bytes(int64_t n_rows);
int spmv_ell_xwin_build(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *col,
                        void *win, size_t win_bytes, int32_t *xcap);
int spmv_ell_run_xwin(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *col,
                      const double *val, const double *x, double *y, const void *win, int32_t xcap);

/* HYB (arrays from spmv_hyb_plan/fill in spmv_host.h):
 * the ELL part writes y, the row-sorted COO tail of the long rows is added
 * by the staged COO kernel in accumulate mode and the deterministic carry
 * pass.  `ws` holds spmv_hyb_ws_bytes(tail_nnz) bytes.                    */
size_t spmv_hyb_ws_bytes(int64_t tail_nnz);
/* HYB over a hot-column table (spmv_hot_columns over the ELL and tail
 * columns together): bit-identical to spmv_hyb_run on the original
 * columns; `ws` holds spmv_hyb_hot_ws_bytes(tail_nnz, H) bytes.          */
size_t spmv_hyb_hot_ws_bytes(int64_t tail_nnz, int64_t H);
int spmv_hyb_run_hot(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col_hot,
                     const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                     const int32_t *tail_col_hot, const double *tail_val, const double *x, double *y,
                     int64_t H, const int32_t *hot, void *ws, size_t ws_bytes);
/* K = 0 (no ELL part; the tail is the whole matrix): every spmv_hyb_run*
 * runs it as COO (spmv_coo_run / spmv_coo_run_tail / spmv_coo_run_hot) and
 * y has COO's bits. */
int spmv_hyb_run(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col,
                 const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                 const int32_t *tail_col, const double *tail_val, const double *x, double *y,
                 void *ws, size_t ws_bytes);
/* HYB with a single-pass tail (no carry pass, no workspace): `tails` built
 * by spmv_coo_tail_build over the tail (dims.nnz = tail_nnz), which refuses
 * a tail row running more than 80 entries past a tile end. */
int spmv_hyb_run_tail(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col,
                      const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                      const int32_t *tail_col, const double *tail_val, const double *x, double *y,
                      const void *tails);

/* spmv_hyb_run_tail with the ELL part through the x-window ELL kernel
 * (`win`, `xcap` from spmv_ell_xwin_build over ell_col); same bits. */
int spmv_hyb_run_tail_xwin(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col,
                           const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                           const int32_t *tail_col, const double *tail_val, const double *x, double *y,
                           const void *tails, const void *win, int32_t xcap);

/* -------------------------------------------------------- SELL-C-sigma ---
 * (spmv_sell_run, spmv_sell_auto_ki and the layout: spmv.h) */
/* SELL with each workgroup's x window staged in LDS (MI355X: 160 KiB LDS
 * per CU).  Build once: spmv_sell_xwin_build scans col (device) for every
 * workgroup's column range into `win` (spmv_sell_xwin_bytes bytes) and
 * returns in *xcap the LDS entries the run needs (0: no window fits, the
 * run gathers from global memory).  spmv_sell_run_xwin copies x[lo..hi]
 * into LDS per workgroup and gathers from there; y is bit-identical to
 * spmv_sell_run's.                                                       */
/* SELL with wide slices split (power-law matrices; plan from
 * spmv_sell_split_plan in spmv_host.h, uploaded): the main kernel covers
 * the first T slot columns of every slice (win = NULL: global x gathers,
 * else the x-window kernel with win/xcap from spmv_sell_xwin_build); chunk
 * c covers columns [chunk_k0[c], +T) of slice chunk_slice[c], one lane per
 * slot, and the chunks of a slice are added to y[perm] in chunk order.
 * `ws` holds spmv_sell_split_ws_bytes(n_chunks, C) bytes.               */
size_t spmv_sell_split_ws_bytes(int64_t n_chunks, int32_t C);
int spmv_sell_run_split(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                        const int64_t *slice_ptr, const int32_t *perm, const int32_t *col,
                        const double *val, const double *x, double *y, const void *win,
                        int32_t xcap, int32_t T, int64_t n_chunks, const int32_t *chunk_slice,
                        const int32_t *chunk_k0, void *ws, size_t ws_bytes);
/* SELL over a hot-column table (col_hot / hot from spmv_hot_columns on the
 * stored SELL columns), global x gathers, with the split plan of
 * spmv_sell_run_split (T = INT32_MAX and n_chunks = 0: no split).  `ws`
 * holds spmv_sell_hot_ws_bytes(n_chunks, C, H) bytes; bit-identical to
 * spmv_sell_run_split on the original columns.                          */
size_t spmv_sell_hot_ws_bytes(int64_t n_chunks, int32_t C, int64_t H);
int spmv_sell_run_hot(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                      const int64_t *slice_ptr, const int32_t *perm, const int32_t *col_hot,
                      const double *val, const double *x, double *y, int32_t T, int64_t n_chunks,
                      const int32_t *chunk_slice, const int32_t *chunk_k0, int64_t H,
                      const int32_t *hot, void *ws, size_t ws_bytes);
size_t spmv_sell_xwin_bytes(int64_t n_slices, int32_t C, int32_t sigma);
int spmv_sell_xwin_build(spmv_dims d, int32_t C, int32_t sigma, int64_t n_slices,
                         const int64_t *slice_ptr, const int32_t *col, void *win,
                         size_t win_bytes, int32_t *xcap);
int spmv_sell_run_xwin(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                       const int64_t *slice_ptr, const int32_t *perm, const int32_t *col,
                       const double *val, const double *x, double *y, const void *win,
                       int32_t xcap);
/* SELL16 (compressed indices; replaces the same
 * reference kernel, kernels/Sigma_C.cl): the SELL-C-σ arrays with every
 * stored column kept as a 16-bit offset from its workgroup's x-window base,
 * 10 instead of 12 bytes per slot.  C must be 64.  Build once: win / xcap
 * from spmv_sell_xwin_build, then spmv_sell16_fill writes col16[stored]
 * from col on the device; it returns SPMV_OTHER_ERROR (nothing written)
 * when some workgroup's columns span more than 65,536 (the caller keeps
 * plain SELL).  spmv_sell16_run gives y bit-identical to spmv_sell_run_xwin
 * with the same ki.                                                      */
int spmv_sell16_fill(spmv_dims d, int32_t C, int32_t sigma, int64_t n_slices,
                     const int64_t *slice_ptr, const int32_t *col, const void *win,
                     uint16_t *col16);
int spmv_sell16_run(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                    const int64_t *slice_ptr, const int32_t *perm, const uint16_t *col16,
                    const double *val, const double *x, double *y, const void *win,
                    int32_t xcap, const void *head);
/* Head copy for small matrices (the ones spmv_sell_auto_ki gives ki = 2:
 * fewer than 14 slices per CU): the first slot groups each wave of the
 * small-matrix kernel reads are also stored at addresses computed from the
 * workgroup and wave ids, so a cold run issues them without first waiting
 * for slice_ptr.  spmv_sell16_head_bytes() is 0 for other matrices (no head;
 * pass head = NULL).  Built once from the SELL16 arrays; y bit-identical.  */
size_t spmv_sell16_head_bytes(int64_t n_slices, int32_t C, int32_t ki);
int spmv_sell16_head_fill(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                          const int64_t *slice_ptr, const double *val, const uint16_t *col16,
                          void *head, size_t head_bytes);
/* The same head for int32 SELL-C-sigma (small matrices only; 12 B per head
 * slot): spmv_sell_head_bytes() is 0 for other matrices.  The run with a
 * head gives the bits of spmv_sell_run_xwin (win/xcap from
 * spmv_sell_xwin_build).  (reference kernels/Sigma_C.cl, sigma_c.c:311)  */
size_t spmv_sell_head_bytes(int64_t n_slices, int32_t C, int32_t ki);
int spmv_sell_head_fill(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                        const int64_t *slice_ptr, const double *val, const int32_t *col, void *head,
                        size_t head_bytes);
int spmv_sell_run_xwin_head(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                            const int64_t *slice_ptr, const int32_t *perm, const int32_t *col,
                            const double *val, const double *x, double *y, const void *win, int32_t xcap,
                            const void *head);

/* --------------------------------------------------------------- CMRS ---
 * (spmv_cmrs_run and the layout: spmv.h) */
/* COO and entry-balanced CMRS over a hot-column table (col_hot / hot from
 * spmv_hot_columns on the format's own column array), as
 * spmv_csr_run_tiled_hot: the CMRS run is bit-identical to
 * spmv_cmrs_run_tiled on the original columns; the COO run cuts 512-entry
 * tiles below a mean row of 96 (R-MAT 1e7/1e8: 0.951 vs 1.242 ms), so a
 * row spanning tiles sums in another order than spmv_coo_run's (within
 * the 1e-6 parity rule; bit-identical for any two tables).  H = 0 is
 * spmv_coo_run / spmv_cmrs_run_tiled.                                     */
size_t spmv_coo_hot_ws_bytes(int64_t nnz, int64_t H);
int spmv_coo_run_hot(spmv_dims d, const int32_t *row, const int32_t *col_hot, const double *val,
                     const double *x, double *y, int64_t H, const int32_t *hot, void *ws, size_t ws_bytes);
size_t spmv_cmrs_hot_ws_bytes(int64_t n_strips, int64_t nnz, int32_t h, int64_t H);
int spmv_cmrs_run_tiled_hot(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                            const uint8_t *row_in_strip, const int32_t *col_hot, const double *val,
                            const double *x, double *y, int64_t H, const int32_t *hot, void *ws,
                            size_t ws_bytes);

/* COO and CMRS with x windows in LDS (the protocol of the CSR/ELL/SELL
 * x-window entry points): *_xwin_bytes sizes the window buffer,
 * *_xwin_build fills it on the device (column range of every COO tile of
 * the staged kernel / every CMRS strip run) and returns xcap, the LDS
 * entries a workgroup stages (<= 2,048; 0 = none fits); *_run_xwin is the
 * plain run with win/xcap appended.  A window wider than xcap gathers
 * from global memory: y is bit-identical to the plain run.  The CMRS
 * windows depend on d (n_rows and nnz pick the lanes per row).          */
size_t spmv_coo_xwin_bytes(int64_t nnz);
int spmv_coo_xwin_build(spmv_dims d, const int32_t *col, void *win, size_t win_bytes, int32_t *xcap);
int spmv_coo_run_xwin(spmv_dims d, const int32_t *row, const int32_t *col, const double *val,
                      const double *x, double *y, void *ws, size_t ws_bytes, const void *win,
                      int32_t xcap);
size_t spmv_cmrs_xwin_bytes(spmv_dims d, int32_t h, int64_t n_strips);
int spmv_cmrs_xwin_build(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                         const int32_t *col, void *win, size_t win_bytes, int32_t *xcap);
int spmv_cmrs_run_xwin(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                       const uint8_t *row_in_strip, const int32_t *col, const double *val,
                       const double *x, double *y, const void *win, int32_t xcap);
/* Entry-balanced CMRS for skewed strips (spmv_cmrs_pick_variant): every
 * workgroup takes a fixed tile of entries; a strip spanning tiles leaves
 * per-row partials for the deterministic carry pass.  `ws` holds
 * spmv_cmrs_tiled_ws_bytes() bytes.  Same arrays as spmv_cmrs_run.      */
size_t spmv_cmrs_tiled_ws_bytes(int64_t n_strips, int64_t nnz, int32_t h);
int spmv_cmrs_run_tiled(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                        const uint8_t *row_in_strip, const int32_t *col, const double *val,
                        const double *x, double *y, void *ws, size_t ws_bytes);

/* ------------------------------------------------- device generator ---
 * Rows [row_begin, row_end) of the banded matrix of BASELINE.json
 * configs[4] (row i: 16 entries at columns (i + o) mod n, o = -8..7),
 * written straight into HBM — values bit-identical to the host's
 * spmv_gen_banded_csr.  layout 0 = CSR: ptr[m+1] (local offsets),
 * col/val[16m]; layout 1 = SELL-C with k-interleave ki (every row has 16
 * entries, so any sigma sort is the identity): ptr = slice_ptr[ns+1],
 * perm[ns*C], col/val[ns*C*16], ns = ceil(m/C).  m = row_end-row_begin. */
int spmv_gen_banded_device(int64_t n, uint64_t seed, int64_t row_begin,
                           int64_t row_end, int layout, int32_t C, int32_t ki,
                           int64_t *ptr, int32_t *perm, int32_t *col, double *val,
                           int device, void *stream);

/* ------------------------------------------- device format builders ---
 * build the formats from a COO (entries in any order,
 * file order kept inside a row) that is already in HBM, without a host
 * round trip.  Every output array equals the host builder's of
 * spmv_host.h element for element (CSR: spmv_csr_from_coo; ELL:
 * spmv_ell_plan/fill; SELL: spmv_sell_plan/fill; CMRS: spmv_cmrs_build).
 * Builders allocate their own scratch, run on d.stream and synchronise it
 * before returning; they are build-time calls, not SpMV-path calls.
 * Sizes: row_ptr[N+1], col_out/val_out[Z]; SELL perm[n_slices*C],
 * slice_ptr[n_slices+1], slice_col[n_slices] (scratch for the fill),
 * n_slices = ceil(N/C), sigma <= 4096; *stored (host) = entries incl.
 * padding, the size of the SELL col/val arrays.                          */
int spmv_dev_csr_from_coo(spmv_dims d, const int32_t *row, const int32_t *col, const double *val,
                          int64_t *row_ptr, int32_t *col_out, double *val_out);
int spmv_dev_ell_plan(spmv_dims d, const int64_t *row_ptr, int32_t ki, int32_t *K, int64_t *ld);
int spmv_dev_ell_fill(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                      int32_t K, int64_t ld, int32_t ki, int32_t *col_out, double *val_out);
int spmv_dev_sell_plan(spmv_dims d, const int64_t *row_ptr, const int32_t *col, int32_t C,
                       int32_t sigma, int32_t ki, int64_t n_slices, int32_t *perm, int64_t *slice_ptr,
                       int32_t *slice_col, int64_t *stored);
int spmv_dev_sell_fill(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                       int32_t C, int32_t ki, int64_t n_slices, const int64_t *slice_ptr,
                       const int32_t *perm, const int32_t *slice_col, int32_t *col_out,
                       double *val_out);
int spmv_dev_cmrs_build(spmv_dims d, const int64_t *row_ptr, int32_t h, int64_t *strip_ptr,
                        uint8_t *row_in_strip);

/* ------------------------------------------------- iterated SpMV -------
 * Vector kernels for power iteration / CG over row shards (SURVEY.md §8f
 * row 3).  The reference stops after one SpMV (reference csr.c:198-236),
 * so nothing here replaces a reference call.  Scalars live in DEVICE
 * memory (num, den, s, out) so an iteration needs no host round trip; the
 * dot product is a fixed two-stage tree: same n and data, same bits.    */
size_t spmv_dot_ws_bytes(int64_t n);
/* *out = sum_i a[i]*b[i]; ws holds spmv_dot_ws_bytes(n) bytes.          */
int spmv_dot(int64_t n, const double *a, const double *b, double *out, void *ws,
             size_t ws_bytes, int device, void *stream);
/* y += sign * (*num / *den) * x   (CG: x += a p, r -= a Ap)             */
int spmv_axpy_ratio(int64_t n, const double *num, const double *den, double sign,
                    const double *x, double *y, int device, void *stream);
/* y = x + (*num / *den) * y       (CG: p = r + b p)                     */
int spmv_xpay_ratio(int64_t n, const double *num, const double *den, const double *x,
                    double *y, int device, void *stream);
/* y = x / sqrt(*s)                (power iteration: normalise)          */
int spmv_scale_rsqrt(int64_t n, const double *s, const double *x, double *y, int device,
                     void *stream);
/* out[k] = x[order[k]]: x in the layout of a matrix whose columns were
 * relabelled by spmv_column_relabel (spmv_host.h), the input its SpMV
 * takes.  out must not alias x.                                          */
int spmv_gather(int64_t n, const int32_t *order, const double *x, double *out, int device, void *stream);

/* ---------------------------------------------------------- switches ---
 * Placement and load-policy switches for A/B runs; each changes speed,
 * never a result bit (tests/test_gpu_parity.py checks that).  The library
 * reads SPMV_XWIN_REMAP, SPMV_XCD_REMAP, SPMV_STREAM_NT and
 * SPMV_CSR_PREFETCH once, when it is loaded, as their initial values; spmv_set_option changes them for
 * the whole process (value -1 = each kernel's measured default, 0 off,
 * 1 on).  Nothing reads the environment on the launch path.             */
enum spmv_option {
    SPMV_OPT_XWIN_REMAP = 1,  /* XCD-contiguous x-window workgroups        */
    SPMV_OPT_XCD_REMAP = 2,   /* XCD-contiguous global-gather workgroups   */
    SPMV_OPT_STREAM_NT = 3,   /* non-temporal matrix loads                 */
    SPMV_OPT_CSR_PREFETCH = 4 /* CSR x-window: first chunk in the prologue */
};
int spmv_set_option(int option, int value);
int spmv_get_option(int option);


#ifdef __cplusplus
}
#endif

#endif /* SPMV_EXT_H */
