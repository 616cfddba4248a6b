// coo.hip — the deterministic carry pass and the COO / CMRS entry points
// for gfx950.
//
// COO replaces the reference's coo kernel (reference kernels/Coo.cl:4-32:
// one work-item per entry, fp64 add built from a 64-bit compare-and-swap
// retry loop, y assumed pre-zeroed).  Entries are sorted by row on the
// host (spmv_coo_sort_by_row), then:
//   pass 1  coo_staged_kernel (staged.hip): each workgroup stages a tile of
//           consecutive entries in LDS and writes every row that begins in
//           it; a row that began in an EARLIER tile is not stored: its
//           partial sum goes to carry[tile].
//   pass 2  coo_carry_kernel (here): one thread per tile; the first tile of
//           every run of carries for the same row adds the run to y[row] —
//           in tile order for a run of <= 8 tiles, lane-strided over the
//           wave plus the butterfly for a longer one (a fixed order).
// No atomics, every y element written by exactly one pass-1 store (plus at
// most one pass-2 update): results are bitwise reproducible.
//
// CMRS replaces the reference's cmrs kernel (reference kernels/Cmrs.cl:
// 1-46: per-lane private LDS row vectors, three barriers per strip,
// uninitialised LDS on the first strip, an out-of-bounds y store in the
// tail strip) with the LDS-staged strip-run kernel (staged.hip).
// (The round-1 wave-per-tile / wave-per-strip segmented-scan kernels were
// slower — COO 0.605 vs 0.487 ms, CMRS 0.549 vs 0.400 ms on the cant batch —
// and were removed.)
#include <limits.h>
#include <stdlib.h>

#include "common.h"

namespace spmv {

__global__ __launch_bounds__(kBlock) void coo_carry_kernel(
    int64_t n_tiles, const int32_t *__restrict__ carry_row,
    const double *__restrict__ carry_val, double *__restrict__ y)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int lane = threadIdx.x & (kWave - 1);
    // The head test and the first 8 tiles' loads are issued together: one
    // round trip for a row over <= 8 tiles (the common case), added in tile
    // order by the head's thread.  (Round 6: the head test first and the
    // run's loads only in head threads measured 14.7 vs 13.9 us average on
    // the R-MAT's CSR / CMRS / COO carries; profiles/round6/ab_cmrs_plan_carry.md.)
    const int32_t prev = t > 0 && t < n_tiles ? carry_row[t - 1] : -1;
    int32_t rr[8];
    double vv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const bool in = t + k < n_tiles;
        rr[k] = in ? carry_row[t + k] : -2;
        vv[k] = in ? carry_val[t + k] : 0.0;
    }
    const int32_t r = rr[0];
    const bool head = t < n_tiles && r >= 0 && prev != r;  // first tile of a run of carries
    const bool lng = head && rr[7] == r;                   // the run goes on past 8 tiles
    if (head && !lng) {
        double s = 0.0;
        for (int k = 0; k < 8 && rr[k] == r; ++k)
            s += vv[k];
        y[r] += s;
    }
    // A hub row's run (R-MAT rows of 1e5 entries span ~100-150 tiles) is
    // summed by the whole wave: 4 x 64 tiles per round trip, lane-strided,
    // then the butterfly (a fixed order, so still bitwise reproducible);
    // one thread walking it 8 tiles per round trip took 13+ dependent round
    // trips (9 us of an R-MAT shard's 145).
    for (uint64_t m = __ballot(lng); m; m &= m - 1) {
        const int l = __builtin_ctzll(m);
        const int32_t hr = __shfl(r, l);
        const int64_t ht = t - lane + l;
        double s = 0.0;
        for (int64_t base = ht;; base += 4 * kWave) {
            int32_t q[4];
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = base + u * kWave + lane;
                q[u] = i < n_tiles ? carry_row[i] : -2;
                v[u] = i < n_tiles ? carry_val[i] : 0.0;
            }
            bool end = false;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (q[u] == hr)
                    s += v[u];
                else
                    end = true;
            }
            if (__ballot(end))
                break;  // the run ended inside this round: rows only grow with the tile
        }
        s = group_sum<kWave>(s);
        if (lane == l)
            y[hr] += s;
    }
}

int launch_carry(int64_t tiles, const int32_t *carry_row, const double *carry_val, double *y,
                 hipStream_t stream)
{
    if (tiles <= 0)
        return SPMV_SUCCESS;
    hipLaunchKernelGGL(coo_carry_kernel, dim3((unsigned)((tiles + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, stream, tiles, carry_row, carry_val, y);
    SPMV_CHECK_LAUNCH("coo_carry_kernel");
    return SPMV_SUCCESS;
}

}  // namespace spmv

using namespace spmv;

extern "C" size_t spmv_coo_ws_bytes(int64_t nnz)
{
    // the carry pass may cut 512-entry tiles (coo_hot_tile): sized for them
    const int64_t t = 2 * kBlock;
    const int64_t tiles = nnz > 0 ? (nnz + t - 1) / t : 0;
    // carry_val (8-byte aligned) first, then carry_row
    return (size_t)(tiles * (int64_t)sizeof(double) + tiles * (int64_t)sizeof(int32_t) + 16);
}

extern "C" int spmv_coo_run(spmv_dims d, const int32_t *row,
                            const int32_t *col, const double *val,
                            const double *x, double *y, void *ws,
                            size_t ws_bytes)
{
    if (d.n_rows < 0 || d.nnz < 0 || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    if (d.nnz == 0) {
        hipError_t e = hipMemsetAsync(y, 0, (size_t)d.n_rows * sizeof(double),
                                      (hipStream_t)d.stream);
        return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "memset y", e);
    }
    if (!ws || ws_bytes < spmv_coo_ws_bytes(d.nnz))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run: workspace too small");
    const int64_t st_tiles = (d.nnz + coo_hot_tile(d.n_rows, d.nnz) - 1) / coo_hot_tile(d.n_rows, d.nnz);
    double *cv = (double *)ws;
    int32_t *cr = (int32_t *)(cv + st_tiles);
    int rc = launch_coo_staged(d, row, col, val, x, y, cr, cv);
    if (rc != SPMV_SUCCESS)
        return rc;
    return launch_carry(st_tiles, cr, cv, y, (hipStream_t)d.stream);
}

// Single-pass COO (no carry pass): every tile also finishes its last row
// from the entries past its end, the tail plan giving their count.  For
// matrices whose rows run at most 80 entries past a tile end (one
// cant-like matrix: the carry kernel was 4.3 of its 20.9 us cold).
extern "C" size_t spmv_coo_tail_bytes(int64_t nnz)
{
    if (nnz <= 0)
        return 0;
    return (size_t)((nnz + coo_staged_tile() - 1) / coo_staged_tile()) * sizeof(int32_t);
}

extern "C" int spmv_coo_tail_build(spmv_dims d, const int32_t *row, void *tails, size_t tails_bytes)
{
    if (d.n_rows < 0 || d.nnz < 0 || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_tail_build: bad sizes");
    if (d.nnz == 0)
        return SPMV_SUCCESS;
    if (!row || !tails || tails_bytes < spmv_coo_tail_bytes(d.nnz))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_tail_build: arrays or buffer missing");
    SPMV_GUARD(d);
    const int64_t mx = coo_tail_build(d, row, (int32_t *)tails);
    if (mx < 0)
        return fail_msg(SPMV_PROGRAM_ERROR, "spmv_coo_tail_build: plan kernel");
    if (mx > coo_tail_cap()) {
        // a refused plan is zeroed, so passing it anyway cannot overrun the
        // kernel's staged tail; its y would be wrong, not unsafe
        (void)hipMemsetAsync(tails, 0, spmv_coo_tail_bytes(d.nnz), (hipStream_t)d.stream);
        return fail_msg(SPMV_OTHER_ERROR,
                        "spmv_coo_tail_build: a row runs more than 80 entries past its tile (use spmv_coo_run)");
    }
    return SPMV_SUCCESS;
}

extern "C" int spmv_coo_run_tail(spmv_dims d, const int32_t *row, const int32_t *col, const double *val,
                                 const double *x, double *y, const void *tails)
{
    if (d.n_rows < 0 || d.nnz < 0 || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_tail: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    if (d.nnz == 0) {
        hipError_t e = hipMemsetAsync(y, 0, (size_t)d.n_rows * sizeof(double), (hipStream_t)d.stream);
        return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "memset y", e);
    }
    if (!tails)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_tail: no tail plan");
    return launch_coo_staged(d, row, col, val, x, y, nullptr, nullptr, nullptr, 0, (const int32_t *)tails);
}

extern "C" int spmv_cmrs_run(spmv_dims d, int32_t h, int64_t n_strips,
                             const int64_t *strip_ptr,
                             const uint8_t *row_in_strip, const int32_t *col,
                             const double *val, const double *x, double *y)
{
    if (d.n_rows < 0 || h < 1 || h > 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run: h must be in [1,64]");
    if (n_strips != (d.n_rows + h - 1) / h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run: n_strips != ceil(N/h)");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    return launch_cmrs_staged(d, h, n_strips, strip_ptr, row_in_strip, col, val, x, y);
}

extern "C" size_t spmv_cmrs_tiled_ws_bytes(int64_t n_strips, int64_t nnz, int32_t h)
{
    (void)n_strips;
    if (h < 1)
        return 0;
    // sized for the smallest tile a run may use
    const int64_t tiles = nnz > 0 ? (nnz + cmrs_tiled_tile_min() - 1) / cmrs_tiled_tile_min() : 0;
    // carry_val[h·tiles] f64, own_lo[tiles+1] i32, carry_row[h·tiles] i32
    return (size_t)(8 * h * tiles + 4 * (tiles + 1) + 4 * h * tiles + 16);
}

// Entry-balanced CMRS (staged.hip cmrs_tiled_kernel): every workgroup
// takes the same number of entries whatever the strips, for skewed
// matrices (spmv_cmrs_pick_variant).  Same y as spmv_cmrs_run up to the
// order of the fp64 sums of strips that span tiles.
extern "C" int spmv_cmrs_run_tiled(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                                   const uint8_t *row_in_strip, const int32_t *col, const double *val,
                                   const double *x, double *y, void *ws, size_t ws_bytes)
{
    if (d.n_rows < 0 || d.nnz < 0 || h < 1 || h > 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled: h must be in [1,64]");
    if (n_strips != (d.n_rows + h - 1) / h || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled: n_strips != ceil(N/h)");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    if (d.nnz == 0) {
        hipError_t e = hipMemsetAsync(y, 0, (size_t)d.n_rows * sizeof(double), (hipStream_t)d.stream);
        return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "memset y", e);
    }
    if (!ws || ws_bytes < spmv_cmrs_tiled_ws_bytes(n_strips, d.nnz, h))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled: workspace too small");
    const int64_t tiles = (d.nnz + cmrs_tiled_tile(d.n_rows, d.nnz) - 1) / cmrs_tiled_tile(d.n_rows, d.nnz);
    if (tiles * h > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled: grid too large");
    double *carry_val = (double *)ws;
    int32_t *own_lo = (int32_t *)(carry_val + (int64_t)h * tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    return launch_cmrs_tiled(d, h, n_strips, strip_ptr, row_in_strip, col, val, x, y, own_lo, carry_row,
                             carry_val);
}

// The plan's tiled CMRS (csrc/plan.hip): the workspace laid out as
// spmv_cmrs_run_tiled (H = 0) or spmv_cmrs_run_tiled_hot (H > 0) lay it out,
// its tile -> first-strip table filled ONCE at plan build (fill = true) and
// reused by every run (fill = false: no csr_tile_rows_kernel per run).
namespace spmv {
int cmrs_tiled_planned(const spmv_dims &d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                       const uint8_t *rin, const int32_t *col, const double *val, const double *x, double *y,
                       int64_t H, const int32_t *hot, void *ws, bool fill)
{
    const int64_t ch = cmrs_tiled_tile(d.n_rows, d.nnz);
    const int64_t tiles = (d.nnz + ch - 1) / ch;
    double *xh = (double *)ws;
    double *carry_val = xh + (H > 0 ? H : 0);
    int32_t *own_lo = (int32_t *)(carry_val + (int64_t)h * tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    const hipStream_t st = (hipStream_t)d.stream;
    if (fill) {
        hipLaunchKernelGGL(csr_tile_rows_kernel, dim3((unsigned)((tiles + 1 + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, n_strips, d.nnz, tiles, ch, strip_ptr, own_lo);
        SPMV_CHECK_LAUNCH("csr_tile_rows_kernel (CMRS plan)");
        return SPMV_SUCCESS;
    }
    return launch_cmrs_tiled(d, h, n_strips, strip_ptr, rin, col, val, x, y, own_lo, carry_row, carry_val, H,
                             hot, H > 0 ? xh : nullptr, true);
}
}  // namespace spmv

extern "C" int spmv_coo_run_xwin(spmv_dims d, const int32_t *row, const int32_t *col, const double *val,
                                 const double *x, double *y, void *ws, size_t ws_bytes, const void *win,
                                 int32_t xcap)
{
    if (d.n_rows < 0 || d.nnz < 0 || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_xwin: bad sizes");
    if (d.n_rows == 0 || d.nnz == 0)
        return spmv_coo_run(d, row, col, val, x, y, ws, ws_bytes);
    if (!win || xcap < 0 || xcap > kStagedXwinCap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_xwin: bad window arguments");
    if (!ws || ws_bytes < spmv_coo_ws_bytes(d.nnz))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_xwin: workspace too small");
    SPMV_GUARD(d);
    const int64_t st_tiles = (d.nnz + coo_hot_tile(d.n_rows, d.nnz) - 1) / coo_hot_tile(d.n_rows, d.nnz);
    double *cv = (double *)ws;
    int32_t *cr = (int32_t *)(cv + st_tiles);
    int rc = launch_coo_staged(d, row, col, val, x, y, cr, cv, (const int2 *)win, xcap);
    if (rc != SPMV_SUCCESS)
        return rc;
    return launch_carry(st_tiles, cr, cv, y, (hipStream_t)d.stream);
}

extern "C" int spmv_cmrs_run_xwin(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                                  const uint8_t *row_in_strip, const int32_t *col, const double *val,
                                  const double *x, double *y, const void *win, int32_t xcap)
{
    if (d.n_rows < 0 || h < 1 || h > 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_xwin: h must be in [1,64]");
    if (n_strips != (d.n_rows + h - 1) / h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_xwin: n_strips != ceil(N/h)");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (d.nnz == 0)  // no windows were built
        return spmv_cmrs_run(d, h, n_strips, strip_ptr, row_in_strip, col, val, x, y);
    if (!win || xcap < 0 || xcap > kStagedXwinCap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_xwin: bad window arguments");
    SPMV_GUARD(d);
    return launch_cmrs_staged(d, h, n_strips, strip_ptr, row_in_strip, col, val, x, y, (const int2 *)win, xcap);
}

extern "C" size_t spmv_coo_hot_ws_bytes(int64_t nnz, int64_t H)
{
    // the hot path may use 512-entry tiles (coo_hot_tile): size the carry
    // for them, at least as large as spmv_coo_ws_bytes (H = 0 runs spmv_coo_run)
    const int64_t t = 2 * kBlock;
    const int64_t tiles = nnz > 0 ? (nnz + t - 1) / t : 0;
    const size_t carry = (size_t)(tiles * (int64_t)(sizeof(double) + sizeof(int32_t)) + 16);
    const size_t base = spmv_coo_ws_bytes(nnz);
    return (size_t)(H > 0 ? H : 0) * sizeof(double) + (carry > base ? carry : base);
}

// COO whose column ids >= n_cols name the hot-column table (host
// spmv_hot_columns, applied to the row-sorted columns): bit-identical to
// spmv_coo_run on the original columns.
extern "C" int spmv_coo_run_hot(spmv_dims d, const int32_t *row, const int32_t *col_hot, const double *val,
                                const double *x, double *y, int64_t H, const int32_t *hot, void *ws,
                                size_t ws_bytes)
{
    if (d.n_rows < 0 || d.nnz < 0 || d.n_rows > INT32_MAX || H < 0 || d.n_cols + H > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_hot: bad sizes");
    if (H == 0 || d.n_rows == 0 || d.nnz == 0)
        return spmv_coo_run(d, row, col_hot, val, x, y, ws, ws_bytes);
    if (!hot || !ws || ws_bytes < spmv_coo_hot_ws_bytes(d.nnz, H))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_hot: hot list or workspace missing");
    SPMV_GUARD(d);
    const int64_t st_tiles = (d.nnz + coo_hot_tile(d.n_rows, d.nnz) - 1) / coo_hot_tile(d.n_rows, d.nnz);
    double *xh = (double *)ws;
    double *cv = xh + H;
    int32_t *cr = (int32_t *)(cv + st_tiles);
    int rc = launch_coo_staged_hot(d, row, col_hot, val, x, y, cr, cv, H, hot, xh);
    if (rc != SPMV_SUCCESS)
        return rc;
    return launch_carry(st_tiles, cr, cv, y, (hipStream_t)d.stream);
}

extern "C" size_t spmv_cmrs_hot_ws_bytes(int64_t n_strips, int64_t nnz, int32_t h, int64_t H)
{
    return (size_t)(H > 0 ? H : 0) * sizeof(double) + spmv_cmrs_tiled_ws_bytes(n_strips, nnz, h);
}

// Entry-balanced CMRS over a hot-column table (as spmv_coo_run_hot).
extern "C" int spmv_cmrs_run_tiled_hot(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                                       const uint8_t *row_in_strip, const int32_t *col_hot, const double *val,
                                       const double *x, double *y, int64_t H, const int32_t *hot, void *ws,
                                       size_t ws_bytes)
{
    if (H < 0 || d.n_cols + H > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled_hot: bad sizes");
    if (H == 0 || d.n_rows <= 0 || d.nnz <= 0)
        return spmv_cmrs_run_tiled(d, h, n_strips, strip_ptr, row_in_strip, col_hot, val, x, y, ws, ws_bytes);
    if (h < 1 || h > 64 || n_strips != (d.n_rows + h - 1) / h || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled_hot: bad strips");
    if (!hot || !ws || ws_bytes < spmv_cmrs_hot_ws_bytes(n_strips, d.nnz, h, H))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled_hot: hot list or workspace missing");
    SPMV_GUARD(d);
    const int64_t tiles = (d.nnz + cmrs_tiled_tile(d.n_rows, d.nnz) - 1) / cmrs_tiled_tile(d.n_rows, d.nnz);
    if (tiles * h > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run_tiled_hot: grid too large");
    double *xh = (double *)ws;
    double *carry_val = xh + H;
    int32_t *own_lo = (int32_t *)(carry_val + (int64_t)h * tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    return launch_cmrs_tiled(d, h, n_strips, strip_ptr, row_in_strip, col_hot, val, x, y, own_lo, carry_row,
                             carry_val, H, hot, xh);
}
