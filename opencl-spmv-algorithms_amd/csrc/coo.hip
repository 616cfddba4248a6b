// coo.hip — atomic-free COO SpMV and CMRS SpMV for gfx950.
//
// COO replaces the reference's coo kernel (reference kernels/Coo.cl:4-32:
// one work-item per entry, fp64 add built from a 64-bit compare-and-swap
// retry loop, y assumed pre-zeroed).  Entries are sorted by row on the
// host (spmv_coo_sort_by_row), then:
//   pass 1  each wave owns a tile of kTile consecutive entries.  Per
//           64-entry step it forms the products, runs a wave-wide
//           segmented inclusive scan keyed by row (6 shuffle steps), and
//           the last lane of every finished row segment stores y[row].
//           A row running past the step is carried in registers.  A row
//           that began in an EARLIER tile is not stored: its partial sum
//           goes to carry[tile].  Rows with no entries get 0.0 from the
//           tile that holds the next non-empty row (and the last tile).
//   pass 2  one thread per tile: the first tile of every run of carries
//           for the same row adds the run, in tile order, to y[row].
// No atomics, every y element written by exactly one pass-1 store (plus
// at most one pass-2 update): results are bitwise reproducible.
//
// CMRS replaces the reference's cmrs kernel (reference kernels/Cmrs.cl:
// 1-46: per-lane private LDS row vectors of h doubles, three barriers
// per strip, uninitialised LDS on the first strip, and an out-of-bounds
// y store in the tail strip).  Here one wave owns one strip: the same
// segmented scan keyed by row_in_strip reduces each 64-entry step, the
// segment tails add into a per-wave LDS strip accumulator of h doubles
// (zeroed first; keys are sorted so the tails of one step hit distinct
// slots), and lanes 0..h-1 store the strip's h contiguous y values,
// bounds-checked.  No barrier: each wave only touches its own LDS slots.
#include <limits.h>
#include <stdlib.h>

#include "common.h"

namespace spmv {

constexpr int kCooIter = 16;                  // 64-entry steps per tile
constexpr int kCooUDefault = 8;               // steps loaded ahead (SPMV_COO_U: 4, 8, 16)

// Kernel choice: "1" = wave segmented scan (this file), "2" = LDS-staged
// (staged.hip, default).  Read once per variable.
static bool staged_variant(const char *env)
{
    const char *s = getenv(env);
    return !(s && s[0] == '1');
}

static int coo_lookahead()
{
    static int cached = -1;
    if (cached < 0) {
        const char *s = getenv("SPMV_COO_U");
        const int u = s ? atoi(s) : kCooUDefault;
        cached = (u == 4 || u == 8 || u == 16) ? u : kCooUDefault;
    }
    return cached;
}
constexpr int64_t kTile = kWave * kCooIter;  // entries per wave

// Inclusive segmented scan over one wave; `key` is non-decreasing across
// lanes, so lane l - off having the same key means every lane between
// does too.
template <typename K>
__device__ __forceinline__ double seg_scan(double p, K key, int lane)
{
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const double pu = __shfl_up(p, off, kWave);
        const K ku = __shfl_up(key, off, kWave);
        if (lane >= off && ku == key)
            p += pu;
    }
    return p;
}

template <int U>
__global__ __launch_bounds__(kBlock) void coo_tile_kernel(
    int64_t n_rows, int64_t nnz, int64_t n_tiles,
    const int32_t *__restrict__ row, const int32_t *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x,
    double *__restrict__ y, int32_t *__restrict__ carry_row,
    double *__restrict__ carry_val, int remap)
{
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t tile = xcd_block(remap) * (kBlock / kWave) + (threadIdx.x >> 6);
    if (tile >= n_tiles)
        return;
    const int64_t t0 = tile * kTile;
    const int64_t t1 = t0 + kTile < nnz ? t0 + kTile : nnz;
    const int32_t first_row = row[t0];
    const int32_t before = t0 > 0 ? row[t0 - 1] : -1;
    const bool first_continues = before == first_row;

    double run = 0.0;      // wave-uniform running sum of row `run_row`
    int32_t run_row = -1;
    int32_t prev_r = before;  // row of the entry just before the step
    double pref = 0.0;     // this lane's share of a continued first row

    // U steps are loaded before any is reduced, so each lane keeps 3·U
    // loads (+ U x gathers) in flight instead of one step's.
    for (int it0 = 0; it0 < kCooIter; it0 += U) {
        if (t0 + (int64_t)it0 * kWave >= t1)
            break;
        int32_t rs[U];
        double ps[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = t0 + (int64_t)(it0 + u) * kWave + lane;
            const bool valid = j < t1;
            rs[u] = valid ? row[j] : INT_MAX;
            ps[u] = valid ? val[j] * x[col[j]] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j0 = t0 + (int64_t)(it0 + u) * kWave;
            if (j0 >= t1)
                break;
            const int nvalid = (int)(t1 - j0 < kWave ? t1 - j0 : kWave);
            const bool valid = lane < nvalid;
            const int32_t r = rs[u];
            double p = ps[u];

            // The row carried from the previous step is finished unless
            // this step starts with the same row.
            const int32_t r0 = __shfl(r, 0, kWave);
            if (lane == 0 && run_row >= 0 && r0 != run_row &&
                !(first_continues && run_row == first_row))
                store_y(y + (run_row), run);

            // Rows strictly between the previous entry's row and r are empty.
            int32_t rp = __shfl_up(r, 1, kWave);
            if (lane == 0)
                rp = prev_r;
            if (valid)
                for (int32_t g = rp + 1; g < r; ++g)
                    store_y(y + (g), 0.0);

            if (first_continues && r == first_row) {
                pref += p;  // goes to the carry, not through the scan
                p = 0.0;
            }
            p = seg_scan(p, r, lane);
            if (r == run_row)
                p += run;
            const int32_t rn = __shfl_down(r, 1, kWave);
            const bool tail = valid && lane < nvalid - 1 && rn != r;
            if (tail && !(first_continues && r == first_row))
                store_y(y + (r), p);
            run_row = __shfl(r, nvalid - 1, kWave);
            run = __shfl(p, nvalid - 1, kWave);
            prev_r = run_row;
        }
    }
    if (lane == 0 && run_row >= 0 && !(first_continues && run_row == first_row))
        store_y(y + (run_row), run);

    // trailing empty rows after the last entry of the matrix
    if (t1 == nnz) {
        const int32_t last = row[nnz - 1];
        for (int64_t g = (int64_t)last + 1 + lane; g < n_rows; g += kWave)
            store_y(y + (g), 0.0);
    }

    pref = group_sum<kWave>(pref);
    if (lane == 0) {
        carry_row[tile] = first_continues ? first_row : -1;
        carry_val[tile] = pref;
    }
}

__global__ __launch_bounds__(kBlock) void coo_carry_kernel(
    int64_t n_tiles, const int32_t *__restrict__ carry_row,
    const double *__restrict__ carry_val, double *__restrict__ y)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n_tiles)
        return;
    // The head test and the first 8 tiles' loads are issued together (one
    // round trip for a row over <= 8 tiles, the common case); a hub row over
    // ~100 tiles then loads 8 tiles per step.  Still added in tile order.
    const int32_t prev = t > 0 ? carry_row[t - 1] : -1;
    int32_t rr[8];
    double vv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const bool in = t + k < n_tiles;
        rr[k] = in ? carry_row[t + k] : -2;
        vv[k] = in ? carry_val[t + k] : 0.0;
    }
    const int32_t r = rr[0];
    if (r < 0 || prev == r)
        return;  // not a carry, or not the head of its run
    double s = 0.0;
    for (int64_t u = t;;) {
        int k = 0;
        for (; k < 8 && rr[k] == r; ++k)
            s += vv[k];
        if (k < 8)
            break;
        u += 8;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const bool in = u + q < n_tiles;
            rr[q] = in ? carry_row[u + q] : -2;
            vv[q] = in ? carry_val[u + q] : 0.0;
        }
    }
    y[r] += s;
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

// ------------------------------------------------------------------ CMRS
template <int U>
__global__ __launch_bounds__(kBlock) void cmrs_kernel(
    int64_t n_rows, int32_t h, int64_t n_strips,
    const int64_t *__restrict__ strip_ptr,
    const uint8_t *__restrict__ row_in_strip,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, int remap)
{
    __shared__ double s_acc[kBlock / kWave][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x >> 6;
    const int64_t s = xcd_block(remap) * (kBlock / kWave) + w;
    if (s >= n_strips)
        return;
    double *acc = s_acc[w];
    acc[lane] = 0.0;
    __builtin_amdgcn_wave_barrier();

    const int64_t beg = strip_ptr[s], end = strip_ptr[s + 1];
    for (int64_t b0 = beg; b0 < end; b0 += U * kWave) {
        int keys[U];
        double ps[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // loads of U steps in flight
            const int64_t j = b0 + u * kWave + lane;
            const bool valid = j < end;
            keys[u] = valid ? (int)row_in_strip[j] : INT_MAX;
            ps[u] = valid ? val[j] * x[col[j]] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j0 = b0 + u * kWave;
            if (j0 >= end)
                break;
            const int nvalid = (int)(end - j0 < kWave ? end - j0 : kWave);
            const bool valid = lane < nvalid;
            const int key = keys[u];
            const double p = seg_scan(ps[u], key, lane);
            const int kn = __shfl_down(key, 1, kWave);
            const bool tail = valid && (lane == nvalid - 1 || kn != key);
            if (tail)
                acc[key] += p;  // distinct keys per step: no two tails collide
            __builtin_amdgcn_wave_barrier();
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < h) {
        const int64_t r = s * h + lane;
        if (r < n_rows)  // reference Cmrs.cl:38-42 stored past y here
            store_y(y + (r), acc[lane]);
    }
}

}  // namespace spmv

using namespace spmv;

extern "C" size_t spmv_coo_ws_bytes(int64_t nnz)
{
    // the wave kernel's kTile and the staged kernels' tile share this
    // workspace: size it for the smaller tile (more tiles)
    const int64_t t = kTile < coo_staged_tile() ? kTile : coo_staged_tile();
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
    if (staged_variant("SPMV_COO_VARIANT")) {
        // spmv_coo_ws_bytes counts the smaller of the two tiles
        const int64_t st_tiles = (d.nnz + coo_staged_tile() - 1) / coo_staged_tile();
        double *cv = (double *)ws;
        int32_t *cr = (int32_t *)(cv + st_tiles);
        int rc = launch_coo_staged(d, row, col, val, x, y, cr, cv);
        if (rc != SPMV_SUCCESS)
            return rc;
        hipLaunchKernelGGL(coo_carry_kernel, dim3((unsigned)((st_tiles + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, (hipStream_t)d.stream, st_tiles, cr, cv, y);
        SPMV_CHECK_LAUNCH("coo_carry_kernel");
        return SPMV_SUCCESS;
    }
    const int64_t tiles = (d.nnz + kTile - 1) / kTile;
    double *carry_val = (double *)ws;
    int32_t *carry_row = (int32_t *)(carry_val + tiles);
    const int64_t blocks = (tiles + (kBlock / kWave) - 1) / (kBlock / kWave);
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run: grid too large");
    const int remap = xcd_remap_enabled() ? 1 : 0;
#define SPMV_COO_LAUNCH(UU)                                                     \
    hipLaunchKernelGGL(coo_tile_kernel<UU>, dim3((unsigned)blocks), dim3(kBlock), 0, \
                       (hipStream_t)d.stream, d.n_rows, d.nnz, tiles, row, col,   \
                       val, x, y, carry_row, carry_val, remap)
    switch (coo_lookahead()) {
    case 8: SPMV_COO_LAUNCH(8); break;
    case 16: SPMV_COO_LAUNCH(16); break;
    default: SPMV_COO_LAUNCH(4); break;
    }
#undef SPMV_COO_LAUNCH
    SPMV_CHECK_LAUNCH("coo_tile_kernel");
    const int64_t cblocks = (tiles + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(coo_carry_kernel, dim3((unsigned)cblocks), dim3(kBlock), 0,
                       (hipStream_t)d.stream, tiles, carry_row, carry_val, y);
    SPMV_CHECK_LAUNCH("coo_carry_kernel");
    return SPMV_SUCCESS;
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
    if (staged_variant("SPMV_CMRS_VARIANT"))
        return launch_cmrs_staged(d, h, n_strips, strip_ptr, row_in_strip, col, val, x, y);
    const int64_t blocks = (n_strips + (kBlock / kWave) - 1) / (kBlock / kWave);
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run: grid too large");
    const int remap = xcd_remap_enabled() ? 1 : 0;
#define SPMV_CMRS_LAUNCH(UU)                                                    \
    hipLaunchKernelGGL(cmrs_kernel<UU>, dim3((unsigned)blocks), dim3(kBlock), 0,    \
                       (hipStream_t)d.stream, d.n_rows, h, n_strips, strip_ptr,   \
                       row_in_strip, col, val, x, y, remap)
    switch (coo_lookahead()) {
    case 8: SPMV_CMRS_LAUNCH(8); break;
    case 16: SPMV_CMRS_LAUNCH(16); break;
    default: SPMV_CMRS_LAUNCH(4); break;
    }
#undef SPMV_CMRS_LAUNCH
    SPMV_CHECK_LAUNCH("cmrs_kernel");
    return SPMV_SUCCESS;
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
    const int64_t st_tiles = (d.nnz + coo_staged_tile() - 1) / coo_staged_tile();
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
