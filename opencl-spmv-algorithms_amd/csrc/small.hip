// small.hip — single-pass CSR for matrices whose whole grid is resident at
// once (BASELINE.json configs[1]: ONE cant-like matrix, 62,451 rows, 4.0 M
// entries, 49.3 MB; ~1,000 workgroups for 256 CUs).
//
// Replaces the reference's scalar CSR kernel (reference kernels/Csr.cl:1-17,
// launched at csr.c:201) for small matrices.  On a matrix this size every
// workgroup is in flight together, so the time is one latency chain plus
// the drain of the stream, not a stream rate: the x-window kernel
// (csr_xwin_kernel) waits for its window bounds, then for its row offsets
// and x range, then streams its chunks one dependent round trip each
// (13.3-13.6 us cold against 8.2 us for a bare 49 MB read, round 3).
//
// Here a workgroup owns a FIXED entry tile [t·E, (t+1)·E), E = 4,096, so
// the addresses of its whole stream are known from blockIdx alone: every
// lane issues all 8 of its value pairs (16 B) and column pairs (8 B) at
// once, before anything else.  The rows the tile OWNS are those whose first
// entry lies in it; a build-time plan (one 32-byte record per tile,
// spmv_csr_small_build) gives them [r0, r1), the entries of the last owned
// row past the tile end (`tail`, at most 512, loaded after the plan
// arrives) and the x range of every entry the tile loads.  The entries of a
// row begun in the previous tile are loaded and never summed.  One barrier
// after the x window and row offsets are in LDS; the products go through
// LDS in 1,024-entry chunks and each owned row is summed by an L-lane group
// (slice_sum + butterfly, as the staged kernels).  No carry pass, no
// atomics: deterministic, one kernel per SpMV.
//
// Row sums are grouped by tile chunks, so the bits differ from
// spmv_csr_run_variant (the parity rule holds); the run is reproducible.
#include <stdio.h>
#include <stdlib.h>

#include "common.h"

namespace spmv {

constexpr int kSmallP = 8;                        // value/column pairs per lane: the whole tile
constexpr int64_t kSmallE = 2 * kBlock * kSmallP;  // 4,096 entries per tile
constexpr int kSmallRC = 2;                       // pairs per lane per LDS product chunk
constexpr int kSmallCH = 2 * kBlock * kSmallRC;   // 1,024 products per chunk
constexpr int kSmallTail = 2 * kBlock;            // tail entries: one pair per lane
constexpr int kSmallNB = 4;                       // row batches of 256/L rows per tile
constexpr int32_t kSmallXcap = 2048;              // x-window entries in LDS (16 KiB)

// One tile's plan record (32 bytes, read once per workgroup as a scalar load).
struct SmallTile {
    int32_t r0, r1;    // owned rows [r0, r1): their first entry lies in the tile
    int32_t xlo, xhi;  // column range of every entry the tile loads ({0, -1}: none)
    int32_t tail;      // entries of the last owned row past the tile end (<= kSmallTail)
    int32_t pad[3];
};
static_assert(sizeof(SmallTile) == 32, "SmallTile is 32 bytes");

// One lane's share of a row's products in an LDS chunk (entries [lo, hi) of
// the chunk, every L-th from lo+lane), two interleaved partial sums.
template <int L>
__device__ __forceinline__ double small_slice_sum(const double *prod, int lo, int hi, int lane)
{
    double a0 = 0.0, a1 = 0.0;
    int j = lo + lane;
    for (; j + 7 * L < hi; j += 8 * L) {
        double p[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            p[k] = prod[j + k * L];
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
            a0 += p[k];
            a1 += p[k + 1];
        }
    }
    for (; j + L < hi; j += 2 * L) {
        a0 += prod[j];
        a1 += prod[j + L];
    }
    if (j < hi)
        a0 += prod[j];
    return a0 + a1;
}

// x[c] from the LDS window or global memory; c < 0 marks an entry that was
// not loaded (past the array; its value is 0 and it is never summed)
struct SmallXWin {
    const double *s;  // LDS
    int32_t lo;
    __device__ __forceinline__ double operator()(int32_t c) const { return s[c >= 0 ? c - lo : 0]; }
};
struct SmallXGlobal {
    const double *__restrict__ x;
    __device__ __forceinline__ double operator()(int32_t c) const { return c >= 0 ? x[c] : 0.0; }
};

// PRE: pairs per lane issued before the plan record arrives (the rest right
// after the x-window / row-offset loads that depend on it).
template <int L, bool NT, int PRE>
__global__ __launch_bounds__(kBlock) void csr_small_kernel(int64_t nz,
                                                           const int64_t *__restrict__ row_ptr,
                                                           const int32_t *__restrict__ col,
                                                           const double *__restrict__ val,
                                                           const double *__restrict__ x, double *__restrict__ y,
                                                           const SmallTile *__restrict__ plan, int32_t xcap,
                                                           int remap)
{
    constexpr int RPB = kBlock / L;
    extern __shared__ double s_x[];
    __shared__ double2 s_prod[kBlock * kSmallRC];
    __shared__ int32_t s_off[kSmallNB * RPB + 1];  // owned rows' offsets, relative to the tile start
    const int64_t t = xcd_block(remap);
    const int64_t tb = t * kSmallE;
    const int tid = threadIdx.x;
    // a pair the lane may always load: the tile's first (its columns are in
    // the window), or any pair of the array when the tile has one entry
    const int64_t spare = tb + 1 < nz ? tb : (nz >= 2 ? ((nz - 2) & ~(int64_t)1) : -1);

    double2 v[kSmallP];
    int2 c[kSmallP];
    auto issue = [&](int k) {
        const int64_t p = tb + 2 * (int64_t)(tid + k * kBlock);
        const bool full = p + 1 < nz;
        if (spare >= 0) {
            const int64_t q = full ? p : spare;
            v[k] = stream_load2<NT>(val + q);
            c[k] = stream_load2<NT>(col + q);
        } else {
            v[k] = double2{0.0, 0.0};
            c[k] = int2{-1, -1};
        }
        if (!full) {  // past the array, or its odd last entry alone
            const bool one = p < nz;
            v[k] = double2{one ? stream_load<NT>(val + p) : 0.0, 0.0};
            c[k] = int2{one ? col[p] : -1, -1};
        }
    };
#pragma unroll
    for (int k = 0; k < PRE; ++k)
        issue(k);

    const SmallTile tp = plan[t];
    const int32_t nr = tp.r1 - tp.r0;  // owned rows (<= kSmallNB * RPB)
    const int64_t te = tb + kSmallE;
    // the tail: entries [te, te + tail) of the last owned row
    double2 tv = {0.0, 0.0};
    int2 tc = {-1, -1};
    {
        const int64_t p = te + 2 * (int64_t)tid;
        const int64_t tend = te + tp.tail;
        if (p + 1 < tend) {
            tv = stream_load2<NT>(val + p);
            tc = stream_load2<NT>(col + p);
        } else if (p < tend) {
            tv.x = stream_load<NT>(val + p);
            tc.x = col[p];
        }
    }
    const int32_t span = tp.xhi - tp.xlo + 1;
    const bool staged = span > 0 && span <= xcap;  // uniform
    if (staged)
        copy_window<kBlock, 4>(s_x, x, tp.xlo, span);
    for (int i = tid; i <= nr; i += kBlock)
        s_off[i] = (int32_t)(row_ptr[tp.r0 + i] - tb);
#pragma unroll
    for (int k = PRE; k < kSmallP; ++k)
        issue(k);
    __syncthreads();  // x window and offsets visible

    const int g = tid / L, lane = tid % L;
    const double *prod = reinterpret_cast<const double *>(s_prod);
    double acc[kSmallNB];
#pragma unroll
    for (int b = 0; b < kSmallNB; ++b)
        acc[b] = 0.0;
    // the owned rows' pieces in one chunk of products [cb, cb + n)
    auto rows = [&](int cb, int n) {
#pragma unroll
        for (int b = 0; b < kSmallNB; ++b) {
            const int i = b * RPB + g;
            if (i < nr) {
                const int beg = s_off[i], end = s_off[i + 1];
                const int lo = beg > cb ? beg - cb : 0;
                const int hi = (end < cb + n ? end : cb + n) - cb;
                if (hi > lo)
                    acc[b] += small_slice_sum<L>(prod, lo, hi, lane);
            }
        }
    };
    auto body = [&](const auto &xs) {
#pragma unroll
        for (int ch = 0; ch < kSmallP / kSmallRC; ++ch) {
#pragma unroll
            for (int kk = 0; kk < kSmallRC; ++kk) {
                const int k = ch * kSmallRC + kk;
                s_prod[tid + kk * kBlock] = double2{v[k].x * xs(c[k].x), v[k].y * xs(c[k].y)};
            }
            __syncthreads();
            rows(ch * kSmallCH, kSmallCH);
            __syncthreads();
        }
        if (tp.tail > 0) {  // uniform
            s_prod[tid] = double2{tv.x * xs(tc.x), tv.y * xs(tc.y)};
            __syncthreads();
            rows((int)kSmallE, kSmallTail);
        }
    };
    if (staged)
        body(SmallXWin{s_x, tp.xlo});
    else
        body(SmallXGlobal{x});
#pragma unroll
    for (int b = 0; b < kSmallNB; ++b) {
        const int i = b * RPB + g;
        const double s = group_sum<L>(acc[b]);
        if (lane == 0 && i < nr)
            store_y(y + tp.r0 + i, s);
    }
}

// Plan of tile t: owned rows, tail and the x range of every loaded entry.
__global__ __launch_bounds__(kBlock) void csr_small_plan_kernel(int64_t n_rows, int64_t nz, int64_t tiles,
                                                                const int64_t *__restrict__ row_ptr,
                                                                const int32_t *__restrict__ col,
                                                                SmallTile *__restrict__ plan)
{
    __shared__ int64_t s_r[2];
    const int64_t t = blockIdx.x;
    const int64_t tb = t * kSmallE, te = tb + kSmallE;
    if (threadIdx.x < 2) {
        // first row whose first entry is >= v (rows past the last tile's
        // start all belong to it)
        const int64_t v = threadIdx.x == 0 ? tb : te;
        int64_t r;
        if (threadIdx.x == 1 && t == tiles - 1) {
            r = n_rows;
        } else if (threadIdx.x == 0 && t == 0) {
            r = 0;
        } else {
            int64_t lo = 0, hi = n_rows;  // row_ptr[n_rows] = nz >= v for the tiles here
            while (lo < hi) {
                const int64_t mid = (lo + hi) / 2;
                if (row_ptr[mid] < v)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            r = lo;
        }
        s_r[threadIdx.x] = r;
    }
    __syncthreads();
    const int64_t r0 = s_r[0], r1 = s_r[1];
    const int64_t tail_end = row_ptr[r1];
    const int64_t tail = tail_end > te ? tail_end - te : 0;
    int64_t loaded_end = te > tail_end ? te : tail_end;
    loaded_end = loaded_end < nz ? loaded_end : nz;
    const int2 xr = block_col_range(col, tb < nz ? tb : nz, loaded_end);
    if (threadIdx.x == 0) {
        SmallTile p;
        p.r0 = (int32_t)r0;
        p.r1 = (int32_t)r1;
        p.xlo = xr.x;
        p.xhi = xr.y;
        p.tail = (int32_t)(tail < INT32_MAX ? tail : INT32_MAX);
        p.pad[0] = p.pad[1] = p.pad[2] = 0;
        plan[t] = p;
    }
}

static int64_t small_tiles(int64_t nz)
{
    const int64_t t = (nz + kSmallE - 1) / kSmallE;
    return t > 0 ? t : 1;
}

static int small_lanes(int64_t n_rows, int64_t nnz, int lanes)
{
    if (lanes > 0)
        return lanes;
    return spmv_csr_auto_lanes(n_rows, nnz) < 16 ? spmv_csr_auto_lanes(n_rows, nnz) : 16;
}

template <int L, bool NT, int PRE>
static void launch_small(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col, const double *val,
                         const double *x, double *y, const SmallTile *plan, int32_t xcap, int remap)
{
    const int64_t tiles = small_tiles(d.nnz);
    hipLaunchKernelGGL((csr_small_kernel<L, NT, PRE>), dim3((unsigned)tiles), dim3(kBlock),
                       (size_t)xcap * sizeof(double), (hipStream_t)d.stream, d.nnz, row_ptr, col, val, x, y, plan,
                       xcap, remap);
}

}  // namespace spmv

using namespace spmv;

extern "C" size_t spmv_csr_small_bytes(int64_t n_rows, int64_t nnz)
{
    if (n_rows <= 0 || nnz < 0 || n_rows > INT32_MAX)
        return 0;
    return (size_t)small_tiles(nnz) * sizeof(SmallTile);
}

extern "C" int spmv_csr_small_suits(int64_t n_rows, int64_t nnz)
{
    // every tile resident at once: about 4 workgroups per CU of the
    // MI355X's 256 (a constant, so the choice never depends on the device)
    return n_rows > 0 && n_rows <= INT32_MAX && small_tiles(nnz) <= 4 * 256 ? 1 : 0;
}

extern "C" int spmv_csr_small_build(spmv_dims d, const int64_t *row_ptr, const int32_t *col, int lanes_per_row,
                                    void *plan, size_t plan_bytes, int32_t *xcap)
{
    if (d.n_rows <= 0 || d.nnz < 0 || d.n_rows > INT32_MAX || !xcap || !row_ptr)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_small_build: bad arguments");
    *xcap = 0;
    const int L = small_lanes(d.n_rows, d.nnz, lanes_per_row);
    if (L != 2 && L != 4 && L != 8 && L != 16)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_small_build: lanes_per_row must be 0, 2, 4, 8 or 16");
    const size_t need = spmv_csr_small_bytes(d.n_rows, d.nnz);
    if (!plan || plan_bytes < need)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_small_build: plan buffer too small");
    SPMV_GUARD(d);
    const int64_t tiles = small_tiles(d.nnz);
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(csr_small_plan_kernel, dim3((unsigned)tiles), dim3(kBlock), 0, st, d.n_rows, d.nnz, tiles,
                       row_ptr, col, (SmallTile *)plan);
    SPMV_CHECK_LAUNCH("csr_small_plan_kernel");
    SmallTile *h = (SmallTile *)malloc(need);
    if (!h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_small_build: out of host memory");
    hipError_t e = hipMemcpyAsync(h, plan, need, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        free(h);
        return fail(SPMV_PROGRAM_ERROR, "spmv_csr_small_build: copy plan", e);
    }
    const int32_t max_rows = kSmallNB * (kBlock / L);
    int32_t best = 0;
    int bad = 0;
    for (int64_t t = 0; t < tiles; ++t) {
        if (h[t].r1 - h[t].r0 > max_rows || h[t].tail > kSmallTail || h[t].r1 < h[t].r0)
            bad = 1;
        const int64_t span = (int64_t)h[t].xhi - h[t].xlo + 1;
        if (span <= kSmallXcap && span > best)
            best = (int32_t)span;
    }
    free(h);
    if (bad)
        return fail_msg(SPMV_OTHER_ERROR,
                        "spmv_csr_small_build: a tile owns too many rows or a row runs too far past its tile "
                        "(use spmv_csr_run_xwin)");
    *xcap = best;
    return SPMV_SUCCESS;
}

extern "C" int spmv_csr_run_small(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                                  const double *x, double *y, int lanes_per_row, const void *plan, int32_t xcap)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || d.n_rows > INT32_MAX || xcap < 0 || xcap > kSmallXcap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_small: bad arguments");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (!plan || !row_ptr || (d.nnz > 0 && (!col || !val || !x)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_small: NULL array");
    const int L = small_lanes(d.n_rows, d.nnz, lanes_per_row);
    SPMV_GUARD(d);
    const bool nt = stream_nt(true);
    const int remap = xwin_remap(true) ? 1 : 0;
    const SmallTile *p = (const SmallTile *)plan;
#define SPMV_SMALL(LL)                                                                    \
    (nt ? launch_small<LL, true, kSmallP>(d, row_ptr, col, val, x, y, p, xcap, remap)   \
        : launch_small<LL, false, kSmallP>(d, row_ptr, col, val, x, y, p, xcap, remap))
    switch (L) {
    case 2: SPMV_SMALL(2); break;
    case 4: SPMV_SMALL(4); break;
    case 8: SPMV_SMALL(8); break;
    case 16: SPMV_SMALL(16); break;
    default:
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_small: lanes_per_row must be 0, 2, 4, 8 or 16");
    }
#undef SPMV_SMALL
    SPMV_CHECK_LAUNCH("csr_small_kernel");
    return SPMV_SUCCESS;
}
