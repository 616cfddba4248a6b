// sell.hip — SELL-C-sigma and ELL SpMV for gfx950.
//
// SELL replaces the reference's sigma_c kernel (reference
// kernels/Sigma_C.cl:1-18: 32-lane work-groups = half a wave64, no row
// sorting, y padded to the slice count).  ELL replaces the reference's
// ell kernel (reference kernels/Ell.cl:1-39: 16 lanes per row over a
// ROW-major N x K array, then an LDS barrier tree).
//
// Both are "one lane per row, column-major slots": at every step the C
// lanes of a slice (or all lanes, for ELL) read C consecutive values, so a
// wave issues one fully coalesced 512-byte (ki = 1) or 1 KiB (ki = 2,
// dwordx4) value load and the matching column load.  No reduction, no
// LDS, no barrier.  SELL writes y[perm[slot]] directly (the sigma-sort is
// undone in the store, not in an extra pass).
// Bytes per slice step: C·ki·(8 + 4) + x gathers; padding slots are
// loaded (that is the format's cost) but re-use the row's own column.
#include <stdio.h>
#include <stdlib.h>

#include "common.h"

#include <type_traits>

namespace spmv {

// Non-temporal matrix loads: SELL-64-1024 0.2955 vs 0.3130 ms and ELL
// 0.3343 vs 0.3429 ms on the 32-copy cant-like batch, one process,
// interleaved (profiles/round1/sweeps.md).  SPMV_STREAM_NT overrides.
constexpr bool kSellStreamNtDefault = true;

// Column sources: int32 columns (SELL), or 16-bit offsets from the
// workgroup's x-window base (SELL16, spmv_sell16_fill): the gathers then
// read s_x[offset] (LDS) or (x + base)[offset].  2 or 4 bytes per lane and
// slot group instead of 4 or 8.
template <bool NT>
__device__ __forceinline__ int32_t col_one(const int32_t *p)
{
    return stream_load<NT>(p);
}

template <bool NT>
__device__ __forceinline__ int32_t col_one(const uint16_t *p)
{
    return (int32_t)stream_load<NT>(p);
}

template <bool NT>
__device__ __forceinline__ int2 col_two(const int32_t *p)
{
    return stream_load2<NT>(p);
}

template <bool NT>
__device__ __forceinline__ int2 col_two(const uint16_t *p)
{
    const uint32_t v = stream_load<NT>(reinterpret_cast<const uint32_t *>(p));
    return int2{(int32_t)(v & 0xFFFFu), (int32_t)(v >> 16)};
}

template <int KI, bool NT>
struct Step;

template <bool NT>
struct Step<1, NT> {
    template <typename XS, typename CT>
    static __device__ __forceinline__ double fma(const double *vp, const CT *cp, const XS &xs, double acc)
    {
        return acc + stream_load<NT>(vp) * xs(col_one<NT>(cp));
    }
};

template <bool NT>
struct Step<2, NT> {
    template <typename XS, typename CT>
    static __device__ __forceinline__ double fma(const double *vp, const CT *cp, const XS &xs, double acc)
    {
        const double2 v = stream_load2<NT>(vp);
        const int2 c = col_two<NT>(cp);
        return acc + v.x * xs(c.x) + v.y * xs(c.y);
    }
};

// Slot-per-lane loop over `w` slots (a multiple of KI) with stride
// `step` elements between consecutive KI-groups; U groups in flight
// (U independent accumulators, combined as a pairwise tree).
template <int KI, bool NT, int U, typename XS, typename CT = int32_t>
__device__ __forceinline__ double slot_dot(const double *__restrict__ vp,
                                           const CT *__restrict__ cp,
                                           int64_t w, int64_t step, const XS &xs)
{
    double a[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        a[u] = 0.0;
    const int64_t groups = w / KI;
    int64_t g = 0;
    for (; g + U <= groups; g += U) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u] = Step<KI, NT>::fma(vp + (g + u) * step, cp + (g + u) * step, xs, a[u]);
    }
    for (; g < groups; ++g)
        a[0] = Step<KI, NT>::fma(vp + g * step, cp + g * step, xs, a[0]);
#pragma unroll
    for (int h = U / 2; h > 0; h /= 2) {
#pragma unroll
        for (int u = 0; u < h; ++u)
            a[u] += a[u + h];
    }
    return a[0];
}

// U slot groups [g, g+U) of one lane, loaded branch-free: a group at or
// past `end` re-loads group g (valid memory, lines the wave reads anyway)
// and is not added, so all U value and column loads are in flight together.
template <int KI, bool NT, int U>
struct SlotBatch;

template <bool NT, int U>
struct SlotBatch<1, NT, U> {
    double v[U];
    int32_t c[U];
    template <typename CT>
    __device__ __forceinline__ void load(const double *vp, const CT *cp, int64_t g, int64_t end, int64_t step)
    {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t gg = g + u < end ? g + u : g;
            v[u] = stream_load<NT>(vp + gg * step);
            c[u] = col_one<NT>(cp + gg * step);
        }
    }
    template <typename XS>
    __device__ __forceinline__ void fma(const XS &xs, int64_t g, int64_t end, double *a) const
    {
#pragma unroll
        for (int u = 0; u < U; ++u)  // branch-free: a guarded add lets the compiler sink the loads into branches
            a[u] += (g + u < end ? v[u] : 0.0) * xs(c[u]);
    }
    template <typename XS>
    __device__ __forceinline__ void fma4(const XS &xs, int64_t g, int64_t end, double *a) const
    {
#pragma unroll
        for (int u = 0; u < U; ++u)
            a[u % 4] += (g + u < end ? v[u] : 0.0) * xs(c[u]);
    }
};

template <bool NT, int U>
struct SlotBatch<2, NT, U> {
    double2 v[U];
    int2 c[U];
    template <typename CT>
    __device__ __forceinline__ void load(const double *vp, const CT *cp, int64_t g, int64_t end, int64_t step)
    {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t gg = g + u < end ? g + u : g;
            v[u] = stream_load2<NT>(vp + gg * step);
            c[u] = col_two<NT>(cp + gg * step);
        }
    }
    template <typename XS>
    __device__ __forceinline__ void fma(const XS &xs, int64_t g, int64_t end, double *a) const
    {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = g + u < end;
            a[u] += (in ? v[u].x : 0.0) * xs(c[u].x) + (in ? v[u].y : 0.0) * xs(c[u].y);
        }
    }
    template <typename XS>
    __device__ __forceinline__ void fma4(const XS &xs, int64_t g, int64_t end, double *a) const
    {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = g + u < end;
            a[u % 4] += (in ? v[u].x : 0.0) * xs(c[u].x) + (in ? v[u].y : 0.0) * xs(c[u].y);
        }
    }
};

// (A software-pipelined slot loop — the next U groups' loads issued before
// the current U's FMAs, same bits — measured SELL 0.2682 vs 0.2624 ms and ELL
// equal: 78 instead of 60 VGPRs halve the 1024-thread workgroups per CU;
// U = 8 groups in flight: equal. profiles/round2/ab_slot_pipe.log,
// ab_rows_sell.log.)

// One workgroup covers one sigma window (up to 1024 slots): every y[perm]
// store of a window then comes from ONE CU, so its L2 merges the window's
// scattered 8-byte stores into whole lines.  With 256-slot workgroups a
// 1024-row window was written from four XCDs and each partially written
// line left the chip up to four times (WRITE_SIZE 2.9x the y bytes,
// profiles/traffic.json), which cost ~10 % of the kernel.
template <int KI, bool NT, int U, typename XS = XGlobal>
__global__ __launch_bounds__(1024) void sell_kernel(
    int32_t C, int64_t n_slices, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ perm, const int32_t *__restrict__ col,
    const double *__restrict__ val, const XS xs,
    double *__restrict__ y, int remap, int64_t wcap)
{
    const int64_t slot = xcd_block(remap) * (int64_t)blockDim.x + threadIdx.x;
    const int64_t s = slot / C;
    if (s >= n_slices)
        return;
    const int64_t r = slot - s * C;
    const int64_t base = slice_ptr[s];
    int64_t w = (slice_ptr[s + 1] - base) / C;
    w = w < wcap ? w : wcap;  // split plan: the rest of a wide slice is sell_split_kernel's
    const int64_t off = base + r * KI;
    const double sum = slot_dot<KI, NT, U>(val + off, col + off, w, (int64_t)C * KI, xs);
    const int32_t row = perm[slot];
    if (row >= 0)
        y[row] = sum;  // scattered by perm: plain stores (sc1 measured 1.8 % slower, profiles/round2/ab_ystore.log)
}

template <int KI, bool NT, int U, typename XS = XGlobal>
__global__ __launch_bounds__(kBlock) void ell_kernel(
    int64_t n_rows, int32_t K, int64_t ld, const int32_t *__restrict__ col,
    const double *__restrict__ val, const XS xs,
    double *__restrict__ y, int remap)
{
    const int64_t i = xcd_block(remap) * kBlock + threadIdx.x;
    if (i >= n_rows)
        return;
    const int64_t off = i * KI;
    store_y(y + (i), slot_dot<KI, NT, U>(val + off, col + off, K, ld * KI, xs));
}

// Column window of every 256-row ELL workgroup: its rows' entries of
// k-group g are the contiguous run [g*ld*ki + b*256*ki, ... + rows*ki).
__global__ __launch_bounds__(kBlock) void ell_window_kernel(int64_t n_rows, int32_t K, int64_t ld, int32_t ki,
                                                            const int32_t *__restrict__ col,
                                                            int2 *__restrict__ win)
{
    const int64_t r0 = (int64_t)blockIdx.x * kBlock;
    const int64_t r1 = r0 + kBlock < n_rows ? r0 + kBlock : n_rows;
    int lo = INT32_MAX, hi = INT32_MIN;
    for (int32_t g = 0; g < K / ki; ++g) {
        const int64_t base = (int64_t)g * ld * ki;
        for (int64_t e = base + r0 * ki + threadIdx.x; e < base + r1 * ki; e += kBlock) {
            const int c = col[e];
            lo = c < lo ? c : lo;
            hi = c > hi ? c : hi;
        }
    }
    const int2 r = block_minmax(lo, hi);
    if (threadIdx.x == 0)
        win[blockIdx.x] = r;
}

// (Round 6: small grids — one cant-like matrix, 244 workgroups, one wave
// per SIMD — with every lane's slot loop in batches of 16 groups (SlotBatch)
// and a one-pass window copy measured slower: 15.3 vs 15.0 us cold with x
// windows, 29.8 vs 16.4 us without; profiles/round6/ab_ell.md.)
// ELL with the workgroup's x window staged in LDS (as sell_xwin_kernel).
// WB: the window copied with 4 loads per thread in flight (copy_window);
// else a strided copy, one round trip per 256 entries.
template <int KI, bool NT, int U, bool WB = false>
__global__ __launch_bounds__(kBlock) void ell_xwin_kernel(
    int64_t n_rows, int32_t K, int64_t ld, const int32_t *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x,
    double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap, int remap = 0)
{
    extern __shared__ double s_x[];
    const int64_t blk = xcd_block(remap);  // remap: neighbouring row blocks (shared x lines) on one XCD
    const int2 wnd = win[blk];
    const int32_t span = wnd.y - wnd.x + 1;
    const bool staged = span > 0 && span <= xcap;  // uniform per workgroup
    if (staged) {
        // the strided copy: the batched copy_window measured 1 % slower on the
        // 32-copy batch (0.3300 / 0.3272 vs 0.3244 / 0.3248 ms,
        // profiles/round2/ab_formats.log) and 1.8 % faster on one cant-like
        // matrix (11.88 -> 11.67 us cold, profiles/round5/ab_ell_wcopy.md),
        // where every workgroup is resident at once and waits out the copy's
        // round trips: batched for a grid of at most 4 workgroups per CU
        if constexpr (WB)
            copy_window<kBlock, 4>(s_x, x, wnd.x, span);
        else
            for (int32_t j = threadIdx.x; j < span; j += kBlock)
                s_x[j] = x[wnd.x + j];
        __syncthreads();
    }
    const int64_t i = blk * kBlock + threadIdx.x;
    if (i >= n_rows)
        return;
    const int64_t off = i * KI;
    store_y(y + i, staged ? slot_dot<KI, NT, U>(val + off, col + off, K, ld * KI, XWindow{s_x, wnd.x})
                          : slot_dot<KI, NT, U>(val + off, col + off, K, ld * KI, XGlobal{x}));
}

constexpr int32_t kEllXwinCap = 2048;  // 16 KiB per 256-row workgroup

}  // namespace spmv

using namespace spmv;

namespace spmv {

// Workgroup geometry of the SELL kernels: one workgroup per sigma window
// when it fits (256..1024 slots, a multiple of the wave), else 256 slots.
// A small matrix (fewer than ~2 windows per CU) needs the parallelism of
// 256-slot groups more than merged stores: one cant-like copy has only 61
// windows of 1024 rows for 256 CUs.
// y of a σ = 1024 window staged in LDS and stored in row order
// (sell_xwin_kernel): cant batch 0.2583 -> 0.2490 ms
// (profiles/round2/ab_sell_ystage.log)
static bool sell_ystage(int bt, int32_t sigma)
{
    return bt == 1024 && sigma == 1024;
}

bool sell_small(int32_t C, int64_t n_slices);
#ifndef SPMV_SELL_SMALL_S  // A/B builds only (tools/gpu_job.sh absingle); the product is built with the default
#define SPMV_SELL_SMALL_S 2
#endif
constexpr int kSellSmallS = SPMV_SELL_SMALL_S;  // sell_small_kernel: waves per slice
#ifndef SPMV_SELL_HEAD_G  // A/B builds only, as SPMV_SELL_SMALL_S
#define SPMV_SELL_HEAD_G 8
#endif
#ifndef SPMV_SELL_SMALL_P  // A/B builds only, as SPMV_SELL_SMALL_S
#define SPMV_SELL_SMALL_P 4
#endif
constexpr int kSellSmallP = SPMV_SELL_SMALL_P;  // sell_small_kernel: slices per workgroup (and per x window)
#ifndef SPMV_SELL_XCOPY  // A/B builds only
#define SPMV_SELL_XCOPY 4
#endif
constexpr int kSellXCopy = SPMV_SELL_XCOPY;  // sell_small_kernel: waves that copy the x window (HEAD)
#ifndef SPMV_SELL_LAST_B  // A/B builds only
#define SPMV_SELL_LAST_B 8
#endif
constexpr int kSellLastB = SPMV_SELL_LAST_B;  // sell_small_kernel: the largest last batch

static void sell_geometry(int32_t C, int32_t sigma, int64_t n_slices, int *bt, int64_t *blocks)
{
    if (sell_small(C, n_slices)) {  // sell_small_kernel: one workgroup (and x window) per 4 slices
        *bt = C * kSellSmallP;
        *blocks = (n_slices + kSellSmallP - 1) / kSellSmallP;
        return;
    }
    const int64_t slots = n_slices * C;
    const int64_t windows = sigma > 1 ? (slots + sigma - 1) / sigma : 0;
    const bool wide = windows >= 512 && sigma >= kBlock && sigma <= 1024 &&
                      sigma % kWave == 0;
    *bt = wide ? sigma : kBlock;
    *blocks = (slots + *bt - 1) / *bt;
}

static int sell_check_args(const spmv_dims &d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                           const char *who)
{
    static thread_local char msg[160];
    if (d.n_rows < 0 || C <= 0 || C > 1024 || n_slices < 0) {
        snprintf(msg, sizeof msg, "%s: bad C / sizes", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    if (ki != 1 && ki != 2) {
        snprintf(msg, sizeof msg, "%s: ki must be 1 or 2", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    if (sigma < 1 || (sigma > 1 && sigma % C != 0)) {
        snprintf(msg, sizeof msg, "%s: sigma must be 1 or a multiple of C", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    if (n_slices * C < d.n_rows) {
        snprintf(msg, sizeof msg, "%s: n_slices*C < n_rows", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    return SPMV_SUCCESS;
}

// Column window [lo, hi] of every SELL workgroup: min/max column over the
// contiguous entries of the slices it covers (one pass over col, build time).
__global__ __launch_bounds__(kBlock) void sell_window_kernel(int32_t C, int bt, int64_t n_slices,
                                                             const int64_t *__restrict__ slice_ptr,
                                                             const int32_t *__restrict__ col,
                                                             int2 *__restrict__ win)
{
    const int64_t b = blockIdx.x;
    const int64_t s0 = b * bt / C;
    int64_t s1 = ((b + 1) * bt + C - 1) / C;
    s1 = s1 < n_slices ? s1 : n_slices;
    const int2 r = block_col_range(col, slice_ptr[s0], slice_ptr[s1]);
    if (threadIdx.x == 0)
        win[b] = r;
}

// SELL with the workgroup's x window staged in LDS.  Cant-like rows of a
// 1024-row sigma window read ~1,600 distinct columns; gathering them from
// global memory costs one TA/TCP address per lane per step (the kernels'
// limiter: TA busy 80 %, requests far below the DRAM credit limit,
// profiles/round1/pmc_stalls.json).  Here the window is copied into LDS
// once with coalesced loads and every gather is a ds_read_b64.  A
// workgroup whose window exceeds xcap entries gathers from global memory.
// CT = uint16_t: SELL16 (columns stored as offsets from wnd.x).
template <int KI, bool NT, int U, typename CT = int32_t>
__device__ __forceinline__ void sell_xwin_body(
    int64_t blk, int32_t C, int64_t n_slices, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ perm, const CT *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x,
    double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap, int64_t wcap,
    int64_t ystage_rows, double *s_x)
{
    const int2 wnd = win[blk];
    const int32_t span = wnd.y - wnd.x + 1;
    const bool staged = span > 0 && span <= xcap;  // uniform per workgroup
    const int64_t slot = blk * blockDim.x + threadIdx.x;
    const int64_t s = slot / C;
    const int32_t row = s < n_slices ? perm[slot] : -1;
    if (staged) {
        if (blockDim.x == 1024)  // one sigma window per workgroup (the default geometry)
            copy_window<1024, 2>(s_x, x, wnd.x, span);
        else
            for (int32_t i = threadIdx.x; i < span; i += blockDim.x)
                s_x[i] = x[wnd.x + i];
    }
    // ystage_rows > 0 (σ = 1024 = the workgroup): does the window keep its
    // rows in order (equal lengths, e.g. the banded matrix)?  Asked at the
    // barrier that publishes the x window anyway.
    bool in_order = false;
    if (ystage_rows > 0)
        in_order = __syncthreads_and(row < 0 || row == slot);  // uniform
    else if (staged)
        __syncthreads();
    double sum = 0.0;
    if (s < n_slices) {
        const int64_t r = slot - s * C;
        const int64_t base = slice_ptr[s];
        int64_t w = (slice_ptr[s + 1] - base) / C;
        w = w < wcap ? w : wcap;
        const int64_t off = base + r * KI;
        constexpr bool c16 = std::is_same<CT, uint16_t>::value;
        sum = staged ? slot_dot<KI, NT, U>(val + off, col + off, w, (int64_t)C * KI, XWindow{s_x, c16 ? 0 : wnd.x})
                     : slot_dot<KI, NT, U>(val + off, col + off, w, (int64_t)C * KI, XGlobal{c16 ? x + wnd.x : x});
    }
    if (ystage_rows > 0) {
        if (in_order) {  // whole rows in order already: written through L2 directly
            if (row >= 0)
                store_y(y + row, sum);
            return;
        }
        // the window's slots hold a permutation of its 1024 rows: y goes
        // through LDS and out in row order (store_y) instead of as 8-byte
        // stores scattered by perm
        __shared__ double s_y[1024];
        const int64_t r0 = blk * 1024;
        if (__syncthreads_and(row < 0 || (row >= r0 && row < r0 + 1024))) {  // uniform
            if (row >= 0)
                s_y[row - r0] = sum;
            __syncthreads();
            const int64_t rr = r0 + threadIdx.x;
            if (rr < ystage_rows)
                store_y(y + rr, s_y[threadIdx.x]);
            return;
        }
    }
    if (row >= 0)
        y[row] = sum;  // scattered by perm: plain stores (sc1 measured 1.8 % slower, profiles/round2/ab_ystore.log)
}

template <int KI, bool NT, int U, typename CT = int32_t>
__global__ __launch_bounds__(1024) void sell_xwin_kernel(
    int32_t C, int64_t n_slices, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ perm, const CT *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x,
    double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap, int64_t wcap, int remap,
    int64_t ystage_rows)
{
    extern __shared__ double s_x[];
    const int64_t blk = xcd_block(remap);  // remap: neighbouring windows on one XCD (shared x lines in L2)
    sell_xwin_body<KI, NT, U, CT>(blk, C, n_slices, slice_ptr, perm, col, val, x, y, win, xcap, wcap, ystage_rows,
                                  s_x);
}

// SELL with a split plan in ONE launch (256-slot workgroups, no y staging):
// the first split_blocks workgroups run the wide slices' chunks
// (sell_split_body, into part[]), the rest the main x-window kernel's
// workgroups (every slice's first T columns).  The chunks — an R-MAT's hub
// rows, long chains of x gathers — then run beside the main stream instead
// of after it; same arithmetic, same bits (sell_split_fix_kernel still adds
// the chunks afterwards).
template <int KI, bool NT, int U, typename XS>
__device__ __forceinline__ void sell_split_body(int64_t gid, int32_t C, int64_t n_chunks, int32_t T,
                                                const int64_t *__restrict__ slice_ptr,
                                                const int32_t *__restrict__ chunk_slice,
                                                const int32_t *__restrict__ chunk_k0, const int32_t *__restrict__ col,
                                                const double *__restrict__ val, const XS xs,
                                                double *__restrict__ part);  // defined with sell_split_kernel

template <int KI, bool NT, int U, int SU>
__global__ __launch_bounds__(kBlock) void sell_split_fused_kernel(
    int64_t split_blocks, int32_t C, int64_t n_slices, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ perm, const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap, int32_t T,
    int64_t n_chunks, const int32_t *__restrict__ chunk_slice, const int32_t *__restrict__ chunk_k0,
    double *__restrict__ part)
{
    extern __shared__ double s_x[];
    const int64_t b = blockIdx.x;
    if (b < split_blocks) {  // uniform
        sell_split_body<KI, NT, SU, XGlobal>(b * kBlock + threadIdx.x, C, n_chunks, T, slice_ptr, chunk_slice,
                                             chunk_k0, col, val, XGlobal{x}, part);
        return;
    }
    sell_xwin_body<KI, NT, U, int32_t>(b - split_blocks, C, n_slices, slice_ptr, perm, col, val, x, y, win, xcap,
                                       (int64_t)T, 0, s_x);
}

// Small matrices (BASELINE.json configs[2]: one cant-like matrix is 976
// slices of C = 64).  With one wave per slice each SIMD holds about one wave
// and every lane walks its ~64-entry row in dependent round trips.  Here a
// workgroup owns P consecutive slices (one σ-window of 1024 rows holds 16)
// with S waves per slice; each wave takes a contiguous range of its slice's
// slot columns (lane = row of the slice).  Every lane issues the value and
// column loads of its first G slot groups at once (branch-free: past its
// range it re-reads its first group, same lines, and adds nothing); with
// those in flight the workgroup copies ONE x window, the union of its P
// slices' columns (XWIN: windows built per workgroup by spmv_sell_xwin_build),
// into LDS, then one barrier and the products.  Groups past G follow in
// batches of 4.  The S partial sums of a row meet in LDS and the slice's
// first wave adds them in wave order.  Deterministic; XWIN and global
// gathers give the same bits (same S, G and batches; P only groups slices);
// a row's sum is grouped differently from sell_kernel's, so the bits differ
// from it (the parity rule holds).  Shape from tools/sell_lab.py (cold
// spans, cant-like single, profiles/round3/sell_lab_multi_slice*.log): one
// slice per workgroup copied a 1,572-entry window per 64 rows (12 MB of L2
// reads for a 49 MB matrix); four slices share it.
template <int KI> constexpr int sell_small_g() { return SPMV_SELL_HEAD_G; }  // first-batch slot groups per lane

// (SELL16 gathering x from global memory instead of the LDS window (xcap 0)
// measured slower on one cant-like copy: 11.6-11.9 vs 10.3-10.6 us cold,
// profiles/round3/ab_sell16_xwindow_vs_global.json.)
// (Also issuing the 12 groups after the head early measured slower for
// SELL16 on one cant-like copy: before the window's loads 10.94-11.0 vs
// 10.36 us cold; after them, before the window barrier, 10.84-10.98 vs
// 10.20-10.24 us in one A/B (profiles/round3/ab_sell16_tail.log).)
// HEAD (SELL16 head copy, spmv_sell16_head_fill): the first G slot groups
// of every wave are also stored in a head array at an address computed from
// the workgroup and wave ids alone, so the first batch goes out without
// waiting for slice_ptr (one dependent HBM round trip fewer on a cold
// matrix); the later groups come from the SELL arrays.  Same values in the
// same accumulators: bit-identical.
// SELL_STAMP(k) / SELL_STAMP_HWID(): per-wave phase hooks, no-ops in the
// product; a lab build (tools/build_variant.sh stamps_sell) injects
// tools/lab_stamps_sell.h (tools/sell_stamps.py reads them)
#ifndef SELL_STAMP
#define SELL_STAMP(k) \
    do {              \
    } while (0)
#define SELL_STAMP_HWID() \
    do {                  \
    } while (0)
#endif
template <int KI, bool NT, bool XWIN, typename XS, typename CT = int32_t, int HG = 0>
__global__ __launch_bounds__(kWave * kSellSmallS * kSellSmallP) void sell_small_kernel(
    int64_t n_slices, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ perm, const CT *__restrict__ col,
    const double *__restrict__ val, const XS xs, double *__restrict__ y, int64_t wcap,
    const double *__restrict__ x, const int2 *__restrict__ win, int32_t xcap,
    const double *__restrict__ hval = nullptr, const CT *__restrict__ hcol = nullptr, int remap = 0)
{
    constexpr bool HEAD = HG > 0;  // HG: the head's slot groups per wave (the first batch)
    // remap: consecutive workgroups (the 1024 / (64 P) of one σ-window, whose
    // y[perm] stores share lines) on one XCD, so its L2 merges those lines
    const int64_t bid = xcd_block(remap);
    constexpr int S = kSellSmallS, P = kSellSmallP, G = HEAD ? HG : sell_small_g<KI>();
    constexpr bool c16 = std::is_same<CT, uint16_t>::value;  // SELL16: offsets from the window base
    static_assert(!c16 || XWIN, "SELL16 needs the workgroup windows");
    static_assert(!HEAD || XWIN, "the head runs with the workgroup windows");
    constexpr int64_t step = (int64_t)kWave * KI;  // elements between slot groups
    extern __shared__ double s_x[];
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    SELL_STAMP(0);
    SELL_STAMP_HWID();
    SlotBatch<KI, NT, G> first;
    // The x window (HEAD + XWIN): the first kSellXCopy waves request it
    // before their heads (its loads then return ahead of theirs) and store
    // it; the others issue their heads at once.  One cant-like matrix cold:
    // SELL16 9.56 -> 9.38 us, SELL 10.33 -> 10.28 (profiles/round5/ab_sell_pipe.md).
    constexpr int XT = kWave * kSellXCopy, XU = 2048 / XT;
    bool xdone = false;
    // (Round 6: the other waves' heads issued before the window bounds
    // arrive, instead of after them, measured 11.5 vs 10.85 us in-process:
    // the x window's loads then queue behind them.)
    if constexpr (HEAD && XWIN) {
        const int64_t hw = bid * (S * P) + wv;
        const int wvu = __builtin_amdgcn_readfirstlane(wv);
        const int2 wq = win[bid];
        const int32_t spq = wq.y - wq.x + 1;
        xdone = spq > 0 && spq <= xcap && spq <= XU * XT;  // uniform per workgroup
        if (xdone && wvu < kSellXCopy) {
            double xv[XU];
#pragma unroll
            for (int k = 0; k < XU; ++k) {
                const int32_t i = (int32_t)threadIdx.x + k * XT;
                xv[k] = x[wq.x + (i < spq ? i : spq - 1)];
            }
            first.load(hval + hw * G * step + lane * KI, hcol + hw * G * step + lane * KI, 0, G, step);
#pragma unroll
            for (int k = 0; k < XU; ++k) {
                const int32_t i = (int32_t)threadIdx.x + k * XT;
                if (i < spq)
                    s_x[i] = xv[k];
            }
        } else {
            first.load(hval + hw * G * step + lane * KI, hcol + hw * G * step + lane * KI, 0, G, step);
        }
    }
    // The slice bounds come through the scalar cache (a wave-uniform index):
    // as vector loads they returned behind the head's loads (loads return in
    // order), so the x window's loads went out only once the whole head had
    // arrived.  Per-wave stamps (tools/sell_stamps.py, cold): 4.4 of 10.4 us
    // from the start to the window barrier.
    const int wu = __builtin_amdgcn_readfirstlane(wv);
    const int64_t s = bid * P + wu / S;
    const int ws = wu % S;  // wave within its slice
    const bool live = s < n_slices;  // uniform per wave
    const int64_t base = live ? slice_ptr[s] : 0;
    int64_t w = live ? (slice_ptr[s + 1] - base) / kWave : 0;
    w = w < wcap ? w : wcap;
    const int64_t groups = w / KI;
    const int64_t per = (groups + S - 1) / S;
    const int64_t g0 = ws * per;
    const int64_t g1 = g0 + per < groups ? g0 + per : groups;
    const bool any = g1 > g0;  // uniform per wave: no loads past the slice
    const double *vp = val + base + lane * KI;
    const CT *cp = col + base + lane * KI;
    if constexpr (!HEAD) {
        if (any)
            first.load(vp, cp, g0, g1, step);
    }
    bool staged = false;
    int2 wnd = make_int2(0, -1);
    if constexpr (XWIN) {
        wnd = win[bid];
        const int32_t span = wnd.y - wnd.x + 1;
        if constexpr (HEAD && !c16) {
            // int32 with a head: only windows the first waves copied are
            // staged; a wider one gathers from global memory (same x values,
            // same bits).  The fallback copy loop joined the straight-line
            // path and made the compiler wait for every head load before the
            // barrier (vmcnt(0): a register of the loop's loads is reused
            // below).  Without it, one cant-like matrix cold: 13.55 -> 13.30
            // us (events); SELL16 measured the other way (12.56 -> 12.78 us)
            // and keeps the loop (profiles/round6/ab_sell_variants.md).
            staged = xdone;
        } else {
            staged = span > 0 && span <= xcap;  // uniform per workgroup
            if (staged && !xdone)
                copy_window<kWave * S * P, 4>(s_x, x, wnd.x, span);
        }
        __syncthreads();
    }
    SELL_STAMP(1);
    // batch 1 (the 4 groups after the first batch) goes out before the first
    // batch's products, later batches one at a time.  One cant-like matrix
    // cold, with the scalar bounds (profiles/round5/ab_sell_pipe.md): SELL
    // 10.80 -> 10.28 us, SELL16 9.70 -> 9.55; keeping two batches in flight
    // throughout, or issuing batch 1 before the window barrier, was slower.
    // (Round 6: every group after the head in ONE batch here — 8 or 16
    // groups, branch-free — measured slower: 13.80 / 14.36 vs 13.30 us cold,
    // profiles/round6/ab_sell_variants.md.)
    SlotBatch<KI, NT, 4> nb;
    if (g0 + G < g1)  // uniform per wave
        nb.load(vp, cp, g0 + G, g1, step);
    const int32_t row = live && ws == 0 ? perm[s * kWave + lane] : -1;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    auto body = [&](const auto &src) {
        if (any)
            first.fma4(src, g0, g1, a);
        SELL_STAMP(2);
        int64_t g = g0 + G;
        if (g < g1)
            nb.fma4(src, g, g1, a);
        // later batches of 4 groups, the last one up to kSellLastB: a short
        // remainder rides with the batch before it instead of costing a
        // round trip of its own (same groups, same accumulators, same order:
        // the same bits).  One cant-like matrix cold, four interleaved rounds:
        // SELL 10.27 -> 10.21 us, SELL16 9.48 -> 9.26; a last batch of up to
        // 6 groups measured slower (profiles/round5/ab_sell_pipe.md)
        for (g += 4; g < g1;) {
            if (g1 - g <= kSellLastB) {
                SlotBatch<KI, NT, kSellLastB> b;
                b.load(vp, cp, g, g1, step);
                b.fma4(src, g, g1, a);
                break;
            }
            SlotBatch<KI, NT, 4> b;
            b.load(vp, cp, g, g1, step);
            b.fma4(src, g, g1, a);
            g += 4;
        }
        SELL_STAMP(3);
    };
    if (staged) {
        body(XWindow{s_x, c16 ? 0 : wnd.x});
    } else {
        if constexpr (c16)
            body(XGlobal{x + wnd.x});
        else
            body(xs);
    }
    double sum = (a[0] + a[2]) + (a[1] + a[3]);
    __shared__ double part[S * P][kWave];
    part[wv][lane] = sum;
    __syncthreads();
    SELL_STAMP(4);
    if (ws == 0) {
#pragma unroll
        for (int k = 1; k < S; ++k)
            sum += part[wv + k][lane];
    }
    // y[perm]: plain stores.  Round 6 (one cant-like matrix cold, in-process):
    // sc1 (store_y) 11.5 and non-temporal 11.4 against 10.85 us plain
    // (profiles/round6/ab_sell_variants.md)
    if (row >= 0)
        y[row] = sum;  // scattered by perm: plain stores, as sell_kernel
    SELL_STAMP(5);
}

// Whether sell_small_kernel runs: C = 64 (a slice is one wave) and fewer
// slices than ~3.5 waves per SIMD of one-wave-per-slice kernels would fill
// on the MI355X's 256 CUs.  A pure function of (C, n_slices), never of the
// current device: it sets the SELL geometry (4-slice workgroups or σ
// windows) that spmv_sell_xwin_bytes/_build, spmv_sell16_fill (16-bit
// offsets from each workgroup's window base), the SELL16 head and
// spmv_sell_auto_ki all bake into the arrays they build, so a matrix built
// under one device must run under the same geometry on any other (ADVICE
// round 3: a CU-count query here made it depend on the current device).
constexpr int64_t kSellSmallCUs = 256;
bool sell_small(int32_t C, int64_t n_slices)
{
    if (C != kWave || n_slices <= 0)
        return false;
    return n_slices < 14 * kSellSmallCUs;
}

// slot groups per wave in the SELL16 head (its kernel's first batch): 8 and
// 12 ran the same (10.36 us cold, cant-like single), 16 slower (11.24 us:
// waves of 9-15 groups read padding); profiles/round3/cant_single_sell16_head_*.json
constexpr int kSell16HeadG = SPMV_SELL_HEAD_G;
static int sell16_head_g() { return kSell16HeadG; }

// XCD-contiguous placement of the x-window ELL workgroups (neighbouring
// 256-row blocks read overlapping x lines; on one XCD they share its L2):
// one cant-like matrix cold 12.28 / 12.16 -> 11.84 / 11.76 us, two
// interleaved rounds (profiles/round5/ab_remap_staged.md).
constexpr bool kEllRemapDefault = true;

// XCD-contiguous placement of the small-matrix kernel's workgroups: the
// workgroups of one σ-window then share one L2, which merges their
// scattered y[perm] stores into whole lines (one cant-like matrix cold,
// interleaved A/B: SELL 11.06 -> 10.86 us, SELL16 10.12 -> 9.80 us,
// profiles/round5/ab_sell_remap.md).  SPMV_XWIN_REMAP=0/1 overrides it per
// call, as for the x-window kernels.  (Round 5 also tried sharing the
// workgroup's 8 waves out over its 4 slices in proportion to their widths,
// instead of 2 per slice: 11.6-11.8 vs 10.5-10.7 us, not kept.)
constexpr bool kSellSmallRemapDefault = true;

template <int KI, bool NT, bool XWIN, typename XS, typename CT = int32_t>
static void launch_sell_small(int64_t n_slices, const int64_t *slice_ptr, const int32_t *perm, const CT *col,
                              const double *val, const XS xs, double *y, int64_t wcap, const double *x,
                              const int2 *win, int32_t xcap, hipStream_t st, const double *hval = nullptr,
                              const CT *hcol = nullptr)
{
    const size_t lds = XWIN ? (size_t)xcap * sizeof(double) : 0;
    const int64_t blocks = (n_slices + kSellSmallP - 1) / kSellSmallP;
    const int remap = xwin_remap(kSellSmallRemapDefault) ? 1 : 0;
#define SPMV_SMALL_HG(HH)                                                                                     \
    hipLaunchKernelGGL((sell_small_kernel<KI, NT, XWIN, XS, CT, HH>), dim3((unsigned)blocks),                 \
                       dim3(kWave * kSellSmallS * kSellSmallP), lds, st, n_slices, slice_ptr, perm, col, val, xs, \
                       y, wcap, x, win, xcap, hval, hcol, remap)
    if constexpr (XWIN) {  // the head (SELL16, or int32 SELL small matrices)
        if (hval)
            SPMV_SMALL_HG(kSell16HeadG);
        else
            SPMV_SMALL_HG(0);
    } else {
        SPMV_SMALL_HG(0);
    }
#undef SPMV_SMALL_HG
}

// SELL16 head copy: waves = 8 per small-kernel workgroup, G groups of
// 64 lanes x ki slots each; padding (a wave with fewer groups) holds value
// 0 and offset 0, and the kernel never adds it.
static int64_t sell16_head_elems(int64_t n_slices, int32_t ki)
{
    const int64_t blocks = (n_slices + kSellSmallP - 1) / kSellSmallP;
    return blocks * kSellSmallS * kSellSmallP * (int64_t)sell16_head_g() * kWave * ki;
}

template <int KI, int G, typename CT>
__global__ __launch_bounds__(kWave * kSellSmallS * kSellSmallP) void sell16_head_kernel(
    int64_t n_slices, const int64_t *__restrict__ slice_ptr, const double *__restrict__ val,
    const CT *__restrict__ col16, double *__restrict__ hval, CT *__restrict__ hcol)
{
    constexpr int S = kSellSmallS, P = kSellSmallP;
    constexpr int64_t step = (int64_t)kWave * KI;
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    const int64_t s = (int64_t)blockIdx.x * P + wv / S;
    const int ws = wv % S;
    const bool live = s < n_slices;
    const int64_t base = live ? slice_ptr[s] : 0;
    const int64_t groups = live ? (slice_ptr[s + 1] - base) / kWave / KI : 0;  // as sell_small_kernel (wcap = max)
    const int64_t per = (groups + S - 1) / S;
    const int64_t g0 = ws * per;
    const int64_t g1 = g0 + per < groups ? g0 + per : groups;
    const int64_t hw = (int64_t)blockIdx.x * (S * P) + wv;
    // groups past the wave's range repeat its first group, exactly as
    // SlotBatch::load re-reads it without a head: the kernel masks their
    // values, and x is read at one of the lane's own columns, so head and
    // no-head give the same bits even for a non-finite x
    for (int u = 0; u < G; ++u)
        for (int k = 0; k < KI; ++k) {
            const int64_t dst = (hw * G + u) * step + lane * KI + k;
            const bool any = g1 > g0;
            const int64_t gg = g0 + u < g1 ? g0 + u : g0;
            const int64_t src = base + gg * step + lane * KI + k;
            hval[dst] = any ? val[src] : 0.0;
            hcol[dst] = any ? col16[src] : (CT)0;
        }
}

// x-window variant when win != NULL (windows from spmv_sell_xwin_build:
// one per workgroup of kSellSmallP slices), else gathers through xs.
template <typename XS>
static void launch_sell_small_any(int32_t ki, bool nt, int64_t n_slices, const int64_t *slice_ptr,
                                  const int32_t *perm, const int32_t *col, const double *val, const XS xs, double *y,
                                  int64_t wcap, hipStream_t st, const double *x = nullptr,
                                  const int2 *win = nullptr, int32_t xcap = 0)
{
    if (win) {
        if constexpr (std::is_same<XS, XGlobal>::value) {
#define SPMV_SMALL_W(K, N) launch_sell_small<K, N, true>(n_slices, slice_ptr, perm, col, val, xs, y, wcap, x, win, xcap, st)
            if (ki == 2) { if (nt) SPMV_SMALL_W(2, true); else SPMV_SMALL_W(2, false); }
            else { if (nt) SPMV_SMALL_W(1, true); else SPMV_SMALL_W(1, false); }
#undef SPMV_SMALL_W
            return;
        }
    }
#define SPMV_SMALL_G(K, N) launch_sell_small<K, N, false>(n_slices, slice_ptr, perm, col, val, xs, y, wcap, x, (const int2 *)nullptr, 0, st)
    if (ki == 2) { if (nt) SPMV_SMALL_G(2, true); else SPMV_SMALL_G(2, false); }
    else { if (nt) SPMV_SMALL_G(1, true); else SPMV_SMALL_G(1, false); }
#undef SPMV_SMALL_G
}

// Wide slices (SELL split plan, spmv_sell_split_plan): a slice wider than
// T slot columns keeps its first T in the main kernel; chunk c covers slot
// columns [k0_c, k0_c + T) of slice s_c, one lane per slot, and leaves the
// slot's partial sum in part[c·C + r].  sell_split_fix_kernel adds each
// slice's chunks in chunk order to y[perm] (deterministic, no atomics).
// An R-MAT hub slice (~1.4e5 slot columns) otherwise keeps one wave busy
// for the whole kernel.
// slot groups per lane per step in a split chunk.  Round 6, R-MAT (bench
// layout, kernel trace): U = 4 / 8 / 16 took 311 / 333 / 336 us — the hub
// chunks' x gathers, not the load chain, set their time
// (profiles/round6/ab_sell_split.md)
constexpr int kSellSplitU = 4;
#ifndef SPMV_SELL_SPLIT_FUSED  // A/B builds only
#define SPMV_SELL_SPLIT_FUSED 1
#endif
constexpr bool kSellSplitFused = SPMV_SELL_SPLIT_FUSED;  // spmv_sell_run_split: one grid (see the fused kernel)
template <int KI, bool NT, int U, typename XS>
__device__ __forceinline__ void sell_split_body(
    int64_t gid, int32_t C, int64_t n_chunks, int32_t T, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ chunk_slice, const int32_t *__restrict__ chunk_k0,
    const int32_t *__restrict__ col, const double *__restrict__ val, const XS xs,
    double *__restrict__ part)
{
    const int64_t c = gid / C;
    if (c >= n_chunks)
        return;
    const int64_t r = gid - c * C;
    const int64_t s = chunk_slice[c];
    const int64_t k0 = chunk_k0[c];
    const int64_t base = slice_ptr[s];
    const int64_t w = (slice_ptr[s + 1] - base) / C;
    const int64_t n = w - k0 < T ? w - k0 : T;
    const int64_t off = base + k0 * C + r * KI;
    part[gid] = slot_dot<KI, NT, U>(val + off, col + off, n, (int64_t)C * KI, xs);
}

template <int KI, bool NT, int U, typename XS = XGlobal>
__global__ __launch_bounds__(kBlock) void sell_split_kernel(
    int32_t C, int64_t n_chunks, int32_t T, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ chunk_slice, const int32_t *__restrict__ chunk_k0,
    const int32_t *__restrict__ col, const double *__restrict__ val, const XS xs,
    double *__restrict__ part)
{
    sell_split_body<KI, NT, U, XS>((int64_t)blockIdx.x * kBlock + threadIdx.x, C, n_chunks, T, slice_ptr,
                                   chunk_slice, chunk_k0, col, val, xs, part);
}

// One 1024-thread workgroup per chunk; only the first chunk of each slice's
// run works.  Thread t takes row r = t % C of segment t / C: the run's
// chunks are cut into W = 1024 / C segments summed side by side (8 loads in
// flight per thread), and the W partial sums of a row are added in segment
// order through LDS — a fixed order, so bitwise reproducible; a run of at
// most W chunks is summed in chunk order exactly as before.  (One wave
// walking an R-MAT hub slice's ~600 chunks 8 per round trip took 57 us.)
constexpr int kSellFixThreads = 1024;
__global__ __launch_bounds__(kSellFixThreads) void sell_split_fix_kernel(int32_t C, int64_t n_chunks,
                                                                         const int32_t *__restrict__ chunk_slice,
                                                                         const int32_t *__restrict__ perm,
                                                                         const double *__restrict__ part,
                                                                         double *__restrict__ y)
{
    const int64_t c = blockIdx.x;
    const int32_t s = chunk_slice[c];
    if (c > 0 && chunk_slice[c - 1] == s)
        return;  // uniform: not the first chunk of its slice
    // the run's end: chunk_slice is sorted by slice, so the chunks equal to
    // s form a prefix of [c, n_chunks); counted 1024 probes at a time
    __shared__ int64_t s_end;
    int64_t lo = c + 1, step = 64;
    for (;;) {  // coarse: probes lo + t * step
        const int64_t q = lo + (int64_t)threadIdx.x * step;
        const int n = __syncthreads_count(q < n_chunks && chunk_slice[q] == s);
        if (n < kSellFixThreads) {  // the end lies in (lo + (n-1)*step, lo + n*step]
            lo = n > 0 ? lo + (int64_t)(n - 1) * step + 1 : lo;
            break;
        }
        lo += (int64_t)kSellFixThreads * step;
    }
    {  // fine: probes lo + t, t < step
        const int64_t q = lo + threadIdx.x;
        const int n = __syncthreads_count(threadIdx.x < step && q < n_chunks && chunk_slice[q] == s);
        if (threadIdx.x == 0)
            s_end = lo + n;
    }
    __syncthreads();
    const int64_t end = s_end;
    const int W = kSellFixThreads / C;
    const int r = threadIdx.x % C, seg = threadIdx.x / C;
    const int64_t len = end - c;
    const int64_t sl = (len + W - 1) / W;
    double acc = 0.0;
    if (seg < W) {
        const int64_t b = c + seg * sl, e = b + sl < end ? b + sl : end;
        for (int64_t u = b; u < e; u += 8) {
            double pp[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                pp[k] = u + k < e ? part[(u + k) * C + r] : 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (u + k < e)
                    acc += pp[k];
        }
    }
    __shared__ double s_p[kSellFixThreads];
    s_p[threadIdx.x] = acc;
    __syncthreads();
    if (seg == 0) {
        double tot = 0.0;
        for (int j = 0; j < W; ++j)
            tot += s_p[j * C + r];
        const int32_t row = perm[(int64_t)s * C + r];
        if (row >= 0)
            y[row] += tot;
    }
}

__global__ __launch_bounds__(kBlock) void sell_hot_gather_kernel(int64_t H, const int32_t *__restrict__ hot,
                                                                 const double *__restrict__ x,
                                                                 double *__restrict__ xh)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < H)
        xh[i] = x[hot[i]];
}

constexpr int32_t kXwinCapWide = 8192;   // 64 KiB of LDS per 1024-slot workgroup (2 per CU)
constexpr int32_t kXwinCapNarrow = 2048; // 16 KiB per 256-slot workgroup

}  // namespace spmv

// k-interleave for a SELL matrix of n_rows built for this device: 2 when
// the small-matrix kernel will run it (16-byte value loads: cant-like single
// 11.3-11.4 vs 12.1-12.2 us cold span with ki = 1, tools/sell_lab.py,
// profiles/round3/sell_lab_multi_slice3.log), else 1 (the σ-window kernel's
// measured best, profiles/round1/sweeps.md).
extern "C" int spmv_sell_auto_ki(int64_t n_rows, int32_t C)
{
    if (n_rows <= 0 || C <= 0)
        return 1;
    return sell_small(C, (n_rows + C - 1) / C) ? 2 : 1;
}

extern "C" int spmv_sell_run(spmv_dims d, int32_t C, int32_t sigma, int32_t ki,
                             int64_t n_slices, const int64_t *slice_ptr,
                             const int32_t *perm, const int32_t *col,
                             const double *val, const double *x, double *y)
{
    int rc = sell_check_args(d, C, sigma, ki, n_slices, "spmv_sell_run");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run: grid too large");
    const int remap = xcd_remap_enabled() ? 1 : 0;
    const bool nt = stream_nt(kSellStreamNtDefault);
    if (sell_small(C, n_slices)) {
        launch_sell_small_any(ki, nt, n_slices, slice_ptr, perm, col, val, XGlobal{x}, y, INT64_MAX,
                              (hipStream_t)d.stream);
        SPMV_CHECK_LAUNCH("sell_small_kernel");
        return SPMV_SUCCESS;
    }
    auto kern = ki == 2 ? (nt ? sell_kernel<2, true, 4> : sell_kernel<2, false, 4>)
                        : (nt ? sell_kernel<1, true, 4> : sell_kernel<1, false, 4>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bt), 0, (hipStream_t)d.stream, C,
                       n_slices, slice_ptr, perm, col, val, XGlobal{x}, y, remap, (int64_t)INT64_MAX);
    SPMV_CHECK_LAUNCH("sell_kernel");
    return SPMV_SUCCESS;
}

extern "C" size_t spmv_sell_xwin_bytes(int64_t n_slices, int32_t C, int32_t sigma)
{
    if (n_slices <= 0 || C <= 0)
        return 0;
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    return (size_t)blocks * sizeof(int2);
}

extern "C" int spmv_sell_xwin_build(spmv_dims d, int32_t C, int32_t sigma, int64_t n_slices,
                                    const int64_t *slice_ptr, const int32_t *col, void *win,
                                    size_t win_bytes, int32_t *xcap)
{
    int rc = sell_check_args(d, C, sigma, 1, n_slices, "spmv_sell_xwin_build");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (!xcap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_xwin_build: xcap is NULL");
    *xcap = 0;
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    if (!win || win_bytes < spmv_sell_xwin_bytes(n_slices, C, sigma))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_xwin_build: window buffer too small");
    SPMV_GUARD(d);
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(sell_window_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, C, bt, n_slices,
                       slice_ptr, col, (int2 *)win);
    SPMV_CHECK_LAUNCH("sell_window_kernel");
    // the LDS size of the run: the widest window, up to the cap (build time,
    // so the one synchronising copy is off the SpMV path)
    int2 *h = (int2 *)malloc((size_t)blocks * sizeof(int2));
    if (!h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_xwin_build: out of host memory");
    hipError_t e = hipMemcpyAsync(h, win, (size_t)blocks * sizeof(int2), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        free(h);
        return fail(SPMV_PROGRAM_ERROR, "spmv_sell_xwin_build: copy windows", e);
    }
    const int32_t cap = bt >= 1024 ? kXwinCapWide : kXwinCapNarrow;
    int32_t need = 0;
    for (int64_t b = 0; b < blocks; ++b) {
        const int64_t span = (int64_t)h[b].y - h[b].x + 1;
        if (span <= cap && span > need)
            need = (int32_t)span;
    }
    free(h);
    *xcap = need;
    return SPMV_SUCCESS;
}

extern "C" int spmv_sell_run_xwin(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                                  const int64_t *slice_ptr, const int32_t *perm, const int32_t *col,
                                  const double *val, const double *x, double *y, const void *win,
                                  int32_t xcap)
{
    int rc = sell_check_args(d, C, sigma, ki, n_slices, "spmv_sell_run_xwin");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    if (!win || xcap < 0 || xcap > kXwinCapWide)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_xwin: bad window arguments");
    SPMV_GUARD(d);
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_xwin: grid too large");
    const bool nt = stream_nt(kSellStreamNtDefault);
    if (sell_small(C, n_slices)) {  // few slices: the waves-per-slice kernel with per-slice x windows (same bits as spmv_sell_run)
        launch_sell_small_any(ki, nt, n_slices, slice_ptr, perm, col, val, XGlobal{x}, y, INT64_MAX,
                              (hipStream_t)d.stream, x, (const int2 *)win, xcap);
        SPMV_CHECK_LAUNCH("sell_small_kernel");
        return SPMV_SUCCESS;
    }
    auto kern = ki == 2 ? (nt ? sell_xwin_kernel<2, true, 4> : sell_xwin_kernel<2, false, 4>)
                        : (nt ? sell_xwin_kernel<1, true, 4> : sell_xwin_kernel<1, false, 4>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bt), (size_t)xcap * sizeof(double),
                       (hipStream_t)d.stream, C, n_slices, slice_ptr, perm, col, val, x, y,
                       (const int2 *)win, xcap, (int64_t)INT64_MAX, xwin_remap(false) ? 1 : 0,
                       sell_ystage(bt, sigma) ? d.n_rows : (int64_t)0);
    SPMV_CHECK_LAUNCH("sell_xwin_kernel");
    return SPMV_SUCCESS;
}

// SELL16: the column of every stored slot as a 16-bit offset from its
// workgroup's x-window base (win[b].x, spmv_sell_xwin_build), so a slot is
// 10 bytes instead of 12.  Workgroup b covers slices [b·bt/C, (b+1)·bt/C)
// exactly (C = 64 divides every SELL workgroup size), so each slot has ONE
// base.  Build time, one workgroup per window.
__global__ __launch_bounds__(kBlock) void sell16_fill_kernel(int32_t C, int bt, int64_t n_slices,
                                                             const int64_t *__restrict__ slice_ptr,
                                                             const int32_t *__restrict__ col,
                                                             const int2 *__restrict__ win,
                                                             uint16_t *__restrict__ col16)
{
    const int64_t b = blockIdx.x;
    const int64_t s0 = b * bt / C;
    int64_t s1 = (b + 1) * bt / C;
    s1 = s1 < n_slices ? s1 : n_slices;
    const int32_t lo = win[b].x;
    for (int64_t e = slice_ptr[s0] + threadIdx.x; e < slice_ptr[s1]; e += kBlock)
        col16[e] = (uint16_t)(col[e] - lo);
}

static int sell16_check(const spmv_dims &d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices, const char *who)
{
    int rc = sell_check_args(d, C, sigma, ki, n_slices, who);
    if (rc != SPMV_SUCCESS)
        return rc;
    if (C != kWave)
        return fail_msg(SPMV_OTHER_ERROR, "SELL16: C must be 64 (one slot column per wave)");
    return SPMV_SUCCESS;
}

extern "C" int spmv_sell16_fill(spmv_dims d, int32_t C, int32_t sigma, int64_t n_slices, const int64_t *slice_ptr,
                                const int32_t *col, const void *win, uint16_t *col16)
{
    int rc = sell16_check(d, C, sigma, 1, n_slices, "spmv_sell16_fill");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    if (!win || !col || !col16 || !slice_ptr)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_fill: NULL array");
    SPMV_GUARD(d);
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    if (bt % C != 0 || blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_fill: workgroups do not hold whole slices");
    const hipStream_t st = (hipStream_t)d.stream;
    // every window must span at most 65,536 columns (build time: one
    // synchronising copy of the window table)
    int2 *h = (int2 *)malloc((size_t)blocks * sizeof(int2));
    if (!h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_fill: out of host memory");
    hipError_t e = hipMemcpyAsync(h, win, (size_t)blocks * sizeof(int2), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        free(h);
        return fail(SPMV_PROGRAM_ERROR, "spmv_sell16_fill: copy windows", e);
    }
    int64_t wide = 0;
    for (int64_t b = 0; b < blocks; ++b)
        wide += (int64_t)h[b].y - h[b].x + 1 > 65536;
    free(h);
    if (wide > 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_fill: a workgroup's columns span more than 65,536");
    hipLaunchKernelGGL(sell16_fill_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, C, bt, n_slices, slice_ptr,
                       col, (const int2 *)win, col16);
    SPMV_CHECK_LAUNCH("sell16_fill_kernel");
    return SPMV_SUCCESS;
}

extern "C" size_t spmv_sell16_head_bytes(int64_t n_slices, int32_t C, int32_t ki)
{
    if (n_slices <= 0 || (ki != 1 && ki != 2) || !sell_small(C, n_slices))
        return 0;
    return (size_t)sell16_head_elems(n_slices, ki) * (sizeof(double) + sizeof(uint16_t));
}

extern "C" int spmv_sell16_head_fill(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                                     const int64_t *slice_ptr, const double *val, const uint16_t *col16, void *head,
                                     size_t head_bytes)
{
    int rc = sell16_check(d, C, sigma, ki, n_slices, "spmv_sell16_head_fill");
    if (rc != SPMV_SUCCESS)
        return rc;
    const size_t need = spmv_sell16_head_bytes(n_slices, C, ki);
    if (need == 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_head_fill: no head (not a small-kernel matrix)");
    if (!head || head_bytes < need || !slice_ptr || !val || !col16)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_head_fill: arrays or head buffer missing");
    SPMV_GUARD(d);
    double *hval = (double *)head;
    uint16_t *hcol = (uint16_t *)(hval + sell16_head_elems(n_slices, ki));
    const int64_t blocks = (n_slices + kSellSmallP - 1) / kSellSmallP;
    const hipStream_t st = (hipStream_t)d.stream;
#define SPMV_HEAD_FILL(K, HH)                                                                                    \
    hipLaunchKernelGGL((sell16_head_kernel<K, HH, uint16_t>), dim3((unsigned)blocks),                             \
                       dim3(kWave * kSellSmallS * kSellSmallP), 0, st, n_slices, slice_ptr, val, col16, hval, hcol)
    if (ki == 2)
        SPMV_HEAD_FILL(2, kSell16HeadG);
    else
        SPMV_HEAD_FILL(1, kSell16HeadG);
#undef SPMV_HEAD_FILL
    SPMV_CHECK_LAUNCH("sell16_head_kernel");
    return SPMV_SUCCESS;
}

// The head for int32 SELL (small matrices): the same copy of every wave's
// first slot groups, with int32 columns (12 B per slot).
extern "C" size_t spmv_sell_head_bytes(int64_t n_slices, int32_t C, int32_t ki)
{
    if (n_slices <= 0 || (ki != 1 && ki != 2) || !sell_small(C, n_slices))
        return 0;
    return (size_t)sell16_head_elems(n_slices, ki) * (sizeof(double) + sizeof(int32_t));
}

extern "C" int spmv_sell_head_fill(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                                   const int64_t *slice_ptr, const double *val, const int32_t *col, void *head,
                                   size_t head_bytes)
{
    int rc = sell_check_args(d, C, sigma, ki, n_slices, "spmv_sell_head_fill");
    if (rc != SPMV_SUCCESS)
        return rc;
    const size_t need = spmv_sell_head_bytes(n_slices, C, ki);
    if (need == 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_head_fill: no head (not a small-kernel matrix)");
    if (!head || head_bytes < need || !slice_ptr || !val || !col)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_head_fill: arrays or head buffer missing");
    SPMV_GUARD(d);
    double *hval = (double *)head;
    int32_t *hcol = (int32_t *)(hval + sell16_head_elems(n_slices, ki));
    const int64_t blocks = (n_slices + kSellSmallP - 1) / kSellSmallP;
    const hipStream_t st = (hipStream_t)d.stream;
    if (ki == 2)
        hipLaunchKernelGGL((sell16_head_kernel<2, kSell16HeadG, int32_t>), dim3((unsigned)blocks),
                           dim3(kWave * kSellSmallS * kSellSmallP), 0, st, n_slices, slice_ptr, val, col, hval, hcol);
    else
        hipLaunchKernelGGL((sell16_head_kernel<1, kSell16HeadG, int32_t>), dim3((unsigned)blocks),
                           dim3(kWave * kSellSmallS * kSellSmallP), 0, st, n_slices, slice_ptr, val, col, hval, hcol);
    SPMV_CHECK_LAUNCH("sell_head_kernel");
    return SPMV_SUCCESS;
}

// spmv_sell_run_xwin with the head (small matrices): same bits.
extern "C" int spmv_sell_run_xwin_head(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                                       const int64_t *slice_ptr, const int32_t *perm, const int32_t *col,
                                       const double *val, const double *x, double *y, const void *win,
                                       int32_t xcap, const void *head)
{
    if (!head || !sell_small(C, n_slices))
        return spmv_sell_run_xwin(d, C, sigma, ki, n_slices, slice_ptr, perm, col, val, x, y, win, xcap);
    int rc = sell_check_args(d, C, sigma, ki, n_slices, "spmv_sell_run_xwin_head");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    if (!win || xcap < 0 || xcap > kXwinCapWide)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_xwin_head: bad window arguments");
    SPMV_GUARD(d);
    const bool nt = stream_nt(kSellStreamNtDefault);
    const hipStream_t st = (hipStream_t)d.stream;
    const int2 *w = (const int2 *)win;
    const double *hval = (const double *)head;
    const int32_t *hcol = (const int32_t *)(hval + sell16_head_elems(n_slices, ki));
#define SPMV_SMALLH(K, N) \
    launch_sell_small<K, N, true, XGlobal, int32_t>(n_slices, slice_ptr, perm, col, val, XGlobal{x}, y, INT64_MAX, x, w, xcap, st, hval, hcol)
    if (ki == 2) { if (nt) SPMV_SMALLH(2, true); else SPMV_SMALLH(2, false); }
    else { if (nt) SPMV_SMALLH(1, true); else SPMV_SMALLH(1, false); }
#undef SPMV_SMALLH
    SPMV_CHECK_LAUNCH("sell_small_kernel (head)");
    return SPMV_SUCCESS;
}

extern "C" int spmv_sell16_run(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                               const int64_t *slice_ptr, const int32_t *perm, const uint16_t *col16,
                               const double *val, const double *x, double *y, const void *win, int32_t xcap,
                               const void *head)
{
    int rc = sell16_check(d, C, sigma, ki, n_slices, "spmv_sell16_run");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    if (!win || xcap < 0 || xcap > kXwinCapWide)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_run: bad window arguments");
    SPMV_GUARD(d);
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell16_run: grid too large");
    const bool nt = stream_nt(kSellStreamNtDefault);
    const hipStream_t st = (hipStream_t)d.stream;
    const int2 *w = (const int2 *)win;
    if (sell_small(C, n_slices)) {
        const double *hval = (const double *)head;
        const uint16_t *hcol = head ? (const uint16_t *)(hval + sell16_head_elems(n_slices, ki)) : nullptr;
#define SPMV_SMALL16(K, N) \
    launch_sell_small<K, N, true, XGlobal, uint16_t>(n_slices, slice_ptr, perm, col16, val, XGlobal{x}, y, INT64_MAX, x, w, xcap, st, hval, hcol)
        if (ki == 2) { if (nt) SPMV_SMALL16(2, true); else SPMV_SMALL16(2, false); }
        else { if (nt) SPMV_SMALL16(1, true); else SPMV_SMALL16(1, false); }
#undef SPMV_SMALL16
        SPMV_CHECK_LAUNCH("sell_small_kernel (SELL16)");
        return SPMV_SUCCESS;
    }
    auto kern = ki == 2 ? (nt ? sell_xwin_kernel<2, true, 4, uint16_t> : sell_xwin_kernel<2, false, 4, uint16_t>)
                        : (nt ? sell_xwin_kernel<1, true, 4, uint16_t> : sell_xwin_kernel<1, false, 4, uint16_t>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bt), (size_t)xcap * sizeof(double), st, C, n_slices,
                       slice_ptr, perm, col16, val, x, y, w, xcap, (int64_t)INT64_MAX, xwin_remap(false) ? 1 : 0,
                       sell_ystage(bt, sigma) ? d.n_rows : (int64_t)0);
    SPMV_CHECK_LAUNCH("sell_xwin_kernel (SELL16)");
    return SPMV_SUCCESS;
}

extern "C" int spmv_ell_run(spmv_dims d, int32_t K, int64_t ld, int32_t ki,
                            const int32_t *col, const double *val,
                            const double *x, double *y)
{
    if (d.n_rows < 0 || K < 0 || ld < d.n_rows || ld % 64 != 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_run: bad K / ld");
    if ((ki != 1 && ki != 2) || K % ki != 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_run: ki must be 1 or 2 and divide K");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    const int64_t blocks = (d.n_rows + kBlock - 1) / kBlock;
    const int remap = xcd_remap_enabled() ? 1 : 0;
    const bool nt = stream_nt(kSellStreamNtDefault);
    auto kern = ki == 2 ? (nt ? ell_kernel<2, true, 4> : ell_kernel<2, false, 4>)
                        : (nt ? ell_kernel<1, true, 4> : ell_kernel<1, false, 4>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)d.stream,
                       d.n_rows, K, ld, col, val, XGlobal{x}, y, remap);
    SPMV_CHECK_LAUNCH("ell_kernel");
    return SPMV_SUCCESS;
}

extern "C" size_t spmv_ell_xwin_bytes(int64_t n_rows)
{
    return n_rows > 0 ? (size_t)((n_rows + kBlock - 1) / kBlock) * sizeof(int2) : 0;
}

extern "C" int spmv_ell_xwin_build(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *col,
                                   void *win, size_t win_bytes, int32_t *xcap)
{
    if (d.n_rows < 0 || K < 0 || ld < d.n_rows || ld % 64 != 0 || (ki != 1 && ki != 2) || K % ki != 0 || !xcap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_xwin_build: bad arguments");
    *xcap = 0;
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    const size_t need = spmv_ell_xwin_bytes(d.n_rows);
    if (!win || win_bytes < need)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_xwin_build: window buffer too small");
    SPMV_GUARD(d);
    const int64_t blocks = (d.n_rows + kBlock - 1) / kBlock;
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(ell_window_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, d.n_rows, K, ld, ki, col,
                       (int2 *)win);
    SPMV_CHECK_LAUNCH("ell_window_kernel");
    int2 *h = (int2 *)malloc(need);
    if (!h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_xwin_build: out of host memory");
    hipError_t e = hipMemcpyAsync(h, win, need, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        free(h);
        return fail(SPMV_PROGRAM_ERROR, "spmv_ell_xwin_build: copy windows", e);
    }
    int32_t best = 0;
    for (int64_t b = 0; b < blocks; ++b) {
        const int64_t span = (int64_t)h[b].y - h[b].x + 1;
        if (span <= kEllXwinCap && span > best)
            best = (int32_t)span;
    }
    free(h);
    *xcap = best;
    return SPMV_SUCCESS;
}

extern "C" int spmv_ell_run_xwin(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *col,
                                 const double *val, const double *x, double *y, const void *win, int32_t xcap)
{
    if (d.n_rows < 0 || K < 0 || ld < d.n_rows || ld % 64 != 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_run_xwin: bad K / ld");
    if ((ki != 1 && ki != 2) || K % ki != 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_run_xwin: ki must be 1 or 2 and divide K");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (!win || xcap < 0 || xcap > kEllXwinCap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_ell_run_xwin: bad window arguments");
    SPMV_GUARD(d);
    const int64_t blocks = (d.n_rows + kBlock - 1) / kBlock;
    const bool nt = stream_nt(kSellStreamNtDefault);
    auto kern = blocks <= 4 * 256
                    ? (ki == 2 ? (nt ? ell_xwin_kernel<2, true, 4, true> : ell_xwin_kernel<2, false, 4, true>)
                               : (nt ? ell_xwin_kernel<1, true, 4, true> : ell_xwin_kernel<1, false, 4, true>))
                    : (ki == 2 ? (nt ? ell_xwin_kernel<2, true, 4> : ell_xwin_kernel<2, false, 4>)
                               : (nt ? ell_xwin_kernel<1, true, 4> : ell_xwin_kernel<1, false, 4>));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), (size_t)xcap * sizeof(double),
                       (hipStream_t)d.stream, d.n_rows, K, ld, col, val, x, y, (const int2 *)win, xcap,
                       xwin_remap(kEllRemapDefault) ? 1 : 0);
    SPMV_CHECK_LAUNCH("ell_xwin_kernel");
    return SPMV_SUCCESS;
}

// HYB with K = 0, the plan's choice where most rows are empty or short (an
// ELL slot would cost more than the tail entry it saves: R-MAT): no ELL
// part, the tail is the whole matrix in row order, so it runs as COO (same
// kernels and workspace; y written, not zeroed and then added to: R-MAT
// 1.587 -> 0.870 ms).  Bad K / ld / ki fall through to the ELL checks.
static bool hyb_is_coo(const spmv_dims &d, int32_t K, int64_t ld, int32_t ki, int64_t tail_nnz)
{
    return K == 0 && d.n_rows > 0 && ld >= d.n_rows && ld % 64 == 0 && (ki == 1 || ki == 2) && tail_nnz > 0;
}

extern "C" size_t spmv_hyb_ws_bytes(int64_t tail_nnz)
{
    return spmv_coo_ws_bytes(tail_nnz);
}

// HYB: the ELL part (first K entries of every row)
// writes y, then the row-sorted COO tail ADDS the remaining entries of the
// long rows (staged COO kernel in accumulate mode + the deterministic carry
// pass).  No atomics: bitwise reproducible.
extern "C" int spmv_hyb_run(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col,
                            const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                            const int32_t *tail_col, const double *tail_val, const double *x, double *y,
                            void *ws, size_t ws_bytes)
{
    if (tail_nnz < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run: negative tail size");
    spmv_dims dt = d;
    dt.nnz = tail_nnz;
    if (hyb_is_coo(d, K, ld, ki, tail_nnz))
        return spmv_coo_run(dt, tail_row, tail_col, tail_val, x, y, ws, ws_bytes);
    int rc = spmv_ell_run(d, K, ld, ki, ell_col, ell_val, x, y);
    if (rc != SPMV_SUCCESS || tail_nnz == 0 || d.n_rows == 0)
        return rc;
    if (!ws || ws_bytes < spmv_hyb_ws_bytes(tail_nnz))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run: workspace too small");
    SPMV_GUARD(d);
    const int64_t tiles = (tail_nnz + coo_staged_tile() - 1) / coo_staged_tile();
    double *carry_val = (double *)ws;
    int32_t *carry_row = (int32_t *)(carry_val + tiles);
    rc = launch_coo_staged_acc(dt, tail_row, tail_col, tail_val, x, y, carry_row, carry_val);
    if (rc != SPMV_SUCCESS)
        return rc;
    return launch_carry(tiles, carry_row, carry_val, y, (hipStream_t)d.stream);
}

// HYB with a single-pass tail: `tails` from spmv_coo_tail_build over the
// tail arrays (dims with nnz = tail_nnz); each tile of the tail finishes its
// last row, so no carry pass and no workspace.
extern "C" int spmv_hyb_run_tail(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col,
                                 const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                                 const int32_t *tail_col, const double *tail_val, const double *x, double *y,
                                 const void *tails)
{
    if (tail_nnz < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run_tail: negative tail size");
    spmv_dims dt = d;
    dt.nnz = tail_nnz;
    if (hyb_is_coo(d, K, ld, ki, tail_nnz))
        return spmv_coo_run_tail(dt, tail_row, tail_col, tail_val, x, y, tails);
    int rc = spmv_ell_run(d, K, ld, ki, ell_col, ell_val, x, y);
    if (rc != SPMV_SUCCESS || tail_nnz == 0 || d.n_rows == 0)
        return rc;
    if (!tails)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run_tail: no tail plan");
    SPMV_GUARD(d);
    return launch_coo_staged_acc(dt, tail_row, tail_col, tail_val, x, y, nullptr, nullptr,
                                 (const int32_t *)tails);
}

// HYB with a single-pass tail and the ELL part through the x-window ELL
// kernel (`win`/`xcap` from spmv_ell_xwin_build over ell_col): same bits as
// spmv_hyb_run_tail (the window only moves where x is read from).
extern "C" int spmv_hyb_run_tail_xwin(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col,
                                      const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                                      const int32_t *tail_col, const double *tail_val, const double *x, double *y,
                                      const void *tails, const void *win, int32_t xcap)
{
    if (tail_nnz < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run_tail_xwin: negative tail size");
    spmv_dims dt = d;
    dt.nnz = tail_nnz;
    if (hyb_is_coo(d, K, ld, ki, tail_nnz))
        return spmv_coo_run_tail(dt, tail_row, tail_col, tail_val, x, y, tails);
    int rc = spmv_ell_run_xwin(d, K, ld, ki, ell_col, ell_val, x, y, win, xcap);
    if (rc != SPMV_SUCCESS || tail_nnz == 0 || d.n_rows == 0)
        return rc;
    if (!tails)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run_tail_xwin: no tail plan");
    SPMV_GUARD(d);
    return launch_coo_staged_acc(dt, tail_row, tail_col, tail_val, x, y, nullptr, nullptr,
                                 (const int32_t *)tails);
}

extern "C" size_t spmv_sell_split_ws_bytes(int64_t n_chunks, int32_t C)
{
    return n_chunks > 0 && C > 0 ? (size_t)n_chunks * C * sizeof(double) : 0;
}

// SELL with the wide slices split (plan from spmv_sell_split_plan): the
// main kernel covers the first T slot columns of every slice and writes y;
// the chunks beyond go to sell_split_kernel, then sell_split_fix_kernel
// adds them.  win = NULL runs the plain main kernel, else the x-window one.
extern "C" int spmv_sell_run_split(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                                   const int64_t *slice_ptr, const int32_t *perm, const int32_t *col,
                                   const double *val, const double *x, double *y, const void *win,
                                   int32_t xcap, int32_t T, int64_t n_chunks, const int32_t *chunk_slice,
                                   const int32_t *chunk_k0, void *ws, size_t ws_bytes)
{
    int rc = sell_check_args(d, C, sigma, ki, n_slices, "spmv_sell_run_split");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (T <= 0 || T % ki != 0 || n_chunks < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_split: T must be a positive multiple of ki");
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    if (n_chunks > 0 && (!chunk_slice || !chunk_k0 || !ws || ws_bytes < spmv_sell_split_ws_bytes(n_chunks, C)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_split: chunk plan or workspace missing");
    if (win && (xcap < 0 || xcap > kXwinCapWide))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_split: bad window arguments");
    SPMV_GUARD(d);
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    const int64_t cblocks = (n_chunks * C + kBlock - 1) / kBlock;
    if (blocks > INT32_MAX || cblocks > INT32_MAX || n_chunks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_split: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    const bool nt = stream_nt(kSellStreamNtDefault);
    double *part = (double *)ws;
    if (win && n_chunks > 0 && !sell_small(C, n_slices) && bt == kBlock && !sell_ystage(bt, sigma) &&
        blocks + cblocks <= INT32_MAX && kSellSplitFused) {
        // chunks and main workgroups in one grid (sell_split_fused_kernel)
        auto kern = ki == 2 ? (nt ? sell_split_fused_kernel<2, true, 4, kSellSplitU>
                                  : sell_split_fused_kernel<2, false, 4, kSellSplitU>)
                            : (nt ? sell_split_fused_kernel<1, true, 4, kSellSplitU>
                                  : sell_split_fused_kernel<1, false, 4, kSellSplitU>);
        hipLaunchKernelGGL(kern, dim3((unsigned)(cblocks + blocks)), dim3(kBlock), (size_t)xcap * sizeof(double), st,
                           cblocks, C, n_slices, slice_ptr, perm, col, val, x, y, (const int2 *)win, xcap, T,
                           n_chunks, chunk_slice, chunk_k0, part);
        SPMV_CHECK_LAUNCH("sell_split_fused_kernel");
        hipLaunchKernelGGL(sell_split_fix_kernel, dim3((unsigned)n_chunks), dim3(kSellFixThreads), 0, st, C, n_chunks,
                           chunk_slice, perm, part, y);
        SPMV_CHECK_LAUNCH("sell_split_fix_kernel");
        return SPMV_SUCCESS;
    }
    if (sell_small(C, n_slices)) {
        launch_sell_small_any(ki, nt, n_slices, slice_ptr, perm, col, val, XGlobal{x}, y, (int64_t)T, st, x,
                              (const int2 *)win, xcap);
    } else if (win) {
        auto kern = ki == 2 ? (nt ? sell_xwin_kernel<2, true, 4> : sell_xwin_kernel<2, false, 4>)
                            : (nt ? sell_xwin_kernel<1, true, 4> : sell_xwin_kernel<1, false, 4>);
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bt), (size_t)xcap * sizeof(double), st, C, n_slices,
                           slice_ptr, perm, col, val, x, y, (const int2 *)win, xcap, (int64_t)T,
                           xwin_remap(false) ? 1 : 0, sell_ystage(bt, sigma) ? d.n_rows : (int64_t)0);
    } else {
        auto kern = ki == 2 ? (nt ? sell_kernel<2, true, 4> : sell_kernel<2, false, 4>)
                            : (nt ? sell_kernel<1, true, 4> : sell_kernel<1, false, 4>);
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bt), 0, st, C, n_slices, slice_ptr, perm, col, val,
                           XGlobal{x}, y, 0, (int64_t)T);
    }
    SPMV_CHECK_LAUNCH("sell kernel (split main)");
    if (n_chunks == 0)
        return SPMV_SUCCESS;
    auto sk = ki == 2 ? (nt ? sell_split_kernel<2, true, kSellSplitU> : sell_split_kernel<2, false, kSellSplitU>)
                      : (nt ? sell_split_kernel<1, true, kSellSplitU> : sell_split_kernel<1, false, kSellSplitU>);
    hipLaunchKernelGGL(sk, dim3((unsigned)cblocks), dim3(kBlock), 0, st, C, n_chunks, T, slice_ptr, chunk_slice,
                       chunk_k0, col, val, XGlobal{x}, part);
    SPMV_CHECK_LAUNCH("sell_split_kernel");
    hipLaunchKernelGGL(sell_split_fix_kernel, dim3((unsigned)n_chunks), dim3(kSellFixThreads), 0, st, C, n_chunks,
                       chunk_slice, perm, part, y);
    SPMV_CHECK_LAUNCH("sell_split_fix_kernel");
    return SPMV_SUCCESS;
}

extern "C" size_t spmv_sell_hot_ws_bytes(int64_t n_chunks, int32_t C, int64_t H)
{
    return (size_t)(H > 0 ? H : 0) * sizeof(double) + spmv_sell_split_ws_bytes(n_chunks, C);
}

// SELL over a hot-column table (col_hot / hot from spmv_hot_columns on the
// stored SELL columns), global gathers (no x windows: renumbered ids are
// not x positions), optional split plan (T = INT32_MAX, n_chunks = 0: none).
// Bit-identical to spmv_sell_run_split on the original columns.
extern "C" int spmv_sell_run_hot(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices,
                                 const int64_t *slice_ptr, const int32_t *perm, const int32_t *col_hot,
                                 const double *val, const double *x, double *y, int32_t T, int64_t n_chunks,
                                 const int32_t *chunk_slice, const int32_t *chunk_k0, int64_t H,
                                 const int32_t *hot, void *ws, size_t ws_bytes)
{
    int rc = sell_check_args(d, C, sigma, ki, n_slices, "spmv_sell_run_hot");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (T <= 0 || T % ki != 0 || n_chunks < 0 || H < 0 || d.n_cols + H > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_hot: bad T / H");
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    if ((n_chunks > 0 && (!chunk_slice || !chunk_k0)) || (H > 0 && !hot) || !ws ||
        ws_bytes < spmv_sell_hot_ws_bytes(n_chunks, C, H))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_hot: plan, hot list or workspace missing");
    SPMV_GUARD(d);
    int bt;
    int64_t blocks;
    sell_geometry(C, sigma, n_slices, &bt, &blocks);
    const int64_t cblocks = (n_chunks * C + kBlock - 1) / kBlock;
    if (blocks > INT32_MAX || cblocks > INT32_MAX || n_chunks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run_hot: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    double *xh = (double *)ws;
    double *part = xh + H;
    if (H > 0)
        hipLaunchKernelGGL(sell_hot_gather_kernel, dim3((unsigned)((H + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           H, hot, x, xh);
    const XHot xs{x, xh, (int32_t)d.n_cols};
    const bool nt = stream_nt(kSellStreamNtDefault);
    if (sell_small(C, n_slices)) {
        launch_sell_small_any(ki, nt, n_slices, slice_ptr, perm, col_hot, val, xs, y, (int64_t)T, st);
    } else {
        auto kern = ki == 2 ? (nt ? sell_kernel<2, true, 4, XHot> : sell_kernel<2, false, 4, XHot>)
                            : (nt ? sell_kernel<1, true, 4, XHot> : sell_kernel<1, false, 4, XHot>);
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bt), 0, st, C, n_slices, slice_ptr, perm, col_hot, val,
                           xs, y, 0, (int64_t)T);
    }
    SPMV_CHECK_LAUNCH("sell kernel (hot columns)");
    if (n_chunks == 0)
        return SPMV_SUCCESS;
    auto sk = ki == 2 ? (nt ? sell_split_kernel<2, true, kSellSplitU, XHot> : sell_split_kernel<2, false, kSellSplitU, XHot>)
                      : (nt ? sell_split_kernel<1, true, kSellSplitU, XHot> : sell_split_kernel<1, false, kSellSplitU, XHot>);
    hipLaunchKernelGGL(sk, dim3((unsigned)cblocks), dim3(kBlock), 0, st, C, n_chunks, T, slice_ptr, chunk_slice,
                       chunk_k0, col_hot, val, xs, part);
    SPMV_CHECK_LAUNCH("sell_split_kernel (hot columns)");
    hipLaunchKernelGGL(sell_split_fix_kernel, dim3((unsigned)n_chunks), dim3(kSellFixThreads), 0, st, C, n_chunks,
                       chunk_slice, perm, part, y);
    SPMV_CHECK_LAUNCH("sell_split_fix_kernel");
    return SPMV_SUCCESS;
}

extern "C" size_t spmv_hyb_hot_ws_bytes(int64_t tail_nnz, int64_t H)
{
    return (size_t)(H > 0 ? H : 0) * sizeof(double) + spmv_hyb_ws_bytes(tail_nnz);
}

// HYB over a hot-column table (ell_col_hot / tail_col_hot renumbered by
// spmv_hot_columns over both column arrays): the ELL part and the COO tail
// read the hottest x values from xh.  Bit-identical to spmv_hyb_run on the
// original columns.
extern "C" int spmv_hyb_run_hot(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *ell_col_hot,
                                const double *ell_val, int64_t tail_nnz, const int32_t *tail_row,
                                const int32_t *tail_col_hot, const double *tail_val, const double *x, double *y,
                                int64_t H, const int32_t *hot, void *ws, size_t ws_bytes)
{
    if (H < 0 || tail_nnz < 0 || d.n_cols + H > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run_hot: bad sizes");
    if (H == 0)
        return spmv_hyb_run(d, K, ld, ki, ell_col_hot, ell_val, tail_nnz, tail_row, tail_col_hot, tail_val, x, y,
                            ws, ws_bytes);
    if (hyb_is_coo(d, K, ld, ki, tail_nnz)) {  // as spmv_hyb_run: the COO over the same table
        spmv_dims dt = d;
        dt.nnz = tail_nnz;
        return spmv_coo_run_hot(dt, tail_row, tail_col_hot, tail_val, x, y, H, hot, ws, ws_bytes);
    }
    if (d.n_rows < 0 || K < 0 || ld < d.n_rows || ld % 64 != 0 || (ki != 1 && ki != 2) || K % ki != 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run_hot: bad K / ld / ki");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (!hot || !ws || ws_bytes < spmv_hyb_hot_ws_bytes(tail_nnz, H))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_hyb_run_hot: hot list or workspace missing");
    SPMV_GUARD(d);
    const hipStream_t st = (hipStream_t)d.stream;
    double *xh = (double *)ws;
    hipLaunchKernelGGL(sell_hot_gather_kernel, dim3((unsigned)((H + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, H,
                       hot, x, xh);
    const XHot xs{x, xh, (int32_t)d.n_cols};
    const int64_t blocks = (d.n_rows + kBlock - 1) / kBlock;
    const bool nt = stream_nt(kSellStreamNtDefault);
    auto kern = ki == 2 ? (nt ? ell_kernel<2, true, 4, XHot> : ell_kernel<2, false, 4, XHot>)
                        : (nt ? ell_kernel<1, true, 4, XHot> : ell_kernel<1, false, 4, XHot>);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), 0, st, d.n_rows, K, ld, ell_col_hot, ell_val, xs,
                       y, 0);
    SPMV_CHECK_LAUNCH("ell_kernel (hot columns)");
    if (tail_nnz == 0)
        return SPMV_SUCCESS;
    const int64_t tiles = (tail_nnz + coo_staged_tile() - 1) / coo_staged_tile();
    double *carry_val = xh + H;
    int32_t *carry_row = (int32_t *)(carry_val + tiles);
    spmv_dims dt = d;
    dt.nnz = tail_nnz;
    int rc = launch_coo_staged_acc_hot(dt, tail_row, tail_col_hot, tail_val, x, y, carry_row, carry_val, xs);
    if (rc != SPMV_SUCCESS)
        return rc;
    return launch_carry(tiles, carry_row, carry_val, y, st);
}
