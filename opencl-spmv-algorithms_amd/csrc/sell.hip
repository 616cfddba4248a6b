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
#include "common.h"

namespace spmv {

// Non-temporal matrix loads: SELL-64-1024 0.2955 vs 0.3130 ms and ELL
// 0.3343 vs 0.3429 ms on the 32-copy cant-like batch, one process,
// interleaved (profiles/round1/sweeps.md).  SPMV_STREAM_NT overrides.
constexpr bool kSellStreamNtDefault = true;

// slot groups in flight per lane: SPMV_SLOT_UNROLL = 4 (default) or 8
static int slot_unroll()
{
    const char *s = getenv("SPMV_SLOT_UNROLL");
    return (s && s[0] == '8') ? 8 : 4;
}

template <int KI, bool NT>
struct Step;

template <bool NT>
struct Step<1, NT> {
    static __device__ __forceinline__ double fma(const double *vp,
                                                 const int32_t *cp,
                                                 const double *__restrict__ x,
                                                 double acc)
    {
        return acc + stream_load<NT>(vp) * x[stream_load<NT>(cp)];
    }
};

template <bool NT>
struct Step<2, NT> {
    static __device__ __forceinline__ double fma(const double *vp,
                                                 const int32_t *cp,
                                                 const double *__restrict__ x,
                                                 double acc)
    {
        const double2 v = stream_load2<NT>(vp);
        const int2 c = stream_load2<NT>(cp);
        return acc + v.x * x[c.x] + v.y * x[c.y];
    }
};

// Slot-per-lane loop over `w` slots (a multiple of KI) with stride
// `step` elements between consecutive KI-groups; U groups in flight
// (U independent accumulators, combined as a pairwise tree).
template <int KI, bool NT, int U>
__device__ __forceinline__ double slot_dot(const double *__restrict__ vp,
                                           const int32_t *__restrict__ cp,
                                           int64_t w, int64_t step,
                                           const double *__restrict__ x)
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
            a[u] = Step<KI, NT>::fma(vp + (g + u) * step, cp + (g + u) * step, x, a[u]);
    }
    for (; g < groups; ++g)
        a[0] = Step<KI, NT>::fma(vp + g * step, cp + g * step, x, a[0]);
#pragma unroll
    for (int h = U / 2; h > 0; h /= 2) {
#pragma unroll
        for (int u = 0; u < h; ++u)
            a[u] += a[u + h];
    }
    return a[0];
}

// One workgroup covers one sigma window (up to 1024 slots): every y[perm]
// store of a window then comes from ONE CU, so its L2 merges the window's
// scattered 8-byte stores into whole lines.  With 256-slot workgroups a
// 1024-row window was written from four XCDs and each partially written
// line left the chip up to four times (WRITE_SIZE 2.9x the y bytes,
// profiles/traffic.json), which cost ~10 % of the kernel.
template <int KI, bool NT, int U>
__global__ __launch_bounds__(1024) void sell_kernel(
    int32_t C, int64_t n_slices, const int64_t *__restrict__ slice_ptr,
    const int32_t *__restrict__ perm, const int32_t *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x,
    double *__restrict__ y, int remap)
{
    const int64_t slot = xcd_block(remap) * (int64_t)blockDim.x + threadIdx.x;
    const int64_t s = slot / C;
    if (s >= n_slices)
        return;
    const int64_t r = slot - s * C;
    const int64_t base = slice_ptr[s];
    const int64_t w = (slice_ptr[s + 1] - base) / C;
    const int64_t off = base + r * KI;
    const double sum = slot_dot<KI, NT, U>(val + off, col + off, w, (int64_t)C * KI, x);
    const int32_t row = perm[slot];
    if (row >= 0)
        y[row] = sum;
}

template <int KI, bool NT, int U>
__global__ __launch_bounds__(kBlock) void ell_kernel(
    int64_t n_rows, int32_t K, int64_t ld, const int32_t *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x,
    double *__restrict__ y, int remap)
{
    const int64_t i = xcd_block(remap) * kBlock + threadIdx.x;
    if (i >= n_rows)
        return;
    const int64_t off = i * KI;
    y[i] = slot_dot<KI, NT, U>(val + off, col + off, K, ld * KI, x);
}

}  // namespace spmv

using namespace spmv;

extern "C" int spmv_sell_run(spmv_dims d, int32_t C, int32_t sigma, int32_t ki,
                             int64_t n_slices, const int64_t *slice_ptr,
                             const int32_t *perm, const int32_t *col,
                             const double *val, const double *x, double *y)
{
    if (d.n_rows < 0 || C <= 0 || C > 1024 || n_slices < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run: bad C / sizes");
    if (ki != 1 && ki != 2)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run: ki must be 1 or 2");
    if (sigma < 1 || (sigma > 1 && sigma % C != 0))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run: sigma must be 1 or a multiple of C");
    if (n_slices * C < d.n_rows)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run: n_slices*C < n_rows");
    if (d.n_rows == 0 || n_slices == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    const int64_t slots = n_slices * C;
    // workgroup = one sigma window when it fits (256..1024 slots, a
    // multiple of the wave), else 256 slots
    static const int force256 = [] {
        const char *s = getenv("SPMV_SELL_BT");  // tuning knob: "256" forces 256-slot groups
        return s && atoi(s) == 256;
    }();
    // A small matrix (fewer than ~2 windows per CU) needs the parallelism of
    // 256-slot groups more than merged stores: one cant-like copy has only
    // 61 windows of 1024 rows for 256 CUs.
    const int64_t windows = sigma > 1 ? (slots + sigma - 1) / sigma : 0;
    const bool wide = !force256 && windows >= 512 && sigma >= kBlock && sigma <= 1024 &&
                      sigma % kWave == 0;
    const int bt = wide ? sigma : kBlock;
    const int64_t blocks = (slots + bt - 1) / bt;
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_sell_run: grid too large");
    const int remap = xcd_remap_enabled() ? 1 : 0;
    const bool nt = stream_nt(kSellStreamNtDefault);
    const bool u8 = slot_unroll() == 8;
    auto kern = ki == 2 ? (nt ? (u8 ? sell_kernel<2, true, 8> : sell_kernel<2, true, 4>)
                              : (u8 ? sell_kernel<2, false, 8> : sell_kernel<2, false, 4>))
                        : (nt ? (u8 ? sell_kernel<1, true, 8> : sell_kernel<1, true, 4>)
                              : (u8 ? sell_kernel<1, false, 8> : sell_kernel<1, false, 4>));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bt), 0, (hipStream_t)d.stream, C,
                       n_slices, slice_ptr, perm, col, val, x, y, remap);
    SPMV_CHECK_LAUNCH("sell_kernel");
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
    const bool u8 = slot_unroll() == 8;
    auto kern = ki == 2 ? (nt ? (u8 ? ell_kernel<2, true, 8> : ell_kernel<2, true, 4>)
                              : (u8 ? ell_kernel<2, false, 8> : ell_kernel<2, false, 4>))
                        : (nt ? (u8 ? ell_kernel<1, true, 8> : ell_kernel<1, true, 4>)
                              : (u8 ? ell_kernel<1, false, 8> : ell_kernel<1, false, 4>));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)d.stream,
                       d.n_rows, K, ld, col, val, x, y, remap);
    SPMV_CHECK_LAUNCH("ell_kernel");
    return SPMV_SUCCESS;
}
