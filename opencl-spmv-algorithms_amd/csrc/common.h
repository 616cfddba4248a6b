// common.h — shared device helpers and launch plumbing for the gfx950
// SpMV kernels (see include/spmv.h for the C-ABI they implement).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spmv.h"
#include "spmv_ext.h"

namespace spmv {

constexpr int kWave = 64;    // CDNA wavefront width
constexpr int kBlock = 256;  // 4 waves per workgroup for every kernel

// ---------------------------------------------------------------- errors
int fail(int rc, const char *where, hipError_t e);
int fail_msg(int rc, const char *msg);

// Sets the device for the duration of one C-ABI call and restores the
// caller's device afterwards.
class DeviceGuard {
  public:
    explicit DeviceGuard(int dev);
    ~DeviceGuard();
    int rc() const { return rc_; }

  private:
    int prev_ = -1;
    int rc_ = SPMV_SUCCESS;
};

// The library's A/B switches (spmv_set_option, spmv_ext.h; initial values
// from SPMV_XCD_REMAP / SPMV_XWIN_REMAP / SPMV_STREAM_NT, read once at load);
// each changes placement or cache policy, never a result bit
// (tests/test_gpu_parity.py checks that):
// XCD-contiguous blockIdx remap of the global-gather kernels (default off).
bool xcd_remap_enabled();
// XCD-contiguous window placement of the x-window kernels; `dflt` = each
// kernel's measured best.
bool xwin_remap(bool dflt);
// CSR x-window kernel: the first chunk prefetched in the prologue (MODE 4)
bool csr_prefetch(bool dflt);
// small-matrix SELL geometry (sell.hip): C = 64 and fewer than 14 slices per CU
bool sell_small(int32_t C, int64_t n_slices);

// LDS-staged CMRS / COO launchers (staged.hip)
// win != nullptr: the x-window kernels (win/xcap from *_xwin_build)
int launch_cmrs_staged(const spmv_dims &d, int32_t h, int64_t n_strips,
                       const int64_t *strip_ptr, const uint8_t *rin, const int32_t *col,
                       const double *val, const double *x, double *y, const int2 *win = nullptr,
                       int32_t xcap = 0);
void cmrs_geometry(const spmv_dims &d, int32_t h, int64_t n_strips, int *L, int *G, int64_t *blocks);
int launch_coo_staged(const spmv_dims &d, const int32_t *row, const int32_t *col,
                      const double *val, const double *x, double *y, int32_t *carry_row,
                      double *carry_val, const int2 *win = nullptr, int32_t xcap = 0,
                      const int32_t *tails = nullptr);
// single-pass COO: the tail plan (tails[tile], staged.hip); returns the
// largest tail, or -1 on a launch / copy error
int64_t coo_tail_build(const spmv_dims &d, const int32_t *row, int32_t *tails);
int64_t coo_tail_cap();
// LDS entries of x a staged COO tile / CMRS strip run may stage (16 KiB)
constexpr int32_t kStagedXwinCap = 2048;
int64_t coo_staged_tile();
// tile of the hot-column COO (spmv_coo_run_hot) for this matrix
int64_t coo_hot_tile(int64_t n_rows, int64_t nnz);
// accumulate mode: y[r] += entries of the rows present (HYB tail)
int launch_coo_staged_acc(const spmv_dims &d, const int32_t *row, const int32_t *col,
                          const double *val, const double *x, double *y, int32_t *carry_row,
                          double *carry_val, const int32_t *tails = nullptr);
int launch_csr_tiled(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                     const double *val, const double *x, double *y, int32_t *own_lo,
                     int32_t *carry_row, double *carry_val);
// entries per tile of the tiled CSR for this matrix, and the smallest it picks
int64_t csr_tiled_tile(int64_t n_rows, int64_t nnz);
int64_t csr_tiled_tile_min();
template <typename V>  // double or float values (instantiated in staged.hip)
int launch_csr_tiled_hot(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                         const V *val, const double *x, double *y, int64_t H, const int32_t *hot,
                         double *xh, const int32_t *own_lo_plan, int32_t *own_lo, int32_t *carry_row,
                         double *carry_val, const int32_t *big = nullptr, int64_t big_len = 0);
int launch_cmrs_tiled(const spmv_dims &d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                      const uint8_t *rin, const int32_t *col, const double *val, const double *x,
                      double *y, int32_t *own_lo, int32_t *carry_row, double *carry_val, int64_t H = 0,
                      const int32_t *hot = nullptr, double *xh = nullptr, bool own_lo_ready = false);
int cmrs_tiled_planned(const spmv_dims &d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                       const uint8_t *rin, const int32_t *col, const double *val, const double *x, double *y,
                       int64_t H, const int32_t *hot, void *ws, bool fill);
__global__ void csr_tile_rows_kernel(int64_t n_rows, int64_t nnz, int64_t tiles, int64_t ch,
                                     const int64_t *__restrict__ ptr, int32_t *__restrict__ own_lo);
struct XHot;
int launch_coo_staged_acc_hot(const spmv_dims &d, const int32_t *row, const int32_t *col,
                              const double *val, const double *x, double *y, int32_t *carry_row,
                              double *carry_val, const XHot xs);
int launch_coo_staged_hot(const spmv_dims &d, const int32_t *row, const int32_t *col, const double *val,
                          const double *x, double *y, int32_t *carry_row, double *carry_val, int64_t H,
                          const int32_t *hot, double *xh);
int64_t cmrs_tiled_tile(int64_t n_rows, int64_t nnz);
int64_t cmrs_tiled_tile_min();
// the deterministic carry pass shared by COO and tiled CSR (coo.hip)
int launch_carry(int64_t tiles, const int32_t *carry_row, const double *carry_val, double *y,
                 hipStream_t stream);

// ------------------------------------------------------- device helpers
// Bijective blockIdx remap: blocks b and b+8 are dealt to the same XCD
// (MI355X_MICROARCH.md §Workgroup dispatch), so give each such group a
// CONTIGUOUS range of logical blocks.  Neighbouring rows/slices then read
// neighbouring x entries through one XCD's L2.  Placement only changes
// speed, never results.
__device__ __forceinline__ int64_t xcd_block(int remap)
{
    const int64_t b = blockIdx.x;
    if (!remap)
        return b;
    const int64_t nb = gridDim.x;
    const int64_t q = nb >> 3, r = nb & 7;
    const int64_t xcd = b & 7, idx = b >> 3;
    return xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
}

// Streamed-once loads of the matrix arrays.  NT = true issues them
// non-temporal (`global_load … nt`), so the values and columns, each read
// exactly once, do not displace x from L2 / the Infinity Cache.
typedef double v2f64 __attribute__((ext_vector_type(2)));
typedef int32_t v2i32 __attribute__((ext_vector_type(2)));

template <bool NT, typename T>
__device__ __forceinline__ T stream_load(const T *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <bool NT>
__device__ __forceinline__ double2 stream_load2(const double *p)
{
    const v2f64 v = stream_load<NT>(reinterpret_cast<const v2f64 *>(p));
    return double2{v.x, v.y};
}

template <bool NT>
__device__ __forceinline__ int2 stream_load2(const int32_t *p)
{
    const v2i32 v = stream_load<NT>(reinterpret_cast<const v2i32 *>(p));
    return int2{v.x, v.y};
}

// Value loads of the staged kernels: fp64 values, or fp32 values (CSR-f32,
// SURVEY.md §8f row 4) widened to fp64 before the product.
typedef float v2f32 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ double2 vpair(const double *p)
{
    return stream_load2<NT>(p);
}

template <bool NT>
__device__ __forceinline__ double2 vpair(const float *p)
{
    const v2f32 v = stream_load<NT>(reinterpret_cast<const v2f32 *>(p));
    return double2{(double)v.x, (double)v.y};
}

template <bool NT, typename V>
__device__ __forceinline__ double vone(const V *p)
{
    return (double)stream_load<NT>(p);
}

// y stores of the SpMV kernels: relaxed agent-scope atomic stores, i.e.
// `global_store … sc1`, written through the XCD's L2 instead of sitting
// there dirty until the matrix stream evicts them into HBM mid-kernel.  The
// 16 MB of y of the cant batch cost the staged stream 0.2254 -> 0.2547 ms as
// plain stores and 0.2428 ms as sc1 stores (csr_stream_probe_kernel P3/P4/PA,
// profiles/round2/probe_ystore.log); the same stores into 64 KiB cost nothing,
// so it is y's HBM write traffic, not the store instructions.
__device__ __forceinline__ void store_y(double *p, double v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Load-policy switch for the streamed arrays (SPMV_OPT_STREAM_NT), otherwise
// `dflt` (each kernel's measured best).
bool stream_nt(bool dflt);

// Where x[c] comes from: global memory (XGlobal) or the workgroup's
// window x[lo..hi] staged in LDS (XWindow: the x-window kernels).
struct XGlobal {
    const double *__restrict__ x;
    __device__ __forceinline__ double operator()(int32_t c) const { return x[c]; }
};

struct XWindow {
    const double *s;  // LDS
    int32_t lo;
    __device__ __forceinline__ double operator()(int32_t c) const { return s[c - lo]; }
};

// Copies x[lo .. lo+span) into LDS (s_x[0 .. span)) with U loads in flight
// per thread: all U loads are issued before the first LDS store (a plain
// strided loop waits out one L2/HBM round trip per T entries).  Lanes past
// the window load its last entry again (same line, never stored).
template <int T = kBlock, int U = 8>
__device__ __forceinline__ void copy_window(double *s_x, const double *__restrict__ x, int32_t lo, int32_t span)
{
    for (int32_t b = 0; b < span; b += U * T) {
        double v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t i = b + (int32_t)threadIdx.x + k * T;
            v[k] = x[lo + (i < span ? i : span - 1)];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t i = b + (int32_t)threadIdx.x + k * T;
            if (i < span)
                s_x[i] = v[k];
        }
    }
}

// copy_window for span <= U·T in ONE straight-line pass (no loop): loads the
// caller issued before it stay in flight behind the window's (a loop header
// merges states and made the compiler wait for them first)
template <int T = kBlock, int U = 8>
__device__ __forceinline__ void copy_window_1pass(double *s_x, const double *__restrict__ x, int32_t lo,
                                                  int32_t span)
{
    double v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int32_t i = (int32_t)threadIdx.x + k * T;
        v[k] = x[lo + (i < span ? i : span - 1)];
    }
    // unconditional stores (lanes past the window write the window's last
    // entry again, the value they loaded): a store under `if (i < span)` let
    // the compiler sink that load into the branch, behind the others
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int32_t i = (int32_t)threadIdx.x + k * T;
        s_x[i < span ? i : span - 1] = v[k];
    }
}

// Hot-column CSR (spmv_csr_run_tiled_hot): ids >= M name the compact table
// xh of the most frequent columns, gathered from x at the start of the run.
struct XHot {
    const double *__restrict__ x;
    const double *__restrict__ xh;
    int32_t M;
    __device__ __forceinline__ double operator()(int32_t c) const { return c >= M ? xh[c - M] : x[c]; }
};

// [min, max] of col[e0..e1) over one 256-thread workgroup ({0, -1} when
// empty); the result is valid in thread 0.  Build-time pass of the
// x-window kernels.
__device__ __forceinline__ int2 block_minmax(int lo, int hi);

__device__ __forceinline__ int2 block_col_range(const int32_t *__restrict__ col, int64_t e0, int64_t e1)
{
    int lo = INT32_MAX, hi = INT32_MIN;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += kBlock) {
        const int c = col[e];
        lo = c < lo ? c : lo;
        hi = c > hi ? c : hi;
    }
    return block_minmax(lo, hi);
}

// workgroup-wide [min lo, max hi] of per-thread partials (valid in thread 0)
__device__ __forceinline__ int2 block_minmax(int lo, int hi)
{
    __shared__ int s_lo[kBlock / kWave], s_hi[kBlock / kWave];
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        const int l2 = __shfl_xor(lo, off), h2 = __shfl_xor(hi, off);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    if (threadIdx.x % kWave == 0) {
        s_lo[threadIdx.x / kWave] = lo;
        s_hi[threadIdx.x / kWave] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWave; ++w) {
            lo = s_lo[w] < lo ? s_lo[w] : lo;
            hi = s_hi[w] > hi ? s_hi[w] : hi;
        }
    }
    return lo <= hi ? int2{lo, hi} : int2{0, -1};
}

// One lane's share of a row's products staged in LDS: entries [lo, hi)
// of the chunk (prod 16-byte aligned) (chunk-relative, < 2^31).  The products are read as
// 16-byte pairs (half the LDS instructions of single reads): lane k takes
// pairs plo+k, plo+k+L, ... into two partial sums (a0 the first product of
// each pair, a1 the second), four pairs read per step before the first add;
// an odd first entry goes to lane 0's a0, an odd last entry to lane L-1's a1.
template <int L>
__device__ __forceinline__ double slice_sum(const double *prod, int64_t lo64, int64_t hi64, int lane)
{
    const int lo = (int)lo64, hi = (int)hi64;
    double a0 = 0.0, a1 = 0.0;
    if (lo >= hi)
        return 0.0;
    if ((lo & 1) && lane == 0)
        a0 = prod[lo];
    if ((hi & 1) && lane == L - 1)
        a1 = prod[hi - 1];
    const double2 *p2 = reinterpret_cast<const double2 *>(prod);
    const int pe = hi >> 1;  // whole pairs [(lo+1)/2, hi/2)
    int k = ((lo + 1) >> 1) + lane;
    for (; k + 3 * L < pe; k += 4 * L) {
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = p2[k + u * L];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a0 += v[u].x;
            a1 += v[u].y;
        }
    }
    for (; k < pe; k += L) {
        const double2 v = p2[k];
        a0 += v.x;
        a1 += v.y;
    }
    return a0 + a1;
}

// v from lane (lane ^ 1) or (lane ^ 2) of its quad by a DPP quad_perm move
// (a VALU operand modifier) instead of __shfl_xor's ds_bpermute through the
// LDS unit; whole quads are active together wherever group_sum runs.
template <int CTRL>
__device__ __forceinline__ double quad_xor(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Butterfly sum over W-lane groups: every lane gets the group's sum, added
// in the same order as the xor butterfly (the last two steps by DPP: same
// bits as __shfl_xor).
template <int W>
__device__ __forceinline__ double group_sum(double v)
{
#pragma unroll
    for (int off = W / 2; off > 2; off >>= 1)
        v += __shfl_xor(v, off, W);
    if constexpr (W >= 4)
        v += quad_xor<0x4E>(v);  // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (W >= 2)
        v += quad_xor<0xB1>(v);  // quad_perm [1,0,3,2]: lane ^ 1
    return v;
}

}  // namespace spmv

#define SPMV_CHECK_LAUNCH(where)                                              \
    do {                                                                      \
        hipError_t e_ = hipGetLastError();                                    \
        if (e_ != hipSuccess)                                                 \
            return ::spmv::fail(SPMV_PROGRAM_ERROR, where, e_);              \
    } while (0)

#define SPMV_GUARD(dims)                                                      \
    ::spmv::DeviceGuard guard_((dims).device);                                \
    if (guard_.rc() != SPMV_SUCCESS)                                          \
        return guard_.rc()
