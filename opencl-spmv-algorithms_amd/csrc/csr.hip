// csr.hip — CSR-vector SpMV for gfx950.
//
// Replaces the reference's scalar CSR kernel (reference kernels/Csr.cl:1-17:
// one work-item per row, 8192 work-items total, reference csr.c:47-48).
// Here a group of L lanes (L | 64) owns one row:
//   * the workgroup's window of row_ptr (256/L + 1 offsets) is staged in
//     LDS once, so each row's bounds cost one LDS read, not two global ones;
//   * the L lanes stride the row's entries together (contiguous, coalesced
//     8-byte value loads and 4-byte column loads), unrolled 4x so every
//     lane keeps 4 value/column/x loads in flight;
//   * the L partial sums are combined with cross-lane shuffles
//     (__shfl_xor butterflies inside the L-lane group).
// Bytes per row: 12·len + 8 (row_ptr) + 8 (y), plus x gathers.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace spmv {

// One L-lane group's row [beg, end) with 16-byte pair loads: the lane
// reads the aligned pair (p, p+1); entries of the pair outside [beg, end)
// are zeroed by value (their column is a valid neighbour column, so the
// gather stays in bounds).  The last pair of the row is loaded as a
// scalar when p+1 == end, so nothing past val[nnz-1] is ever read.
template <int L, typename XS>
__device__ __forceinline__ double row_dot_pairs(int64_t beg, int64_t end, int lane,
                                                const int32_t *__restrict__ col,
                                                const double *__restrict__ val, const XS &xs)
{
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int64_t p = (beg & ~(int64_t)1) + 2 * lane;
    for (; p + 1 + 2 * L < end; p += 4 * L) {
        const double2 va = *reinterpret_cast<const double2 *>(val + p);
        const int2 ca = *reinterpret_cast<const int2 *>(col + p);
        const double2 vb = *reinterpret_cast<const double2 *>(val + p + 2 * L);
        const int2 cb = *reinterpret_cast<const int2 *>(col + p + 2 * L);
        s0 += (p >= beg ? va.x : 0.0) * xs(ca.x);
        s1 += va.y * xs(ca.y);
        s2 += vb.x * xs(cb.x);
        s3 += vb.y * xs(cb.y);
    }
    for (; p < end; p += 2 * L) {
        if (p + 1 < end) {
            const double2 va = *reinterpret_cast<const double2 *>(val + p);
            const int2 ca = *reinterpret_cast<const int2 *>(col + p);
            s0 += (p >= beg ? va.x : 0.0) * xs(ca.x);
            s1 += va.y * xs(ca.y);
        } else if (p >= beg) {
            s0 += val[p] * xs(col[p]);
        }
    }
    return group_sum<L>((s0 + s1) + (s2 + s3));
}

template <int L, bool PAIR>
__global__ __launch_bounds__(kBlock) void csr_vector_kernel(
    int64_t n_rows, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, int remap)
{
    constexpr int RPB = kBlock / L;  // rows per workgroup
    __shared__ int64_t s_ptr[RPB + 1];

    const int64_t row0 = xcd_block(remap) * RPB;
    if (threadIdx.x <= RPB) {
        int64_t r = row0 + threadIdx.x;
        s_ptr[threadIdx.x] = row_ptr[r < n_rows ? r : n_rows];
    }
    __syncthreads();

    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    const int64_t row = row0 + g;
    const int64_t beg = s_ptr[g], end = s_ptr[g + 1];  // empty past n_rows

    if constexpr (PAIR) {
        const double sum = row_dot_pairs<L>(beg, end, lane, col, val, XGlobal{x});
        if (lane == 0 && row < n_rows)
            store_y(y + (row), sum);
        return;
    }
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int64_t j = beg + lane;
    for (; j + 3 * L < end; j += 4 * L) {
        const int32_t c0 = col[j], c1 = col[j + L], c2 = col[j + 2 * L],
                      c3 = col[j + 3 * L];
        const double v0 = val[j], v1 = val[j + L], v2 = val[j + 2 * L],
                     v3 = val[j + 3 * L];
        s0 += v0 * x[c0];
        s1 += v1 * x[c1];
        s2 += v2 * x[c2];
        s3 += v3 * x[c3];
    }
    for (; j < end; j += L)
        s0 += val[j] * x[col[j]];
    double sum = group_sum<L>((s0 + s1) + (s2 + s3));
    if (lane == 0 && row < n_rows)
        store_y(y + (row), sum);
}

// CSR-vector (direct: every L-lane group walks its own row) with the
// workgroup's x window staged in LDS first; windows from
// spmv_csr_xwin_build (one per gpw workgroups of 256/L rows).
template <int L>
__global__ __launch_bounds__(kBlock) void csr_vector_xwin_kernel(
    int64_t n_rows, int64_t gpw, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap)
{
    constexpr int RPB = kBlock / L;
    extern __shared__ double s_x[];
    __shared__ int64_t s_ptr[RPB + 1];
    const int64_t row0 = (int64_t)blockIdx.x * RPB;
    if (threadIdx.x <= RPB) {
        const int64_t r = row0 + threadIdx.x;
        s_ptr[threadIdx.x] = row_ptr[r < n_rows ? r : n_rows];
    }
    const int2 wnd = win[blockIdx.x / gpw];  // the window covering this workgroup's rows
    const int32_t span = wnd.y - wnd.x + 1;
    const bool staged = span > 0 && span <= xcap;  // uniform per workgroup
    if (staged)
        for (int32_t i = threadIdx.x; i < span; i += kBlock)
            s_x[i] = x[wnd.x + i];
    __syncthreads();
    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    const int64_t row = row0 + g;
    const int64_t beg = s_ptr[g], end = s_ptr[g + 1];
    const double sum = staged ? row_dot_pairs<L>(beg, end, lane, col, val, XWindow{s_x, wnd.x})
                              : row_dot_pairs<L>(beg, end, lane, col, val, XGlobal{x});
    if (lane == 0 && row < n_rows)
        store_y(y + (row), sum);
}

// CSR-vector with the entry stream staged through LDS ("staged" variant).
// The workgroup's rows occupy one contiguous range of entries
// [ptr[row0], ptr[row0+RPB]).  Instead of every L-lane group walking its
// own row (ragged trip counts, loads that straddle row ends), all 256
// lanes stream that range like a copy kernel — aligned 16-byte value
// pairs + 8-byte column pairs, kStageRounds pairs per lane in flight —
// and store the products a·x in LDS.  After one barrier each L-lane group
// sums its row's slice of the products (conflict-free ds_read_b64, stride
// 1 across lanes) and reduces with the same shuffle butterfly.  Ranges
// longer than the LDS chunk are processed in chunks; a row's partial sum
// stays in its lanes' registers across chunks.
constexpr int kStageRoundsDefault = 3;  // pairs per lane per chunk: 1536 products, 12 KiB
// (round 1, persistent kernel: R = 3 0.3008 ms, R = 4 0.3013, R = 5 and
// R = 8 slower; round 2, x-window kernel MODE 3: R = 3 0.2591-0.2607 ms,
// R = 4 0.2639-0.2642 — one default for every staged CSR kernel keeps
// their chunk boundaries, hence their bits, identical)
// Chunks of the staged kernels start on a kChunkAlign-entry boundary at or
// before the row group's first entry (up to 31 entries of the previous group
// are loaded and never summed), so a wave's 64 value pairs (1 KiB) and column
// pairs (512 B) cover whole 128-B lines, 8 + 4 instead of 9 + 5: the
// CSR-shaped stream probe reads 6.81 TB/s from aligned tiles and 6.47 TB/s
// from tiles that start on any even entry (tools/bw_probe,
// csr_prologue_dep1[_unaligned]).  Every staged CSR kernel cuts the same
// chunks, so their sums stay bit-identical to each other.
constexpr int64_t kChunkAlign = 32;
__host__ __device__ __forceinline__ int64_t chunk_start(int64_t e) { return e & ~(kChunkAlign - 1); }
constexpr bool kCsrStreamNtDefault = false;  // SPMV_STREAM_NT overrides
// the x-window kernel (x gathers from LDS) streams faster non-temporal:
// 0.2991 vs 0.3077 ms on the cant-like batch
constexpr bool kCsrXwinNtDefault = true;
// Stage load schedule (SPMV_CSR_BATCH overrides): 0 = per-round guarded
// loads measured 0.313 ms against 0.350 ms for loads + gathers batched
// (mode 2: 76 VGPRs, 6 waves/SIMD) on the cant-like batch.
constexpr int kCsrBatchDefault = 0;

// One row group (RPB = 256/L rows) of the staged scheme; s_ptr holds the
// group's RPB+1 row offsets.  Ends with a barrier, so the caller may
// overwrite s_ptr / s_prod afterwards.
// Column sources of the staged kernels: where the column of entry p comes
// from.  Col32 = the CSR int32 array.  Col16 = compressed 16-bit indices
// (SURVEY.md §8f row 4): entry p's column is base[p/64] + off[p] when the
// 64-entry block's columns span < 65536, else the block is stored whole in
// esc (base = -1 - slot).  10.06 instead of 12 bytes per entry; the
// columns, hence products and sums, are exactly CSR's.
// Two-phase form for the pipelined kernels: raw(p) only issues loads (no
// load depends on another), decode(raw, p) turns them into the column pair
// (CSR16's escaped blocks load their int32 columns there, a second round
// trip for those blocks only).
template <bool NT>
struct Col32 {
    const int32_t *__restrict__ col;
    using Raw = int2;
    __device__ __forceinline__ int2 pair(int64_t p) const { return stream_load2<NT>(col + p); }
    __device__ __forceinline__ int32_t one(int64_t p) const { return stream_load<NT>(col + p); }
    __device__ __forceinline__ Raw raw(int64_t p) const { return stream_load2<NT>(col + p); }
    __device__ __forceinline__ int2 decode(Raw r, int64_t) const { return r; }
};

template <bool NT>
struct Col16 {
    const int32_t *__restrict__ base;
    const uint16_t *__restrict__ off;
    const int32_t *__restrict__ esc;
    // p even: entries p, p+1 share a 64-entry block and a 4-byte word
    __device__ __forceinline__ int2 pair(int64_t p) const
    {
        const int32_t b = base[p >> 6];
        if (b >= 0) {
            const uint32_t w = stream_load<NT>(reinterpret_cast<const uint32_t *>(off + p));
            return int2{b + (int32_t)(w & 0xffffu), b + (int32_t)(w >> 16)};
        }
        return stream_load2<NT>(esc + (int64_t)(-1 - b) * 64 + (p & 63));
    }
    __device__ __forceinline__ int32_t one(int64_t p) const
    {
        const int32_t b = base[p >> 6];
        return b >= 0 ? b + (int32_t)stream_load<NT>(off + p) : esc[(int64_t)(-1 - b) * 64 + (p & 63)];
    }
    struct Raw {
        int32_t b;   // the block's base, or -1 - escape slot
        uint32_t w;  // the pair's two 16-bit offsets
    };
    __device__ __forceinline__ Raw raw(int64_t p) const
    {
        return Raw{base[p >> 6], stream_load<NT>(reinterpret_cast<const uint32_t *>(off + p))};
    }
    __device__ __forceinline__ int2 decode(Raw r, int64_t p) const
    {
        if (r.b >= 0)
            return int2{r.b + (int32_t)(r.w & 0xffffu), r.b + (int32_t)(r.w >> 16)};
        return stream_load2<NT>(esc + (int64_t)(-1 - r.b) * 64 + (p & 63));
    }
};

// One chunk of a staged range, [cb, ce), cb even: every lane loads its R
// value/column pairs FIRST (branch-free, so all 2R loads are in flight
// together), then gathers x and stores the products in LDS.  A lane whose
// pair starts at or past ce, or would reach past the array (nz entries),
// loads the chunk's first pair instead — valid memory on a line the wave
// reads anyway (pair 0 of the array, the former fallback, was one line
// every workgroup of the grid hit) — and its products are never read: the
// reductions only read [cb, ce).  The one
// entry that can need more is the array's last entry when nz is odd; it
// is loaded singly in a branch almost every wave skips.  (With the guarded
// loads inside per-round branches the compiler serialised the rounds:
// one round's loads in flight at a time.)
// GATHERS_TOGETHER: also issue all 2R x gathers before the first product
// (more loads in flight per wave, more VGPRs, lower occupancy) instead of
// gathering round by round.
template <int R, bool NT, bool GATHERS_TOGETHER, typename Cols, typename XS, typename V = double>
__device__ __forceinline__ void stage_products(int64_t cb, int64_t ce, int64_t nz, const Cols &cols,
                                               const V *__restrict__ val, const XS &xs,
                                               double2 *s_prod)
{
    double2 v[R];
    int2 c[R];
    if (nz >= 2) {  // uniform; a 1-entry array has no pair 0
        const int64_t spare = cb + 1 < nz ? cb : (nz - 2) & ~(int64_t)1;  // this chunk's first pair
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t p = cb + 2 * (int64_t)(threadIdx.x + k * kBlock);
            const int64_t q = (p < ce && p + 1 < nz) ? p : spare;
            v[k] = vpair<NT>(val + q);
            c[k] = cols.pair(q);
        }
    } else {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            v[k] = double2{0.0, 0.0};
            c[k] = int2{0, 0};
        }
    }
    if constexpr (GATHERS_TOGETHER) {
        double2 xv[R];
#pragma unroll
        for (int k = 0; k < R; ++k)  // all 2R gathers in flight together
            xv[k] = double2{xs(c[k].x), xs(c[k].y)};
#pragma unroll
        for (int k = 0; k < R; ++k)
            s_prod[threadIdx.x + k * kBlock] = double2{v[k].x * xv[k].x, v[k].y * xv[k].y};
    } else {
#pragma unroll
        for (int k = 0; k < R; ++k)
            s_prod[threadIdx.x + k * kBlock] = double2{v[k].x * xs(c[k].x), v[k].y * xs(c[k].y)};
    }
    // the array's odd last entry (at most one lane of one chunk)
    const int64_t tail = nz - 1 - cb;
    if ((nz & 1) && nz - 1 < ce && tail >= 0 && tail < 2 * R * kBlock && (tail >> 1) % kBlock == threadIdx.x) {
        const int64_t p = nz - 1;
        s_prod[tail >> 1].x = vone<NT>(val + p) * xs(cols.one(p));
    }
}

// BATCH: 0 = per-round guarded loads, 1 = stream loads batched (gathers
// per round), 2 = stream loads and gathers batched (stage_products)
// One lane's share of a row's products in the staged chunk: entries
// [lo, hi) of the chunk (chunk-relative, < 2^31), every L-th from lo+lane,
// two partial sums so consecutive LDS reads do not wait on each other.
// Eight products are read per step before the first add (one LDS round
// trip per 8·L entries instead of per 2·L); the adds keep the a0/a1
// alternation, so the sums are the same bits as the two-at-a-time loop.
template <int L>
__device__ __forceinline__ double slice_sum(const double *prod, int64_t lo64, int64_t hi64, int lane)
{
    const int lo = (int)lo64, hi = (int)hi64;
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

template <int L, int R, bool NT, typename Cols = Col32<NT>, int BATCH = 0, typename XS = XGlobal,
          typename V = double>
__device__ __forceinline__ void staged_group(
    int64_t row, const int64_t *s_ptr, double2 *s_prod,
    const Cols cols, const V *__restrict__ val,
    const XS xs, double *__restrict__ y, int64_t n_rows, int64_t nz)
{
    constexpr int RPB = kBlock / L;
    constexpr int CH = 2 * kBlock * R;  // products per chunk
    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    const int64_t beg = s_ptr[g], end = s_ptr[g + 1];
    const int64_t blk_end = s_ptr[RPB];
    const double *prod = reinterpret_cast<const double *>(s_prod);

    double acc = 0.0;
    // chunks start on a kChunkAlign boundary (whole cache lines per wave);
    // entries before the group's range are loaded but never summed.
    for (int64_t cb = chunk_start(s_ptr[0]); cb < blk_end; cb += CH) {
        const int64_t ce = cb + CH < blk_end ? cb + CH : blk_end;
        if constexpr (BATCH > 0) {
            stage_products<R, NT, BATCH == 2>(cb, ce, nz, cols, val, xs, s_prod);
        } else {  // per-round guarded loads
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int t = threadIdx.x + k * kBlock;
                const int64_t p = cb + 2 * (int64_t)t;
                double2 pr = {0.0, 0.0};
                if (p + 1 < ce) {
                    const double2 v = vpair<NT>(val + p);
                    const int2 c = cols.pair(p);
                    pr.x = v.x * xs(c.x);
                    pr.y = v.y * xs(c.y);
                } else if (p < ce) {
                    pr.x = vone<NT>(val + p) * xs(cols.one(p));
                }
                s_prod[t] = pr;
            }
        }
        __syncthreads();
        acc += slice_sum<L>(prod, beg > cb ? beg - cb : 0, (end < ce ? end : ce) - cb, lane);
        __syncthreads();
    }
    acc = group_sum<L>(acc);
    if (lane == 0 && row < n_rows)
        store_y(y + (row), acc);
    __syncthreads();
}

// SPMV_XWIN_PROBE (timing-only builds, tools/gpu_job.sh abprobe; y is WRONG
// in them): bit 1 no x gathers, 2 no row reduction, 8 no x-window copy —
// prices each part of the MODE 3 kernel
#ifndef SPMV_XWIN_PROBE
#define SPMV_XWIN_PROBE 0
#endif
struct XConst {
    __device__ __forceinline__ double operator()(int32_t c) const { return (double)c; }
};

// One lane's share of a staged chunk in flight: R value pairs and R column
// pairs, loaded branch-free (pairs past the chunk load the chunk's first
// pair again and are never summed), so all 2R loads are outstanding together and can stay in
// flight across a barrier while the previous chunk is reduced.
template <int R, bool NT, typename V, typename Cols = Col32<NT>>
struct StreamRegs {
    double2 v[R];
    typename Cols::Raw c[R];
    int64_t q[R];  // the pair each lane loaded (decode needs it for escaped blocks only)

    __device__ __forceinline__ void issue(int64_t cb, int64_t ce, int64_t nz, const Cols &cols,
                                          const V *__restrict__ val)
    {
        if (nz < 2) {  // uniform; a 0/1-entry array has no pair 0 (its entry: products()), nothing is loaded
#pragma unroll
            for (int k = 0; k < R; ++k) {
                v[k] = double2{0.0, 0.0};
                c[k] = typename Cols::Raw{};
                q[k] = 0;
            }
            return;
        }
        const int64_t spare = cb + 1 < nz ? cb : (nz - 2) & ~(int64_t)1;  // this chunk's first pair
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t p = cb + 2 * (int64_t)(threadIdx.x + k * kBlock);
            q[k] = (p < ce && p + 1 < nz) ? p : spare;
            v[k] = vpair<NT>(val + q[k]);
            c[k] = cols.raw(q[k]);
        }
    }

    // products of the issued chunk [cb, ce) into s_prod (as stage_products)
    template <typename XS>
    __device__ __forceinline__ void products(int64_t cb, int64_t ce, int64_t nz, const Cols &cols,
                                             const V *__restrict__ val, const XS &xs, double2 *s_prod) const
    {
        if (nz >= 2) {  // uniform (no gathers for a 0/1-entry array: x may be empty)
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int2 cc = cols.decode(c[k], q[k]);
                s_prod[threadIdx.x + k * kBlock] = double2{v[k].x * xs(cc.x), v[k].y * xs(cc.y)};
            }
        } else {
#pragma unroll
            for (int k = 0; k < R; ++k)
                s_prod[threadIdx.x + k * kBlock] = double2{0.0, 0.0};
        }
        const int64_t tail = nz - 1 - cb;  // the array's odd last entry
        if ((nz & 1) && nz - 1 < ce && tail >= 0 && tail < 2 * R * kBlock && (tail >> 1) % kBlock == threadIdx.x) {
            const int64_t p = nz - 1;
            s_prod[tail >> 1].x = vone<NT>(val + p) * xs(cols.one(p));
        }
    }
};

// The row groups of one x window, software-pipelined (csr_xwin_kernel
// MODE 3): the loads of the NEXT chunk — of this row group or of the
// window's next group — are issued right after the current chunk's
// products are in LDS, so they are in flight during the barrier and the
// L-lane reduction instead of after it.  s_off holds the window's
// ngroups·RPB + 1 row offsets.  Chunks and per-row sums are exactly those
// of staged_group (same boundaries, same order): the same bits.
// NBUF = 2 (MODE 4): chunks alternate between two product buffers, so the
// barrier that protected the buffer from the next chunk's products is gone
// (one barrier per chunk); the caller adds a barrier before reusing LDS.
template <int L, int R, bool NT, typename XS, typename V, int NBUF = 1, bool PRE = false,
          typename Cols = Col32<NT>>
__device__ __forceinline__ void staged_window_pipelined(int64_t row0, int ngroups, const int64_t *s_off,
                                                        double2 *s_prod_base, const Cols cols,
                                                        const V *__restrict__ val, const XS xs,
                                                        double *__restrict__ y, int64_t n_rows, int64_t nz,
                                                        const StreamRegs<R, NT, V, Cols> pre_st = {},
                                                        bool pre = false)
{
    constexpr int RPB = kBlock / L;
    constexpr int CH = 2 * kBlock * R;
    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    int buf = 0;
    // first chunk of group j at or after `from` that has one (staged_group's
    // loop runs a chunk iff chunk_start(start) < end); ngroups when none
    auto next_group = [&](int from) {
        int j = from;
        while (j < ngroups && chunk_start(s_off[j * RPB]) >= s_off[(j + 1) * RPB])
            ++j;
        return j;
    };
    StreamRegs<R, NT, V, Cols> st;
    int jn;
    if (PRE && pre) {  // the caller issued group 0's first chunk (it has one)
        st = pre_st;
        jn = 0;
    } else {
        jn = next_group(0);
        if (jn < ngroups) {
            const int64_t b = chunk_start(s_off[jn * RPB]), e = s_off[(jn + 1) * RPB];
            st.issue(b, b + CH < e ? b + CH : e, nz, cols, val);
        }
    }
    for (int gi = 0; gi < ngroups; ++gi) {
        const int64_t *gp = s_off + gi * RPB;
        const int64_t beg = gp[g], end = gp[g + 1];
        const int64_t blk_end = gp[RPB];
        double acc = 0.0;
        for (int64_t cb = chunk_start(gp[0]); cb < blk_end; cb += CH) {
            const int64_t ce = cb + CH < blk_end ? cb + CH : blk_end;
            double2 *s_prod = s_prod_base + buf * (kBlock * R);
            const double *prod = reinterpret_cast<const double *>(s_prod);
#if SPMV_XWIN_PROBE & 1  // timing probe: no x gathers (wrong y)
            st.products(cb, ce, nz, cols, val, XConst{}, s_prod);
#else
            st.products(cb, ce, nz, cols, val, xs, s_prod);
#endif
            // the next chunk: this group's, else the next group's first
            if (cb + CH < blk_end) {
                const int64_t nb = cb + CH;
                st.issue(nb, nb + CH < blk_end ? nb + CH : blk_end, nz, cols, val);
            } else if ((jn = next_group(gi + 1)) < ngroups) {
                const int64_t b = chunk_start(s_off[jn * RPB]), e = s_off[(jn + 1) * RPB];
                st.issue(b, b + CH < e ? b + CH : e, nz, cols, val);
            }
            __syncthreads();
#if SPMV_XWIN_PROBE & 2  // timing probe: one product per lane instead of the row slice (wrong y)
            acc += prod[threadIdx.x];
#else
            acc += slice_sum<L>(prod, beg > cb ? beg - cb : 0, (end < ce ? end : ce) - cb, lane);
#endif
            if constexpr (NBUF == 1)
                __syncthreads();
            else
                buf ^= 1;
        }
        acc = group_sum<L>(acc);
        const int64_t row = row0 + (int64_t)gi * RPB + g;
        // (the window's y staged in LDS and stored once at its end measured
        // the same: 0.2481 vs 0.2478 ms, profiles/round2/ab_ystage.log)
        if (lane == 0 && row < n_rows)
            store_y(y + (row), acc);
    }
}

// The window's rows as ONE entry range (csr_xwin_kernel MODE 5): instead of
// chunking each 256/L-row group on its own (a 64-row group of the cant
// batch is 4,107 entries: two full 2,048-entry chunks and an 11-entry one,
// every chunk one memory round trip and two barriers), the window's whole
// range [s_off[0], s_off[WR]) is cut into the fewest chunks of at most
// 2·256·R entries, all of (nearly) equal size, streamed pipelined as in
// MODE 3.  L-lane group g owns the RW consecutive rows g·RW .. g·RW+RW-1 of
// the window (WR = RW·256/L rows) and adds each chunk's slice of each row.
// Rows that lie in one chunk sum exactly as in the other modes; a row cut
// by a chunk boundary is summed in the same order over other boundaries.
template <int L, int R, int RW, bool NT, typename XS, typename V, typename Cols>
__device__ __forceinline__ void staged_window_flat(int64_t row0, const int64_t *s_off, double2 *s_prod,
                                                   const Cols cols, const V *__restrict__ val,
                                                   const XS xs, double *__restrict__ y, int64_t n_rows, int64_t nz)
{
    constexpr int G = kBlock / L;
    constexpr int64_t CHMAX = 2 * kBlock * R;
    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    const double *prod = reinterpret_cast<const double *>(s_prod);
    int64_t rb[RW + 1];
#pragma unroll
    for (int k = 0; k <= RW; ++k)
        rb[k] = s_off[g * RW + k];
    const int64_t e0 = chunk_start(s_off[0]), e1 = s_off[G * RW];
    const int64_t nch = e1 > e0 ? (e1 - e0 + CHMAX - 1) / CHMAX : 0;
    const int64_t cs = nch > 0 ? chunk_start(((e1 - e0 + nch - 1) / nch) + kChunkAlign - 1) : 0;  // aligned, <= CHMAX
    double acc[RW];
#pragma unroll
    for (int k = 0; k < RW; ++k)
        acc[k] = 0.0;
    StreamRegs<R, NT, V, Cols> st;
    if (nch > 0)
        st.issue(e0, e0 + cs < e1 ? e0 + cs : e1, nz, cols, val);
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t cb = e0 + c * cs;
        const int64_t ce = cb + cs < e1 ? cb + cs : e1;
        st.products(cb, ce, nz, cols, val, xs, s_prod);
        if (c + 1 < nch)
            st.issue(ce, ce + cs < e1 ? ce + cs : e1, nz, cols, val);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RW; ++k) {
            const int64_t lo = rb[k] > cb ? rb[k] : cb;
            const int64_t hi = rb[k + 1] < ce ? rb[k + 1] : ce;
            if (lo < hi)  // uniform over the L-lane group
                acc[k] += slice_sum<L>(prod, lo - cb, hi - cb, lane);
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < RW; ++k) {
        const double s = group_sum<L>(acc[k]);
        const int64_t row = row0 + (int64_t)g * RW + k;
        if (lane == 0 && row < n_rows)
            store_y(y + (row), s);
    }
}

// Variant 2: one workgroup per row group.
template <int L, int R>
__global__ __launch_bounds__(kBlock) void csr_staged_kernel(
    int64_t n_rows, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, int remap)
{
    constexpr int RPB = kBlock / L;
    __shared__ int64_t s_ptr[RPB + 1];
    __shared__ double2 s_prod[kBlock * R];
    const int64_t row0 = xcd_block(remap) * RPB;
    if (threadIdx.x <= RPB) {
        int64_t r = row0 + threadIdx.x;
        s_ptr[threadIdx.x] = row_ptr[r < n_rows ? r : n_rows];
    }
    __syncthreads();
    staged_group<L, R, false>(row0 + threadIdx.x / L, s_ptr, s_prod, Col32<false>{col}, val, XGlobal{x}, y, n_rows,
                              row_ptr[n_rows]);
}

// Variant 3: persistent workgroups (a few per CU) walk the row groups
// grid-stride and PREFETCH the next group's row offsets into registers
// while the current group streams, so a group no longer starts with a
// dependent round trip for its offsets.  Cols = Col32 (CSR) or Col16
// (compressed column indices, spmv_csr16_run).
template <int L, int R, bool NT, typename Cols, int BATCH = 0>
__global__ __launch_bounds__(kBlock) void csr_staged_persistent_kernel(
    int64_t n_rows, int64_t n_groups, const int64_t *__restrict__ row_ptr,
    const Cols cols, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y)
{
    constexpr int RPB = kBlock / L;
    __shared__ int64_t s_ptr[RPB + 1];
    __shared__ double2 s_prod[kBlock * R];
    const int64_t nz = row_ptr[n_rows];
    int64_t grp = blockIdx.x;
    int64_t next = 0;
    if (threadIdx.x <= RPB) {
        int64_t r = grp * RPB + threadIdx.x;
        next = row_ptr[r < n_rows ? r : n_rows];
    }
    for (; grp < n_groups; grp += gridDim.x) {
        if (threadIdx.x <= RPB)
            s_ptr[threadIdx.x] = next;
        __syncthreads();
        const int64_t g2 = grp + gridDim.x;
        if (threadIdx.x <= RPB && g2 < n_groups) {
            int64_t r = g2 * RPB + threadIdx.x;
            next = row_ptr[r < n_rows ? r : n_rows];
        }
        staged_group<L, R, NT, Cols, BATCH>(grp * RPB + threadIdx.x / L, s_ptr, s_prod, cols, val, XGlobal{x}, y, n_rows,
                                            nz);
    }
}

// Column window of every row group (RPB rows): [min, max] column of its
// entry range (one pass over col, build time).
__global__ __launch_bounds__(kBlock) void csr_window_kernel(int64_t n_rows, int64_t rpb,
                                                            const int64_t *__restrict__ row_ptr,
                                                            const int32_t *__restrict__ col,
                                                            int2 *__restrict__ win)
{
    const int64_t g = blockIdx.x;
    const int64_t r1 = (g + 1) * rpb < n_rows ? (g + 1) * rpb : n_rows;
    const int2 r = block_col_range(col, row_ptr[g * rpb], row_ptr[r1]);
    if (threadIdx.x == 0)
        win[g] = r;
}

// The persistent staged kernel with x windows in LDS.  A window covers
// gpw consecutive row groups (rows_per_window = gpw * 256/L rows): the
// workgroup copies x[win.x .. win.y] into LDS (dynamic, xcap entries) once
// and then streams the gpw groups, whose products gather from LDS instead
// of global memory — the limiter of the staged kernel (TA busy, requests
// well below the DRAM credit limit: profiles/round1/pmc_stalls.json).
// Windows of several groups overlap less than per-group windows, so less
// x is re-read.  A window wider than xcap gathers from global memory.
// Same products, same order: y is bit-identical to variant 3.
// MODE (load schedule; products, sums and y are the same bits in every mode):
//   0 = window copied by a strided loop (one round trip per 256 entries),
//       each stream round's loads waited for before the next round's issue;
//   1 = the window's row offsets (all its groups, staged in LDS after the x
//       range: dynamic LDS of xcap + rows_per_window + 1 doubles) and its x
//       range loaded together, 8 loads in flight per thread, before ONE
//       barrier; no offset loads between the groups;
//   2 = as 1, and all R value/column pair loads of a chunk issued together
//       before the first product (stage_products; x gathers from LDS);
//   3 = as 2, software-pipelined: the next chunk's loads are issued before
//       the current chunk's barrier and reduction (staged_window_pipelined);
//   4 = as 3 with two product buffers: one barrier per chunk;
//   5 = as 3, the window's rows chunked as one entry range
//       (staged_window_flat; gpw in {1, 2, 4}, else MODE 3).
// MODE 3/4 kernels are built for kXwinWaves waves per SIMD (workgroups per
// CU), which caps their VGPRs (8 -> 64)
#ifndef SPMV_XWIN_WAVES
#define SPMV_XWIN_WAVES 1
#endif
constexpr int kXwinWaves = SPMV_XWIN_WAVES;
template <int L, int R, bool NT, typename V = double, int MODE = 0, bool PRE = false, typename Cols = Col32<NT>>
__global__ __launch_bounds__(kBlock, MODE >= 3 ? kXwinWaves : 1) void csr_xwin_kernel(
    int64_t n_rows, int64_t n_groups, int64_t gpw, const int64_t *__restrict__ row_ptr,
    const Cols cols, const V *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap,
    int remap)
{
    constexpr int RPB = kBlock / L;
    constexpr int BATCH = MODE == 2 ? 1 : 0;
    extern __shared__ double s_x[];
    __shared__ int64_t s_ptr[MODE > 0 ? 1 : RPB + 1];
    __shared__ double2 s_prod[kBlock * R * (MODE == 4 ? 2 : 1)];
    int64_t *s_off = reinterpret_cast<int64_t *>(s_x + xcap);  // MODE > 0: the window's offsets
    const int64_t nz = row_ptr[n_rows];
    const int64_t n_win = (n_groups + gpw - 1) / gpw;
    // remap: consecutive windows on one XCD, so the overlapping x ranges of
    // neighbouring windows are copied from that XCD's L2
    for (int64_t wi = xcd_block(remap); wi < n_win; wi += gridDim.x) {
        const int64_t g_beg = wi * gpw;
        const int64_t g_end = (wi + 1) * gpw < n_groups ? (wi + 1) * gpw : n_groups;
        const int2 wnd = win[wi];
        const int32_t span = wnd.y - wnd.x + 1;
        const bool staged = span > 0 && span <= xcap;  // uniform per workgroup
        // MODE 3 (kCsrXwinPre): group 0's first chunk is issued before the
        // window copy — its range needs only two row offsets, loaded beside
        // the window bounds — so the copy and the first chunk's loads share
        // one round trip instead of following each other
        StreamRegs<R, NT, V, Cols> st_pre;
        bool pre = false;
        if constexpr (MODE == 3 && PRE) {
            const int64_t rr0 = g_beg * RPB;
            const int64_t rr1 = rr0 + RPB < n_rows ? rr0 + RPB : n_rows;
            const int64_t b = chunk_start(row_ptr[rr0]), e = row_ptr[rr1];
            pre = b < e;  // uniform
            if (pre)
                st_pre.issue(b, b + 2 * kBlock * R < e ? b + 2 * kBlock * R : e, nz, cols, val);
        }
        if constexpr (MODE > 0) {
            // offsets r0 .. r0 + nr of the window's rows (clamped past
            // n_rows), then the x range: every load issued before the stores.
            // The flat modes read all gpw groups' offsets, also in a last
            // window with fewer groups (clamped: empty rows)
            const int64_t r0 = g_beg * RPB;
            const int32_t nr = (int32_t)((MODE >= 5 ? gpw : g_end - g_beg) * RPB) + 1;
            constexpr int U = 2;  // offsets per thread per pass (nr <= U·256 in one pass)
            for (int32_t b = 0; b < nr; b += U * kBlock) {
                int64_t o[U];
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int64_t r = r0 + b + threadIdx.x + k * kBlock;
                    o[k] = row_ptr[r < n_rows ? r : n_rows];
                }
                if (staged && b == 0)
#if !(SPMV_XWIN_PROBE & 8)  // timing probe: no window copy (wrong y)
                    copy_window(s_x, x, wnd.x, span);
#endif
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int32_t i = b + (int32_t)threadIdx.x + k * kBlock;
                    if (i < nr)
                        s_off[i] = o[k];
                }
            }
        } else if (staged) {
            for (int32_t i = threadIdx.x; i < span; i += kBlock)
                s_x[i] = x[wnd.x + i];
        }
        if constexpr (MODE >= 5) {  // flat chunks; MODE 5/6/7 = gpw 1/2/4 (the launcher's pick)
            constexpr int RW = MODE == 5 ? 1 : MODE == 6 ? 2 : 4;
            __syncthreads();  // window and offsets visible
            const int64_t r0 = g_beg * RPB;
            if (staged)
                staged_window_flat<L, R, RW, NT>(r0, s_off, s_prod, cols, val, XWindow{s_x, wnd.x}, y, n_rows, nz);
            else
                staged_window_flat<L, R, RW, NT>(r0, s_off, s_prod, cols, val, XGlobal{x}, y, n_rows, nz);
            continue;
        }
        if constexpr (MODE >= 3) {
            constexpr int NB = MODE == 4 ? 2 : 1;
            __syncthreads();  // window and offsets visible
            if (staged)
                staged_window_pipelined<L, R, NT, XWindow, V, NB, PRE, Cols>(
                    g_beg * RPB, (int)(g_end - g_beg), s_off, s_prod, cols, val, XWindow{s_x, wnd.x}, y, n_rows, nz,
                    st_pre, pre);
            else
                staged_window_pipelined<L, R, NT, XGlobal, V, NB, PRE, Cols>(
                    g_beg * RPB, (int)(g_end - g_beg), s_off, s_prod, cols, val, XGlobal{x}, y, n_rows, nz, st_pre,
                    pre);
            if constexpr (NB == 2)
                __syncthreads();  // the last chunk's buffer is read before the next window writes LDS
            continue;
        }
        for (int64_t grp = g_beg; grp < g_end; ++grp) {
            const int64_t *gp = s_ptr;
            if constexpr (MODE > 0) {
                gp = s_off + (grp - g_beg) * RPB;
                if (grp == g_beg)
                    __syncthreads();  // window and offsets visible
            } else {
                if (threadIdx.x <= RPB) {
                    const int64_t r = grp * RPB + threadIdx.x;
                    s_ptr[threadIdx.x] = row_ptr[r < n_rows ? r : n_rows];
                }
                __syncthreads();  // offsets (and, for the first group, the window) visible
            }
            const int64_t row = grp * RPB + threadIdx.x / L;
            if (staged)
                staged_group<L, R, NT, Cols, BATCH, XWindow, V>(row, gp, s_prod, cols, val,
                                                                     XWindow{s_x, wnd.x}, y, n_rows, nz);
            else
                staged_group<L, R, NT, Cols, BATCH, XGlobal, V>(row, gp, s_prod, cols, val,
                                                                     XGlobal{x}, y, n_rows, nz);
        }
    }
}

// Timing probes on the matrix's own arrays (SPMV_CSR_STREAM_PROBE=P; y is
// WRONG): tools/bw_probe's staged stream — 1536-entry chunks of value/column
// pairs, products to LDS, barrier, a 6-product read per lane, barrier — made
// step by step more like csr_xwin_kernel, to find what the structure costs:
//   P = 1: fixed 8192-entry tiles of the entry array (the bare probe);
//   P = 2: one tile per 128-row window, bounds from row_ptr (chunk_start);
//   P = 3: as 2, chunks restart at every 64-row group (as the kernel);
//   P = 4: as 3, plus one y store per row (lane 0 of 4-lane groups);
//   P = 5: as 4, windows placed XCD-contiguously;
//   P = 6: as 3, the window's y values stored once at its end (128 lanes);
//   P = 7: as 4 with non-temporal y stores;
//   P = 8: as 6 with non-temporal y stores;
//   P = 9 / A: as 4 with relaxed system- / agent-scope atomic stores;
//   P = B: as 3 with one y store at the START of each workgroup;
//   P = C: as 4 with two windows per workgroup;
//   P = D / E: as 4 with "sc1 nt" / "sc0 sc1 nt" stores;
//   P = F: as 4 with every store into the first 64 KiB of y;
//   P = G / H / I: as 4, the stream loaded "sc1 nt" / "sc0 sc1 nt" / "sc1";
//   P = J: as G with sc1 y stores.
template <int P>
__global__ __launch_bounds__(kBlock) void csr_stream_probe_kernel(const int64_t *__restrict__ row_ptr, int64_t n_rows,
                                                                  const double *__restrict__ val,
                                                                  const int32_t *__restrict__ col, int64_t nnz,
                                                                  double *__restrict__ y)
{
    constexpr int R = 3;
    constexpr int64_t CH = 2 * kBlock * R, TILE = 8192;
    __shared__ double2 s_prod[kBlock * R];
    const double *prod = reinterpret_cast<const double *>(s_prod);
    const int64_t w = P >= 5 ? xcd_block(1) : blockIdx.x;
    double s = 0.0;
    auto stream = [&](int64_t t0, int64_t t1) {
        for (int64_t cb = t0; cb < t1; cb += CH) {
            double2 v[R];
            int2 c[R];
            if constexpr (P >= 16 && P <= 19) {  // stream loads with explicit cache-policy bits
                v2f64 va[R];
                v2i32 ca[R];
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int64_t p = cb + 2 * (int64_t)(threadIdx.x + k * kBlock);
                    const int64_t q = p + 1 < t1 ? p : t0;
                    if constexpr (P == 16 || P == 19) {
                        asm volatile("global_load_dwordx4 %0, %1, off sc1 nt" : "=v"(va[k]) : "v"(val + q));
                        asm volatile("global_load_dwordx2 %0, %1, off sc1 nt" : "=v"(ca[k]) : "v"(col + q));
                    } else if constexpr (P == 17) {
                        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt" : "=v"(va[k]) : "v"(val + q));
                        asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1 nt" : "=v"(ca[k]) : "v"(col + q));
                    } else {
                        asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(va[k]) : "v"(val + q));
                        asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(ca[k]) : "v"(col + q));
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)"
                             : "+v"(va[0]), "+v"(va[1]), "+v"(va[2]), "+v"(ca[0]), "+v"(ca[1]), "+v"(ca[2])
                             :
                             : "memory");
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    v[k] = double2{va[k].x, va[k].y};
                    c[k] = int2{ca[k].x, ca[k].y};
                }
            } else {
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const int64_t p = cb + 2 * (int64_t)(threadIdx.x + k * kBlock);
                    const int64_t q = p + 1 < t1 ? p : t0;
                    v[k] = stream_load2<true>(val + q);
                    c[k] = stream_load2<true>(col + q);
                }
            }
#pragma unroll
            for (int k = 0; k < R; ++k)
                s_prod[threadIdx.x + k * kBlock] = double2{v[k].x * (double)c[k].x, v[k].y * (double)c[k].y};
            __syncthreads();
            const int g = threadIdx.x / 4, lane = threadIdx.x % 4;
#pragma unroll
            for (int k = 0; k < 2 * R; ++k)
                s += prod[g * 8 * R + lane + 4 * k];
            __syncthreads();
        }
    };
    if constexpr (P == 11) {  // a y store at the START of the workgroup only (then the P3 stream)
        const int64_t row = w * 128 + threadIdx.x;
        if (threadIdx.x < 128 && row < n_rows)
            y[row] = 0.0;
    }
    if constexpr (P == 12) {  // as 4, two windows per workgroup (one end-of-workgroup per 256 rows)
        for (int64_t ww = 2 * (int64_t)blockIdx.x; ww < 2 * (int64_t)blockIdx.x + 2; ++ww)
            for (int gi = 0; gi < 2; ++gi) {
                const int64_t r0 = ww * 128 + gi * 64;
                if (r0 >= n_rows)
                    break;
                const int64_t r1 = r0 + 64 < n_rows ? r0 + 64 : n_rows;
                stream(chunk_start(row_ptr[r0]), row_ptr[r1]);
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1)
                    y[row] = s;
            }
    } else if constexpr (P == 1) {
        const int64_t t0 = w * TILE;
        stream(t0, t0 + TILE < nnz ? t0 + TILE : nnz);
    } else if constexpr (P == 2) {
        const int64_t r0 = w * 128, r1 = r0 + 128 < n_rows ? r0 + 128 : n_rows;
        stream(chunk_start(row_ptr[r0]), row_ptr[r1]);
    } else {
        for (int gi = 0; gi < 2; ++gi) {
            const int64_t r0 = w * 128 + gi * 64;
            if (r0 >= n_rows)
                break;
            const int64_t r1 = r0 + 64 < n_rows ? r0 + 64 : n_rows;
            stream(chunk_start(row_ptr[r0]), row_ptr[r1]);
            if constexpr (P == 4 || P == 5) {
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1)
                    y[row] = s;
            } else if constexpr (P == 7) {
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1)
                    __builtin_nontemporal_store(s, y + row);
            } else if constexpr (P == 13 || P == 14) {
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1) {
                    if constexpr (P == 13)
                        asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(y + row), "v"(s) : "memory");
                    else
                        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt" ::"v"(y + row), "v"(s) : "memory");
                }
            } else if constexpr (P == 15) {  // plain stores into 64 KiB of y (no HBM write traffic to speak of)
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1)
                    y[row & 8191] = s;
            } else if constexpr (P >= 16 && P <= 18) {  // plain y stores beside the policy loads
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1)
                    y[row] = s;
            } else if constexpr (P == 19) {
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1)
                    store_y(y + row, s);
            } else if constexpr (P == 9 || P == 10) {
                const int64_t row = r0 + threadIdx.x / 4;
                if (threadIdx.x % 4 == 0 && row < r1)
                    __hip_atomic_store(y + row, s, __ATOMIC_RELAXED,
                                       P == 9 ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if constexpr (P == 6 || P == 8) {  // the window's 128 y values at its end, one coalesced store
            const int64_t row = w * 128 + threadIdx.x;
            if (threadIdx.x < 128 && row < n_rows) {
                if constexpr (P == 8)
                    __builtin_nontemporal_store(s, y + row);
                else
                    y[row] = s;
            }
        }
    }
    if (s == 123.456)
        y[0] = s;
}

// x ring of csr_xstream_kernel: column c lives in slot c & mask of a
// power-of-two LDS array at least as long as the widest row group's column
// span, so the ranges of consecutive groups share every column they overlap
// on and a new group copies only the columns the previous one lacked.
struct XRing {
    const double *s;  // LDS
    int32_t mask;
    __device__ __forceinline__ double operator()(int32_t c) const { return s[c & mask]; }
};

// x[lo .. lo+span) into the ring, U loads in flight per thread
template <int U = 8>
__device__ __forceinline__ void copy_ring(double *s_x, const double *__restrict__ x, int32_t lo, int32_t span,
                                          int32_t mask)
{
    for (int32_t b = 0; b < span; b += U * kBlock) {
        double v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t i = b + (int32_t)threadIdx.x + k * kBlock;
            v[k] = x[lo + (i < span ? i : span - 1)];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int32_t i = b + (int32_t)threadIdx.x + k * kBlock;
            if (i < span)
                s_x[(lo + i) & mask] = v[k];
        }
    }
}

// The streaming CSR kernel (spmv_csr_run_xwin with one row group per window
// and SPMV_CSR_XSTREAM=1): persistent workgroups, each owning ONE contiguous
// range of row groups (256/L rows each; the ranges differ by at most one
// group), streamed as one software pipeline that does not stop at group
// boundaries.  Per chunk: products of chunk k (x from the ring) -> the loads
// of chunk k+1 issued (the next group's first chunk at a group's end) ->
// barrier -> the L-lane row slices of chunk k -> barrier.  What the x-window
// kernel pays per window, this kernel hides inside that pipeline:
//  - the next group's row offsets are loaded two groups ahead (three LDS
//    offset buffers), so issuing its first chunk never waits on them;
//  - the next group's column range (win, one int2 per group) is loaded a
//    group ahead, and the columns it adds to the ring are loaded beside the
//    next chunk's stream and stored after the first barrier, when no lane
//    gathers from the ring any more.
// Chunks, products and sums are those of staged_group: y is bit-identical to
// the other staged CSR kernels.  A group whose range does not fit in the ring
// gathers from global memory.
template <int L, int R, bool NT, typename V = double, typename Cols = Col32<NT>>
__global__ __launch_bounds__(kBlock) void csr_xstream_kernel(
    int64_t n_rows, int64_t n_groups, const int64_t *__restrict__ row_ptr, const Cols cols,
    const V *__restrict__ val, const double *__restrict__ x, double *__restrict__ y,
    const int2 *__restrict__ gwin, int32_t cap)
{
    constexpr int RPB = kBlock / L;
    constexpr int CH = 2 * kBlock * R;
    constexpr int U = 2;  // new ring columns per thread loaded ahead of the barrier
    extern __shared__ double s_x[];
    __shared__ int64_t s_off[3][RPB + 1];
    __shared__ double2 s_prod[kBlock * R];
    const double *prod = reinterpret_cast<const double *>(s_prod);
    const int64_t nz = row_ptr[n_rows];
    const int64_t gb = (int64_t)blockIdx.x * n_groups / gridDim.x;
    const int64_t ge = ((int64_t)blockIdx.x + 1) * n_groups / gridDim.x;
    if (gb >= ge)
        return;  // uniform
    const int t = threadIdx.x, g = t / L, lane = t % L;
    const int32_t mask = cap - 1;
    const XRing xr{s_x, mask};
    auto offs = [&](int64_t j) {  // offset of row j·RPB + t (threads 0..RPB), clamped
        const int64_t r = j * RPB + t;
        return row_ptr[r < n_rows ? r : n_rows];
    };
    auto fits = [&](int2 w) { return w.x <= w.y && (int64_t)w.y - w.x + 1 <= cap; };

    // prologue: offsets of the first two groups (the third's in a register),
    // the first group's columns copied whole
    int64_t onext = 0;
    {
        int64_t o0 = 0, o1 = 0;
        if (t <= RPB) {
            o0 = offs(gb);
            o1 = offs(gb + 1);
            onext = offs(gb + 2);
        }
        const int2 w = gwin[gb];
        if (fits(w))
            copy_ring(s_x, x, w.x, w.y - w.x + 1, mask);
        if (t <= RPB) {
            s_off[0][t] = o0;
            s_off[1][t] = o1;
        }
    }
    int2 w0 = gwin[gb];
    bool fit = fits(w0);
    int32_t rlo = fit ? w0.x : 1, rhi = fit ? w0.y : 0;  // columns the ring holds (none: rlo > rhi)
    int2 wnext = gwin[gb + 1 < n_groups ? gb + 1 : gb];
    __syncthreads();

    StreamRegs<R, NT, V, Cols> st;
    {
        const int64_t b = chunk_start(s_off[0][0]), e = s_off[0][RPB];
        st.issue(b, b + CH < e ? b + CH : e, nz, cols, val);
    }
    int bi = 0;  // s_off buffer of group gi
    for (int64_t gi = gb; gi < ge; ++gi) {
        const int64_t *gp = s_off[bi];
        const int64_t beg = gp[g], end = gp[g + 1];
        const int64_t gend = gp[RPB];
        const int bn = bi == 2 ? 0 : bi + 1, bnn = bn == 2 ? 0 : bn + 1;
        double acc = 0.0;
        // chunks as staged_group's; a group without one runs one empty chunk
        for (int64_t cb = chunk_start(gp[0]), k = 0;; ++k) {
            const int64_t ce = cb + CH < gend ? cb + CH : gend;
            const bool last = ce >= gend;
            if (fit)
                st.products(cb, ce, nz, cols, val, xr, s_prod);
            else
                st.products(cb, ce, nz, cols, val, XGlobal{x}, s_prod);
            if (k == 0) {  // the group after next: offsets to LDS, the one after that loaded
                if (t <= RPB)
                    s_off[bnn][t] = onext;
                if (t <= RPB)
                    onext = offs(gi + 3);
            }
            // the next group's new ring columns: [A0, A1] below the ring's
            // range and [B0, B1] above it
            const bool more = last && gi + 1 < ge;
            const int2 wn = wnext;
            const bool nfit = more && fits(wn);
            int32_t A0 = 0, nA = 0, B0 = 0, nB = 0;
            double rv[U];
            if (nfit) {
                if (rlo > rhi) {
                    A0 = wn.x;
                    nA = wn.y - wn.x + 1;
                } else {
                    const int32_t a1 = wn.y < rlo - 1 ? wn.y : rlo - 1;
                    A0 = wn.x;
                    nA = a1 >= A0 ? a1 - A0 + 1 : 0;
                    B0 = wn.x > rhi + 1 ? wn.x : rhi + 1;
                    nB = wn.y >= B0 ? wn.y - B0 + 1 : 0;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t i = t + u * kBlock;
                    const int32_t c = i < nA ? A0 + i : i < nA + nB ? B0 + (i - nA) : wn.x;
                    rv[u] = x[c];
                }
            }
            if (more) {  // the next group's first chunk
                const int64_t *np = s_off[bn];
                const int64_t b = chunk_start(np[0]), e = np[RPB];
                st.issue(b, b + CH < e ? b + CH : e, nz, cols, val);
                wnext = gwin[gi + 2 < n_groups ? gi + 2 : gi + 1];
            } else if (!last) {
                st.issue(ce, ce + CH < gend ? ce + CH : gend, nz, cols, val);
            }
            __syncthreads();  // products visible; nobody gathers from the ring any more
            acc += slice_sum<L>(prod, beg > cb ? beg - cb : 0, (end < ce ? end : ce) - cb, lane);
            if (nfit) {
                const int32_t n = nA + nB;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t i = t + u * kBlock;
                    if (i < n)
                        s_x[(i < nA ? A0 + i : B0 + (i - nA)) & mask] = rv[u];
                }
                for (int32_t i = t + U * kBlock; i < n; i += kBlock) {
                    const int32_t c = i < nA ? A0 + i : B0 + (i - nA);
                    s_x[c & mask] = x[c];
                }
                rlo = wn.x;
                rhi = wn.y;
                fit = true;
            } else if (more && wn.x <= wn.y) {  // too wide: global gathers, ring forgotten
                rlo = 1;
                rhi = 0;
                fit = false;
            }  // an empty next group keeps the ring (and `fit`)
            __syncthreads();
            if (last)
                break;
            cb = ce;
        }
        acc = group_sum<L>(acc);
        const int64_t row = gi * RPB + g;
        if (lane == 0 && row < n_rows)
            store_y(y + (row), acc);
        bi = bn;
    }
}

// One lane's share of a staged chunk held in registers: R value pairs,
// R column pairs and how many entries of each pair are inside the chunk.
template <int R, bool NT>
struct ChunkRegs {
    double2 v[R];
    int2 c[R];
    uint32_t live;  // bit 2k: entry 2k+... of pair k inside the chunk; bit 2k+1: its partner

    __device__ __forceinline__ void issue(const int32_t *__restrict__ col,
                                          const double *__restrict__ val, int64_t cb, int64_t ce)
    {
        // one 64-bit base, 32-bit per-pair offsets (a chunk is < 2^31 entries)
        const int32_t left = (int32_t)(ce - cb);
        const double *vb = val + cb;
        const int32_t *cbp = col + cb;
        live = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int32_t q = 2 * (int32_t)(threadIdx.x + k * kBlock);
            if (q + 1 < left) {
                v[k] = stream_load2<NT>(vb + q);
                c[k] = stream_load2<NT>(cbp + q);
                live |= 3u << (2 * k);
            } else if (q < left) {  // odd tail: never read past the range
                v[k] = double2{stream_load<NT>(vb + q), 0.0};
                c[k] = int2{stream_load<NT>(cbp + q), 0};
                live |= 1u << (2 * k);
            }
        }
    }

    template <typename XS>
    __device__ __forceinline__ void products_xs(const XS &xs, double2 *s_prod) const
    {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            double2 pr = {0.0, 0.0};
            if (live & (1u << (2 * k)))
                pr.x = v[k].x * xs(c[k].x);
            if (live & (2u << (2 * k)))
                pr.y = v[k].y * xs(c[k].y);
            s_prod[threadIdx.x + k * kBlock] = pr;
        }
    }

    __device__ __forceinline__ void products(const double *__restrict__ x, double2 *s_prod) const
    {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            double2 pr = {0.0, 0.0};
            if (live & (1u << (2 * k)))
                pr.x = v[k].x * x[c[k].x];
            if (live & (2u << (2 * k)))
                pr.y = v[k].y * x[c[k].y];
            s_prod[threadIdx.x + k * kBlock] = pr;
        }
    }
};

// The x-window kernel with the first chunk of every window PREFETCHED: its
// value/column loads are issued (into registers, ChunkRegs) before the
// window's x range is copied into LDS, so the window copy and the first
// barrier no longer sit in front of the stream.  Same products, same order:
// bit-identical to csr_xwin_kernel.  SPMV_CSR_XWIN_PF=0 turns it off.
template <int L, int R, bool NT, typename XS>
__device__ __forceinline__ void staged_group_pf(int64_t row, const int64_t *s_ptr, double2 *s_prod,
                                                const int32_t *__restrict__ col, const double *__restrict__ val,
                                                const XS xs, double *__restrict__ y, int64_t n_rows,
                                                const ChunkRegs<R, NT> &pre)
{
    constexpr int RPB = kBlock / L;
    constexpr int CH = 2 * kBlock * R;
    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    const int64_t beg = s_ptr[g], end = s_ptr[g + 1];
    const int64_t blk_end = s_ptr[RPB];
    const double *prod = reinterpret_cast<const double *>(s_prod);
    double acc = 0.0;
    bool first = true;
    for (int64_t cb = chunk_start(s_ptr[0]); cb < blk_end; cb += CH) {
        const int64_t ce = cb + CH < blk_end ? cb + CH : blk_end;
        if (first) {
            pre.products_xs(xs, s_prod);
            first = false;
        } else {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int t = threadIdx.x + k * kBlock;
                const int64_t p = cb + 2 * (int64_t)t;
                double2 pr = {0.0, 0.0};
                if (p + 1 < ce) {
                    const double2 v = stream_load2<NT>(val + p);
                    const int2 c = stream_load2<NT>(col + p);
                    pr.x = v.x * xs(c.x);
                    pr.y = v.y * xs(c.y);
                } else if (p < ce) {
                    pr.x = stream_load<NT>(val + p) * xs(stream_load<NT>(col + p));
                }
                s_prod[t] = pr;
            }
        }
        __syncthreads();
        acc += slice_sum<L>(prod, beg > cb ? beg - cb : 0, (end < ce ? end : ce) - cb, lane);
        __syncthreads();
    }
    acc = group_sum<L>(acc);
    if (lane == 0 && row < n_rows)
        store_y(y + (row), acc);
    __syncthreads();
}

template <int L, int R, bool NT>
__global__ __launch_bounds__(kBlock) void csr_xwin_pf_kernel(
    int64_t n_rows, int64_t n_groups, int64_t gpw, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap)
{
    constexpr int RPB = kBlock / L;
    constexpr int CH = 2 * kBlock * R;
    extern __shared__ double s_x[];
    __shared__ int64_t s_ptr[RPB + 1];
    __shared__ double2 s_prod[kBlock * R];
    const int64_t nz = row_ptr[n_rows];
    const int64_t n_win = (n_groups + gpw - 1) / gpw;
    for (int64_t wi = blockIdx.x; wi < n_win; wi += gridDim.x) {
        const int64_t g_beg = wi * gpw;
        ChunkRegs<R, NT> pre;
        {
            const int64_t r0 = g_beg * RPB;
            const int64_t r1 = r0 + RPB < n_rows ? r0 + RPB : n_rows;
            const int64_t b0 = chunk_start(row_ptr[r0]);
            const int64_t e0 = row_ptr[r1];
            pre.issue(col, val, b0, b0 + CH < e0 ? b0 + CH : e0);
        }
        const int2 wnd = win[wi];
        const int32_t span = wnd.y - wnd.x + 1;
        const bool staged = span > 0 && span <= xcap;  // uniform per workgroup
        if (staged)
            for (int32_t i = threadIdx.x; i < span; i += kBlock)
                s_x[i] = x[wnd.x + i];
        const int64_t g_end = (wi + 1) * gpw < n_groups ? (wi + 1) * gpw : n_groups;
        for (int64_t grp = g_beg; grp < g_end; ++grp) {
            if (threadIdx.x <= RPB) {
                const int64_t r = grp * RPB + threadIdx.x;
                s_ptr[threadIdx.x] = row_ptr[r < n_rows ? r : n_rows];
            }
            __syncthreads();  // offsets (and, for the first group, the window) visible
            const int64_t row = grp * RPB + threadIdx.x / L;
            if (grp == g_beg) {
                if (staged)
                    staged_group_pf<L, R, NT>(row, s_ptr, s_prod, col, val, XWindow{s_x, wnd.x}, y, n_rows, pre);
                else
                    staged_group_pf<L, R, NT>(row, s_ptr, s_prod, col, val, XGlobal{x}, y, n_rows, pre);
            } else if (staged) {
                staged_group<L, R, NT, Col32<NT>, 0, XWindow>(row, s_ptr, s_prod, Col32<NT>{col}, val,
                                                              XWindow{s_x, wnd.x}, y, n_rows, nz);
            } else {
                staged_group<L, R, NT, Col32<NT>, 0, XGlobal>(row, s_ptr, s_prod, Col32<NT>{col}, val,
                                                              XGlobal{x}, y, n_rows, nz);
            }
        }
    }
}

// Variant 5: the persistent staged scheme, software-pipelined.  The value
// and column loads of the NEXT chunk (of this row group or of the block's
// next group) are issued right after the barrier that publishes the
// current chunk's products, so HBM keeps streaming while the L-lane
// groups reduce from LDS; variant 3 issued them only after its second
// barrier.  Row offsets are double-buffered in LDS and fetched two groups
// ahead.  Same products, same per-row summation order as variants 2/3,
// so the results are bit-identical to them.
template <int L, int R, bool NT>
__global__ __launch_bounds__(kBlock) void csr_pipelined_kernel(
    int64_t n_rows, int64_t n_groups, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y)
{
    constexpr int RPB = kBlock / L;
    constexpr int CH = 2 * kBlock * R;
    __shared__ int64_t s_ptr[2][RPB + 1];
    __shared__ double2 s_prod[kBlock * R];
    const double *prod = reinterpret_cast<const double *>(s_prod);
    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    const int64_t grid = gridDim.x;
    int64_t grp = blockIdx.x;
    if (grp >= n_groups)
        return;  // whole workgroup
    auto offsets = [&](int64_t gg) {
        const int64_t r = gg * RPB + threadIdx.x;
        return row_ptr[r < n_rows ? r : n_rows];
    };
    int64_t next = 0;  // offsets of group grp + grid, two groups ahead of use
    if (threadIdx.x <= RPB) {
        s_ptr[0][threadIdx.x] = offsets(grp);
        if (grp + grid < n_groups)
            next = offsets(grp + grid);
    }
    __syncthreads();
    int b = 0;
    int64_t beg, end, blk_end;
    auto start_group = [&]() {
        // the other buffer was last read before the previous barrier
        if (threadIdx.x <= RPB) {
            s_ptr[1 - b][threadIdx.x] = next;
            if (grp + 2 * grid < n_groups)
                next = offsets(grp + 2 * grid);
        }
        beg = s_ptr[b][g];
        end = s_ptr[b][g + 1];
        blk_end = s_ptr[b][RPB];
    };
    start_group();
    int64_t cb = chunk_start(s_ptr[b][0]);
    int64_t ce = cb + CH < blk_end ? cb + CH : blk_end;
    ChunkRegs<R, NT> regs;
    regs.issue(col, val, cb, ce);
    double acc = 0.0;
    for (;;) {
        regs.products(x, s_prod);
        __syncthreads();  // products (and the next group's offsets) visible
        const bool last = ce >= blk_end;
        int64_t ngrp = grp, ncb = 0, nce = 0;
        if (!last) {
            ncb = ce;
            nce = ncb + CH < blk_end ? ncb + CH : blk_end;
        } else {
            ngrp = grp + grid;
            if (ngrp < n_groups) {
                const int64_t nend = s_ptr[1 - b][RPB];
                ncb = chunk_start(s_ptr[1 - b][0]);
                nce = ncb + CH < nend ? ncb + CH : nend;
            }
        }
        if (ngrp < n_groups)
            regs.issue(col, val, ncb, nce);
        acc += slice_sum<L>(prod, beg > cb ? beg - cb : 0, (end < ce ? end : ce) - cb, lane);
        if (last) {
            acc = group_sum<L>(acc);
            const int64_t row = grp * RPB + g;
            if (lane == 0 && row < n_rows)
                store_y(y + (row), acc);
            acc = 0.0;
        }
        __syncthreads();  // s_prod free again
        if (ngrp >= n_groups)
            break;
        if (last) {
            grp = ngrp;
            b = 1 - b;
            start_group();
        }
        cb = ncb;
        ce = nce;
    }
}

static bool csr_pair_loads()
{
    static int cached = -1;
    if (cached < 0) {
        const char *s = getenv("SPMV_CSR_PAIR");
        cached = (s && s[0] == '0') ? 0 : 1;
    }
    return cached == 1;
}

// variant: 1 = direct (each L-lane group streams its own row),
//          2 = staged (the group's entry range streamed through LDS),
//          3 = staged, persistent workgroups with offset prefetch
static int csr_default_variant()
{
    static int cached = -1;
    if (cached < 0) {
        const char *s = getenv("SPMV_CSR_VARIANT");
        cached = (s && ((s[0] >= '1' && s[0] <= '3') || s[0] == '5')) ? s[0] - '0' : 3;
    }
    return cached;
}

// Chunk size of the staged CSR kernels for a matrix: R = 3 (1,536-entry
// chunks) unless R = 4 (2,048) cuts a row group of 256/L rows of the mean
// length into FEWER chunks — every chunk is a memory round trip and two
// barriers.  Cant-like (L = 4, 64 rows x 64.2 = 4,107 entries): 3 chunks
// either way, R = 3 (measured 0.2591 vs 0.2639 ms).  Banded (L = 2, 128
// rows x 16 = 2,048): 1 chunk with R = 4 against 2 with R = 3 (configs[4]
// measured 4.50 ms with R = 3).  Every staged CSR path uses this rule, so
// their chunk boundaries, hence their bits, stay identical.
static int csr_auto_rounds(int64_t n_rows, int64_t nnz, int L)
{
    if (n_rows <= 0 || L <= 0)
        return kStageRoundsDefault;
    const double eg = (double)(kBlock / L) * ((double)nnz / (double)n_rows);
    const int64_t c3 = (int64_t)((eg + 1535.0) / 1536.0), c4 = (int64_t)((eg + 2047.0) / 2048.0);
    return c4 < c3 ? 4 : 3;
}

// SPMV_CSR_STAGE_ROUNDS in {2,3,4,5,8} overrides the rule (tuning knob,
// read per call so a sweep can change it inside one process)
static int csr_stage_rounds(int64_t n_rows, int64_t nnz, int L)
{
    const char *s = getenv("SPMV_CSR_STAGE_ROUNDS");
    const int r = s ? atoi(s) : csr_auto_rounds(n_rows, nnz, L);
    return (r == 2 || r == 3 || r == 4 || r == 5 || r == 8) ? r : csr_auto_rounds(n_rows, nnz, L);
}

static int cu_count()
{
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
    return n;
}

// Resident workgroups per CU for a persistent kernel, from the occupancy
// calculator (VGPRs, LDS and the wave limit together), at most 8.  Sizing
// the grid by hand once launched 8 per CU of a kernel that fit only 7,
// and the 256 stragglers ran as a second wave.
template <typename K>
static int64_t persistent_grid(K kernel, int64_t groups, size_t dyn_lds = 0)
{
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, dyn_lds) != hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    if (per_cu > 8)
        per_cu = 8;
    const int64_t grid = (int64_t)cu_count() * per_cu;
    return grid < groups ? grid : groups;
}

// SPMV_CSR_BATCH = 0 / 1 / 2 selects the stage's load schedule (see
// staged_group); read per call so a sweep can flip it in-process
static int csr_batch_mode(int dflt)
{
    const char *s = getenv("SPMV_CSR_BATCH");
    return (s && s[0] >= '0' && s[0] <= '2') ? s[0] - '0' : dflt;
}

template <int L, int R, bool NT, typename Cols, int BATCH>
static void launch_persistent_cols(const spmv_dims &d, const int64_t *row_ptr, const Cols cols,
                                   const double *val, const double *x, double *y, int64_t groups)
{
    static const int64_t per = persistent_grid(csr_staged_persistent_kernel<L, R, NT, Cols, BATCH>, INT64_MAX);
    const int64_t grid = per < groups ? per : groups;
    hipLaunchKernelGGL((csr_staged_persistent_kernel<L, R, NT, Cols, BATCH>), dim3((unsigned)grid),
                       dim3(kBlock), 0, (hipStream_t)d.stream, d.n_rows, groups, row_ptr, cols, val, x, y);
}

template <int L, int R, bool NT>
static void launch_persistent(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                              const double *val, const double *x, double *y, int variant,
                              int64_t groups)
{
    const hipStream_t st = (hipStream_t)d.stream;
    using K = Col32<NT>;
    if (variant == 5) {
        static const int64_t per = persistent_grid(csr_pipelined_kernel<L, R, NT>, INT64_MAX);
        const int64_t grid = per < groups ? per : groups;
        hipLaunchKernelGGL((csr_pipelined_kernel<L, R, NT>), dim3((unsigned)grid), dim3(kBlock), 0, st,
                           d.n_rows, groups, row_ptr, col, val, x, y);
        return;
    }
    switch (csr_batch_mode(kCsrBatchDefault)) {
    case 1: launch_persistent_cols<L, R, NT, K, 1>(d, row_ptr, K{col}, val, x, y, groups); break;
    case 2: launch_persistent_cols<L, R, NT, K, 2>(d, row_ptr, K{col}, val, x, y, groups); break;
    default: launch_persistent_cols<L, R, NT, K, 0>(d, row_ptr, K{col}, val, x, y, groups); break;
    }
}

// compressed-index CSR: the persistent staged kernel with Col16 columns
template <int L, bool NT>
static void launch_csr16(const spmv_dims &d, const int64_t *row_ptr, const Col16<NT> cols,
                         const double *val, const double *x, double *y)
{
    constexpr int RPB = kBlock / L;
    const int64_t groups = (d.n_rows + RPB - 1) / RPB;
    const bool r4 = csr_stage_rounds(d.n_rows, d.nnz, L) == 4;  // R = 3 or 4 (the rule)
    switch (csr_batch_mode(kCsrBatchDefault)) {
    case 1:
        if (r4) launch_persistent_cols<L, 4, NT, Col16<NT>, 1>(d, row_ptr, cols, val, x, y, groups);
        else launch_persistent_cols<L, 3, NT, Col16<NT>, 1>(d, row_ptr, cols, val, x, y, groups);
        break;
    case 2:
        if (r4) launch_persistent_cols<L, 4, NT, Col16<NT>, 2>(d, row_ptr, cols, val, x, y, groups);
        else launch_persistent_cols<L, 3, NT, Col16<NT>, 2>(d, row_ptr, cols, val, x, y, groups);
        break;
    default:
        if (r4) launch_persistent_cols<L, 4, NT, Col16<NT>, 0>(d, row_ptr, cols, val, x, y, groups);
        else launch_persistent_cols<L, 3, NT, Col16<NT>, 0>(d, row_ptr, cols, val, x, y, groups);
        break;
    }
}

template <int L, int R>
static void launch_staged(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                          const double *val, const double *x, double *y, int variant)
{
    constexpr int RPB = kBlock / L;
    const int64_t groups = (d.n_rows + RPB - 1) / RPB;
    if (variant == 3 || variant == 5) {
        if (stream_nt(kCsrStreamNtDefault))
            launch_persistent<L, R, true>(d, row_ptr, col, val, x, y, variant, groups);
        else
            launch_persistent<L, R, false>(d, row_ptr, col, val, x, y, variant, groups);
    } else {
        hipLaunchKernelGGL((csr_staged_kernel<L, R>), dim3((unsigned)groups), dim3(kBlock), 0,
                           (hipStream_t)d.stream, d.n_rows, row_ptr, col, val, x, y,
                           xcd_remap_enabled() ? 1 : 0);
    }
}

template <int L>
static void launch_csr(const spmv_dims &d, const int64_t *row_ptr,
                       const int32_t *col, const double *val, const double *x,
                       double *y, int variant)
{
    constexpr int RPB = kBlock / L;
    const int64_t blocks = (d.n_rows + RPB - 1) / RPB;
    const int remap = xcd_remap_enabled() ? 1 : 0;
    const hipStream_t st = (hipStream_t)d.stream;
    if (variant >= 2) {
        switch (csr_stage_rounds(d.n_rows, d.nnz, L)) {
        case 2: launch_staged<L, 2>(d, row_ptr, col, val, x, y, variant); break;
        case 3: launch_staged<L, 3>(d, row_ptr, col, val, x, y, variant); break;
        case 4: launch_staged<L, 4>(d, row_ptr, col, val, x, y, variant); break;
        case 5: launch_staged<L, 5>(d, row_ptr, col, val, x, y, variant); break;
        case 8: launch_staged<L, 8>(d, row_ptr, col, val, x, y, variant); break;
        default: launch_staged<L, 4>(d, row_ptr, col, val, x, y, variant); break;
        }
    } else if (csr_pair_loads()) {
        hipLaunchKernelGGL((csr_vector_kernel<L, true>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, st, d.n_rows, row_ptr, col, val, x, y, remap);
    } else {
        hipLaunchKernelGGL((csr_vector_kernel<L, false>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, st, d.n_rows, row_ptr, col, val, x, y, remap);
    }
}

}  // namespace spmv

using namespace spmv;

extern "C" int spmv_csr_auto_lanes(int64_t n_rows, int64_t nnz)
{
    // Lanes per row for the default (staged) variant: about one lane per 16
    // entries of the mean row, a power of two in [2, 64].  The reduction
    // reads LDS, so a few lanes per row suffice, and more rows per group
    // amortise the group's offset fetch (mean 64 -> L = 4: 0.320 ms vs
    // 0.328 ms at L = 8 on the cant-like batch, profiles/round1_sweep.md).
    // The direct variant uses twice this (L = 8: 0.353 ms vs 0.383 at 16).
    double mean = n_rows > 0 ? (double)nnz / (double)n_rows : 0.0;
    int L = 2;
    while (L < 64 && (double)(2 * L) * 16.0 <= mean * 1.5)
        L *= 2;
    return L;
}

extern "C" int spmv_csr_run_variant(spmv_dims d, const int64_t *row_ptr,
                                    const int32_t *col, const double *val,
                                    const double *x, double *y, int lanes_per_row,
                                    int variant)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run: negative size");
    if (variant < 0 || variant > 5 || variant == 4)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run: variant must be 0..3 or 5 (4 = spmv_csr_run_tiled)");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if ((d.n_rows + 1) / 2 > (int64_t)INT32_MAX * 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run: too many rows");
    SPMV_GUARD(d);
    const int v = variant ? variant : csr_default_variant();
    int L = lanes_per_row;
    if (L <= 0) {
        L = spmv_csr_auto_lanes(d.n_rows, d.nnz);
        if (v == 1 && L < 64)
            L *= 2;
    }
    switch (L) {
    case 2: launch_csr<2>(d, row_ptr, col, val, x, y, v); break;
    case 4: launch_csr<4>(d, row_ptr, col, val, x, y, v); break;
    case 8: launch_csr<8>(d, row_ptr, col, val, x, y, v); break;
    case 16: launch_csr<16>(d, row_ptr, col, val, x, y, v); break;
    case 32: launch_csr<32>(d, row_ptr, col, val, x, y, v); break;
    case 64: launch_csr<64>(d, row_ptr, col, val, x, y, v); break;
    default:
        return fail_msg(SPMV_OTHER_ERROR,
                        "spmv_csr_run: lanes_per_row must be 0 or a power of two in [2,64]");
    }
    SPMV_CHECK_LAUNCH("csr kernel");
    return SPMV_SUCCESS;
}

extern "C" int spmv_csr_run(spmv_dims d, const int64_t *row_ptr,
                            const int32_t *col, const double *val,
                            const double *x, double *y, int lanes_per_row)
{
    return spmv_csr_run_variant(d, row_ptr, col, val, x, y, lanes_per_row, 0);
}

namespace spmv {

constexpr int32_t kCsrXwinCap = 2048;  // 16 KiB of LDS: 32 KiB per workgroup with the stage
constexpr int32_t kCsrXwinRows = 128;  // rows per x window (rows_per_window = 0): 0.2836 ms vs 0.2907 (64), 0.2938 (256), 0.2964 (512), 0.3397 (1024)

// SPMV_CSR_XWIN_PF: 1 = csr_xwin_pf_kernel (first chunk prefetched before
// the window copy), 0 = csr_xwin_kernel.  Read on every call (sweeps).
static bool csr_xwin_prefetch()
{
    const char *s = getenv("SPMV_CSR_XWIN_PF");
    return s && s[0] == '1';
}

// Load schedule of csr_xwin_kernel (its MODE): SPMV_CSR_XWIN_MODE=0..3,
// read on every call (A/B runs, tools/ab_env.py); default kCsrXwinMode.
// MODE 3 with XCD-contiguous windows: 0.2644 ms vs 0.2678 (MODE 3, round
// robin), 0.2701 (MODE 0, remap) and 0.2717 (MODE 0, round robin), five
// interleaved rounds on one box (profiles/round2/ab_csr_xwin.log)
constexpr int kCsrXwinMode = 3;
constexpr bool kCsrXwinRemap = true;
// pairs per lane per chunk of the x-window kernel: csr_stage_rounds (the
// chunk-count rule; R = 3 on the cant batch, 4 on the banded matrix)
// Without the knob: MODE 3 when a window's entries make more than one
// chunk (there is a next chunk to pipeline: cant-like, 128 rows x 64.2 =
// 8,214 entries in 1,536-entry chunks), else MODE 0 — a one-chunk window
// gains nothing from the pipeline and its 86 instead of 64 VGPRs cost
// workgroups per CU (banded, 128 rows x 16 = one 2,048-entry chunk: 0.765
// ms MODE 0 vs 0.815 ms MODE 3, profiles/round2/ab_banded.log).
static int csr_xwin_mode(int64_t n_rows, int64_t nnz, int64_t rows_per_window, int R)
{
    const char *s = getenv("SPMV_CSR_XWIN_MODE");
    if (s && s[0] >= '0' && s[0] <= '5' && s[1] == 0)
        return s[0] - '0';
    const double ew = n_rows > 0 ? (double)rows_per_window * ((double)nnz / (double)n_rows) : 0.0;
    return ew > 2.0 * kBlock * R ? kCsrXwinMode : 0;
}

// XCD-contiguous windows pay when neighbouring windows share x lines: the
// widest window spans several times its rows (cant-like: 678 columns for 128
// rows; on), not when each row reads a narrow band (banded: 143 columns for
// 128 rows; 0.765 vs 0.782 ms with remap, off)
static bool csr_xwin_remap_rule(int32_t xcap, int64_t rows_per_window)
{
    return xwin_remap(kCsrXwinRemap && (int64_t)xcap > 2 * rows_per_window);
}

// SPMV_CSR_XWIN_PRE=1: MODE 3 issues the first chunk before the window copy
// (read per call; A/B knob).  Off: the prefetched registers live across the
// copy (100 VGPRs instead of 78, 4 instead of 6 workgroups per CU) and it
// measured 0.2646 vs 0.2589 ms (profiles/round2/ab_csr_xwin_pre.log)
constexpr bool kCsrXwinPre = false;
static bool csr_xwin_pre()
{
    const char *s = getenv("SPMV_CSR_XWIN_PRE");
    return s && (s[0] == '0' || s[0] == '1') ? s[0] == '1' : kCsrXwinPre;
}

// SPMV_CSR_XWIN_R in {2,3,4,6,8}: value/column pairs per lane per chunk of
// the MODE 3 kernel (non-temporal loads only; sweep knob, read per call);
// 0 = the launcher's R
static int csr_xwin_rounds()
{
    const char *s = getenv("SPMV_CSR_XWIN_R");
    return s ? atoi(s) : 0;
}

// dynamic LDS of csr_xwin_kernel: the x window, and from MODE 1 on the
// window's row offsets behind it
static size_t csr_xwin_lds(int mode, int32_t xcap, int64_t gpw, int rpb)
{
    return ((size_t)xcap + (mode > 0 ? (size_t)(gpw * rpb + 1) : 0)) * sizeof(double);
}

// rows per x window: a multiple of the row group (256/L rows), default
// kCsrXwinRows but at least two groups, so a window whose groups are one
// chunk each still has a next chunk to pipeline (MODE 3): the banded matrix
// (L = 2, 128-row groups of 2,048 entries) 0.7534 ms with one-group windows
// (MODE 0) against 0.7261 ms with two (profiles/round2/ab_banded3.log);
// explicit rows_per_window: at least one group.  Same chunks, same bits.
static int64_t csr_xwin_gpw(int L, int32_t rows_per_window)
{
    const int64_t rpb = kBlock / L;
    const int64_t rows = rows_per_window > 0 ? rows_per_window : kCsrXwinRows;
    const int64_t g = (rows + rpb - 1) / rpb;
    return g < (rows_per_window > 0 ? 1 : 2) ? (rows_per_window > 0 ? 1 : 2) : g;
}

// SPMV_CSR_LDS_PAD=<bytes>: extra dynamic LDS per workgroup of the x-window
// kernels (an occupancy sweep knob: fewer workgroups per CU); default 0
static size_t csr_lds_pad()
{
    const char *s = getenv("SPMV_CSR_LDS_PAD");
    return s ? (size_t)atol(s) : 0;
}

// SPMV_CSR_XSTREAM=1 / 0: csr_xstream_kernel for x windows of one row group
// (read per call; default kCsrXstream)
constexpr bool kCsrXstream = false;
static bool csr_xstream()
{
    const char *s = getenv("SPMV_CSR_XSTREAM");
    return (s && (s[0] == '0' || s[0] == '1')) ? s[0] == '1' : kCsrXstream;
}

// win: one column range per row group; the ring is the smallest power of
// two >= xcap (at least 64 entries)
template <int L, int R, bool NT, typename Cols, typename V>
static void launch_csr_xstream(const spmv_dims &d, const int64_t *row_ptr, const Cols cols, const V *val,
                               const double *x, double *y, const int2 *win, int32_t xcap)
{
    constexpr int RPB = kBlock / L;
    const int64_t groups = (d.n_rows + RPB - 1) / RPB;
    int lg = 6;
    while ((1 << lg) < xcap)
        ++lg;
    const int32_t cap = 1 << lg;
    const size_t lds = (size_t)cap * sizeof(double) + csr_lds_pad();
    // (capping its VGPRs for 6 waves per SIMD spills 13 registers)
    static int64_t resident[16] = {};  // per ring size (the occupancy calculator once per size)
    if (resident[lg] == 0 || csr_lds_pad() != 0)
        resident[lg] = persistent_grid(csr_xstream_kernel<L, R, NT, V, Cols>, INT64_MAX, lds);
    const int64_t grid = resident[lg] < groups ? resident[lg] : groups;
    hipLaunchKernelGGL((csr_xstream_kernel<L, R, NT, V, Cols>), dim3((unsigned)grid), dim3(kBlock), lds,
                       (hipStream_t)d.stream, d.n_rows, groups, row_ptr, cols, val, x, y, win, cap);
}

template <int L, int R, bool NT, typename Cols, typename V = double>
static void launch_csr_xwin(const spmv_dims &d, const int64_t *row_ptr, const Cols cols,
                            const V *val, const double *x, double *y, const int2 *win, int32_t xcap,
                            int64_t gpw)
{
    constexpr int RPB = kBlock / L;
    if (gpw == 1 && csr_xstream()) {
        launch_csr_xstream<L, R, NT, Cols, V>(d, row_ptr, cols, val, x, y, win, xcap);
        return;
    }
    const int64_t groups = (d.n_rows + RPB - 1) / RPB;
    const int64_t n_win = (groups + gpw - 1) / gpw;
    int mode = csr_xwin_mode(d.n_rows, d.nnz, gpw * RPB, R);
    // a very tall window's offsets would not fit beside the x range in the
    // 64 KiB of dynamic LDS: MODE 0 stages them per row group instead
    if (mode > 0 && csr_xwin_lds(mode, xcap, gpw, RPB) + sizeof(double2) * kBlock * R * 2 > 64 * 1024)
        mode = 0;
    const size_t lds = csr_xwin_lds(mode, xcap, gpw, RPB) + csr_lds_pad();
    // one workgroup per window (the dispatcher balances) unless
    // SPMV_CSR_XWIN_PERSISTENT=1 (resident workgroups walk the windows)
    const char *ps = getenv("SPMV_CSR_XWIN_PERSISTENT");
    const int64_t grid = (ps && ps[0] == '1') ? persistent_grid(csr_xwin_kernel<L, R, NT, V, 0, false, Cols>, n_win, lds) : n_win;
    if (grid > INT32_MAX)
        return;
    const int remap = csr_xwin_remap_rule(xcap, gpw * RPB) ? 1 : 0;
    const hipStream_t st = (hipStream_t)d.stream;
    constexpr bool kFp64 = std::is_same<V, double>::value;  // fp32 values: modes 0 and 3 only
    if (!kFp64 && mode != 0)
        mode = 3;
    if constexpr (kFp64 && std::is_same<Cols, Col32<NT>>::value) {  // the round-1 prefetch kernel reads int32 columns
        if (csr_xwin_prefetch()) {
            const size_t lds0 = (size_t)xcap * sizeof(double);
            hipLaunchKernelGGL((csr_xwin_pf_kernel<L, R, NT>), dim3((unsigned)grid), dim3(kBlock), lds0, st, d.n_rows,
                               groups, gpw, row_ptr, cols.col, val, x, y, win, xcap);
            return;
        }
    }
    switch (mode) {
    case 0:
        hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 0, false, Cols>), dim3((unsigned)grid), dim3(kBlock), lds, st,
                           d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
        break;
    case 1:
        if constexpr (kFp64)
        hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 1, false, Cols>), dim3((unsigned)grid), dim3(kBlock), lds, st,
                           d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
        break;
    case 2:
        if constexpr (kFp64)
        hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 2, false, Cols>), dim3((unsigned)grid), dim3(kBlock), lds, st,
                           d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
        break;
    case 3:
        if constexpr (NT && kFp64) {  // SPMV_CSR_XWIN_R: pairs per lane per chunk (sweep knob)
            const int rr = csr_xwin_rounds();
            if (rr != 0 && rr != R) {
                const size_t l2 = lds;  // the chunk buffer is static LDS
#define SPMV_XWIN_R(RR)                                                                                      \
    hipLaunchKernelGGL((csr_xwin_kernel<L, RR, NT, V, 3, false, Cols>), dim3((unsigned)grid), dim3(kBlock), l2, st, \
                       d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap)
                switch (rr) {
                case 2: SPMV_XWIN_R(2); return;
                case 3: SPMV_XWIN_R(3); return;
                case 4: SPMV_XWIN_R(4); return;
                case 6: SPMV_XWIN_R(6); return;
                case 8: SPMV_XWIN_R(8); return;
                default: break;
                }
#undef SPMV_XWIN_R
            }
        }
        if (kFp64 && csr_xwin_pre())
            hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 3, kFp64, Cols>), dim3((unsigned)grid), dim3(kBlock), lds,
                               st, d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
        else
            hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 3, false, Cols>), dim3((unsigned)grid), dim3(kBlock), lds, st,
                               d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
        break;
    case 4:
        if constexpr (kFp64)
        hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 4, false, Cols>), dim3((unsigned)grid), dim3(kBlock), lds, st,
                           d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
        break;
    case 5:
        if constexpr (!kFp64) {
            break;
        } else if (gpw == 1 || gpw == 2 || gpw == 4) {
            const bool r3 = NT && csr_xwin_rounds() == 3 && R != 3;  // SPMV_CSR_XWIN_R (sweep knob)
#define SPMV_FLAT(RR, MM)                                                                                     \
    hipLaunchKernelGGL((csr_xwin_kernel<L, RR, NT, V, MM, false, Cols>), dim3((unsigned)grid), dim3(kBlock), lds, st, \
                       d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap)
            if (gpw == 1) {
                if (r3) SPMV_FLAT(3, 5); else SPMV_FLAT(R, 5);
            } else if (gpw == 2) {
                if (r3) SPMV_FLAT(3, 6); else SPMV_FLAT(R, 6);
            } else {
                if (r3) SPMV_FLAT(3, 7); else SPMV_FLAT(R, 7);
            }
#undef SPMV_FLAT
        } else {
            hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 3, false, Cols>), dim3((unsigned)grid), dim3(kBlock), lds, st,
                               d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
        }
        break;
    }
}

template <int L>
static void launch_csr_vector_xwin(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                                   const double *val, const double *x, double *y, const int2 *win,
                                   int32_t xcap, int64_t gpw)
{
    constexpr int RPB = kBlock / L;
    const int64_t blocks = (d.n_rows + RPB - 1) / RPB;
    hipLaunchKernelGGL((csr_vector_xwin_kernel<L>), dim3((unsigned)blocks), dim3(kBlock),
                       (size_t)xcap * sizeof(double), (hipStream_t)d.stream, d.n_rows, gpw, row_ptr, col, val, x,
                       y, win, xcap);
}

// SPMV_CSR_XWIN_DIRECT=1: the x-window run uses the direct (row-walking)
// kernel instead of the staged one (read per call: sweep knob)
static bool csr_xwin_direct()
{
    const char *s = getenv("SPMV_CSR_XWIN_DIRECT");
    return s && s[0] == '1';
}

}  // namespace spmv

extern "C" size_t spmv_csr_xwin_bytes(int64_t n_rows, int64_t nnz, int lanes_per_row, int32_t rows_per_window)
{
    const int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(n_rows, nnz);
    if (L < 2 || L > 64 || (L & (L - 1)) || n_rows <= 0 || rows_per_window < 0)
        return 0;
    const int64_t rpw = csr_xwin_gpw(L, rows_per_window) * (kBlock / L);
    return (size_t)((n_rows + rpw - 1) / rpw) * sizeof(int2);
}

extern "C" int spmv_csr_xwin_build(spmv_dims d, const int64_t *row_ptr, const int32_t *col,
                                   int lanes_per_row, int32_t rows_per_window, void *win, size_t win_bytes,
                                   int32_t *xcap)
{
    if (d.n_rows < 0 || d.nnz < 0 || !xcap || rows_per_window < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_xwin_build: bad arguments");
    *xcap = 0;
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    const int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    const size_t need = spmv_csr_xwin_bytes(d.n_rows, d.nnz, L, rows_per_window);
    if (need == 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_xwin_build: lanes_per_row must be 0 or a power of two in [2,64]");
    if (!win || win_bytes < need)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_xwin_build: window buffer too small");
    SPMV_GUARD(d);
    const int64_t rpw = csr_xwin_gpw(L, rows_per_window) * (kBlock / L);
    const int64_t n_win = (d.n_rows + rpw - 1) / rpw;
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(csr_window_kernel, dim3((unsigned)n_win), dim3(kBlock), 0, st, d.n_rows, rpw, row_ptr,
                       col, (int2 *)win);
    SPMV_CHECK_LAUNCH("csr_window_kernel");
    int2 *h = (int2 *)malloc(need);
    if (!h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_xwin_build: out of host memory");
    hipError_t e = hipMemcpyAsync(h, win, need, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        free(h);
        return fail(SPMV_PROGRAM_ERROR, "spmv_csr_xwin_build: copy windows", e);
    }
    int32_t best = 0;
    for (int64_t g = 0; g < n_win; ++g) {
        const int64_t span = (int64_t)h[g].y - h[g].x + 1;
        if (span <= kCsrXwinCap && span > best)
            best = (int32_t)span;
    }
    free(h);
    *xcap = best;
    return SPMV_SUCCESS;
}

extern "C" int spmv_csr_run_xwin(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                                 const double *x, double *y, int lanes_per_row, int32_t rows_per_window,
                                 const void *win, int32_t xcap)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || rows_per_window < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_xwin: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (!win || xcap < 0 || xcap > kCsrXwinCap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_xwin: bad window arguments");
    SPMV_GUARD(d);
    const int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    if (L < 2 || L > 64 || (L & (L - 1)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_xwin: lanes_per_row must be 0 or a power of two in [2,64]");
    const int64_t gpw = csr_xwin_gpw(L, rows_per_window);
    {
        const char *pr = getenv("SPMV_CSR_STREAM_PROBE");
        if (pr && pr[0] == 'P' && d.nnz >= 2) {  // timing probes P1..P5 (y wrong)
            const unsigned gt = (unsigned)((d.nnz + 8191) / 8192), gw = (unsigned)((d.n_rows + 127) / 128);
            const hipStream_t st = (hipStream_t)d.stream;
            switch (pr[1]) {
            case '2': hipLaunchKernelGGL((csr_stream_probe_kernel<2>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case '3': hipLaunchKernelGGL((csr_stream_probe_kernel<3>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case '4': hipLaunchKernelGGL((csr_stream_probe_kernel<4>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case '5': hipLaunchKernelGGL((csr_stream_probe_kernel<5>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case '6': hipLaunchKernelGGL((csr_stream_probe_kernel<6>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case '7': hipLaunchKernelGGL((csr_stream_probe_kernel<7>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case '8': hipLaunchKernelGGL((csr_stream_probe_kernel<8>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case '9': hipLaunchKernelGGL((csr_stream_probe_kernel<9>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'A': hipLaunchKernelGGL((csr_stream_probe_kernel<10>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'B': hipLaunchKernelGGL((csr_stream_probe_kernel<11>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'C': hipLaunchKernelGGL((csr_stream_probe_kernel<12>), dim3((gw + 1) / 2), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'D': hipLaunchKernelGGL((csr_stream_probe_kernel<13>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'E': hipLaunchKernelGGL((csr_stream_probe_kernel<14>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'F': hipLaunchKernelGGL((csr_stream_probe_kernel<15>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'G': hipLaunchKernelGGL((csr_stream_probe_kernel<16>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'H': hipLaunchKernelGGL((csr_stream_probe_kernel<17>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'I': hipLaunchKernelGGL((csr_stream_probe_kernel<18>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            case 'J': hipLaunchKernelGGL((csr_stream_probe_kernel<19>), dim3(gw), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            default: hipLaunchKernelGGL((csr_stream_probe_kernel<1>), dim3(gt), dim3(kBlock), 0, st, row_ptr, d.n_rows, val, col, d.nnz, y); break;
            }
            SPMV_CHECK_LAUNCH("csr_stream_probe_kernel");
            return SPMV_SUCCESS;
        }
    }
    const bool nt = stream_nt(kCsrXwinNtDefault);
    const bool r4 = csr_stage_rounds(d.n_rows, d.nnz, L) == 4;  // R = 3 or 4 (the rule)
    const int2 *w = (const int2 *)win;
    const bool direct = csr_xwin_direct();
#define SPMV_XWIN(LL)                                                                          \
    (direct ? launch_csr_vector_xwin<LL>(d, row_ptr, col, val, x, y, w, xcap, gpw)             \
     : nt   ? (r4 ? launch_csr_xwin<LL, 4, true>(d, row_ptr, Col32<true>{col}, val, x, y, w, xcap, gpw)   \
                  : launch_csr_xwin<LL, 3, true>(d, row_ptr, Col32<true>{col}, val, x, y, w, xcap, gpw))  \
            : (r4 ? launch_csr_xwin<LL, 4, false>(d, row_ptr, Col32<false>{col}, val, x, y, w, xcap, gpw) \
                  : launch_csr_xwin<LL, 3, false>(d, row_ptr, Col32<false>{col}, val, x, y, w, xcap, gpw)))
    switch (L) {
    case 2: SPMV_XWIN(2); break;
    case 4: SPMV_XWIN(4); break;
    case 8: SPMV_XWIN(8); break;
    case 16: SPMV_XWIN(16); break;
    case 32: SPMV_XWIN(32); break;
    default: SPMV_XWIN(64); break;
    }
#undef SPMV_XWIN
    SPMV_CHECK_LAUNCH("csr_xwin_kernel");
    return SPMV_SUCCESS;
}

extern "C" int spmv_csr16_run(spmv_dims d, const int64_t *row_ptr, const int32_t *blk_base,
                              const uint16_t *col_off, const int32_t *col_esc, const double *val,
                              const double *x, double *y, int lanes_per_row)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr16_run: negative size");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (d.nnz > 0 && (!blk_base || !col_off))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr16_run: missing index arrays");
    SPMV_GUARD(d);
    const int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    const bool nt = stream_nt(kCsrStreamNtDefault);
#define SPMV_CSR16(LL)                                                                          \
    (nt ? launch_csr16<LL, true>(d, row_ptr, Col16<true>{blk_base, col_off, col_esc}, val, x, y) \
        : launch_csr16<LL, false>(d, row_ptr, Col16<false>{blk_base, col_off, col_esc}, val, x, y))
    switch (L) {
    case 2: SPMV_CSR16(2); break;
    case 4: SPMV_CSR16(4); break;
    case 8: SPMV_CSR16(8); break;
    case 16: SPMV_CSR16(16); break;
    case 32: SPMV_CSR16(32); break;
    case 64: SPMV_CSR16(64); break;
    default:
        return fail_msg(SPMV_OTHER_ERROR,
                        "spmv_csr16_run: lanes_per_row must be 0 or a power of two in [2,64]");
    }
#undef SPMV_CSR16
    SPMV_CHECK_LAUNCH("csr16 kernel");
    return SPMV_SUCCESS;
}

// CSR16 on the x-window pipeline: the same kernel, load schedule and chunks
// as spmv_csr_run_xwin with the columns decoded from the 16-bit offsets
// (escaped blocks from their int32 copy), so y is bit-identical to it.
// Windows from spmv_csr_xwin_build over the CSR's int32 columns (the same
// column values) with the same lanes_per_row and rows_per_window.
extern "C" int spmv_csr16_run_xwin(spmv_dims d, const int64_t *row_ptr, const int32_t *blk_base,
                                   const uint16_t *col_off, const int32_t *col_esc, const double *val,
                                   const double *x, double *y, int lanes_per_row, int32_t rows_per_window,
                                   const void *win, int32_t xcap)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || rows_per_window < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr16_run_xwin: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (d.nnz > 0 && (!blk_base || !col_off))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr16_run_xwin: missing index arrays");
    if (!win || xcap < 0 || xcap > kCsrXwinCap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr16_run_xwin: bad window arguments");
    SPMV_GUARD(d);
    const int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    if (L < 2 || L > 64 || (L & (L - 1)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr16_run_xwin: lanes_per_row must be 0 or a power of two in [2,64]");
    const int64_t gpw = csr_xwin_gpw(L, rows_per_window);
    const bool nt = stream_nt(kCsrXwinNtDefault);
    const bool r4 = csr_stage_rounds(d.n_rows, d.nnz, L) == 4;
    const int2 *w = (const int2 *)win;
#define SPMV_XWIN16(LL)                                                                                           \
    do {                                                                                                          \
        if (nt) {                                                                                                 \
            const Col16<true> cs{blk_base, col_off, col_esc};                                                     \
            if (r4) launch_csr_xwin<LL, 4, true>(d, row_ptr, cs, val, x, y, w, xcap, gpw);                        \
            else launch_csr_xwin<LL, 3, true>(d, row_ptr, cs, val, x, y, w, xcap, gpw);                           \
        } else {                                                                                                  \
            const Col16<false> cs{blk_base, col_off, col_esc};                                                    \
            if (r4) launch_csr_xwin<LL, 4, false>(d, row_ptr, cs, val, x, y, w, xcap, gpw);                       \
            else launch_csr_xwin<LL, 3, false>(d, row_ptr, cs, val, x, y, w, xcap, gpw);                          \
        }                                                                                                         \
    } while (0)
    switch (L) {
    case 2: SPMV_XWIN16(2); break;
    case 4: SPMV_XWIN16(4); break;
    case 8: SPMV_XWIN16(8); break;
    case 16: SPMV_XWIN16(16); break;
    case 32: SPMV_XWIN16(32); break;
    default: SPMV_XWIN16(64); break;
    }
#undef SPMV_XWIN16
    SPMV_CHECK_LAUNCH("csr_xwin_kernel (16-bit columns)");
    return SPMV_SUCCESS;
}

extern "C" size_t spmv_csr_tiled_ws_bytes(int64_t n_rows, int64_t nnz)
{
    (void)n_rows;
    // sized for the smallest tile the run may pick
    const int64_t tiles = nnz > 0 ? (nnz + csr_tiled_tile_min() - 1) / csr_tiled_tile_min() : 0;
    // carry_val[tiles] f64, own_lo[tiles+1] i32, carry_row[tiles] i32
    return (size_t)(8 * tiles + 4 * (tiles + 1) + 4 * tiles + 16);
}

extern "C" int spmv_csr_run_tiled(spmv_dims d, const int64_t *row_ptr, const int32_t *col,
                                  const double *val, const double *x, double *y, void *ws,
                                  size_t ws_bytes)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    if (d.nnz == 0) {
        hipError_t e = hipMemsetAsync(y, 0, (size_t)d.n_rows * sizeof(double), (hipStream_t)d.stream);
        return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "memset y", e);
    }
    if (!ws || ws_bytes < spmv_csr_tiled_ws_bytes(d.n_rows, d.nnz))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled: workspace too small");
    const int64_t tiles = (d.nnz + csr_tiled_tile(d.n_rows, d.nnz) - 1) / csr_tiled_tile(d.n_rows, d.nnz);
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled: grid too large");
    double *carry_val = (double *)ws;
    int32_t *own_lo = (int32_t *)(carry_val + tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    int rc = launch_csr_tiled(d, row_ptr, col, val, x, y, own_lo, carry_row, carry_val);
    if (rc != SPMV_SUCCESS)
        return rc;
    return launch_carry(tiles, carry_row, carry_val, y, (hipStream_t)d.stream);
}

extern "C" size_t spmv_csr_hot_ws_bytes(int64_t n_rows, int64_t nnz, int64_t H)
{
    return (size_t)(H > 0 ? H : 0) * sizeof(double) + spmv_csr_tiled_ws_bytes(n_rows, nnz);
}

// Entry-balanced CSR whose column ids >= n_cols name the hot-column table
// (host spmv_hot_columns): xh[i] = x[hot[i]] is gathered first, then the
// tiled kernel reads the H hottest x values from that compact, L2-resident
// table.  Same products in the same order as spmv_csr_run_tiled on the
// un-renumbered columns, so y is bit-identical to it.
extern "C" int spmv_csr_run_tiled_hot(spmv_dims d, const int64_t *row_ptr, const int32_t *col_hot,
                                      const double *val, const double *x, double *y, int64_t H,
                                      const int32_t *hot, const int32_t *own_lo_plan, void *ws,
                                      size_t ws_bytes)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || d.n_rows > INT32_MAX || H < 0 ||
        d.n_cols + H > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_hot: bad sizes");
    if (d.n_rows == 0 || d.nnz == 0 || (H == 0 && !own_lo_plan))
        return spmv_csr_run_tiled(d, row_ptr, col_hot, val, x, y, ws, ws_bytes);
    if ((H > 0 && !hot) || !ws || ws_bytes < spmv_csr_hot_ws_bytes(d.n_rows, d.nnz, H))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_hot: hot list or workspace missing");
    SPMV_GUARD(d);
    const int64_t tiles = (d.nnz + csr_tiled_tile(d.n_rows, d.nnz) - 1) / csr_tiled_tile(d.n_rows, d.nnz);
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_hot: grid too large");
    double *xh = (double *)ws;
    double *carry_val = xh + H;
    int32_t *own_lo = (int32_t *)(carry_val + tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    return launch_csr_tiled_hot(d, row_ptr, col_hot, val, x, y, H, hot, xh, own_lo_plan, own_lo, carry_row,
                                carry_val);
}

// CSR with fp32 values (8 bytes per entry instead of
// 12): the x-window kernel widens each value to fp64 before the product
// and sums in fp64, so y equals spmv_csr_run_xwin's on the fp32-rounded
// values bit for bit.  Windows from spmv_csr_xwin_build on the same
// row_ptr/col with the same lanes_per_row and rows_per_window.
extern "C" int spmv_csr_f32v_run_xwin(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const float *val,
                                      const double *x, double *y, int lanes_per_row, int32_t rows_per_window,
                                      const void *win, int32_t xcap)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || rows_per_window < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_xwin: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if (!win || xcap < 0 || xcap > kCsrXwinCap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_xwin: bad window arguments");
    SPMV_GUARD(d);
    const int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    if (L < 2 || L > 64 || (L & (L - 1)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_xwin: lanes_per_row must be 0 or a power of two in [2,64]");
    const int64_t gpw = csr_xwin_gpw(L, rows_per_window);
    const bool nt = stream_nt(kCsrXwinNtDefault);
    const int2 *w = (const int2 *)win;
    const int64_t groups_base = d.n_rows;
#define SPMV_XWIN32(LL)                                                                                     \
    do {                                                                                                    \
        constexpr int RPB = kBlock / LL;                                                                    \
        const int64_t groups = (groups_base + RPB - 1) / RPB;                                               \
        if ((groups + gpw - 1) / gpw > INT32_MAX)                                                           \
            return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_xwin: grid too large");                    \
        const bool r4 = csr_stage_rounds(d.n_rows, d.nnz, LL) == 4;                                         \
        if (nt && r4)                                                                                       \
            launch_csr_xwin<LL, 4, true>(d, row_ptr, Col32<true>{col}, val, x, y, w, xcap, gpw);            \
        else if (nt)                                                                                        \
            launch_csr_xwin<LL, 3, true>(d, row_ptr, Col32<true>{col}, val, x, y, w, xcap, gpw);            \
        else if (r4)                                                                                        \
            launch_csr_xwin<LL, 4, false>(d, row_ptr, Col32<false>{col}, val, x, y, w, xcap, gpw);          \
        else                                                                                                \
            launch_csr_xwin<LL, 3, false>(d, row_ptr, Col32<false>{col}, val, x, y, w, xcap, gpw);          \
    } while (0)
    switch (L) {
    case 2: SPMV_XWIN32(2); break;
    case 4: SPMV_XWIN32(4); break;
    case 8: SPMV_XWIN32(8); break;
    case 16: SPMV_XWIN32(16); break;
    case 32: SPMV_XWIN32(32); break;
    default: SPMV_XWIN32(64); break;
    }
#undef SPMV_XWIN32
    SPMV_CHECK_LAUNCH("csr_xwin_kernel (fp32 values)");
    return SPMV_SUCCESS;
}

// fp32 values, entry-balanced tiles (+ hot-column table, build-once tile
// plan), as spmv_csr_run_tiled_hot: bit-identical to it on the fp32-rounded
// values.  own_lo_plan from spmv_csr_tiled_plan, or NULL.
extern "C" int spmv_csr_f32v_run_tiled_hot(spmv_dims d, const int64_t *row_ptr, const int32_t *col_hot,
                                           const float *val, const double *x, double *y, int64_t H,
                                           const int32_t *hot, const int32_t *own_lo_plan, void *ws,
                                           size_t ws_bytes)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || d.n_rows > INT32_MAX || H < 0 ||
        d.n_cols + H > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_tiled_hot: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    if (d.nnz == 0) {
        hipError_t e = hipMemsetAsync(y, 0, (size_t)d.n_rows * sizeof(double), (hipStream_t)d.stream);
        return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "memset y", e);
    }
    if ((H > 0 && !hot) || !ws || ws_bytes < spmv_csr_hot_ws_bytes(d.n_rows, d.nnz, H))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_tiled_hot: hot list or workspace missing");
    const int64_t tiles = (d.nnz + csr_tiled_tile(d.n_rows, d.nnz) - 1) / csr_tiled_tile(d.n_rows, d.nnz);
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_tiled_hot: grid too large");
    double *xh = (double *)ws;
    double *carry_val = xh + H;
    int32_t *own_lo = (int32_t *)(carry_val + tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    return launch_csr_tiled_hot(d, row_ptr, col_hot, val, x, y, H, hot, xh, own_lo_plan, own_lo, carry_row,
                                carry_val);
}
