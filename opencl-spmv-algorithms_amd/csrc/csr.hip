// csr.hip — CSR-vector SpMV for gfx950.
//
// Replaces the reference's scalar CSR kernel (reference kernels/Csr.cl:1-17:
// one work-item per row, 8192 work-items total, reference csr.c:47-48).
// Here a group of L lanes (L | 64) owns one row.  Variants (the `variant`
// argument of spmv_csr_run_variant):
//   1 = direct: every L-lane group walks its own row with 16-byte pair loads
//       and reduces with a __shfl_xor butterfly;
//   2 = staged: the row group's entry range is streamed through LDS by all
//       256 lanes like a copy kernel, then each L-lane group sums its row;
//   3 = staged, persistent workgroups with the next group's offsets
//       prefetched (default; spmv_csr_run_xwin adds the LDS x windows);
//   4 = entry-balanced tiles for skewed rows (spmv_csr_run_tiled, staged.hip).
// Bytes per row: 12·len + 8 (row_ptr) + 8 (y), plus x gathers.
#include <stdio.h>
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

// Variant 1: the workgroup's 256/L + 1 row offsets staged in LDS, then
// every L-lane group walks its row (row_dot_pairs).
template <int L>
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
    const double sum = row_dot_pairs<L>(beg, end, lane, col, val, XGlobal{x});
    if (lane == 0 && row < n_rows)
        store_y(y + (row), sum);
}

// CSR-vector with the entry stream staged through LDS ("staged" variants).
// The workgroup's rows occupy one contiguous range of entries
// [ptr[row0], ptr[row0+RPB]).  Instead of every L-lane group walking its
// own row (ragged trip counts, loads that straddle row ends), all 256
// lanes stream that range like a copy kernel — aligned 16-byte value
// pairs + 8-byte column pairs, R pairs per lane in flight — and store the
// products a·x in LDS.  After one barrier each L-lane group sums its row's
// slice of the products (conflict-free ds_read_b64, stride 1 across lanes)
// and reduces with the same shuffle butterfly.  Ranges longer than the LDS
// chunk are processed in chunks; a row's partial sum stays in its lanes'
// registers across chunks.
constexpr int kStageRoundsDefault = 3;  // pairs per lane per chunk: 1536 products, 12 KiB
// (round 1, persistent kernel: R = 3 0.3008 ms, R = 4 0.3013, R = 5 and
// R = 8 slower; round 2, x-window kernel MODE 3: R = 3 0.2591-0.2607 ms,
// R = 4 0.2639-0.2642 — one rule for every staged CSR kernel keeps their
// chunk boundaries, hence their bits, identical)
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

// One row group (RPB = 256/L rows) of the staged scheme; s_ptr holds the
// group's RPB+1 row offsets.  Ends with a barrier, so the caller may
// overwrite s_ptr / s_prod afterwards.  Per-round guarded loads (the batched
// schedule measured 0.350 against 0.313 ms here: 76 VGPRs, 6 waves/SIMD).
template <int L, int R, bool NT, typename Cols = Col32<NT>, typename XS = XGlobal, typename V = double>
__device__ __forceinline__ void staged_group(
    int64_t row, const int64_t *s_ptr, double2 *s_prod,
    const Cols cols, const V *__restrict__ val,
    const XS xs, double *__restrict__ y, int64_t n_rows)
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
        __syncthreads();
        acc += slice_sum<L>(prod, beg > cb ? beg - cb : 0, (end < ce ? end : ce) - cb, lane);
        __syncthreads();
    }
    acc = group_sum<L>(acc);
    if (lane == 0 && row < n_rows)
        store_y(y + (row), acc);
    __syncthreads();
}

// One lane's share of a staged chunk in flight: R value pairs and R column
// pairs, loaded branch-free (pairs past the chunk load the chunk's first
// pair again and are never summed), so all 2R loads are outstanding
// together and can stay in flight across a barrier while the previous chunk
// is reduced.  (With the guarded loads inside per-round branches the
// compiler serialised the rounds: one round's loads in flight at a time.)
template <int R, bool NT, typename V, typename Cols = Col32<NT>>
struct StreamRegs {
    double2 v[R];
    typename Cols::Raw c[R];
    int64_t q[R];  // the pair each lane loaded (decode needs it for escaped blocks only)

    // issue() for an array known to hold at least 2 entries: branch-free, so
    // a caller may issue it inside straight-line code whose later waits must
    // leave these loads in flight (a branch around loads makes the compiler's
    // wait counts conservative at the join: vmcnt(0) for everything)
    __device__ __forceinline__ void issue_nz2(int64_t cb, int64_t ce, int64_t nz, const Cols &cols,
                                              const V *__restrict__ val)
    {
        const int64_t spare = cb + 1 < nz ? cb : (nz - 2) & ~(int64_t)1;  // this chunk's first pair
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t p = cb + 2 * (int64_t)(threadIdx.x + k * kBlock);
            q[k] = (p < ce && p + 1 < nz) ? p : spare;
            v[k] = vpair<NT>(val + q[k]);
            c[k] = cols.raw(q[k]);
        }
    }

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

    // products of the issued chunk [cb, ce) into s_prod
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
// CSR_STAMP(k): per-wave phase hooks, no-ops in the product; a lab build
// (tools/build_variant.sh stamps_csr) injects tools/lab_stamps_csr.h
#ifndef CSR_STAMP
#define CSR_STAMP(k) \
    do {             \
    } while (0)
#endif
// st: the chunk loads in flight; prefetched = the caller already issued
// group 0's first chunk into st (csr_xwin_kernel MODE 4), so the first issue
// here is skipped (the same chunk, the same bits).
template <int L, int R, bool NT, typename XS, typename V, typename Cols = Col32<NT>>
__device__ __forceinline__ void staged_window_pipelined(int64_t row0, int ngroups, const int64_t *s_off,
                                                        double2 *s_prod, const Cols cols,
                                                        const V *__restrict__ val, const XS xs,
                                                        double *__restrict__ y, int64_t n_rows, int64_t nz,
                                                        StreamRegs<R, NT, V, Cols> &st, bool prefetched)
{
    constexpr int RPB = kBlock / L;
    constexpr int CH = 2 * kBlock * R;
    const int g = threadIdx.x / L;
    const int lane = threadIdx.x % L;
    const double *prod = reinterpret_cast<const double *>(s_prod);
    // first group at or after `from` that has a chunk (staged_group's loop
    // runs a chunk iff chunk_start(start) < end); ngroups when none
    auto next_group = [&](int from) {
        int j = from;
        while (j < ngroups && chunk_start(s_off[j * RPB]) >= s_off[(j + 1) * RPB])
            ++j;
        return j;
    };
    int jn = next_group(0);
    if (jn < ngroups && !prefetched) {
        const int64_t b = chunk_start(s_off[jn * RPB]), e = s_off[(jn + 1) * RPB];
        st.issue(b, b + CH < e ? b + CH : e, nz, cols, val);
    }
    int nchunk = 0;
    (void)nchunk;
    for (int gi = 0; gi < ngroups; ++gi) {
        const int64_t *gp = s_off + gi * RPB;
        const int64_t beg = gp[g], end = gp[g + 1];
        const int64_t blk_end = gp[RPB];
        double acc = 0.0;
        for (int64_t cb = chunk_start(gp[0]); cb < blk_end; cb += CH) {
            const int64_t ce = cb + CH < blk_end ? cb + CH : blk_end;
            st.products(cb, ce, nz, cols, val, xs, s_prod);
            CSR_STAMP(nchunk == 0 ? 2 : 5 + nchunk);  // 2: chunk 0's products; 6, 7: chunks 1, 2
            ++nchunk;
            // the next chunk: this group's, else the next group's first
            if (cb + CH < blk_end) {
                const int64_t nb = cb + CH;
                st.issue(nb, nb + CH < blk_end ? nb + CH : blk_end, nz, cols, val);
            } else if ((jn = next_group(gi + 1)) < ngroups) {
                const int64_t b = chunk_start(s_off[jn * RPB]), e = s_off[(jn + 1) * RPB];
                st.issue(b, b + CH < e ? b + CH : e, nz, cols, val);
            }
            __syncthreads();
            if (nchunk == 1)
                CSR_STAMP(3);  // chunk 0: products published
            acc += slice_sum<L>(prod, beg > cb ? beg - cb : 0, (end < ce ? end : ce) - cb, lane);
            if (nchunk == 1)
                CSR_STAMP(4);  // chunk 0: row sums read
            __syncthreads();
            if (nchunk == 1)
                CSR_STAMP(5);  // chunk 0: second barrier
        }
        acc = group_sum<L>(acc);
        const int64_t row = row0 + (int64_t)gi * RPB + g;
        // (the window's y staged in LDS and stored once at its end measured
        // the same: 0.2481 vs 0.2478 ms, profiles/round2/ab_ystage.log)
        if (lane == 0 && row < n_rows)
            store_y(y + (row), acc);
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
    staged_group<L, R, false>(row0 + threadIdx.x / L, s_ptr, s_prod, Col32<false>{col}, val, XGlobal{x}, y, n_rows);
}

// Variant 3: persistent workgroups (a few per CU) walk the row groups
// grid-stride and PREFETCH the next group's row offsets into registers
// while the current group streams, so a group no longer starts with a
// dependent round trip for its offsets.  Cols = Col32 (CSR) or Col16
// (compressed column indices, spmv_csr16_run).
template <int L, int R, bool NT, typename Cols>
__global__ __launch_bounds__(kBlock) void csr_staged_persistent_kernel(
    int64_t n_rows, int64_t n_groups, const int64_t *__restrict__ row_ptr,
    const Cols cols, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y)
{
    constexpr int RPB = kBlock / L;
    __shared__ int64_t s_ptr[RPB + 1];
    __shared__ double2 s_prod[kBlock * R];
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
        staged_group<L, R, NT, Cols>(grp * RPB + threadIdx.x / L, s_ptr, s_prod, cols, val, XGlobal{x}, y, n_rows);
    }
}

// Column window of every x window (rpb rows): [min, max] column over every
// entry a staged kernel LOADS for those rows — from two entries before the
// first chunk's 32-entry-aligned start (the lead-in entries of the previous
// rows, and the spare pair of a chunk starting at the array's last entry) to
// one past the rows' last entry (the partner of a pair that straddles the
// range end).  Those entries are never summed, but their gathers read LDS,
// so every one of them must lie inside the window.  One pass over col,
// build time.
__global__ __launch_bounds__(kBlock) void csr_window_kernel(int64_t n_rows, int64_t rpb,
                                                            const int64_t *__restrict__ row_ptr,
                                                            const int32_t *__restrict__ col,
                                                            int2 *__restrict__ win)
{
    const int64_t g = blockIdx.x;
    const int64_t r1 = (g + 1) * rpb < n_rows ? (g + 1) * rpb : n_rows;
    const int64_t nz = row_ptr[n_rows];
    const int64_t b = row_ptr[g * rpb], e = row_ptr[r1];
    int2 r = {0, -1};
    if (b < e) {  // uniform: rows without entries load nothing
        const int64_t lo = chunk_start(b) >= 2 ? chunk_start(b) - 2 : 0;
        const int64_t hi = e + 1 < nz ? e + 1 : nz;
        r = block_col_range(col, lo, hi);
    }
    if (threadIdx.x == 0)
        win[g] = r;
}

// The staged kernel with x windows in LDS.  A window covers gpw consecutive
// row groups (rows_per_window = gpw * 256/L rows), one workgroup per window:
// the workgroup copies x[win.x .. win.y] into LDS (dynamic, xcap entries)
// once and then streams the gpw groups, whose products gather from LDS
// instead of global memory — the limiter of the staged kernel (TA busy,
// requests well below the DRAM credit limit: profiles/round1/pmc_stalls.json).
// A window wider than xcap gathers from global memory.  Same products, same
// order: y is bit-identical to variant 3.
// MODE (load schedule; products, sums and y are the same bits in both):
//   0 = window copied by a strided loop, each group's offsets staged in LDS
//       before it, each stream round's loads waited for before the next;
//   3 = the window's row offsets (all its groups, in dynamic LDS behind the
//       x range) and its x range loaded together, 8 loads in flight per
//       thread, before ONE barrier; the chunks software-pipelined: the next
//       chunk's loads are issued before the current chunk's barrier and
//       reduction (staged_window_pipelined);
//   4 = MODE 3 with the window's first chunk also issued in the prologue,
//       right behind the x-range and offset loads, from two scalar loads of
//       its bounds: its HBM round trip overlaps the window's instead of
//       following the window barrier (a small grid, all windows resident:
//       the per-window chain is the kernel's time).
// (Modes 1/2/4/5-7, a prefetched first chunk, a persistent streaming kernel
// with an x ring and a per-entry-range flat schedule were measured slower
// or equal and removed: profiles/round2/ab_csr_xwin*.log, ab_csr_flat.log,
// ab_xstream.log.)
template <int L, int R, bool NT, typename V, int MODE, typename Cols>
__global__ __launch_bounds__(kBlock) void csr_xwin_kernel(
    int64_t n_rows, int64_t n_groups, int64_t gpw, const int64_t *__restrict__ row_ptr,
    const Cols cols, const V *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, const int2 *__restrict__ win, int32_t xcap,
    int remap)
{
    static_assert(MODE == 0 || MODE == 3 || MODE == 4, "csr_xwin_kernel: MODE 0, 3 or 4");
    CSR_STAMP(0);
    constexpr int RPB = kBlock / L;
    extern __shared__ double s_x[];
    __shared__ int64_t s_ptr[MODE >= 3 ? 1 : RPB + 1];
    __shared__ double2 s_prod[kBlock * R];
    int64_t *s_off = reinterpret_cast<int64_t *>(s_x + xcap);  // MODE 3: the window's offsets
    const int64_t nz = row_ptr[n_rows];
    // remap: consecutive windows on one XCD, so the overlapping x ranges of
    // neighbouring windows are copied from that XCD's L2
    const int64_t wi = xcd_block(remap);
    const int64_t g_beg = wi * gpw;
    const int64_t g_end = (wi + 1) * gpw < n_groups ? (wi + 1) * gpw : n_groups;
    // MODE 4: group 0's bounds, uniform addresses (scalar loads, their own
    // counter), requested together with the window bounds and pinned by the
    // empty asm (a scheduling boundary) so that ONE scalar round trip
    // precedes every vector load
    int64_t pb = 0, pe = 0, b0 = 0;
    if constexpr (MODE == 4) {
        const int64_t r0p = g_beg * RPB;
        const int64_t r1 = r0p + RPB < n_rows ? r0p + RPB : n_rows;
        b0 = row_ptr[r0p];
        pe = row_ptr[r1];
    }
    const int2 wnd = win[wi];
    if constexpr (MODE == 4) {
        asm volatile("" ::"s"(b0), "s"(pe), "s"(wnd.x), "s"(wnd.y), "s"(nz));
        pb = chunk_start(b0);
    }
    const int32_t span = wnd.y - wnd.x + 1;
    const bool staged = span > 0 && span <= xcap;  // uniform per workgroup
    if constexpr (MODE >= 3) {
        // offsets r0 .. r0 + nr of the window's rows (clamped past n_rows),
        // then the x range: every load issued before the stores
        const int64_t r0 = g_beg * RPB;
        StreamRegs<R, NT, V, Cols> st;
        bool pre = MODE == 4 && pb < pe;  // group 0 has a chunk (next_group(0) == 0)
        const int32_t nr = (int32_t)((g_end - g_beg) * RPB) + 1;
        constexpr int U = 2;  // offsets per thread per pass (nr <= U·256 in one pass)
        constexpr int XU = 8;  // window entries per thread (copy_window's default)
        if (nr <= U * kBlock && span <= XU * kBlock) {
            // one pass, branch-free: the offsets' and the window's loads all
            // go out before the first store (with the loop below the compiler
            // waited for the offsets before requesting the window)
            int64_t o[U];
            double xv[XU];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int64_t r = r0 + threadIdx.x + k * kBlock;
                o[k] = row_ptr[r < n_rows ? r : n_rows];
            }
            const int32_t xl = span > 0 ? span - 1 : 0;  // clamped (loaded, never stored past span)
#pragma unroll
            for (int k = 0; k < XU; ++k) {
                const int32_t i = (int32_t)threadIdx.x + k * kBlock;
                xv[k] = x[wnd.x + (i < xl ? i : xl)];
            }
            // MODE 4: the first chunk behind them (loads return in order:
            // storing the offsets and the window waits for those only).
            // Unconditional (an empty group 0 loads its spare pair, then the
            // pipeline issues its real first chunk); the launcher picks MODE
            // 4 only for nnz >= 2
            if constexpr (MODE == 4) {
                st.issue_nz2(pb, pre ? (pb + 2 * kBlock * R < pe ? pb + 2 * kBlock * R : pe) : pb, nz, cols, val);
                // the offsets' loads stay here, ahead of the chunk's (the
                // compiler otherwise sinks o[0] into its conditional store,
                // behind every load of the prologue, and waits for all)
                asm volatile("" ::"v"(o[0]), "v"(o[1]));
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int32_t i = (int32_t)threadIdx.x + k * kBlock;
                if (i < nr)
                    s_off[i] = o[k];
            }
            if (staged) {
#pragma unroll
                for (int k = 0; k < XU; ++k) {
                    const int32_t i = (int32_t)threadIdx.x + k * kBlock;
                    if (i < span)
                        s_x[i] = xv[k];
                }
            }
        } else {
        pre = false;  // a window too big for the one-pass prologue: issued after the barrier
        for (int32_t b = 0; b < nr; b += U * kBlock) {
            int64_t o[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int64_t r = r0 + b + threadIdx.x + k * kBlock;
                o[k] = row_ptr[r < n_rows ? r : n_rows];
            }
            if (staged && b == 0)
                copy_window(s_x, x, wnd.x, span);
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int32_t i = b + (int32_t)threadIdx.x + k * kBlock;
                if (i < nr)
                    s_off[i] = o[k];
            }
        }
        }
        __syncthreads();  // window and offsets visible
        CSR_STAMP(1);
        if (staged)
            staged_window_pipelined<L, R, NT, XWindow, V, Cols>(r0, (int)(g_end - g_beg), s_off, s_prod, cols, val,
                                                               XWindow{s_x, wnd.x}, y, n_rows, nz, st, pre);
        else
            staged_window_pipelined<L, R, NT, XGlobal, V, Cols>(r0, (int)(g_end - g_beg), s_off, s_prod, cols, val,
                                                               XGlobal{x}, y, n_rows, nz, st, pre);
        return;
    }
    if (staged)
        for (int32_t i = threadIdx.x; i < span; i += kBlock)
            s_x[i] = x[wnd.x + i];
    for (int64_t grp = g_beg; grp < g_end; ++grp) {
        if (threadIdx.x <= RPB) {
            const int64_t r = grp * RPB + threadIdx.x;
            s_ptr[threadIdx.x] = row_ptr[r < n_rows ? r : n_rows];
        }
        __syncthreads();  // offsets (and, for the first group, the window) visible
        const int64_t row = grp * RPB + threadIdx.x / L;
        if (staged)
            staged_group<L, R, NT, Cols, XWindow, V>(row, s_ptr, s_prod, cols, val, XWindow{s_x, wnd.x}, y, n_rows);
        else
            staged_group<L, R, NT, Cols, XGlobal, V>(row, s_ptr, s_prod, cols, val, XGlobal{x}, y, n_rows);
    }
}

// (Round 6, one cant-like matrix cold, events: R = 2 / 5 / 6 pairs per lane
// 15.5 / 14.9 / 15.6 us against 15.0 us for R = 3, profiles/round6/ab_csr_r.md.)
// Chunk size of the staged CSR kernels for a matrix: R = 3 (1,536-entry
// chunks) unless R = 4 (2,048) cuts a row group of 256/L rows of the mean
// length into FEWER chunks — every chunk is a memory round trip and two
// barriers.  Cant-like (L = 4, 64 rows x 64.2 = 4,107 entries): 3 chunks
// either way, R = 3 (measured 0.2591 vs 0.2639 ms).  Banded (L = 2, 128
// rows x 16 = 2,048): 1 chunk with R = 4 against 2 with R = 3 (configs[4]
// measured 4.50 ms with R = 3).  Every staged CSR path uses this rule, so
// their chunk boundaries, hence their bits, stay identical.
static int csr_stage_rounds(int64_t n_rows, int64_t nnz, int L)
{
    if (n_rows <= 0 || L <= 0)
        return kStageRoundsDefault;
    const double eg = (double)(kBlock / L) * ((double)nnz / (double)n_rows);
    const int64_t c3 = (int64_t)((eg + 1535.0) / 1536.0), c4 = (int64_t)((eg + 2047.0) / 2048.0);
    return c4 < c3 ? 4 : 3;
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

template <int L, int R, bool NT, typename Cols>
static void launch_persistent(const spmv_dims &d, const int64_t *row_ptr, const Cols cols, const double *val,
                              const double *x, double *y, int64_t groups)
{
    static const int64_t per = persistent_grid(csr_staged_persistent_kernel<L, R, NT, Cols>, INT64_MAX);
    const int64_t grid = per < groups ? per : groups;
    hipLaunchKernelGGL((csr_staged_persistent_kernel<L, R, NT, Cols>), dim3((unsigned)grid), dim3(kBlock), 0,
                       (hipStream_t)d.stream, d.n_rows, groups, row_ptr, cols, val, x, y);
}

// compressed-index CSR: the persistent staged kernel with Col16 columns
template <int L, bool NT>
static void launch_csr16(const spmv_dims &d, const int64_t *row_ptr, const Col16<NT> cols,
                         const double *val, const double *x, double *y)
{
    constexpr int RPB = kBlock / L;
    const int64_t groups = (d.n_rows + RPB - 1) / RPB;
    if (csr_stage_rounds(d.n_rows, d.nnz, L) == 4)
        launch_persistent<L, 4, NT, Col16<NT>>(d, row_ptr, cols, val, x, y, groups);
    else
        launch_persistent<L, 3, NT, Col16<NT>>(d, row_ptr, cols, val, x, y, groups);
}

template <int L, int R>
static void launch_staged(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                          const double *val, const double *x, double *y, int variant)
{
    constexpr int RPB = kBlock / L;
    const int64_t groups = (d.n_rows + RPB - 1) / RPB;
    if (variant == 3) {
        if (stream_nt(kCsrStreamNtDefault))
            launch_persistent<L, R, true>(d, row_ptr, Col32<true>{col}, val, x, y, groups);
        else
            launch_persistent<L, R, false>(d, row_ptr, Col32<false>{col}, val, x, y, groups);
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
    if (variant >= 2) {
        if (csr_stage_rounds(d.n_rows, d.nnz, L) == 4)
            launch_staged<L, 4>(d, row_ptr, col, val, x, y, variant);
        else
            launch_staged<L, 3>(d, row_ptr, col, val, x, y, variant);
    } else {
        hipLaunchKernelGGL((csr_vector_kernel<L>), dim3((unsigned)blocks), dim3(kBlock), 0, (hipStream_t)d.stream,
                           d.n_rows, row_ptr, col, val, x, y, xcd_remap_enabled() ? 1 : 0);
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
    if (variant < 0 || variant > 3)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run: variant must be 0..3 (4 = spmv_csr_run_tiled)");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if ((d.n_rows + 1) / 2 > (int64_t)INT32_MAX * 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run: too many rows");
    SPMV_GUARD(d);
    const int v = variant ? variant : 3;
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

// Load schedule of csr_xwin_kernel: MODE 3 when a window's entries make
// more than one chunk (there is a next chunk to pipeline: cant-like, 128
// rows x 64.2 = 8,214 entries in 1,536-entry chunks), else MODE 0 — a
// one-chunk window gains nothing from the pipeline and its 86 instead of 64
// VGPRs cost workgroups per CU (banded, 128 rows x 16 = one 2,048-entry
// chunk: 0.765 ms MODE 0 vs 0.815 ms MODE 3, profiles/round2/ab_banded.log).
// MODE 3 with XCD-contiguous windows: 0.2644 ms vs 0.2678 (MODE 3, round
// robin), 0.2701 (MODE 0, remap) and 0.2717 (MODE 0, round robin), five
// interleaved rounds on one box (profiles/round2/ab_csr_xwin.log).
static int csr_xwin_mode(int64_t n_rows, int64_t nnz, int64_t rows_per_window, int R)
{
    const double ew = n_rows > 0 ? (double)rows_per_window * ((double)nnz / (double)n_rows) : 0.0;
    return ew > 2.0 * kBlock * R ? 3 : 0;
}

// XCD-contiguous windows pay when neighbouring windows share x lines: the
// widest window spans several times its rows (cant-like: 678 columns for 128
// rows; on), not when each row reads a narrow band (banded: 143 columns for
// 128 rows; 0.765 vs 0.782 ms with remap, off).  SPMV_XWIN_REMAP forces it
// (placement only: same bits).
// Round 5: only for grids of many rounds on the chip (>= 8 windows per CU).
// On ONE cant-like matrix (488 windows, one round, all windows resident at
// once) the round-robin placement ran 1.5 % faster in three interleaved A/Bs
// (12.08 / 11.98 vs 12.18 / 12.26 us cold, profiles/round5/ab_remap_staged.md;
// 12.12 vs 12.20-12.30 in round 4, profiles/round4/ab_csr_single.md T).
static bool csr_xwin_remap_rule(int32_t xcap, int64_t rows_per_window, int64_t n_windows)
{
    return xwin_remap((int64_t)xcap > 2 * rows_per_window && n_windows >= 8 * 256);
}

// dynamic LDS of csr_xwin_kernel: the x window, and in MODE 3 the window's
// row offsets behind it
static size_t csr_xwin_lds(int mode, int32_t xcap, int64_t gpw, int rpb)
{
    return ((size_t)xcap + (mode >= 3 ? (size_t)(gpw * rpb + 1) : 0)) * sizeof(double);
}

// MODE 4 (the first chunk prefetched in the prologue, behind the x window's
// and offsets' loads) is opt-in: on one cant-like matrix (976 windows of 64
// rows, all resident at once) it measured 15.6 us cold against MODE 3's
// 14.8 us (profiles/round6/csr_prefetch_ab.md) — its 90 VGPRs cost a wave per
// SIMD and the barrier already waits on the x window's HBM round trip.
// SPMV_OPT_CSR_PREFETCH (spmv_set_option) = 1 selects it (same bits).
static bool csr_xwin_prefetch_rule(int64_t n_windows)
{
    (void)n_windows;
    return csr_prefetch(false);
}

// rows per x window: a multiple of the row group (256/L rows), default
// kCsrXwinRows but at least two groups, so a window whose groups are one
// chunk each still has a next chunk to pipeline (MODE 3): the banded matrix
// (L = 2, 128-row groups of 2,048 entries) 0.7534 ms with one-group windows
// (MODE 0) against 0.7261 ms with two (profiles/round2/ab_banded3.log);
// explicit rows_per_window: at least one group.  Same chunks, same bits.
// A small matrix (fewer than 4 default windows per CU) gets one-group
// windows instead, twice the workgroups to spread over the CUs: one
// cant-like matrix (488 windows of 128 rows) 13.28 vs 13.74 us cold, 10.5 vs
// 12.1 us warm (rocprof, profiles/round3/cant_single_csr_windows.log).
static int64_t csr_xwin_gpw(int L, int32_t rows_per_window, int64_t n_rows)
{
    const int64_t rpb = kBlock / L;
    if (rows_per_window > 0) {
        const int64_t g = (rows_per_window + rpb - 1) / rpb;
        return g < 1 ? 1 : g;
    }
    int64_t g = (kCsrXwinRows + rpb - 1) / rpb;
    g = g < 2 ? 2 : g;
    // the MI355X's 256 CUs as a constant, not the current device's count:
    // the window table (spmv_csr_xwin_build) bakes this choice in, so it
    // must not change with the device a matrix is later run on
    if (n_rows < 4 * (int64_t)256 * g * rpb)
        g = 1;
    return g;
}

template <int L, int R, bool NT, typename Cols, typename V = double>
static void launch_csr_xwin(const spmv_dims &d, const int64_t *row_ptr, const Cols cols,
                            const V *val, const double *x, double *y, const int2 *win, int32_t xcap,
                            int64_t gpw)
{
    constexpr int RPB = kBlock / L;
    const int64_t groups = (d.n_rows + RPB - 1) / RPB;
    const int64_t n_win = (groups + gpw - 1) / gpw;
    int mode = csr_xwin_mode(d.n_rows, d.nnz, gpw * RPB, R);
    // a very tall window's offsets would not fit beside the x range in the
    // 64 KiB of dynamic LDS: MODE 0 stages them per row group instead
    if (mode == 3 && csr_xwin_lds(mode, xcap, gpw, RPB) + sizeof(double2) * kBlock * R * 2 > 64 * 1024)
        mode = 0;
    const size_t lds = csr_xwin_lds(mode, xcap, gpw, RPB);
    if (n_win > INT32_MAX)
        return;
    const int remap = csr_xwin_remap_rule(xcap, gpw * RPB, n_win) ? 1 : 0;
    const hipStream_t st = (hipStream_t)d.stream;
    if (mode == 3 && d.nnz >= 2 && csr_xwin_prefetch_rule(n_win))
        hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 4, Cols>), dim3((unsigned)n_win), dim3(kBlock), lds, st,
                           d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
    else if (mode == 3)
        hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 3, Cols>), dim3((unsigned)n_win), dim3(kBlock), lds, st,
                           d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
    else
        hipLaunchKernelGGL((csr_xwin_kernel<L, R, NT, V, 0, Cols>), dim3((unsigned)n_win), dim3(kBlock), lds, st,
                           d.n_rows, groups, gpw, row_ptr, cols, val, x, y, win, xcap, remap);
}

// One launcher per column source / value type: L from the switch, R and the
// load policy from the rules above.
template <int L, typename V, typename MakeCols>
static void launch_xwin_l(const spmv_dims &d, const int64_t *row_ptr, MakeCols mk, const V *val, const double *x,
                          double *y, const int2 *w, int32_t xcap, int64_t gpw)
{
    const bool nt = stream_nt(kCsrXwinNtDefault);
    const bool r4 = csr_stage_rounds(d.n_rows, d.nnz, L) == 4;  // R = 3 or 4 (the rule)
    if (nt && r4)
        launch_csr_xwin<L, 4, true>(d, row_ptr, mk.template get<true>(), val, x, y, w, xcap, gpw);
    else if (nt)
        launch_csr_xwin<L, 3, true>(d, row_ptr, mk.template get<true>(), val, x, y, w, xcap, gpw);
    else if (r4)
        launch_csr_xwin<L, 4, false>(d, row_ptr, mk.template get<false>(), val, x, y, w, xcap, gpw);
    else
        launch_csr_xwin<L, 3, false>(d, row_ptr, mk.template get<false>(), val, x, y, w, xcap, gpw);
}

struct MakeCol32 {
    const int32_t *col;
    template <bool NT>
    Col32<NT> get() const { return Col32<NT>{col}; }
};

struct MakeCol16 {
    const int32_t *base;
    const uint16_t *off;
    const int32_t *esc;
    template <bool NT>
    Col16<NT> get() const { return Col16<NT>{base, off, esc}; }
};

template <typename V, typename MakeCols>
static int launch_xwin_any(const spmv_dims &d, int L, const int64_t *row_ptr, MakeCols mk, const V *val,
                           const double *x, double *y, const int2 *w, int32_t xcap, int64_t gpw)
{
    switch (L) {
    case 2: launch_xwin_l<2>(d, row_ptr, mk, val, x, y, w, xcap, gpw); break;
    case 4: launch_xwin_l<4>(d, row_ptr, mk, val, x, y, w, xcap, gpw); break;
    case 8: launch_xwin_l<8>(d, row_ptr, mk, val, x, y, w, xcap, gpw); break;
    case 16: launch_xwin_l<16>(d, row_ptr, mk, val, x, y, w, xcap, gpw); break;
    case 32: launch_xwin_l<32>(d, row_ptr, mk, val, x, y, w, xcap, gpw); break;
    case 64: launch_xwin_l<64>(d, row_ptr, mk, val, x, y, w, xcap, gpw); break;
    default: return fail_msg(SPMV_OTHER_ERROR, "csr x-window run: lanes_per_row must be 0 or a power of two in [2,64]");
    }
    return SPMV_SUCCESS;
}

}  // namespace spmv

extern "C" size_t spmv_csr_xwin_bytes(int64_t n_rows, int64_t nnz, int lanes_per_row, int32_t rows_per_window)
{
    const int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(n_rows, nnz);
    if (L < 2 || L > 64 || (L & (L - 1)) || n_rows <= 0 || rows_per_window < 0)
        return 0;
    const int64_t rpw = csr_xwin_gpw(L, rows_per_window, n_rows) * (kBlock / L);
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
    const int64_t rpw = csr_xwin_gpw(L, rows_per_window, d.n_rows) * (kBlock / L);
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

static int xwin_args(spmv_dims d, int32_t rows_per_window, const void *win, int32_t xcap, int lanes_per_row,
                     int *L, const char *who)
{
    static thread_local char msg[160];
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || rows_per_window < 0) {
        snprintf(msg, sizeof msg, "%s: bad sizes", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    if (d.n_rows > 0 && (!win || xcap < 0 || xcap > kCsrXwinCap)) {
        snprintf(msg, sizeof msg, "%s: bad window arguments", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    *L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    if (*L < 2 || *L > 64 || (*L & (*L - 1))) {
        snprintf(msg, sizeof msg, "%s: lanes_per_row must be 0 or a power of two in [2,64]", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    return SPMV_SUCCESS;
}

extern "C" int spmv_csr_run_xwin(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                                 const double *x, double *y, int lanes_per_row, int32_t rows_per_window,
                                 const void *win, int32_t xcap)
{
    int L = 0;
    int rc = xwin_args(d, rows_per_window, win, xcap, lanes_per_row, &L, "spmv_csr_run_xwin");
    if (rc != SPMV_SUCCESS || d.n_rows == 0)
        return rc;
    SPMV_GUARD(d);
    rc = launch_xwin_any(d, L, row_ptr, MakeCol32{col}, val, x, y, (const int2 *)win, xcap,
                         csr_xwin_gpw(L, rows_per_window, d.n_rows));
    if (rc != SPMV_SUCCESS)
        return rc;
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
    int L = 0;
    int rc = xwin_args(d, rows_per_window, win, xcap, lanes_per_row, &L, "spmv_csr16_run_xwin");
    if (rc != SPMV_SUCCESS || d.n_rows == 0)
        return rc;
    if (d.nnz > 0 && (!blk_base || !col_off))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr16_run_xwin: missing index arrays");
    SPMV_GUARD(d);
    rc = launch_xwin_any(d, L, row_ptr, MakeCol16{blk_base, col_off, col_esc}, val, x, y, (const int2 *)win, xcap,
                         csr_xwin_gpw(L, rows_per_window, d.n_rows));
    if (rc != SPMV_SUCCESS)
        return rc;
    SPMV_CHECK_LAUNCH("csr_xwin_kernel (16-bit columns)");
    return SPMV_SUCCESS;
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
    int L = 0;
    int rc = xwin_args(d, rows_per_window, win, xcap, lanes_per_row, &L, "spmv_csr_f32v_run_xwin");
    if (rc != SPMV_SUCCESS || d.n_rows == 0)
        return rc;
    SPMV_GUARD(d);
    const int64_t gpw = csr_xwin_gpw(L, rows_per_window, d.n_rows);
    const int64_t groups = (d.n_rows + kBlock / L - 1) / (kBlock / L);
    if ((groups + gpw - 1) / gpw > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_f32v_run_xwin: grid too large");
    rc = launch_xwin_any(d, L, row_ptr, MakeCol32{col}, val, x, y, (const int2 *)win, xcap, gpw);
    if (rc != SPMV_SUCCESS)
        return rc;
    SPMV_CHECK_LAUNCH("csr_xwin_kernel (fp32 values)");
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
template <typename V>
static int run_tiled_hot(spmv_dims d, const int64_t *row_ptr, const int32_t *col_hot, const V *val,
                         const double *x, double *y, int64_t H, const int32_t *hot, const int32_t *own_lo_plan,
                         void *ws, const char *who)
{
    static thread_local char msg[160];
    const int64_t tiles = (d.nnz + csr_tiled_tile(d.n_rows, d.nnz) - 1) / csr_tiled_tile(d.n_rows, d.nnz);
    if (tiles > INT32_MAX) {
        snprintf(msg, sizeof msg, "%s: grid too large", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    double *xh = (double *)ws;
    double *carry_val = xh + H;
    int32_t *own_lo = (int32_t *)(carry_val + tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    return launch_csr_tiled_hot(d, row_ptr, col_hot, val, x, y, H, hot, xh, own_lo_plan, own_lo, carry_row,
                                carry_val);
}

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
    return run_tiled_hot(d, row_ptr, col_hot, val, x, y, H, hot, own_lo_plan, ws,
                         "spmv_csr_run_tiled_hot");
}

extern "C" int64_t spmv_csr_tiled_tile(int64_t n_rows, int64_t nnz)
{
    return csr_tiled_tile(n_rows, nnz);
}

// spmv_csr_run_tiled_hot with the big-tile plan of the host builder
// spmv_csr_tiled_bigplan (uploaded; built for tile = spmv_csr_tiled_tile):
// tiles owning more than 1,024 rows write their rows without entries as
// zeros and sum only the listed ones, instead of reading every owned row's
// offsets from global memory.  big = NULL: spmv_csr_run_tiled_hot.
extern "C" int spmv_csr_run_tiled_plan(spmv_dims d, const int64_t *row_ptr, const int32_t *col_hot,
                                       const double *val, const double *x, double *y, int64_t H,
                                       const int32_t *hot, const int32_t *own_lo_plan, const int32_t *big,
                                       int64_t big_len, int64_t big_tile, void *ws, size_t ws_bytes)
{
    if (!big)
        return spmv_csr_run_tiled_hot(d, row_ptr, col_hot, val, x, y, H, hot, own_lo_plan, ws, ws_bytes);
    // the plan must be this matrix's: built for the tile the run cuts, and
    // at least as long as its tile index (the kernel bounds-checks the rest)
    if (big_tile != csr_tiled_tile(d.n_rows, d.nnz) || big_tile != csr_tiled_tile_min())
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_plan: plan built for another tile size");
    if (d.nnz > 0 && big_len < (d.nnz + big_tile - 1) / big_tile + 1)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_plan: plan shorter than its tile index");
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || d.n_rows > INT32_MAX || H < 0 ||
        d.n_cols + H > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_plan: bad sizes");
    if (d.n_rows == 0 || d.nnz == 0)
        return spmv_csr_run_tiled(d, row_ptr, col_hot, val, x, y, ws, ws_bytes);
    if (!own_lo_plan || (H > 0 && !hot) || !ws || ws_bytes < spmv_csr_hot_ws_bytes(d.n_rows, d.nnz, H))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_plan: tile plan, hot list or workspace missing");
    SPMV_GUARD(d);
    const int64_t tiles = (d.nnz + csr_tiled_tile(d.n_rows, d.nnz) - 1) / csr_tiled_tile(d.n_rows, d.nnz);
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run_tiled_plan: grid too large");
    double *xh = (double *)ws;
    double *carry_val = xh + H;
    int32_t *own_lo = (int32_t *)(carry_val + tiles);
    int32_t *carry_row = own_lo + tiles + 1;
    return launch_csr_tiled_hot(d, row_ptr, col_hot, val, x, y, H, hot, xh, own_lo_plan, own_lo, carry_row,
                                carry_val, big, big_len);
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
    return run_tiled_hot(d, row_ptr, col_hot, val, x, y, H, hot, own_lo_plan, ws,
                         "spmv_csr_f32v_run_tiled_hot");
}

// ------------------------------------------------- column-grouped CSR (CSRG)
// Power-law matrices (R-MAT, configs[3]) are bound by their x gathers: a
// cold column fills a whole 128-byte L2 line for 8 bytes, and the R-MAT's
// ~4 M used columns (33 MB of x lines) do not fit one XCD's 4 MiB L2, so
// the tiled kernel moved 3.46x bytes_alg (profiles/traffic_rmat.json).
// CSRG (host spmv_csrg_fill) stores the entries group after group, each
// group owning the x lines of 1/G of the columns; the tiled kernel runs the
// (row, group) pairs in that order, so the tiles in flight gather from one
// group's lines (~5 MB at G = 16) and mostly hit L2.  Each pair's sum goes
// to yp; csrg_reduce_kernel then adds a row block's pair sums in group order
// in LDS: every group's pairs of the block are one contiguous run of yp
// (blk_off), read as a stream.  Deterministic; the row sums are grouped
// differently from CSR's, so y agrees with it to the parity rule.
__global__ __launch_bounds__(kBlock) void csrg_reduce_kernel(int64_t n_rows, int32_t groups, int64_t nb,
                                                             const int32_t *__restrict__ blk_off,
                                                             const uint16_t *__restrict__ pair_row,
                                                             const double *__restrict__ yp, double *__restrict__ y)
{
    constexpr int B = SPMV_CSRG_ROWS;
    __shared__ double s_y[B];
    const int64_t b = blockIdx.x;
    for (int i = threadIdx.x; i < B; i += kBlock)
        s_y[i] = 0.0;
    __syncthreads();
    for (int32_t g = 0; g < groups; ++g) {  // group order: a row's pair sums added g = 0, 1, ...
        const int32_t p0 = blk_off[(int64_t)g * (nb + 1) + b], p1 = blk_off[(int64_t)g * (nb + 1) + b + 1];
        for (int32_t p = p0 + (int32_t)threadIdx.x; p < p1; p += 4 * kBlock) {
            double v[4];
            int r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // 4 loads in flight; a row appears once per group
                const int32_t pk = p + k * kBlock;
                r[k] = pk < p1 ? (int)pair_row[pk] : -1;
                v[k] = pk < p1 ? yp[pk] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (r[k] >= 0)
                    s_y[r[k]] += v[k];
        }
        __syncthreads();
    }
    const int64_t r0 = b * B;
    for (int i = threadIdx.x; i < B; i += kBlock)
        if (r0 + i < n_rows)
            store_y(y + r0 + i, s_y[i]);
}

extern "C" size_t spmv_csrg_ws_bytes(int64_t n_pairs, int64_t nnz)
{
    return (size_t)(n_pairs > 0 ? n_pairs : 0) * sizeof(double) + spmv_csr_tiled_ws_bytes(n_pairs, nnz);
}

extern "C" int spmv_csrg_run(spmv_dims d, int32_t groups, int64_t n_pairs, const int64_t *pair_ptr,
                             const int32_t *col_g, const double *val_g, const int32_t *own_lo_plan,
                             const int32_t *blk_off, const uint16_t *pair_row, const double *x, double *y,
                             void *ws, size_t ws_bytes)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0 || d.n_rows > INT32_MAX || n_pairs < 0 ||
        n_pairs > INT32_MAX || n_pairs > d.nnz || (d.nnz > 0 && n_pairs == 0) || groups < 1 || groups > 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csrg_run: bad sizes");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    if (d.nnz == 0) {
        hipError_t e = hipMemsetAsync(y, 0, (size_t)d.n_rows * sizeof(double), (hipStream_t)d.stream);
        return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "memset y", e);
    }
    if (!pair_ptr || !col_g || !val_g || !blk_off || !pair_row || !ws ||
        ws_bytes < spmv_csrg_ws_bytes(n_pairs, d.nnz))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csrg_run: arrays or workspace missing");
    double *yp = (double *)ws;
    spmv_dims pd = d;  // the pair CSR: one "row" per (row, group) pair
    pd.n_rows = n_pairs;
    int rc = run_tiled_hot(pd, pair_ptr, col_g, val_g, x, yp, 0, nullptr, own_lo_plan, yp + n_pairs,
                           "spmv_csrg_run");
    if (rc != SPMV_SUCCESS)
        return rc;
    const int64_t nb = (d.n_rows + SPMV_CSRG_ROWS - 1) / SPMV_CSRG_ROWS;
    hipLaunchKernelGGL(csrg_reduce_kernel, dim3((unsigned)nb), dim3(kBlock), 0, (hipStream_t)d.stream, d.n_rows,
                       groups, nb, blk_off, pair_row, yp, y);
    SPMV_CHECK_LAUNCH("csrg_reduce_kernel");
    return SPMV_SUCCESS;
}
