// staged.hip — LDS-staged CMRS and COO kernels for gfx950.
//
// Both formats store each workgroup's entries as ONE contiguous range
// (CMRS: a run of strips; COO: a fixed tile of the row-sorted entries).
// Like the staged CSR kernel (csr.hip), all 256 lanes stream that range
// as aligned 16-byte value pairs + column pairs, form the products a·x and
// store them in LDS together with the per-entry row key; after one barrier
// every row's slice of the products is found by a binary search over the
// sorted keys in LDS and summed by an L-lane group (shuffle butterfly).
// Compared with the wave-per-strip / wave-per-tile segmented scans
// (coo.hip), no lane waits on a global load between scan steps, so the
// kernels stream at the CSR rate.
//
// CMRS replaces the reference's cmrs kernel (reference kernels/Cmrs.cl:
// 1-46: per-lane partial rows in LDS, three barriers per strip, an
// out-of-bounds tail store); COO replaces the reference's CAS-atomic coo
// kernel (reference kernels/Coo.cl:4-32) — rows that start in an earlier
// tile go through the same deterministic carry pass as coo.hip.
#include <stdlib.h>

#include "common.h"

namespace spmv {

// first index in [lo, hi) whose key is >= k (keys sorted)
template <typename K>
__device__ __forceinline__ int lower_bound_lds(const K *keys, int lo, int hi, int k)
{
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int)keys[mid] < k)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// Row keys staged next to the products, in two phases so their loads are
// batched with the value/column loads: load(q) the key pair of entries
// (q, q+1), store(t, pair), and one(t, p) for the array's odd last entry.
// COO: int32 row ids (int2 pairs); CMRS: uint8 row-in-strip (2-byte pairs).
template <bool NT>
struct KeysRow32 {
    const int32_t *__restrict__ k;
    int2 *s;
    using P = int2;
    __device__ __forceinline__ P load(int64_t q) const { return stream_load2<NT>(k + q); }
    __device__ __forceinline__ void store(int t, P v) const { s[t] = v; }
    __device__ __forceinline__ void one(int t, int64_t p) const { s[t] = make_int2(stream_load<NT>(k + p), 0); }
};

struct KeysU8 {
    const uint8_t *__restrict__ k;
    uint16_t *s;
    using P = uint16_t;
    __device__ __forceinline__ P load(int64_t q) const { return *reinterpret_cast<const uint16_t *>(k + q); }
    __device__ __forceinline__ void store(int t, P v) const { s[t] = v; }
    __device__ __forceinline__ void one(int t, int64_t p) const { s[t] = (uint16_t)k[p]; }
};

struct KeysNone {  // the tiled CSR: rows come from row_ptr, no keys
    using P = uint8_t;
    __device__ __forceinline__ P load(int64_t) const { return 0; }
    __device__ __forceinline__ void store(int, P) const {}
    __device__ __forceinline__ void one(int, int64_t) const {}
};

// Streams entries [cb, ce) (cb even) of an nz-entry array into LDS:
// products in s_prod, row keys through `keys`.  Every lane issues its R
// value, column and key pair loads before the first product (branch-free:
// a pair starting at or past ce loads the chunk's first pair again, a line
// the wave already reads, and is never read back), so 3R loads per lane are
// in flight together; a pair that
// straddles ce reads one entry past the chunk, inside the array, that no
// reduction reads.  The array's odd last entry is loaded singly.
// NT: non-temporal stream loads.
// stage_chunk in two halves: issue() puts a lane's 3R pair loads in flight,
// commit() writes the products and keys of the issued chunk to LDS.  A
// kernel may issue the next chunk between a commit and the barrier that
// publishes it (software pipelining), with the same result as stage_chunk.
// SAFE2: the caller guarantees nz >= 2 (no branch on it: with one, the
// compiler widened the column indices on the load path before the merge, so
// it waited for the columns right after issuing them, before anything else)
template <int R, bool NT, typename V, typename Keys, bool SAFE2 = false>
struct StageRegs {
    double2 v[R];
    int2 c[R];
    typename Keys::P kp[R];

    __device__ __forceinline__ void issue(int64_t cb, int64_t ce, int64_t nz, const int32_t *__restrict__ col,
                                          const V *__restrict__ val, const Keys &keys)
    {
        if constexpr (!SAFE2)
            if (nz < 2)  // uniform; a 1-entry array has no pair 0 (its entry: the tail in commit)
                return;
        const int64_t spare = cb + 1 < nz ? cb : (nz - 2) & ~(int64_t)1;  // this chunk's first pair
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t p = cb + 2 * (int64_t)(threadIdx.x + k * kBlock);
            const int64_t q = (p < ce && p + 1 < nz) ? p : spare;
            v[k] = vpair<NT>(val + q);
            c[k] = stream_load2<NT>(col + q);
            kp[k] = keys.load(q);
        }
    }

    template <typename XS>
    __device__ __forceinline__ void commit(int64_t cb, int64_t ce, int64_t nz, const int32_t *__restrict__ col,
                                           const V *__restrict__ val, const XS &xs, double2 *s_prod,
                                           const Keys &keys) const
    {
        if (SAFE2 || nz >= 2) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const int t = threadIdx.x + k * kBlock;
                s_prod[t] = double2{v[k].x * xs(c[k].x), v[k].y * xs(c[k].y)};
                keys.store(t, kp[k]);
            }
        }
        const int64_t tail = nz - 1 - cb;
        if ((nz & 1) && nz - 1 < ce && tail >= 0 && tail < 2 * R * kBlock && (tail >> 1) % kBlock == threadIdx.x) {
            const int64_t p = nz - 1;
            const int t = (int)(tail >> 1);
            s_prod[t] = double2{vone<NT>(val + p) * xs(stream_load<NT>(col + p)), 0.0};
            keys.one(t, p);
        }
    }
};

// Streams entries [cb, ce) (cb even) of an nz-entry array into LDS:
// products in s_prod, row keys through `keys`.  Every lane issues its R
// value, column and key pair loads before the first product (branch-free:
// a pair starting at or past ce loads the chunk's first pair again, a line
// the wave already reads, and is never read back), so 3R loads per lane are
// in flight together; a pair that
// straddles ce reads one entry past the chunk, inside the array, that no
// reduction reads.  The array's odd last entry is loaded singly.
// NT: non-temporal stream loads.
template <int R, bool NT = false, typename XS, typename Keys, typename V>
__device__ __forceinline__ void stage_chunk(int64_t cb, int64_t ce, int64_t nz, const int32_t *__restrict__ col,
                                            const V *__restrict__ val, const XS &xs,
                                            double2 *s_prod, const Keys &keys)
{
    StageRegs<R, NT, V, Keys> st;
    st.issue(cb, ce, nz, col, val, keys);
    st.commit(cb, ce, nz, col, val, xs, s_prod, keys);
}

// ------------------------------------------------------------------ CMRS
// A workgroup owns G consecutive strips (G·h rows, L lanes per row).
// XW: the workgroup's x window x[win.x .. win.y] (the column range of its
// entry run, spmv_cmrs_xwin_build) is copied into LDS first and the
// products gather from LDS; a window wider than xcap gathers from global
// memory.  Same products, same order: y is bit-identical either way.
// NT: non-temporal loads of the entry stream.
template <int L, int R, bool XW, bool NT = false>
__global__ __launch_bounds__(kBlock) void cmrs_staged_kernel(
    int64_t n_rows, int32_t h, int32_t G, int64_t n_strips,
    const int64_t *__restrict__ strip_ptr, const uint8_t *__restrict__ rin,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y,
    const int2 *__restrict__ win, int32_t xcap, int remap = 0)
{
    constexpr int CH = 2 * kBlock * R;
    extern __shared__ double s_x[];
    __shared__ int64_t s_sp[kBlock + 1];
    const int64_t blk = xcd_block(remap);  // remap: neighbouring strip runs (shared x lines) on one XCD
    __shared__ double2 s_prod[kBlock * R];
    __shared__ uint16_t s_key2[kBlock * R];  // keys of entry pairs
    const uint8_t *s_key = reinterpret_cast<const uint8_t *>(s_key2);
    const double *prod = reinterpret_cast<const double *>(s_prod);

    const int64_t s0 = blk * G;
    // the entry count bounds every chunk load: requested first, with the
    // strip offsets and the x window (read after the barrier it was one more
    // dependent round trip before the first chunk's loads could go out)
    const int64_t nz = strip_ptr[n_strips];
    // the run's strip offsets: loaded by every thread (clamped), stored to
    // LDS only after the window's loads are out — stored right after their
    // load, inside the branch, the compiler waited for them before
    // requesting the x window (two dependent round trips instead of one)
    const int64_t sv = strip_ptr[s0 + threadIdx.x < n_strips ? s0 + threadIdx.x : n_strips];
    bool staged = false;  // uniform per workgroup
    int32_t wlo = 0;
    if constexpr (XW) {
        const int2 wnd = win[blk];
        const int32_t span = wnd.y - wnd.x + 1;
        // a window wider than one pass of the copy gathers from global
        // memory instead (same x values, same bits): a copy loop here would
        // join the one-pass path and make it wait for the offsets first
        staged = span > 0 && span <= xcap && span <= 8 * kBlock;
        wlo = wnd.x;
        if (staged)  // uniform
            copy_window_1pass(s_x, x, wlo, span);
    }
    if ((int)threadIdx.x <= G)
        s_sp[threadIdx.x] = sv;
    asm volatile("" ::"s"(nz));  // in a register by the barrier (the read-only load was sunk past it)
    __syncthreads();

    const int rl = threadIdx.x / L, lane = threadIdx.x % L;
    const bool active = rl < G * h;
    const int si = active ? rl / h : 0;
    const int key = active ? rl % h : 0;
    const int64_t sb = s_sp[si], se = active ? s_sp[si + 1] : s_sp[si];
    const int64_t row = (s0 + si) * h + key;
    const int64_t blk_end = s_sp[G];
    const KeysU8 keys{rin, s_key2};

    double acc = 0.0;
    // chunks start on a 32-entry boundary: whole 128-B lines per wave (as
    // csr.hip kChunkAlign); the previous strip's entries are never summed.
    // (A software-pipelined chunk loop, the next chunk's loads issued before
    // this chunk's barrier, measured 0.3227 vs 0.2896 ms: 78 instead of 66
    // VGPRs; profiles/round2/ab_cmrs_pipe.log.  On ONE cant-like matrix, with
    // the first chunk also issued before the x window, 18.9 vs 16.4 us cold:
    // profiles/round4/ab_csr_single.md J.)
    const int64_t c0 = s_sp[0] & ~(int64_t)31;
    for (int64_t cb = c0; cb < blk_end; cb += CH) {
        const int64_t ce = cb + CH < blk_end ? cb + CH : blk_end;
        if (staged) {
            stage_chunk<R, NT>(cb, ce, nz, col, val, XWindow{s_x, wlo}, s_prod, keys);
        } else {
            stage_chunk<R, NT>(cb, ce, nz, col, val, XGlobal{x}, s_prod, keys);
        }
        __syncthreads();
        const int64_t lo = sb > cb ? sb : cb;
        const int64_t hi = se < ce ? se : ce;
        if (lo < hi) {  // this strip has entries in the chunk: find the row
            // the row's two bounds searched at once by lanes 0 and 1 of its
            // group (one dependent LDS chain instead of two; the same a, b)
            int a, b;
            if constexpr (L >= 2) {
                const int f = lower_bound_lds(s_key, (int)(lo - cb), (int)(hi - cb), key + (lane & 1));
                a = __shfl(f, 0, L);
                b = __shfl(f, 1, L);
            } else {
                a = lower_bound_lds(s_key, (int)(lo - cb), (int)(hi - cb), key);
                b = lower_bound_lds(s_key, a, (int)(hi - cb), key + 1);
            }
            acc += slice_sum<L>(prod, a, b, lane);
        }
        __syncthreads();
    }
    acc = group_sum<L>(acc);
    if (active && lane == 0 && row < n_rows && s0 + si < n_strips)
        store_y(y + (row), acc);
}

// ------------------------------------------------------------------- COO
constexpr int kCooRowCap = 1024;
// Rows of row-start table per tile for mean rows >= 12 (a 1,536-entry tile
// spans ~128 rows or fewer): the table shrinks from 4 to 1 KiB, so 8 tiles fit
// a CU's LDS instead of 7 (the single-pass form: 8 instead of 5); a tile
// spanning more rows keeps the binary searches (same bits).
constexpr int kCooRowCapShort = 250;
// entries a single-pass COO tile may load past its end (pairs staged in LDS
// behind the tile: 40; the cant-like matrix's rows reach 81 entries, so its
// tails stay within 80).  With 256 pairs (512 entries) the tail's LDS left
// 5 tiles per CU: 21.8 us cold on one cant-like matrix, against 18.0 us now
// and 20.6 us for the carry pass
constexpr int kCooTailCap = 80;
// entry pairs staged per thread by the COO kernels (tile = 2·256·kCooR entries)
constexpr int kCooR = 3;
// XCD-contiguous placement of the single-pass COO tiles and the x-window
// CMRS strip runs (neighbours read overlapping x lines; on one XCD they share
// its L2).  SPMV_XWIN_REMAP=0/1 overrides it per call.  One cant-like matrix
// cold, two interleaved rounds (profiles/round5/ab_remap_staged.md): COO
// 16.68 / 16.88 -> 16.54 / 16.52 us (on), CMRS 13.34 / 13.48 -> 13.52 / 13.58
// (off).
constexpr bool kCooRemapDefault = true;
constexpr bool kCmrsRemapDefault = false;

// A workgroup owns one tile of CH consecutive row-sorted entries and
// writes y for rows (row[t0-1], row[t1-1]] (rows without entries get 0;
// the last tile also covers the trailing rows).  A first row that began
// in an earlier tile goes to carry[tile] for coo_carry_kernel (coo.hip).
// XW: the tile's x window in LDS (as cmrs_staged_kernel), bit-identical.
// XS/NT: x accessor of the global gathers (XHot: hot-column table) and the
// stream load policy.
// TAIL (single pass, spmv_coo_run_tail): the tile also loads the entries of
// its last row that run past the tile end (tails[tile] of them, at most
// kCooTailCap, from spmv_coo_tail_build) and finishes that row itself; a row begun
// in an earlier tile is skipped, so no carry pass runs.
// COO_STAMP(k) / COO_NOTE(k, v): per-tile phase hooks, no-ops in the
// product; a lab build (tools/build_variant.sh stamps_coo) injects
// tools/lab_stamps_coo.h (tools/coo_stamps.py reads them)
#ifndef COO_STAMP
#define COO_STAMP(k) \
    do {             \
    } while (0)
#define COO_NOTE(k, v) \
    do {               \
    } while (0)
#define COO_STAMP_END() \
    do {                \
    } while (0)
#endif
template <int L, int R, bool ACC, bool XW, bool NT = false, typename XS = XGlobal, bool TAIL = false,
          int RC = kCooRowCap>
__global__ __launch_bounds__(kBlock) void coo_staged_kernel(
    int64_t n_rows, int64_t nnz, const int32_t *__restrict__ row,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, int32_t *__restrict__ carry_row,
    double *__restrict__ carry_val, const int2 *__restrict__ win, int32_t xcap, const XS xs,
    const int32_t *__restrict__ tails = nullptr, int remap = 0)
{
    constexpr int CH = 2 * kBlock * R;
    extern __shared__ double s_x[];
    constexpr int GROUPS = kBlock / L;
    constexpr int TP = TAIL ? (kCooTailCap + 1) / 2 : 0;  // tail entry pairs staged behind the tile
    __shared__ double2 s_prod[kBlock * R + TP];
    __shared__ int2 s_row2[kBlock * R + TP];
    __shared__ int32_t s_prev;
    __shared__ int32_t s_start[RC + 1];  // owned rows' first entries
    __shared__ double s_sum[ACC ? RC : 1];  // ACC: the owned rows' sums
    const int32_t *s_row = reinterpret_cast<const int32_t *>(s_row2);
    const double *prod = reinterpret_cast<const double *>(s_prod);

    const int64_t tile = xcd_block(remap);  // remap: neighbouring tiles (shared x lines) on one XCD
    COO_STAMP(0);
    const int64_t t0 = tile * CH;
    const int64_t t1 = t0 + CH < nnz ? t0 + CH : nnz;
    const int n = (int)(t1 - t0);
    // uniform; > 0 only for full tiles (n even).  Clamped to the staged
    // capacity, so a plan built for other row arrays cannot write past the
    // LDS tail (spmv_coo_tail_build zeroes a plan it refuses)
    int tail = TAIL ? tails[tile] : 0;
    tail = tail < 0 ? 0 : (tail > 2 * TP ? 2 * TP : tail);
    if (threadIdx.x == 0)
        s_prev = t0 > 0 ? row[t0 - 1] : -1;
    const KeysRow32<NT> keys{row, s_row2};
    bool staged = false;  // uniform per workgroup
    int32_t wlo = 0;
    if constexpr (XW) {
        const int2 wnd = win[tile];
        const int32_t span = wnd.y - wnd.x + 1;
        staged = span > 0 && span <= xcap;
        wlo = wnd.x;
        if (staged) {
            copy_window(s_x, x, wlo, span);
            __syncthreads();
        }
    }
    if constexpr (TAIL) {
        // the tile's pairs and the last row's entries past t1 (pair j at
        // t1 + 2j) in flight together, then the products of both
        static_assert(!XW, "the single-pass COO gathers x through xs");
        StageRegs<R, NT, double, KeysRow32<NT>, true> st;  // nnz >= 2 (coo_tiny_kernel below that)
        st.issue(t0, t1, nnz, col, val, keys);
        const int j = threadIdx.x;
        const int64_t p = t1 + 2 * (int64_t)j;
        const bool tpair = 2 * j + 1 < tail, tone = 2 * j + 1 == tail;  // tail > 0 only for full tiles
        static_assert(TP <= kBlock, "one tail pair per thread");
        double2 tv = {0.0, 0.0};
        int2 tc = {0, 0}, tk = {0, 0};
        // a pair, or the lone last entry p = nnz - 1 (nnz odd): element
        // loads, so the lone entry is read on its own, aligned, instead of
        // as an odd pair (p - 1, p) (the tail is < kCooTailCap
        // entries per tile, the extra instructions are a few per thread)
        const bool tsh = p + 1 >= nnz;
        if (tpair || tone) {  // ONE branch: with two, a merge made the waves wait for the tile's loads first
            const int64_t q1 = tsh ? p : p + 1;
            tv = double2{stream_load<NT>(val + p), stream_load<NT>(val + q1)};
            tc = int2{stream_load<NT>(col + p), stream_load<NT>(col + q1)};
            tk = int2{stream_load<NT>(row + p), stream_load<NT>(row + q1)};
        }
        // (Round 6: the tail's x values gathered before commit, branch-free
        // with the tile's, measured 18.72 vs 18.59 us cold on one cant-like
        // matrix, events; profiles/round6/ab_coo_cmrs.md.)
        st.commit(t0, t1, nnz, col, val, xs, s_prod, keys);
        if (tpair || tone) {
            s_prod[n / 2 + j] = tpair ? double2{tv.x * xs(tc.x), tv.y * xs(tc.y)} : double2{tv.x * xs(tc.x), 0.0};
            s_row2[n / 2 + j] = tsh ? make_int2(tk.x, tk.x) : tk;  // (.y of a lone entry is never read)
        }
    } else if (staged) {
        stage_chunk<R, NT>(t0, t1, nnz, col, val, XWindow{s_x, wlo}, s_prod, keys);
    } else {
        stage_chunk<R, NT>(t0, t1, nnz, col, val, xs, s_prod, keys);
    }
    __syncthreads();
    COO_STAMP(1);  // products and keys in LDS

    const int32_t prev = s_prev;
    const int32_t first = s_row[0], last = s_row[n - 1];
    const int ne = n + tail;  // staged entries: the tile, then its last row's tail
    const bool first_continues = prev == first;
    const int g = threadIdx.x / L, lane = threadIdx.x % L;
    // Row starts from the key changes (one pass over the staged keys, every
    // row of (prev, last] written by exactly one thread) instead of two
    // binary searches per row; a tile spanning more than RC rows
    // (long runs of empty rows) keeps the searches.
    const int64_t r_lo = (int64_t)prev + 1;
    const int64_t span = (int64_t)last - r_lo + 1;  // rows (prev, last]
    bool heads = false;  // uniform per workgroup
    {
        heads = span >= 0 && span <= RC;
        if (heads) {
            // a pair of keys per read (and the key before it): 3 instead
            // of 8 bytes of LDS reads per entry
            for (int t = threadIdx.x; 2 * t < n; t += kBlock) {
                const int j = 2 * t;
                const int2 kk = s_row2[t];
                const int32_t kp = j > 0 ? s_row[j - 1] : prev;
                for (int32_t r = kp + 1; r <= kk.x; ++r)
                    s_start[r - r_lo] = j;
                if (j + 1 < n)
                    for (int32_t r = kk.x + 1; r <= kk.y; ++r)
                        s_start[r - r_lo] = j + 1;
            }
            if (threadIdx.x == 0)
                s_start[span] = ne;
            __syncthreads();
        }
    }
    // Tiles over more than RC rows (long runs of rows without entries): the
    // entries that begin a row after prev as a bitmap over the tile's n
    // entries (one ballot per 64), so a row's end is the next set bit (or ne)
    // — the range [first, end) a search over s_row gives it, so the same
    // bits.  Searching per row-first entry instead (lower_bound over the
    // rest of the tile, 11 dependent LDS reads, the wave waiting on its
    // slowest group in nearly every step of a walk over all entries) took
    // 13-23 us per such tile (tools/coo_stamps.py; profiles/round6/ab_coo_first.md).
    // (The words live in s_start, behind the span bitmap where there is one:
    // a __shared__ array of their own took one tile per CU off the
    // cant-like single pass, 20,592 B of LDS > 160 KiB / 8.)
    constexpr int FW = (2 * kBlock * R + 63) / 64 * 2;  // row-first words of a tile
    static_assert(FW < RC, "the row-first words fit in s_start");
    auto build_first = [&](uint32_t *s_first) {
        const int lw = (int)threadIdx.x & (kWave - 1);
        for (int j0 = (int)threadIdx.x - lw; j0 < n; j0 += kBlock) {  // wave-uniform
            const int j = j0 + lw;
            bool f = false;
            if (j < n) {
                const int32_t r = s_row[j];
                f = r > prev && (j == 0 || s_row[j - 1] != r);
            }
            const uint64_t bal = __ballot(f);
            if (lw == 0) {
                s_first[j0 >> 5] = (uint32_t)bal;
                s_first[(j0 >> 5) + 1] = (uint32_t)(bal >> 32);
            }
        }
    };
    // fn(first, end) for every row that begins in the tile, one 32-entry
    // word of s_first per group at a time (uniform over the group)
    auto for_each_row = [&](const uint32_t *s_first, auto &&fn) {
        const int nfw = (n + 31) >> 5;
        for (int w = g; w < nfw; w += GROUPS) {
            uint32_t m = s_first[w];
            while (m) {
                const int j = w * 32 + __builtin_ctz(m);
                m &= m - 1;
                int b = ne;
                if (m) {
                    b = w * 32 + __builtin_ctz(m);
                } else {
                    for (int w2 = w + 1; w2 < nfw; ++w2) {
                        const uint32_t m2 = s_first[w2];
                        if (m2) {
                            b = w2 * 32 + __builtin_ctz(m2);
                            break;
                        }
                    }
                }
                fn(j, b);
            }
        }
    };
    COO_STAMP(2);  // row starts in LDS (heads)
    COO_NOTE(4, (uint64_t)span);
    COO_NOTE(5, (uint64_t)(heads ? 0 : span <= 32 * (int64_t)(RC + 1 - FW) ? 1 : 2));

    // carry: the first row's entries when it began in an earlier tile (with
    // TAIL the earlier tile summed them from its tail)
    if (!TAIL && g == 0) {
        double c = 0.0;
        if (first_continues) {
            const int b = heads ? s_start[0] : lower_bound_lds(s_row, 0, n, first + 1);
            c = slice_sum<L>(prod, 0, b, lane);
        }
        c = group_sum<L>(c);
        if (lane == 0) {
            carry_row[tile] = first_continues ? first : -1;
            carry_val[tile] = c;
        }
    }
    if constexpr (ACC) {
        // accumulate mode (HYB tail): y[r] += the tile's entries of every row
        // that begins here; rows without entries in the tail are left
        // untouched.  One L-lane group per row (a hub row's 1,536 tile
        // entries no longer fall to one thread).
        if (!heads) {  // uniform
            // a tile over a long run of rows without tail entries (a HYB
            // tail of a few rows' remainders): the rows that begin here from
            // the row-first bitmap, instead of two binary searches per
            // spanned row
            uint32_t *s_first = reinterpret_cast<uint32_t *>(s_start);
            build_first(s_first);
            __syncthreads();
            for_each_row(s_first, [&](int j, int b) {
                double s = slice_sum<L>(prod, j, b, lane);
                s = group_sum<L>(s);
                if (lane == 0)
                    y[s_row[j]] += s;
            });
            return;
        }
        // the row sums into LDS, then y[r] += sum in one coalesced pass with
        // every thread's y loads in flight together, instead of y[r] += s
        // inside the row loop (one dependent read of y per row per group):
        // one cant-like HYB's K = 52 tail 9.08 / 9.16 -> 8.64 / 8.72 us
        // (rocprof trace, same box; K = 72's tail, 30.4 us, did not move:
        // profiles/round6/ab_hyb_k.md)
        for (int64_t r = r_lo + g; r <= (int64_t)last; r += GROUPS) {
            const int a = s_start[r - r_lo], b = s_start[r - r_lo + 1];
            if (a == b)
                continue;  // uniform over the group
            double s = slice_sum<L>(prod, a, b, lane);
            s = group_sum<L>(s);
            if (lane == 0)
                s_sum[r - r_lo] = s;
        }
        __syncthreads();
        const int sp = (int)span;  // <= RC
        for (int i0 = 0; i0 < sp; i0 += 4 * kBlock) {
            double yv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // clamped: every load valid, none behind a branch
                const int i = i0 + (int)threadIdx.x + k * kBlock;
                yv[k] = y[r_lo + (i < sp ? i : sp - 1)];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = i0 + (int)threadIdx.x + k * kBlock;
                if (i < sp && s_start[i] != s_start[i + 1])
                    y[r_lo + i] = yv[k] + s_sum[i];
            }
        }
        return;
    }
    // owned rows: (prev, last], plus the trailing empty rows in the last
    // tile; a continued first row equals prev, so it is excluded here
    const int64_t r_hi = t1 == nnz ? n_rows - 1 : (int64_t)last;
    if (!heads && span > RC && span <= 32 * (int64_t)(RC + 1 - FW)) {  // uniform
        // A tile over a long run of mostly empty rows (R-MAT: up to ~28 K
        // rows per 512-entry tile): the rows WITH entries come from the
        // row-first bitmap, each summed over [first, end) exactly as the
        // search path sums it (the same bits), and marked in a bitmap over
        // the span (s_start's words); then the others are written as zeros,
        // coalesced.  The search path did two binary searches per owned row.
        uint32_t *s_bits = reinterpret_cast<uint32_t *>(s_start);
        const int nw = (int)((span + 31) >> 5);
        for (int i = threadIdx.x; i < nw; i += kBlock)
            s_bits[i] = 0u;
        uint32_t *s_first = s_bits + nw;
        build_first(s_first);
        __syncthreads();
        for_each_row(s_first, [&](int j, int b) {
            const int32_t r = s_row[j];
            double sm = slice_sum<L>(prod, j, b, lane);
            sm = group_sum<L>(sm);
            if (lane == 0) {
                store_y(y + r, sm);
                atomicOr(&s_bits[(r - r_lo) >> 5], 1u << ((r - r_lo) & 31));
            }
        });
        __syncthreads();
        for (int64_t r = r_lo + threadIdx.x; r <= r_hi; r += kBlock) {
            const bool has = r <= last && ((s_bits[(r - r_lo) >> 5] >> ((r - r_lo) & 31)) & 1u);
            if (!has)
                store_y(y + r, 0.0);
        }
        COO_STAMP_END();
        return;
    }
    for (int64_t r = r_lo + g; r <= r_hi; r += GROUPS) {
        double s = 0.0;
        if (r <= last) {
            int a, b;
            if (heads) {
                a = s_start[r - r_lo];
                b = s_start[r - r_lo + 1];
            } else {
                a = lower_bound_lds(s_row, 0, ne, (int)r);
                b = lower_bound_lds(s_row, a, ne, (int)r + 1);
            }
            s = slice_sum<L>(prod, a, b, lane);
        }
        s = group_sum<L>(s);
        if (lane == 0)
            store_y(y + (r), s);
    }
    COO_STAMP_END();
}

// ------------------------------------------------------------ CSR tiled
// Entry-balanced CSR for skewed row lengths (R-MAT hubs of ~1e5 entries):
// a workgroup owns a fixed tile of CH entries, never a fixed row count, so
// no workgroup streams more than CH entries.  A row is OWNED by the tile
// holding its first offset row_ptr[r] (trailing empty rows: the last
// tile); the owner writes y[r] = its partial sum, later tiles that the row
// runs into write carry[tile], finished by coo_carry_kernel.
// own_lo[t] = first row with row_ptr >= t·CH (pre-pass, one binary search
// per tile over row_ptr).
__global__ __launch_bounds__(kBlock) void csr_tile_rows_kernel(int64_t n_rows, int64_t nnz,
                                                               int64_t tiles, int64_t ch,
                                                               const int64_t *__restrict__ row_ptr,
                                                               int32_t *__restrict__ own_lo)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t > tiles)
        return;
    const int64_t off = t * ch < nnz ? t * ch : nnz + 1;  // t = tiles: past every row
    int64_t lo = 0, hi = n_rows;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (row_ptr[mid] < off)
            lo = mid + 1;
        else
            hi = mid;
    }
    own_lo[t] = (int32_t)lo;
}

// The tile's row offsets (rows r_lo..r_hi+1, clipped to the tile, relative
// to t0) are staged in LDS together with the products, so the row phase
// makes no dependent global loads; a tile spanning more than kTiledRowCap
// rows (long runs of empty rows) reads them from global memory.  With a
// stream-only x this phase, not the gathers, held the kernel to 2.6 TB/s
// on R-MAT (tools/rmat_exp.hip mode 2).
constexpr int kTiledRowCap = 1024;
// A tile owning more rows (R-MAT: 1,329 of 195,313 512-entry tiles, up to
// 28,255 rows, almost all empty) read their offsets from global memory one
// 64-row run per wave at a time: one such tile took most of an R-MAT
// shard's time.  With the big-tile plan (spmv_csr_tiled_bigplan) it lists
// its owned rows that HAVE entries and writes the rest as zeros from a bitmap
// of up to kTiledBigRowCap rows; more than that keeps the old path.
constexpr int kTiledBigRowCap = 65536;

// (A fused carry — the last-arriving tile of a spanning row finishing it —
// was bit-identical but slower: 0.890 vs 0.856 ms on R-MAT with the
// partials passed through RMW atomics, 5.9 ms with agent-scope
// release/acquire; removed, profiles/HISTORY.md §H6.  A persistent form with the
// hottest 16 K table entries in LDS, one 1024-thread workgroup per CU:
// bit-identical, 2.21 vs 0.83 ms — four tiles in flight per CU instead of
// eight; removed, profiles/HISTORY.md §H9.)
//
// Load order: a tile's dependent round trips are the latency the grid
// waits out.  The value/column pairs need the tile index only, so they are
// issued first; own_lo (a scalar load) and then the row offsets go out
// behind them into registers; the gathers follow once the columns land;
// offsets and products reach LDS together before the one barrier.
//
// Row phase: wave w takes the tile's rows in runs of 64 (runs w, w+4, ...);
// a lane sums a row of at most kTiledShort entries alone, in entry order;
// a longer row (R-MAT hub rows fill whole tiles) is summed by the whole
// wave, lane j taking entries j, j+64, ..., then a butterfly.  With one L-lane
// group per row, a tile inside a hub row was summed by L = 2 lanes, 256
// dependent adds, while the other 254 lanes waited.  The carry (the
// entries before the first row that starts in the tile) is wave 0's, the
// same way.  Deterministic (fixed per-row order); the grouping differs from
// an L-lane sum, so y agrees with the other CSR kernels to the parity rule.
constexpr int kTiledShort = 16;

// sum of p[a..b) by the whole wave (all lanes call it with the same a, b)
__device__ __forceinline__ double wave_sum(const double *p, int a, int b)
{
    const int lane = threadIdx.x & (kWave - 1);
    double s = 0.0;
    for (int j = a + lane; j < b; j += kWave)
        s += p[j];
    return group_sum<kWave>(s);
}

template <int R, bool NT, typename XS, typename V = double>
__global__ __launch_bounds__(kBlock) void csr_tiled_kernel(
    int64_t n_rows, int64_t nnz, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const V *__restrict__ val,
    const XS xs, double *__restrict__ y,
    const int32_t *__restrict__ own_lo, int32_t *__restrict__ carry_row,
    double *__restrict__ carry_val, const int32_t *__restrict__ big = nullptr, int64_t big_len = 0)
{
    constexpr int CH = 2 * kBlock * R;
    constexpr int RPK = (kTiledRowCap + 1 + kBlock - 1) / kBlock;  // staged offsets per thread
    constexpr int NW = kBlock / kWave;
    // only the R = 1 instantiation takes a big-tile plan (launch_tiled_r):
    // the others keep 4 KiB of LDS for s_rp instead of the 8 KiB bitmap
    constexpr int kBitWords = R == 1 ? kTiledBigRowCap / 32 : kTiledRowCap + 1;
    static_assert(kBitWords >= kTiledRowCap + 1, "s_rp lives in the big-tile bitmap");
    __shared__ double2 s_prod[kBlock * R];
    __shared__ uint32_t s_bits[kBitWords];  // big tiles: owned rows with entries; else s_rp
    int32_t *s_rp = reinterpret_cast<int32_t *>(s_bits);
    const double *prod = reinterpret_cast<const double *>(s_prod);
    const int64_t tile = blockIdx.x;
    const int64_t t0 = tile * CH;
    const int64_t t1 = t0 + CH < nnz ? t0 + CH : nnz;
    StageRegs<R, NT, V, KeysNone, true> st;  // nnz >= 2 (launch_tiled_xs)
    st.issue(t0, t1, nnz, col, val, KeysNone{});
    const int64_t r_lo = own_lo[tile];
    const int64_t r_hi = t1 == nnz ? n_rows - 1 : (int64_t)own_lo[tile + 1] - 1;
    const int64_t nr = r_hi - r_lo + 1;  // owned rows (may be 0)
    const bool rp_lds = nr >= 0 && nr <= kTiledRowCap;  // uniform
    // big tile (more owned rows than the offset table, at most the bitmap's):
    // the plan lists its owned rows WITH entries, [a, b) relative to t0
    // (every plan read is bounds-checked against big_len, so a plan of
    // another matrix or tile size cannot read past its buffer)
    const int64_t tiles = (nnz + CH - 1) / CH;
    int32_t bk = R == 1 && !rp_lds && big && nr <= kTiledBigRowCap && tile < big_len ? big[tile] : -1;  // uniform
    if (bk >= 0 && tiles + bk + 1 >= big_len)
        bk = -1;
    int32_t b_beg = 0, b_end = 0;
    int2 item[2] = {{0, 0}, {0, 0}};
    int64_t rpv[RPK];
    // (Round 6: awaiting the tile's columns here, before requesting the
    // offsets branch-free, so commit's gathers overlap the offsets: R-MAT
    // 0.700-0.705 vs 0.674 ms, profiles/round6/ab_tiled.md.  With ~8
    // tiles per CU the other tiles hide this chain; loads in flight count.)
    if (rp_lds) {
#pragma unroll
        for (int k = 0; k < RPK; ++k) {  // r_lo + nr <= n_rows
            const int i = (int)threadIdx.x + k * kBlock;
            rpv[k] = i <= nr ? row_ptr[r_lo + i] : 0;
        }
    } else if (bk >= 0) {
        b_beg = big[tiles + bk];
        b_end = big[tiles + bk + 1];
        b_beg = b_beg > 0 ? b_beg : 0;
        b_end = (int64_t)b_end < big_len ? b_end : (int32_t)big_len;
#pragma unroll
        for (int k = 0; k < 2; ++k) {  // at most CH listed rows; CH <= 2·kBlock for R = 1
            const int32_t i = b_beg + 2 * ((int32_t)threadIdx.x + k * kBlock);
            if (i + 1 < b_end)
                item[k] = *reinterpret_cast<const int2 *>(big + i);
        }
        for (int32_t i = threadIdx.x; i < (int32_t)((nr + 31) >> 5); i += kBlock)
            s_bits[i] = 0u;
    }
    st.commit(t0, t1, nnz, col, val, xs, s_prod, KeysNone{});
    if (rp_lds) {
#pragma unroll
        for (int k = 0; k < RPK; ++k) {
            const int i = (int)threadIdx.x + k * kBlock;
            if (i <= nr)
                s_rp[i] = (int32_t)((rpv[k] < t1 ? rpv[k] : t1) - t0);
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    if (bk >= 0) {
        // carry: the entries before the first listed row (the owned rows
        // before it have none) belong to row r_lo - 1
        if (wv == 0) {
            const int n_t = (int)(t1 - t0);
            int e_rel = b_end > b_beg + 1 ? (big[b_beg + 1] & 0xFFFF) : n_t;
            e_rel = e_rel < n_t ? e_rel : n_t;
            const bool has = r_lo > 0 && e_rel > 0;
            const double c = has ? wave_sum(prod, 0, e_rel) : 0.0;
            if (lane == 0) {
                carry_row[tile] = has ? (int32_t)(r_lo - 1) : -1;
                carry_val[tile] = c;
            }
        }
        // the listed rows, summed as the offset-table path sums them (the
        // same bits): up to kTiledShort entries by one lane in entry order,
        // longer rows by the whole wave; each row marked in the bitmap
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int32_t i = b_beg + 2 * ((int32_t)threadIdx.x + k * kBlock);
            // (bounds re-checked so a plan of another matrix cannot index
            // past the bitmap or the products)
            const bool ok = i + 1 < b_end && item[k].x >= 0 && item[k].x < nr;
            const int32_t rr = item[k].x, a = item[k].y & 0xFFFF;
            int32_t b = (int32_t)((uint32_t)item[k].y >> 16);
            b = b < CH ? b : CH;
            const bool lng = ok && b - a > kTiledShort;
            if (ok && !lng) {
                double sum = 0.0;
                for (int j = a; j < b; ++j)
                    sum += prod[j];
                store_y(y + r_lo + rr, sum);
            }
            if (ok)
                atomicOr(&s_bits[rr >> 5], 1u << (rr & 31));
            for (uint64_t m = __ballot(lng); m; m &= m - 1) {
                const int l = __builtin_ctzll(m);
                const int la = __shfl(a, l), lb = __shfl(b, l), lr = __shfl(rr, l);
                const double sum = wave_sum(prod, la, lb);
                if (lane == 0)
                    store_y(y + r_lo + lr, sum);
            }
        }
        __syncthreads();
        // every other owned row has no entries: y = 0, coalesced, no row_ptr reads
        for (int32_t i = threadIdx.x; i < (int32_t)nr; i += kBlock)
            if (!((s_bits[i >> 5] >> (i & 31)) & 1u))
                store_y(y + r_lo + i, 0.0);
        return;
    }
    // [a, b) of owned row r (relative to t0)
    auto range = [&](int64_t r, int &a, int &b) {
        if (rp_lds) {
            a = s_rp[r - r_lo];
            b = s_rp[r - r_lo + 1];
        } else {
            const int64_t a64 = row_ptr[r], b64 = row_ptr[r + 1];
            a = (int)(a64 - t0);
            b = (int)((b64 < t1 ? b64 : t1) - t0);
        }
    };
    // carry: entry t0 lies in row r_lo-1 when no row starts exactly at t0
    // (row_ptr[r_lo] > t0; for r_lo = n_rows, row_ptr = nnz >= t1 > t0)
    if (wv == 0) {
        int64_t e_rel;  // min(row_ptr[r_lo], t1) - t0
        if (rp_lds) {
            e_rel = s_rp[0];
        } else {
            const int64_t o = r_lo < n_rows ? row_ptr[r_lo] : nnz;
            e_rel = (o < t1 ? o : t1) - t0;
        }
        const bool has = r_lo > 0 && e_rel > 0;
        const double c = has ? wave_sum(prod, 0, (int)e_rel) : 0.0;
        if (lane == 0) {
            carry_row[tile] = has ? (int32_t)(r_lo - 1) : -1;
            carry_val[tile] = c;
        }
    }
    for (int64_t r0 = r_lo + (int64_t)wv * kWave; r0 <= r_hi; r0 += NW * kWave) {
        const int64_t r = r0 + lane;
        int a = 0, b = 0;
        if (r <= r_hi)
            range(r, a, b);
        const bool lng = b - a > kTiledShort;
        if (r <= r_hi && !lng) {
            double sum = 0.0;
            for (int j = a; j < b; ++j)
                sum += prod[j];
            store_y(y + r, sum);
        }
        for (uint64_t m = __ballot(r <= r_hi && lng); m; m &= m - 1) {  // long rows: the whole wave
            const int l = __builtin_ctzll(m);
            const int la = __shfl(a, l), lb = __shfl(b, l);
            const double sum = wave_sum(prod, la, lb);
            if (lane == 0)
                store_y(y + r0 + l, sum);
        }
    }
}

// ------------------------------------------------------------ CMRS tiled
// Entry-balanced CMRS for skewed strips (the R-MAT strip of rows 0-7 holds
// ~3e5 entries; with one workgroup per run of strips that workgroup
// streams it alone).  As csr_tiled_kernel: a workgroup owns a fixed tile of
// CH entries; strip s is OWNED by the tile holding strip_ptr[s] (own_lo
// from csr_tile_rows_kernel over strip_ptr), which writes all h rows of it
// from its part of the strip.  The strip running into a tile from an
// earlier one leaves up to h partial rows: carry[k·tiles + tile] for row
// key k (k-major, so each row's continuation tiles are consecutive and
// coo_carry_kernel adds them: a run of <= 8 tiles in tile order by one
// thread, a longer run lane-strided over a wave and then the butterfly —
// a fixed order either way, so bitwise reproducible).  Needs kBlock / L >= h.
template <int L, int R, typename XS>
__global__ __launch_bounds__(kBlock) void cmrs_tiled_kernel(
    int64_t n_rows, int32_t h, int64_t n_strips, int64_t nnz, int64_t tiles,
    const int64_t *__restrict__ strip_ptr, const uint8_t *__restrict__ rin,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const XS xs, double *__restrict__ y,
    const int32_t *__restrict__ own_lo, int32_t *__restrict__ carry_row,
    double *__restrict__ carry_val)
{
    constexpr int CH = 2 * kBlock * R;
    constexpr int GROUPS = kBlock / L;
    __shared__ double2 s_prod[kBlock * R];
    __shared__ uint16_t s_key2[kBlock * R];  // row keys of entry pairs
    const uint8_t *s_key = reinterpret_cast<const uint8_t *>(s_key2);
    const double *prod = reinterpret_cast<const double *>(s_prod);
    const int64_t tile = blockIdx.x;
    const int64_t t0 = tile * CH;
    const int64_t t1 = t0 + CH < nnz ? t0 + CH : nnz;
    const int64_t s_lo = own_lo[tile];
    const int64_t s_hi = t1 == nnz ? n_strips - 1 : (int64_t)own_lo[tile + 1] - 1;
    stage_chunk<R, true>(t0, t1, nnz, col, val, xs, s_prod, KeysU8{rin, s_key2});
    __syncthreads();
    const int g = threadIdx.x / L, lane = threadIdx.x % L;

    // carried strip: entry t0 lies in strip s_lo-1 when no strip starts at t0
    if (g < h) {
        double c = 0.0;
        int32_t cr = -1;
        if (s_lo > 0 && (s_lo == n_strips || strip_ptr[s_lo] > t0)) {
            const int64_t e64 = s_lo < n_strips && strip_ptr[s_lo] < t1 ? strip_ptr[s_lo] : t1;
            const int e = (int)(e64 - t0);
            const int a = lower_bound_lds(s_key, 0, e, g);
            const int b = lower_bound_lds(s_key, a, e, g + 1);
            for (int j = a + lane; j < b; j += L)
                c += prod[j];
            const int64_t r = (s_lo - 1) * h + g;
            if (b > a && r < n_rows)
                cr = (int32_t)r;
        }
        c = group_sum<L>(c);
        if (lane == 0) {
            carry_row[(int64_t)g * tiles + tile] = cr;
            carry_val[(int64_t)g * tiles + tile] = c;
        }
    }
    // owned strips, one L-lane group per row.  (Round 6: staging the offsets
    // in LDS 256 strips per pass measured slower for every tile, 791 vs 748
    // us on the R-MAT, and equal when kept to tiles over > 256 strips;
    // profiles/round6/ab_cmrs_plan_carry.md.)
    const int64_t items = (s_hi - s_lo + 1) * h;
    for (int64_t it = g; it < items; it += GROUPS) {
        const int64_t s = s_lo + it / h;
        const int k = (int)(it % h);
        const int64_t sa = strip_ptr[s];
        int64_t sb = strip_ptr[s + 1];
        sb = sb < t1 ? sb : t1;
        double acc = 0.0;
        if (sa < sb) {
            const int a = lower_bound_lds(s_key, (int)(sa - t0), (int)(sb - t0), k);
            const int b = lower_bound_lds(s_key, a, (int)(sb - t0), k + 1);
            for (int j = a + lane; j < b; j += L)
                acc += prod[j];
        }
        acc = group_sum<L>(acc);
        const int64_t r = s * h + k;
        if (lane == 0 && r < n_rows)
            store_y(y + (r), acc);
    }
}

// CMRS tile = 2·kBlock·R entries, R as the tiled CSR's rule (1 below a mean
// row of 96, else 3): R-MAT 1e7/1e8 0.877 vs 0.902 ms, 8 row shards max
// 0.166 vs 0.244 ms (profiles/round2/ab_cmrs_tiled_r.log).
// Workspaces are sized for R = 1.
static int cmrs_tiled_r(int64_t n_rows, int64_t nnz)
{
    return n_rows > 0 && (double)nnz >= 96.0 * (double)n_rows ? 3 : 1;
}

int64_t cmrs_tiled_tile(int64_t n_rows, int64_t nnz) { return 2 * kBlock * cmrs_tiled_r(n_rows, nnz); }
int64_t cmrs_tiled_tile_min() { return 2 * kBlock; }

// xh[i] = x[hot[i]], 4 entries per thread: the 4 index loads go out as one
// 16-byte load, then the 4 gathers together (two round trips per thread,
// a quarter of the workgroups).  vec: hot and xh 16-byte aligned (checked
// by the launcher; otherwise element loads)
__global__ __launch_bounds__(kBlock) void hot_gather_kernel(int64_t H, const int32_t *__restrict__ hot,
                                                            const double *__restrict__ x,
                                                            double *__restrict__ xh, int vec)
{
    const int64_t i = 4 * ((int64_t)blockIdx.x * kBlock + threadIdx.x);
    if (vec && i + 3 < H) {
        const int4 c = *reinterpret_cast<const int4 *>(hot + i);
        const double a = x[c.x], b = x[c.y], d = x[c.z], e = x[c.w];
        *reinterpret_cast<double2 *>(xh + i) = double2{a, b};
        *reinterpret_cast<double2 *>(xh + i + 2) = double2{d, e};
    } else {
        for (int64_t j = i; j < i + 4 && j < H; ++j)
            xh[j] = x[hot[j]];
    }
}

static void launch_hot_gather(int64_t H, const int32_t *hot, const double *x, double *xh, hipStream_t st)
{
    if (H > 0)
        hipLaunchKernelGGL(hot_gather_kernel, dim3((unsigned)((H + 4 * kBlock - 1) / (4 * kBlock))), dim3(kBlock), 0,
                           st, H, hot, x, xh, (int)((((uintptr_t)hot | (uintptr_t)xh) & 15) == 0));
}

int launch_cmrs_tiled(const spmv_dims &d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                      const uint8_t *rin, const int32_t *col, const double *val, const double *x,
                      double *y, int32_t *own_lo, int32_t *carry_row, double *carry_val, int64_t H,
                      const int32_t *hot, double *xh, bool own_lo_ready)
{
    const int64_t ch = cmrs_tiled_tile(d.n_rows, d.nnz);
    const int64_t tiles = (d.nnz + ch - 1) / ch;
    const hipStream_t st = (hipStream_t)d.stream;
    launch_hot_gather(H, hot, x, xh, st);
    if (!own_lo_ready) {  // (a plan fills it once: cmrs_tiled_planned)
        hipLaunchKernelGGL(csr_tile_rows_kernel, dim3((unsigned)((tiles + 1 + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, n_strips, d.nnz, tiles, ch, strip_ptr, own_lo);
        SPMV_CHECK_LAUNCH("csr_tile_rows_kernel (strips)");
    }
    // lanes per row as the staged kernels (one per ~16 entries of the mean
    // row), at most kBlock / h so every carried row key has its group
    int L = spmv_csr_auto_lanes(d.n_rows, d.nnz);
    while (L > 1 && L * h > kBlock)
        L >>= 1;
#define SPMV_CMRS_TILED_R(LL, R)                                                                     \
    do {                                                                                             \
        if (H > 0)                                                                                   \
            hipLaunchKernelGGL((cmrs_tiled_kernel<LL, R, XHot>), dim3((unsigned)tiles), dim3(kBlock), 0, \
                               st, d.n_rows, h, n_strips, d.nnz, tiles, strip_ptr, rin, col, val,       \
                               XHot{x, xh, (int32_t)d.n_cols}, y, own_lo, carry_row, carry_val);       \
        else                                                                                         \
            hipLaunchKernelGGL((cmrs_tiled_kernel<LL, R, XGlobal>), dim3((unsigned)tiles), dim3(kBlock), \
                               0, st, d.n_rows, h, n_strips, d.nnz, tiles, strip_ptr, rin, col, val,    \
                               XGlobal{x}, y, own_lo, carry_row, carry_val);                            \
    } while (0)
#define SPMV_CMRS_TILED(LL)                 \
    do {                                    \
        if (ch == 2 * kBlock)               \
            SPMV_CMRS_TILED_R(LL, 1);       \
        else                                \
            SPMV_CMRS_TILED_R(LL, 3);       \
    } while (0)
    switch (L) {
    case 1: SPMV_CMRS_TILED(1); break;
    case 2: SPMV_CMRS_TILED(2); break;
    case 4: SPMV_CMRS_TILED(4); break;
    case 8: SPMV_CMRS_TILED(8); break;
    case 16: SPMV_CMRS_TILED(16); break;
    case 32: SPMV_CMRS_TILED(32); break;
    default: SPMV_CMRS_TILED(64); break;
    }
#undef SPMV_CMRS_TILED
#undef SPMV_CMRS_TILED_R
    SPMV_CHECK_LAUNCH("cmrs_tiled_kernel");
    return launch_carry((int64_t)h * tiles, carry_row, carry_val, y, st);
}

// Tile = 2·kBlock·R entries.  Round 5: R = 1 (512-entry tiles) for every
// matrix.  With the R-MAT's columns relabelled by degree (no hot table) the
// whole matrix ran 0.772-0.777 ms cold with R = 1 against 0.784-0.785 with
// the round-4 rule (R = 2 for mean rows of 6-95 entries, 3 from 96) and
// 0.806 with R = 3, and every 8-way shard was as fast or faster, the hub
// shard (mean row 179) 0.124 vs 0.130 ms (profiles/round5/ab_tiled_r.md):
// a shard's ~1e4 tiles fill the chip ~6 times, so halving the tile halves
// the grid's tail.  History: round 2 picked R = 1 for R-MAT-like rows
// (0.826 / 0.831 / 0.861 ms with R = 1 / 2 / 3, profiles/round2/ab_tiled_r.log);
// with round 3's wave-per-long-row phase the hot-table R-MAT ran 0.800 /
// 0.785 / 0.788 ms (profiles/round3/rmat_tiled_r.log).  Workspaces and plans
// are sized for the smallest tile (R = 1).
static int tiled_r(int64_t n_rows, int64_t nnz)
{
    (void)n_rows;
    (void)nnz;
    return 1;
}

int64_t csr_tiled_tile(int64_t n_rows, int64_t nnz) { return 2 * kBlock * tiled_r(n_rows, nnz); }
int64_t csr_tiled_tile_min() { return 2 * kBlock; }

template <int R, typename XS, typename V>
static void launch_tiled_r(const spmv_dims &d, int64_t tiles, const int64_t *row_ptr, const int32_t *col,
                           const V *val, XS xs, double *y, const int32_t *own_lo, int32_t *carry_row,
                           double *carry_val, const int32_t *big, int64_t big_len)
{
    const hipStream_t st = (hipStream_t)d.stream;
    // the plain-load variant exists for R = 3 only
    if (R == 3 && !stream_nt(true))
        hipLaunchKernelGGL((csr_tiled_kernel<R, false, XS, V>), dim3((unsigned)tiles), dim3(kBlock), 0, st, d.n_rows,
                           d.nnz, row_ptr, col, val, xs, y, own_lo, carry_row, carry_val, R == 1 ? big : nullptr, big_len);
    else
        hipLaunchKernelGGL((csr_tiled_kernel<R, true, XS, V>), dim3((unsigned)tiles), dim3(kBlock), 0, st, d.n_rows,
                           d.nnz, row_ptr, col, val, xs, y, own_lo, carry_row, carry_val, R == 1 ? big : nullptr, big_len);
}

// A matrix of fewer than two entries (the tiled kernel loads entry pairs):
// one workgroup, a row per thread; the carry pass that follows finds none.
template <typename XS, typename V>
__global__ __launch_bounds__(kBlock) void csr_tiny_kernel(int64_t n_rows, int64_t tiles,
                                                          const int64_t *__restrict__ row_ptr,
                                                          const int32_t *__restrict__ col, const V *__restrict__ val,
                                                          const XS xs, double *__restrict__ y,
                                                          int32_t *__restrict__ carry_row)
{
    for (int64_t r = threadIdx.x; r < n_rows; r += kBlock) {
        double s = 0.0;
        for (int64_t j = row_ptr[r]; j < row_ptr[r + 1]; ++j)
            s += (double)val[j] * xs(col[j]);
        y[r] = s;
    }
    if (threadIdx.x < tiles)
        carry_row[threadIdx.x] = -1;
}

template <typename XS, typename V>
static void launch_tiled_xs(const spmv_dims &d, int64_t tiles, const int64_t *row_ptr, const int32_t *col,
                            const V *val, XS xs, double *y, const int32_t *own_lo, int32_t *carry_row,
                            double *carry_val, const int32_t *big = nullptr, int64_t big_len = 0)
{
    if (d.nnz < 2) {
        hipLaunchKernelGGL((csr_tiny_kernel<XS, V>), dim3(1), dim3(kBlock), 0, (hipStream_t)d.stream, d.n_rows,
                           tiles, row_ptr, col, val, xs, y, carry_row);
        return;
    }
    switch (tiled_r(d.n_rows, d.nnz)) {
    case 1: launch_tiled_r<1>(d, tiles, row_ptr, col, val, xs, y, own_lo, carry_row, carry_val, big, big_len); break;
    case 2: launch_tiled_r<2>(d, tiles, row_ptr, col, val, xs, y, own_lo, carry_row, carry_val, big, big_len); break;
    default: launch_tiled_r<3>(d, tiles, row_ptr, col, val, xs, y, own_lo, carry_row, carry_val, big, big_len); break;
    }
}

int launch_csr_tiled(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                     const double *val, const double *x, double *y, int32_t *own_lo,
                     int32_t *carry_row, double *carry_val)
{
    const int64_t ch = csr_tiled_tile(d.n_rows, d.nnz);
    const int64_t tiles = (d.nnz + ch - 1) / ch;
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(csr_tile_rows_kernel, dim3((unsigned)((tiles + 1 + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, st, d.n_rows, d.nnz, tiles, ch, row_ptr, own_lo);
    SPMV_CHECK_LAUNCH("csr_tile_rows_kernel");
    launch_tiled_xs(d, tiles, row_ptr, col, val, XGlobal{x}, y, own_lo, carry_row, carry_val);
    SPMV_CHECK_LAUNCH("csr_tiled_kernel");
    return SPMV_SUCCESS;
}

template <typename V>
int launch_csr_tiled_hot(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                         const V *val, const double *x, double *y, int64_t H, const int32_t *hot,
                         double *xh, const int32_t *own_lo_plan, int32_t *own_lo, int32_t *carry_row,
                         double *carry_val, const int32_t *big, int64_t big_len)
{
    const int64_t ch = csr_tiled_tile(d.n_rows, d.nnz);
    const int64_t tiles = (d.nnz + ch - 1) / ch;
    const hipStream_t st = (hipStream_t)d.stream;
    launch_hot_gather(H, hot, x, xh, st);
    if (!own_lo_plan) {
        hipLaunchKernelGGL(csr_tile_rows_kernel, dim3((unsigned)((tiles + 1 + kBlock - 1) / kBlock)),
                           dim3(kBlock), 0, st, d.n_rows, d.nnz, tiles, ch, row_ptr, own_lo);
        SPMV_CHECK_LAUNCH("csr_tile_rows_kernel");
        own_lo_plan = own_lo;
    }
    if (H > 0)
        launch_tiled_xs(d, tiles, row_ptr, col, val, XHot{x, xh, (int32_t)d.n_cols}, y, own_lo_plan, carry_row,
                        carry_val, big, big_len);
    else
        launch_tiled_xs(d, tiles, row_ptr, col, val, XGlobal{x}, y, own_lo_plan, carry_row, carry_val, big, big_len);
    SPMV_CHECK_LAUNCH("csr_tiled_kernel (hot columns)");
    return launch_carry(tiles, carry_row, carry_val, y, st);
}

template int launch_csr_tiled_hot<double>(const spmv_dims &, const int64_t *, const int32_t *, const double *,
                                          const double *, double *, int64_t, const int32_t *, double *,
                                          const int32_t *, int32_t *, int32_t *, double *, const int32_t *, int64_t);
template int launch_csr_tiled_hot<float>(const spmv_dims &, const int64_t *, const int32_t *, const float *,
                                         const double *, double *, int64_t, const int32_t *, double *,
                                         const int32_t *, int32_t *, int32_t *, double *, const int32_t *, int64_t);

// ----------------------------------------------------------- launchers
// Geometry of the strip-run CMRS kernel: lanes per row as the staged CSR
// (one per ~16 entries of the mean row), at most 256/h so one strip fits a
// workgroup; G strips per workgroup.  The x windows use the same G.
void cmrs_geometry(const spmv_dims &d, int32_t h, int64_t n_strips, int *L, int *G, int64_t *blocks)
{
    int l = spmv_csr_auto_lanes(d.n_rows, d.nnz);
    while (l > 1 && l * h > kBlock)
        l >>= 1;
    *L = l;
    *G = kBlock / (l * h) > 0 ? kBlock / (l * h) : 1;
    *blocks = (n_strips + *G - 1) / *G;
}

int launch_cmrs_staged(const spmv_dims &d, int32_t h, int64_t n_strips,
                       const int64_t *strip_ptr, const uint8_t *rin, const int32_t *col,
                       const double *val, const double *x, double *y, const int2 *win, int32_t xcap)
{
    int L, G;
    int64_t blocks;
    cmrs_geometry(d, h, n_strips, &L, &G, &blocks);
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    constexpr int R = 3;
    const size_t lds = win ? (size_t)xcap * sizeof(double) : 0;
    const bool nt = stream_nt(true);  // +5 % on the cant batch (0.321 vs 0.338 ms)
    const int remap = xwin_remap(kCmrsRemapDefault) ? 1 : 0;
#define SPMV_CMRS_STAGED(LL)                                                                            \
    do {                                                                                                \
        if (win && nt)                                                                             \
            hipLaunchKernelGGL((cmrs_staged_kernel<LL, R, true, true>), dim3((unsigned)blocks),          \
                               dim3(kBlock), lds, st, d.n_rows, h, G, n_strips, strip_ptr, rin, col, val, \
                               x, y, win, xcap, remap);                                                 \
        else if (win)                                                                                   \
            hipLaunchKernelGGL((cmrs_staged_kernel<LL, R, true>), dim3((unsigned)blocks), dim3(kBlock),  \
                               lds, st, d.n_rows, h, G, n_strips, strip_ptr, rin, col, val, x, y, win,   \
                               xcap, remap);                                                            \
        else                                                                                            \
            hipLaunchKernelGGL((cmrs_staged_kernel<LL, R, false>), dim3((unsigned)blocks), dim3(kBlock), \
                               0, st, d.n_rows, h, G, n_strips, strip_ptr, rin, col, val, x, y,          \
                               (const int2 *)nullptr, 0);                                               \
    } while (0)
    switch (L) {
    case 1: SPMV_CMRS_STAGED(1); break;
    case 2: SPMV_CMRS_STAGED(2); break;
    case 4: SPMV_CMRS_STAGED(4); break;
    case 8: SPMV_CMRS_STAGED(8); break;
    case 16: SPMV_CMRS_STAGED(16); break;
    case 32: SPMV_CMRS_STAGED(32); break;
    default: SPMV_CMRS_STAGED(64); break;
    }
#undef SPMV_CMRS_STAGED
    SPMV_CHECK_LAUNCH("cmrs_staged_kernel");
    return SPMV_SUCCESS;
}

int64_t coo_staged_tile() { return 2 * kBlock * kCooR; }


// COO over the hot-column table (power-law matrices): 512-entry tiles (R =
// 1) below a mean row of 96, as the tiled CSR and CMRS.
static int coo_hot_r(int64_t n_rows, int64_t nnz)
{
    return n_rows > 0 && (double)nnz < 96.0 * (double)n_rows ? 1 : kCooR;
}

int64_t coo_hot_tile(int64_t n_rows, int64_t nnz) { return 2 * kBlock * coo_hot_r(n_rows, nnz); }

// The single pass on fewer than two entries (its kernel loads entry pairs):
// one workgroup; ACC adds into y, else y is written (zeros, then the entry).
template <bool ACC>
__global__ __launch_bounds__(kBlock) void coo_tiny_kernel(int64_t n_rows, int64_t nnz, const int32_t *__restrict__ row,
                                                          const int32_t *__restrict__ col,
                                                          const double *__restrict__ val,
                                                          const double *__restrict__ x, double *__restrict__ y)
{
    if constexpr (!ACC)
        for (int64_t r = threadIdx.x; r < n_rows; r += kBlock)
            y[r] = 0.0;
    __syncthreads();
    if (threadIdx.x == 0 && nnz == 1)
        y[row[0]] = (ACC ? y[row[0]] : 0.0) + val[0] * x[col[0]];
}

int launch_coo_staged_acc(const spmv_dims &d, const int32_t *row, const int32_t *col,
                          const double *val, const double *x, double *y, int32_t *carry_row,
                          double *carry_val, const int32_t *tails)
{
    constexpr int R = kCooR;
    const int64_t tiles = (d.nnz + coo_staged_tile() - 1) / coo_staged_tile();
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "coo tail: grid too large");
    if (tiles == 0)
        return SPMV_SUCCESS;
    if (tails && d.nnz < 2)
        hipLaunchKernelGGL(coo_tiny_kernel<true>, dim3(1), dim3(kBlock), 0, (hipStream_t)d.stream, d.n_rows, d.nnz,
                           row, col, val, x, y);
    else if (tails)  // single pass: every tile finishes its last row (no carry)
        hipLaunchKernelGGL((coo_staged_kernel<4, R, true, false, false, XGlobal, true>), dim3((unsigned)tiles),
                           dim3(kBlock), 0, (hipStream_t)d.stream, d.n_rows, d.nnz, row, col, val, x, y,
                           carry_row, carry_val, (const int2 *)nullptr, 0, XGlobal{x}, tails,
                           xwin_remap(kCooRemapDefault) ? 1 : 0);
    else
        hipLaunchKernelGGL((coo_staged_kernel<4, R, true, false>), dim3((unsigned)tiles), dim3(kBlock), 0,
                           (hipStream_t)d.stream, d.n_rows, d.nnz, row, col, val, x, y, carry_row, carry_val,
                           (const int2 *)nullptr, 0, XGlobal{x});
    SPMV_CHECK_LAUNCH("coo_staged_kernel (accumulate)");
    return SPMV_SUCCESS;
}

int launch_coo_staged_acc_hot(const spmv_dims &d, const int32_t *row, const int32_t *col,
                              const double *val, const double *x, double *y, int32_t *carry_row,
                              double *carry_val, const XHot xs)
{
    constexpr int R = kCooR;
    const int64_t tiles = (d.nnz + coo_staged_tile() - 1) / coo_staged_tile();
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "hyb tail: grid too large");
    if (tiles == 0)
        return SPMV_SUCCESS;
    hipLaunchKernelGGL((coo_staged_kernel<4, R, true, false, true, XHot>), dim3((unsigned)tiles), dim3(kBlock), 0,
                       (hipStream_t)d.stream, d.n_rows, d.nnz, row, col, val, x, y, carry_row, carry_val,
                       (const int2 *)nullptr, 0, xs);
    SPMV_CHECK_LAUNCH("coo_staged_kernel (accumulate, hot columns)");
    return SPMV_SUCCESS;
}

// Tail plan of the single-pass COO: for every full tile, how many entries
// of its last row lie past its end (kCooTailCap + 1 = too many).
__global__ __launch_bounds__(kBlock) void coo_tail_kernel(int64_t nnz, int64_t tiles, int64_t CH,
                                                          const int32_t *__restrict__ row,
                                                          int32_t *__restrict__ tails)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= tiles)
        return;
    const int64_t t1 = (t + 1) * CH;
    int32_t k = 0;
    if (t1 < nnz) {
        const int32_t last = row[t1 - 1];
        while (k <= kCooTailCap && t1 + k < nnz && row[t1 + k] == last)
            ++k;
    }
    tails[t] = k;
}

int64_t coo_tail_build(const spmv_dims &d, const int32_t *row, int32_t *tails)
{
    const int64_t CH = coo_staged_tile();
    const int64_t tiles = (d.nnz + CH - 1) / CH;
    if (tiles <= 0)
        return 0;
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(coo_tail_kernel, dim3((unsigned)((tiles + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, d.nnz,
                       tiles, CH, row, tails);
    if (hipGetLastError() != hipSuccess)
        return -1;
    int32_t *h = (int32_t *)malloc((size_t)tiles * sizeof(int32_t));
    if (!h)
        return -1;
    hipError_t e = hipMemcpyAsync(h, tails, (size_t)tiles * sizeof(int32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    int64_t mx = 0;
    for (int64_t t = 0; e == hipSuccess && t < tiles; ++t)
        mx = h[t] > mx ? h[t] : mx;
    free(h);
    return e == hipSuccess ? mx : -1;
}

int64_t coo_tail_cap() { return kCooTailCap; }

int launch_coo_staged(const spmv_dims &d, const int32_t *row, const int32_t *col,
                      const double *val, const double *x, double *y, int32_t *carry_row,
                      double *carry_val, const int2 *win, int32_t xcap, const int32_t *tails)
{
    constexpr int R = kCooR;
    // the carry pass (with or without x windows) cuts the hot path's tiles
    // (512 entries below a mean row of 96: R-MAT 1.046 -> 0.872 ms warm), so
    // all three keep the same bits; the single pass, 1536
    const int64_t tile = tails ? coo_staged_tile() : coo_hot_tile(d.n_rows, d.nnz);
    const bool r1 = tile != coo_staged_tile();
    const int64_t tiles = (d.nnz + tile - 1) / tile;
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    const size_t lds = win ? (size_t)xcap * sizeof(double) : 0;
    // rows per tile ~ tile / mean row length; 4 lanes per row unless rows are long
    const double mean = d.n_rows > 0 ? (double)d.nnz / (double)d.n_rows : 0.0;
    // non-temporal stream loads: 0.4451 vs 0.4570 ms on the cant batch
    // (SPMV_STREAM_NT=0), three interleaved pairs on one box,
    // profiles/round2/ab_coo_nt.log
    const bool nt = stream_nt(true);
    const int remap = xwin_remap(kCooRemapDefault) ? 1 : 0;  // the single pass (tails) only
    if (tails && d.nnz < 2) {
        hipLaunchKernelGGL(coo_tiny_kernel<false>, dim3(1), dim3(kBlock), 0, st, d.n_rows, d.nnz, row, col, val, x, y);
        SPMV_CHECK_LAUNCH("coo_tiny_kernel");
        return SPMV_SUCCESS;
    }
#define SPMV_COO_STAGED(LL)                                                                              \
    do {                                                                                                 \
        if (tails)                                                                                       \
            hipLaunchKernelGGL((coo_staged_kernel<LL, R, false, false, true, XGlobal, true, RC>),        \
                               dim3((unsigned)tiles), dim3(kBlock), 0, st, d.n_rows, d.nnz, row, col, val, \
                               x, y, carry_row, carry_val, (const int2 *)nullptr, 0, XGlobal{x}, tails,   \
                               remap);                                                                   \
        else if (win && r1)                                                                              \
            hipLaunchKernelGGL((coo_staged_kernel<LL, 1, false, true>), dim3((unsigned)tiles),            \
                               dim3(kBlock), lds, st, d.n_rows, d.nnz, row, col, val, x, y, carry_row,    \
                               carry_val, win, xcap, XGlobal{x});                                        \
        else if (win)                                                                                    \
            hipLaunchKernelGGL((coo_staged_kernel<LL, R, false, true>), dim3((unsigned)tiles),            \
                               dim3(kBlock), lds, st, d.n_rows, d.nnz, row, col, val, x, y, carry_row,    \
                               carry_val, win, xcap, XGlobal{x});                                        \
        else if (nt && r1)                                                                               \
            hipLaunchKernelGGL((coo_staged_kernel<LL, 1, false, false, true, XGlobal, false, RC>),       \
                               dim3((unsigned)tiles), dim3(kBlock), 0, st, d.n_rows, d.nnz, row, col, val, \
                               x, y, carry_row, carry_val, (const int2 *)nullptr, 0, XGlobal{x});         \
        else if (nt)                                                                                     \
            hipLaunchKernelGGL((coo_staged_kernel<LL, R, false, false, true, XGlobal, false, RC>),       \
                               dim3((unsigned)tiles),                                                    \
                               dim3(kBlock), 0, st, d.n_rows, d.nnz, row, col, val, x, y, carry_row,      \
                               carry_val, (const int2 *)nullptr, 0, XGlobal{x});                         \
        else if (r1)                                                                                     \
            hipLaunchKernelGGL((coo_staged_kernel<LL, 1, false, false>), dim3((unsigned)tiles),           \
                               dim3(kBlock), 0, st, d.n_rows, d.nnz, row, col, val, x, y, carry_row,      \
                               carry_val, (const int2 *)nullptr, 0, XGlobal{x});                         \
        else                                                                                             \
            hipLaunchKernelGGL((coo_staged_kernel<LL, R, false, false>), dim3((unsigned)tiles),           \
                               dim3(kBlock), 0, st, d.n_rows, d.nnz, row, col, val, x, y, carry_row,      \
                               carry_val, (const int2 *)nullptr, 0, XGlobal{x});                         \
    } while (0)
    // long rows: 8 lanes. Round 6 on the cant-like single pass, event-cold
    // µs over two pairs: L=8 18.56/18.60, L=4 18.44/18.54 (noise), L=16
    // 19.40/19.36 (profiles/round6/ab_coo_lanes.md)
    if (mean >= 48.0) {
        constexpr int RC = kCooRowCapShort;
        SPMV_COO_STAGED(8);
    } else if (mean >= 12.0) {
        constexpr int RC = kCooRowCapShort;
        SPMV_COO_STAGED(4);
    } else {
        constexpr int RC = kCooRowCap;
        SPMV_COO_STAGED(2);
    }
#undef SPMV_COO_STAGED
    SPMV_CHECK_LAUNCH("coo_staged_kernel");
    return SPMV_SUCCESS;
}

// COO over a hot-column table (power-law columns): non-temporal stream
// loads, the H hottest x values gathered into xh first (as the tiled CSR).
int launch_coo_staged_hot(const spmv_dims &d, const int32_t *row, const int32_t *col, const double *val,
                          const double *x, double *y, int32_t *carry_row, double *carry_val, int64_t H,
                          const int32_t *hot, double *xh)
{
    const int R = coo_hot_r(d.n_rows, d.nnz);
    const int64_t tiles = (d.nnz + coo_hot_tile(d.n_rows, d.nnz) - 1) / coo_hot_tile(d.n_rows, d.nnz);
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run_hot: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    launch_hot_gather(H, hot, x, xh, st);
    const XHot xs{x, xh, (int32_t)d.n_cols};
    const double mean = d.n_rows > 0 ? (double)d.nnz / (double)d.n_rows : 0.0;
#define SPMV_COO_HOT_R(LL, RR)                                                                           \
    hipLaunchKernelGGL((coo_staged_kernel<LL, RR, false, false, true, XHot>), dim3((unsigned)tiles),      \
                       dim3(kBlock), 0, st, d.n_rows, d.nnz, row, col, val, x, y, carry_row, carry_val,    \
                       (const int2 *)nullptr, 0, xs)
#define SPMV_COO_HOT(LL)                \
    do {                                \
        if (R == 1)                     \
            SPMV_COO_HOT_R(LL, 1);      \
        else                            \
            SPMV_COO_HOT_R(LL, kCooR);  \
    } while (0)
    if (mean >= 48.0)
        SPMV_COO_HOT(8);
    else if (mean >= 12.0)
        SPMV_COO_HOT(4);
    else
        SPMV_COO_HOT(2);
#undef SPMV_COO_HOT
#undef SPMV_COO_HOT_R
    SPMV_CHECK_LAUNCH("coo_staged_kernel (hot columns)");
    return SPMV_SUCCESS;
}

// ------------------------------------------------------------ x windows
// Column range of every COO tile / CMRS strip run (build time, one pass
// over col), and the LDS size of a run: the widest window up to the cap.
__global__ __launch_bounds__(kBlock) void tile_window_kernel(int64_t nnz, int64_t per,
                                                             const int32_t *__restrict__ col,
                                                             int2 *__restrict__ win)
{
    const int64_t e0 = (int64_t)blockIdx.x * per;
    const int64_t e1 = e0 + per < nnz ? e0 + per : nnz;
    const int2 r = block_col_range(col, e0, e1);
    if (threadIdx.x == 0)
        win[blockIdx.x] = r;
}

__global__ __launch_bounds__(kBlock) void cmrs_window_kernel(int64_t n_strips, int32_t G,
                                                             const int64_t *__restrict__ strip_ptr,
                                                             const int32_t *__restrict__ col,
                                                             int2 *__restrict__ win)
{
    // every entry the staged kernel LOADS for the run (as csr.hip
    // csr_window_kernel): from two before the 32-entry-aligned first chunk to
    // one past the run's last entry; those outside the run are never summed,
    // but their gathers read LDS and must stay inside the window
    const int64_t s0 = (int64_t)blockIdx.x * G;
    const int64_t s1 = s0 + G < n_strips ? s0 + G : n_strips;
    const int64_t nz = strip_ptr[n_strips];
    const int64_t b = strip_ptr[s0], e = strip_ptr[s1];
    int2 r = {0, -1};
    if (b < e) {  // uniform
        const int64_t c0 = b & ~(int64_t)31;
        r = block_col_range(col, c0 >= 2 ? c0 - 2 : 0, e + 1 < nz ? e + 1 : nz);
    }
    if (threadIdx.x == 0)
        win[blockIdx.x] = r;
}

static int windows_xcap(const int2 *win, int64_t n, int32_t cap, hipStream_t st, int32_t *xcap,
                        const char *who)
{
    int2 *h = (int2 *)malloc((size_t)n * sizeof(int2));
    if (!h)
        return fail_msg(SPMV_OTHER_ERROR, who);
    hipError_t e = hipMemcpyAsync(h, win, (size_t)n * sizeof(int2), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        free(h);
        return fail(SPMV_PROGRAM_ERROR, who, e);
    }
    int32_t best = 0;
    for (int64_t b = 0; b < n; ++b) {
        const int64_t span = (int64_t)h[b].y - h[b].x + 1;
        if (span <= cap && span > best)
            best = (int32_t)span;
    }
    free(h);
    *xcap = best;
    return SPMV_SUCCESS;
}

}  // namespace spmv

using namespace spmv;

extern "C" size_t spmv_coo_xwin_bytes(int64_t nnz)
{
    // one window per carry-pass tile (coo_hot_tile: 512 or 1536 entries)
    return nnz > 0 ? (size_t)((nnz + 2 * kBlock - 1) / (2 * kBlock)) * sizeof(int2) : 0;
}

extern "C" int spmv_coo_xwin_build(spmv_dims d, const int32_t *col, void *win, size_t win_bytes, int32_t *xcap)
{
    if (d.nnz < 0 || !xcap)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_xwin_build: bad arguments");
    *xcap = 0;
    if (d.nnz == 0 || d.n_rows == 0)
        return SPMV_SUCCESS;
    if (!win || win_bytes < spmv_coo_xwin_bytes(d.nnz))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_xwin_build: window buffer too small");
    SPMV_GUARD(d);
    const int64_t tile = coo_hot_tile(d.n_rows, d.nnz);
    const int64_t tiles = (d.nnz + tile - 1) / tile;
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_xwin_build: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(tile_window_kernel, dim3((unsigned)tiles), dim3(kBlock), 0, st, d.nnz, tile, col,
                       (int2 *)win);
    SPMV_CHECK_LAUNCH("tile_window_kernel");
    return windows_xcap((const int2 *)win, tiles, kStagedXwinCap, st, xcap, "spmv_coo_xwin_build: copy windows");
}

extern "C" size_t spmv_cmrs_xwin_bytes(spmv_dims d, int32_t h, int64_t n_strips)
{
    if (h < 1 || h > 64 || n_strips <= 0 || d.nnz <= 0)
        return 0;
    int L, G;
    int64_t blocks;
    cmrs_geometry(d, h, n_strips, &L, &G, &blocks);
    return (size_t)blocks * sizeof(int2);
}

extern "C" int spmv_cmrs_xwin_build(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr,
                                    const int32_t *col, void *win, size_t win_bytes, int32_t *xcap)
{
    if (d.n_rows < 0 || d.nnz < 0 || h < 1 || h > 64 || !xcap || n_strips != (d.n_rows + h - 1) / h)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_xwin_build: bad arguments");
    *xcap = 0;
    if (d.n_rows == 0 || d.nnz == 0)
        return SPMV_SUCCESS;
    if (!win || win_bytes < spmv_cmrs_xwin_bytes(d, h, n_strips))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_xwin_build: window buffer too small");
    SPMV_GUARD(d);
    int L, G;
    int64_t blocks;
    cmrs_geometry(d, h, n_strips, &L, &G, &blocks);
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_xwin_build: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(cmrs_window_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, n_strips, G, strip_ptr, col,
                       (int2 *)win);
    SPMV_CHECK_LAUNCH("cmrs_window_kernel");
    return windows_xcap((const int2 *)win, blocks, kStagedXwinCap, st, xcap, "spmv_cmrs_xwin_build: copy windows");
}

// The tile -> first owned row table of the entry-balanced CSR depends on
// row_ptr only: built once here, the runs skip their pre-pass.
extern "C" int64_t spmv_csr_tiled_plan_len(int64_t nnz)
{
    // own_lo[tiles + 1]
    return nnz > 0 ? (nnz + csr_tiled_tile_min() - 1) / csr_tiled_tile_min() + 1 : 0;
}

extern "C" int spmv_csr_tiled_plan(spmv_dims d, const int64_t *row_ptr, int32_t *own_lo)
{
    if (d.n_rows < 0 || d.nnz < 0 || d.n_rows > INT32_MAX || (d.nnz > 0 && !own_lo))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_tiled_plan: bad arguments");
    if (d.nnz == 0 || d.n_rows == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    const int64_t ch = csr_tiled_tile(d.n_rows, d.nnz);
    const int64_t tiles = (d.nnz + ch - 1) / ch;
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_tiled_plan: grid too large");
    hipLaunchKernelGGL(csr_tile_rows_kernel, dim3((unsigned)((tiles + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)d.stream, d.n_rows, d.nnz, tiles, ch, row_ptr, own_lo);
    SPMV_CHECK_LAUNCH("csr_tile_rows_kernel (plan)");
    return SPMV_SUCCESS;
}
