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

// Streams entries [cb, ce) into LDS: products in s_prod, keys via `key`.
// cb is even, so value pairs are 16-byte aligned; nothing at or past ce
// is read.
template <int R, typename KeyFn>
__device__ __forceinline__ void stage_chunk(int64_t cb, int64_t ce, const int32_t *__restrict__ col,
                                            const double *__restrict__ val,
                                            const double *__restrict__ x, double2 *s_prod,
                                            KeyFn key)
{
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int t = threadIdx.x + k * kBlock;
        const int64_t p = cb + 2 * (int64_t)t;
        double2 pr = {0.0, 0.0};
        if (p + 1 < ce) {
            const double2 v = *reinterpret_cast<const double2 *>(val + p);
            const int2 c = *reinterpret_cast<const int2 *>(col + p);
            pr.x = v.x * x[c.x];
            pr.y = v.y * x[c.y];
            key(t, p, 2);
        } else if (p < ce) {
            pr.x = val[p] * x[col[p]];
            key(t, p, 1);
        }
        s_prod[t] = pr;
    }
}

// ------------------------------------------------------------------ CMRS
// A workgroup owns G consecutive strips (G·h rows, L lanes per row).
template <int L, int R>
__global__ __launch_bounds__(kBlock) void cmrs_staged_kernel(
    int64_t n_rows, int32_t h, int32_t G, int64_t n_strips,
    const int64_t *__restrict__ strip_ptr, const uint8_t *__restrict__ rin,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y)
{
    constexpr int CH = 2 * kBlock * R;
    __shared__ int64_t s_sp[kBlock + 1];
    __shared__ double2 s_prod[kBlock * R];
    __shared__ uint16_t s_key2[kBlock * R];  // keys of entry pairs
    const uint8_t *s_key = reinterpret_cast<const uint8_t *>(s_key2);
    const double *prod = reinterpret_cast<const double *>(s_prod);

    const int64_t s0 = (int64_t)blockIdx.x * G;
    if ((int)threadIdx.x <= G) {
        const int64_t s = s0 + threadIdx.x;
        s_sp[threadIdx.x] = strip_ptr[s < n_strips ? s : n_strips];
    }
    __syncthreads();

    const int rl = threadIdx.x / L, lane = threadIdx.x % L;
    const bool active = rl < G * h;
    const int si = active ? rl / h : 0;
    const int key = active ? rl % h : 0;
    const int64_t sb = s_sp[si], se = active ? s_sp[si + 1] : s_sp[si];
    const int64_t row = (s0 + si) * h + key;
    const int64_t blk_end = s_sp[G];

    double acc = 0.0;
    for (int64_t cb = s_sp[0] & ~(int64_t)1; cb < blk_end; cb += CH) {
        const int64_t ce = cb + CH < blk_end ? cb + CH : blk_end;
        stage_chunk<R>(cb, ce, col, val, x, s_prod, [&](int t, int64_t p, int n) {
            s_key2[t] = n == 2 ? *reinterpret_cast<const uint16_t *>(rin + p) : (uint16_t)rin[p];
        });
        __syncthreads();
        const int64_t lo = sb > cb ? sb : cb;
        const int64_t hi = se < ce ? se : ce;
        if (lo < hi) {  // this strip has entries in the chunk: find the row
            const int a = lower_bound_lds(s_key, (int)(lo - cb), (int)(hi - cb), key);
            const int b = lower_bound_lds(s_key, a, (int)(hi - cb), key + 1);
            for (int j = a + lane; j < b; j += L)
                acc += prod[j];
        }
        __syncthreads();
    }
    acc = group_sum<L>(acc);
    if (active && lane == 0 && row < n_rows && s0 + si < n_strips)
        y[row] = acc;
}

// ------------------------------------------------------------------- COO
// A workgroup owns one tile of CH consecutive row-sorted entries and
// writes y for rows (row[t0-1], row[t1-1]] (rows without entries get 0;
// the last tile also covers the trailing rows).  A first row that began
// in an earlier tile goes to carry[tile] for coo_carry_kernel (coo.hip).
template <int L, int R, bool ACC = false>
__global__ __launch_bounds__(kBlock) void coo_staged_kernel(
    int64_t n_rows, int64_t nnz, const int32_t *__restrict__ row,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y, int32_t *__restrict__ carry_row,
    double *__restrict__ carry_val)
{
    constexpr int CH = 2 * kBlock * R;
    constexpr int GROUPS = kBlock / L;
    __shared__ double2 s_prod[kBlock * R];
    __shared__ int2 s_row2[kBlock * R];
    __shared__ int32_t s_prev;
    const int32_t *s_row = reinterpret_cast<const int32_t *>(s_row2);
    const double *prod = reinterpret_cast<const double *>(s_prod);

    const int64_t tile = blockIdx.x;
    const int64_t t0 = tile * CH;
    const int64_t t1 = t0 + CH < nnz ? t0 + CH : nnz;
    const int n = (int)(t1 - t0);
    if (threadIdx.x == 0)
        s_prev = t0 > 0 ? row[t0 - 1] : -1;
    stage_chunk<R>(t0, t1, col, val, x, s_prod, [&](int t, int64_t p, int cnt) {
        s_row2[t] = cnt == 2 ? *reinterpret_cast<const int2 *>(row + p) : make_int2(row[p], 0);
    });
    __syncthreads();

    const int32_t prev = s_prev;
    const int32_t first = s_row[0], last = s_row[n - 1];
    const bool first_continues = prev == first;
    const int g = threadIdx.x / L, lane = threadIdx.x % L;

    // carry: the first row's entries when it began in an earlier tile
    if (g == 0) {
        double c = 0.0;
        if (first_continues) {
            const int b = lower_bound_lds(s_row, 0, n, first + 1);
            for (int j = lane; j < b; j += L)
                c += prod[j];
        }
        c = group_sum<L>(c);
        if (lane == 0) {
            carry_row[tile] = first_continues ? first : -1;
            carry_val[tile] = c;
        }
    }
    if constexpr (ACC) {
        // accumulate mode (HYB tail): y[r] += the tile's entries of every row
        // that begins here; rows without entries are left untouched, so only
        // the row keys present are visited: one thread per run of equal keys,
        // summed in entry order
        for (int j = threadIdx.x; j < n; j += kBlock) {
            const int32_t r = s_row[j];
            const bool head = j == 0 ? r != prev : r != s_row[j - 1];
            if (!head || (j == 0 && first_continues))
                continue;
            double s = 0.0;
            int k = j;
            for (; k < n && s_row[k] == r; ++k)
                s += prod[k];
            y[r] += s;
        }
        return;
    }
    // owned rows: (prev, last], plus the trailing empty rows in the last
    // tile; a continued first row equals prev, so it is excluded here
    const int64_t r_lo = (int64_t)prev + 1;
    const int64_t r_hi = t1 == nnz ? n_rows - 1 : (int64_t)last;
    for (int64_t r = r_lo + g; r <= r_hi; r += GROUPS) {
        double s = 0.0;
        if (r <= last) {
            const int a = lower_bound_lds(s_row, 0, n, (int)r);
            const int b = lower_bound_lds(s_row, a, n, (int)r + 1);
            for (int j = a + lane; j < b; j += L)
                s += prod[j];
        }
        s = group_sum<L>(s);
        if (lane == 0)
            y[r] = s;
    }
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

template <int L, int R>
__global__ __launch_bounds__(kBlock) void csr_tiled_kernel(
    int64_t n_rows, int64_t nnz, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ x, double *__restrict__ y,
    const int32_t *__restrict__ own_lo, int32_t *__restrict__ carry_row,
    double *__restrict__ carry_val)
{
    constexpr int CH = 2 * kBlock * R;
    constexpr int GROUPS = kBlock / L;
    __shared__ double2 s_prod[kBlock * R];
    const double *prod = reinterpret_cast<const double *>(s_prod);
    const int64_t tile = blockIdx.x;
    const int64_t t0 = tile * CH;
    const int64_t t1 = t0 + CH < nnz ? t0 + CH : nnz;
    const int64_t r_lo = own_lo[tile];
    const int64_t r_hi = t1 == nnz ? n_rows - 1 : (int64_t)own_lo[tile + 1] - 1;
    stage_chunk<R>(t0, t1, col, val, x, s_prod, [](int, int64_t, int) {});
    __syncthreads();
    const int g = threadIdx.x / L, lane = threadIdx.x % L;

    // carry: entry t0 lies in row r_lo-1 when no row starts exactly at t0
    if (g == 0) {
        double c = 0.0;
        int32_t cr = -1;
        if (r_lo > 0 && (r_lo == n_rows || row_ptr[r_lo] > t0)) {
            cr = (int32_t)(r_lo - 1);
            const int64_t e = row_ptr[r_lo - 1 + 1] < t1 ? row_ptr[r_lo] : t1;
            for (int64_t j = t0 + lane; j < e; j += L)
                c += prod[j - t0];
        }
        c = group_sum<L>(c);
        if (lane == 0) {
            carry_row[tile] = cr;
            carry_val[tile] = c;
        }
    }
    for (int64_t r = r_lo + g; r <= r_hi; r += GROUPS) {
        const int64_t a = row_ptr[r];
        int64_t b = row_ptr[r + 1];
        b = b < t1 ? b : t1;
        double s = 0.0;
        for (int64_t j = a + lane; j < b; j += L)
            s += prod[j - t0];
        s = group_sum<L>(s);
        if (lane == 0)
            y[r] = s;
    }
}

int64_t csr_tiled_tile() { return 2 * kBlock * 3; }

int launch_csr_tiled(const spmv_dims &d, const int64_t *row_ptr, const int32_t *col,
                     const double *val, const double *x, double *y, int32_t *own_lo,
                     int32_t *carry_row, double *carry_val)
{
    constexpr int R = 3;
    const int64_t ch = csr_tiled_tile();
    const int64_t tiles = (d.nnz + ch - 1) / ch;
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(csr_tile_rows_kernel, dim3((unsigned)((tiles + 1 + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, st, d.n_rows, d.nnz, tiles, ch, row_ptr, own_lo);
    SPMV_CHECK_LAUNCH("csr_tile_rows_kernel");
    const double mean = d.n_rows > 0 ? (double)d.nnz / (double)d.n_rows : 0.0;
    if (mean >= 48.0)
        hipLaunchKernelGGL((csr_tiled_kernel<8, R>), dim3((unsigned)tiles), dim3(kBlock), 0, st,
                           d.n_rows, d.nnz, row_ptr, col, val, x, y, own_lo, carry_row, carry_val);
    else if (mean >= 12.0)
        hipLaunchKernelGGL((csr_tiled_kernel<4, R>), dim3((unsigned)tiles), dim3(kBlock), 0, st,
                           d.n_rows, d.nnz, row_ptr, col, val, x, y, own_lo, carry_row, carry_val);
    else
        hipLaunchKernelGGL((csr_tiled_kernel<2, R>), dim3((unsigned)tiles), dim3(kBlock), 0, st,
                           d.n_rows, d.nnz, row_ptr, col, val, x, y, own_lo, carry_row, carry_val);
    SPMV_CHECK_LAUNCH("csr_tiled_kernel");
    return SPMV_SUCCESS;
}

// ----------------------------------------------------------- launchers
int launch_cmrs_staged(const spmv_dims &d, int32_t h, int64_t n_strips,
                       const int64_t *strip_ptr, const uint8_t *rin, const int32_t *col,
                       const double *val, const double *x, double *y)
{
    // lanes per row: one per ~16 entries of the mean row (as staged CSR),
    // at most 256/h so one strip fits a workgroup
    int L = spmv_csr_auto_lanes(d.n_rows, d.nnz);
    while (L > 1 && L * h > kBlock)
        L >>= 1;
    const int G = kBlock / (L * h) > 0 ? kBlock / (L * h) : 1;
    const int64_t blocks = (n_strips + G - 1) / G;
    if (blocks > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_cmrs_run: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    constexpr int R = 3;
#define SPMV_CMRS_STAGED(LL)                                                                    \
    hipLaunchKernelGGL((cmrs_staged_kernel<LL, R>), dim3((unsigned)blocks), dim3(kBlock), 0, st, \
                       d.n_rows, h, G, n_strips, strip_ptr, rin, col, val, x, y)
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

int64_t coo_staged_tile() { return 2 * kBlock * 3; }

int launch_coo_staged_acc(const spmv_dims &d, const int32_t *row, const int32_t *col,
                          const double *val, const double *x, double *y, int32_t *carry_row,
                          double *carry_val)
{
    constexpr int R = 3;
    const int64_t tiles = (d.nnz + coo_staged_tile() - 1) / coo_staged_tile();
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "coo tail: grid too large");
    if (tiles == 0)
        return SPMV_SUCCESS;
    hipLaunchKernelGGL((coo_staged_kernel<4, R, true>), dim3((unsigned)tiles), dim3(kBlock), 0,
                       (hipStream_t)d.stream, d.n_rows, d.nnz, row, col, val, x, y, carry_row, carry_val);
    SPMV_CHECK_LAUNCH("coo_staged_kernel (accumulate)");
    return SPMV_SUCCESS;
}

int launch_coo_staged(const spmv_dims &d, const int32_t *row, const int32_t *col,
                      const double *val, const double *x, double *y, int32_t *carry_row,
                      double *carry_val)
{
    constexpr int R = 3;
    const int64_t tiles = (d.nnz + coo_staged_tile() - 1) / coo_staged_tile();
    if (tiles > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_coo_run: grid too large");
    const hipStream_t st = (hipStream_t)d.stream;
    // rows per tile ~ tile / mean row length; 4 lanes per row unless rows are long
    const double mean = d.n_rows > 0 ? (double)d.nnz / (double)d.n_rows : 0.0;
    if (mean >= 48.0)
        hipLaunchKernelGGL((coo_staged_kernel<8, R>), dim3((unsigned)tiles), dim3(kBlock), 0, st,
                           d.n_rows, d.nnz, row, col, val, x, y, carry_row, carry_val);
    else if (mean >= 12.0)
        hipLaunchKernelGGL((coo_staged_kernel<4, R>), dim3((unsigned)tiles), dim3(kBlock), 0, st,
                           d.n_rows, d.nnz, row, col, val, x, y, carry_row, carry_val);
    else
        hipLaunchKernelGGL((coo_staged_kernel<2, R>), dim3((unsigned)tiles), dim3(kBlock), 0, st,
                           d.n_rows, d.nnz, row, col, val, x, y, carry_row, carry_val);
    SPMV_CHECK_LAUNCH("coo_staged_kernel");
    return SPMV_SUCCESS;
}

}  // namespace spmv
