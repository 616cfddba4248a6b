// build.hip — format construction on the device.
//
// The reference builds every format on the host while parsing the file
// (reference csr.c:68-91, ell.c:68-164, sigma_c.c:71-202, cmrs.c:72-117),
// and so do the host builders of this suite (host/formats.c).  For the
// 1e9-entry configurations (BASELINE.json configs[4]) the host round trip
// is the bottleneck, so these entry points build CSR, ELL, SELL-C-sigma and
// CMRS from a COO that is already in HBM.  Every array they produce is
// element-for-element the host builders' (tests/test_build_gpu.py):
//   CSR   stable by row (file order inside a row): a stable LSD radix sort
//         of the row keys with the entry index as payload, then a gather;
//   ELL   K = longest row rounded up to ki, ld = round_up(N, 64), padding
//         value 0.0 and column = the row's last column (0 for empty rows);
//   SELL  rows sorted by (length descending, row ascending) inside every
//         sigma-window — one workgroup per window, a bitonic sort of packed
//         64-bit keys in LDS — slice widths = longest row of the slice,
//         padding column = the row's last column, else the first column of
//         the first non-empty row of the slice;
//   CMRS  strip_ptr from row_ptr, row_in_strip = row % h.
// Builders allocate their scratch, run on d.stream and synchronise it
// before returning (build time, never on the SpMV path).
#include <hipcub/hipcub.hpp>
#include <stdlib.h>

#include "common.h"

namespace spmv {

// ------------------------------------------------------------------ CSR
__global__ void coo_rows_check_kernel(int64_t nnz, int64_t n_rows, const int32_t *__restrict__ row,
                                      uint32_t *__restrict__ keys, int *__restrict__ bad)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride) {
        const int32_t r = row[i];
        if (r < 0 || r >= n_rows)
            *bad = 1;
        keys[i] = (uint32_t)(r < 0 ? 0 : r);
    }
}

template <typename I>
__global__ void iota_kernel(int64_t n, I *__restrict__ v)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        v[i] = (I)i;
}

// row_ptr from the sorted row keys: entry i opens rows (key[i-1], key[i]]
__global__ void row_ptr_from_sorted_kernel(int64_t nnz, int64_t n_rows, const uint32_t *__restrict__ keys,
                                           int64_t *__restrict__ row_ptr)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= nnz; i += stride) {
        const int64_t prev = i == 0 ? -1 : (int64_t)keys[i - 1];
        const int64_t cur = i == nnz ? n_rows : (int64_t)keys[i];
        for (int64_t r = prev + 1; r <= cur; ++r)
            row_ptr[r] = i;
    }
}

template <typename I>
__global__ void gather_entries_kernel(int64_t nnz, const I *__restrict__ idx, const int32_t *__restrict__ col,
                                      const double *__restrict__ val, int32_t *__restrict__ col_out,
                                      double *__restrict__ val_out)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += stride) {
        const int64_t j = (int64_t)idx[i];
        col_out[i] = col[j];
        val_out[i] = val[j];
    }
}

static unsigned grid_for(int64_t n)
{
    const int64_t g = (n + kBlock - 1) / kBlock;
    return (unsigned)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

// Scratch that frees itself; every builder synchronises its stream first.
struct Scratch {
    void *p = nullptr;
    hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 1); }
    ~Scratch()
    {
        if (p)
            (void)hipFree(p);
    }
};

template <typename I>
static int csr_from_coo_impl(const spmv_dims &d, const int32_t *row, const int32_t *col, const double *val,
                             int64_t *row_ptr, int32_t *col_out, double *val_out)
{
    const hipStream_t st = (hipStream_t)d.stream;
    const int64_t nnz = d.nnz, n = d.n_rows;
    Scratch keys_in, keys_out, idx_in, idx_out, bad, tmp;
    hipError_t e;
    if ((e = keys_in.alloc(nnz * 4)) != hipSuccess || (e = keys_out.alloc(nnz * 4)) != hipSuccess ||
        (e = idx_in.alloc(nnz * sizeof(I))) != hipSuccess || (e = idx_out.alloc(nnz * sizeof(I))) != hipSuccess ||
        (e = bad.alloc(sizeof(int))) != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_dev_csr_from_coo: scratch", e);
    if ((e = hipMemsetAsync(bad.p, 0, sizeof(int), st)) != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_dev_csr_from_coo: memset", e);
    hipLaunchKernelGGL(coo_rows_check_kernel, dim3(grid_for(nnz)), dim3(kBlock), 0, st, nnz, n, row,
                       (uint32_t *)keys_in.p, (int *)bad.p);
    hipLaunchKernelGGL((iota_kernel<I>), dim3(grid_for(nnz)), dim3(kBlock), 0, st, nnz, (I *)idx_in.p);
    int end_bit = 1;
    while (end_bit < 32 && ((int64_t)1 << end_bit) < n)
        ++end_bit;
    size_t tbytes = 0;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, tbytes, (const uint32_t *)keys_in.p, (uint32_t *)keys_out.p,
                                           (const I *)idx_in.p, (I *)idx_out.p, nnz, 0, end_bit, st);
    if (e == hipSuccess)
        e = tmp.alloc(tbytes);
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(tmp.p, tbytes, (const uint32_t *)keys_in.p, (uint32_t *)keys_out.p,
                                               (const I *)idx_in.p, (I *)idx_out.p, nnz, 0, end_bit, st);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_dev_csr_from_coo: radix sort", e);
    hipLaunchKernelGGL(row_ptr_from_sorted_kernel, dim3(grid_for(nnz + 1)), dim3(kBlock), 0, st, nnz, n,
                       (const uint32_t *)keys_out.p, row_ptr);
    hipLaunchKernelGGL((gather_entries_kernel<I>), dim3(grid_for(nnz)), dim3(kBlock), 0, st, nnz,
                       (const I *)idx_out.p, col, val, col_out, val_out);
    SPMV_CHECK_LAUNCH("csr build kernels");
    int h_bad = 0;
    if ((e = hipMemcpyAsync(&h_bad, bad.p, sizeof(int), hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_dev_csr_from_coo: sync", e);
    return h_bad ? fail_msg(SPMV_OTHER_ERROR, "spmv_dev_csr_from_coo: row index out of range") : SPMV_SUCCESS;
}

// ------------------------------------------------------------------ ELL
__global__ void row_len_max_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr,
                                   unsigned long long *__restrict__ out)
{
    int64_t m = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_rows; i += stride) {
        const int64_t l = row_ptr[i + 1] - row_ptr[i];
        m = l > m ? l : m;
    }
    atomicMax(out, (unsigned long long)m);  // max is order-independent
}

__global__ void ell_fill_kernel(int64_t n_rows, const int64_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
                                const double *__restrict__ val, int32_t K, int64_t ld, int32_t ki,
                                int32_t *__restrict__ col_out, double *__restrict__ val_out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ld)
        return;
    int64_t b = 0, e = 0;
    if (i < n_rows) {
        b = row_ptr[i];
        e = row_ptr[i + 1];
    }
    const int32_t pad_col = e > b ? col[e - 1] : 0;
    for (int64_t k = 0; k < K; ++k) {
        const int64_t pos = (k / ki) * ld * ki + i * ki + (k % ki);
        if (b + k < e) {
            col_out[pos] = col[b + k];
            val_out[pos] = val[b + k];
        } else {
            col_out[pos] = pad_col;
            val_out[pos] = 0.0;
        }
    }
}

// ----------------------------------------------------------------- SELL
// One workgroup per sigma-window: bitonic sort of (INT32_MAX - len, row)
// packed in 64 bits, ascending = length descending, row ascending (the
// host's qsort order, host/formats.c cmp_len_desc).
constexpr int kSortMax = 4096;  // largest sigma sorted on the device (32 KiB of keys)

__global__ __launch_bounds__(1024) void sell_window_sort_kernel(int64_t n_rows, int32_t sigma,
                                                                const int64_t *__restrict__ row_ptr,
                                                                int32_t *__restrict__ perm)
{
    __shared__ unsigned long long s_k[kSortMax];
    const int64_t r0 = (int64_t)blockIdx.x * sigma;
    const int64_t n = r0 + sigma < n_rows ? sigma : n_rows - r0;
    int P = 1;
    while (P < n)
        P <<= 1;
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
        unsigned long long k = ~0ull;
        if (i < n) {
            const int64_t len = row_ptr[r0 + i + 1] - row_ptr[r0 + i];
            k = ((unsigned long long)(uint32_t)(INT32_MAX - (int32_t)len) << 32) | (uint32_t)i;
        }
        s_k[i] = k;
    }
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;
                    const unsigned long long a = s_k[i], b = s_k[j];
                    if ((a > b) == up) {
                        s_k[i] = b;
                        s_k[j] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        perm[r0 + i] = (int32_t)(r0 + (int64_t)(uint32_t)(s_k[i] & 0xffffffffu));
}

__global__ void sell_perm_init_kernel(int64_t slots, int64_t n_rows, int32_t *__restrict__ perm)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slots; i += stride)
        perm[i] = i < n_rows ? (int32_t)i : -1;
}

// per slice: width (longest row, rounded to ki) * C, and the padding
// column of empty rows (first column of the first non-empty row)
__global__ void sell_slice_kernel(int64_t n_slices, int32_t C, int32_t ki, const int64_t *__restrict__ row_ptr,
                                  const int32_t *__restrict__ col, const int32_t *__restrict__ perm,
                                  int64_t *__restrict__ slice_len, int32_t *__restrict__ slice_col)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slices)
        return;
    int64_t w = 0;
    int32_t sc = 0;
    bool found = false;
    for (int32_t r = 0; r < C; ++r) {
        const int32_t row = perm[s * C + r];
        if (row < 0)
            continue;
        const int64_t b = row_ptr[row], l = row_ptr[row + 1] - b;
        w = l > w ? l : w;
        if (!found && l > 0) {
            sc = col[b];
            found = true;
        }
    }
    slice_len[s] = (w + ki - 1) / ki * ki * C;
    slice_col[s] = sc;
}

__global__ void sell_fill_kernel(int64_t n_slices, int32_t C, int32_t ki, const int64_t *__restrict__ row_ptr,
                                 const int32_t *__restrict__ col, const double *__restrict__ val,
                                 const int64_t *__restrict__ slice_ptr, const int32_t *__restrict__ perm,
                                 const int32_t *__restrict__ slice_col, int32_t *__restrict__ col_out,
                                 double *__restrict__ val_out)
{
    const int64_t slot = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = slot / C;
    if (s >= n_slices)
        return;
    const int64_t r = slot - s * C;
    const int64_t base = slice_ptr[s];
    const int64_t w = (slice_ptr[s + 1] - base) / C;
    const int32_t row = perm[slot];
    int64_t b = 0, e = 0;
    if (row >= 0) {
        b = row_ptr[row];
        e = row_ptr[row + 1];
    }
    const int32_t pad_col = e > b ? col[e - 1] : slice_col[s];
    for (int64_t k = 0; k < w; ++k) {
        const int64_t pos = base + (k / ki) * (int64_t)C * ki + r * ki + (k % ki);
        if (b + k < e) {
            col_out[pos] = col[b + k];
            val_out[pos] = val[b + k];
        } else {
            col_out[pos] = pad_col;
            val_out[pos] = 0.0;
        }
    }
}

// ----------------------------------------------------------------- CMRS
__global__ void cmrs_strip_kernel(int64_t n_rows, int32_t h, int64_t n_strips, const int64_t *__restrict__ row_ptr,
                                  int64_t *__restrict__ strip_ptr)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s > n_strips)
        return;
    const int64_t r = s * h < n_rows ? s * h : n_rows;
    strip_ptr[s] = row_ptr[r];
}

__global__ void cmrs_rin_kernel(int64_t n_rows, int32_t h, const int64_t *__restrict__ row_ptr,
                                uint8_t *__restrict__ rin)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows)
        return;
    for (int64_t j = row_ptr[r]; j < row_ptr[r + 1]; ++j)
        rin[j] = (uint8_t)(r % h);
}

static int sync_or_fail(hipStream_t st, const char *who)
{
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, who, e);
}

}  // namespace spmv

using namespace spmv;

extern "C" int spmv_dev_csr_from_coo(spmv_dims d, const int32_t *row, const int32_t *col, const double *val,
                                     int64_t *row_ptr, int32_t *col_out, double *val_out)
{
    if (d.n_rows < 0 || d.nnz < 0 || d.n_rows > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_csr_from_coo: bad sizes");
    SPMV_GUARD(d);
    if (d.nnz == 0) {
        hipError_t e = hipMemsetAsync(row_ptr, 0, (size_t)(d.n_rows + 1) * sizeof(int64_t), (hipStream_t)d.stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize((hipStream_t)d.stream);
        return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "spmv_dev_csr_from_coo", e);
    }
    return d.nnz <= (int64_t)UINT32_MAX
               ? csr_from_coo_impl<uint32_t>(d, row, col, val, row_ptr, col_out, val_out)
               : csr_from_coo_impl<uint64_t>(d, row, col, val, row_ptr, col_out, val_out);
}

extern "C" int spmv_dev_ell_plan(spmv_dims d, const int64_t *row_ptr, int32_t ki, int32_t *K, int64_t *ld)
{
    if (d.n_rows < 0 || (ki != 1 && ki != 2) || !K || !ld)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_ell_plan: bad arguments");
    SPMV_GUARD(d);
    const hipStream_t st = (hipStream_t)d.stream;
    Scratch mx;
    hipError_t e = mx.alloc(sizeof(unsigned long long));
    if (e == hipSuccess)
        e = hipMemsetAsync(mx.p, 0, sizeof(unsigned long long), st);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_dev_ell_plan: scratch", e);
    hipLaunchKernelGGL(row_len_max_kernel, dim3(grid_for(d.n_rows)), dim3(kBlock), 0, st, d.n_rows, row_ptr,
                       (unsigned long long *)mx.p);
    unsigned long long h = 0;
    e = hipMemcpyAsync(&h, mx.p, sizeof h, hipMemcpyDeviceToHost, st);
    int rc = e == hipSuccess ? sync_or_fail(st, "spmv_dev_ell_plan") : fail(SPMV_PROGRAM_ERROR, "spmv_dev_ell_plan", e);
    if (rc != SPMV_SUCCESS)
        return rc;
    const int64_t k = ((int64_t)h + ki - 1) / ki * ki;
    if (k > INT32_MAX)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_ell_plan: K too large");
    *K = (int32_t)k;
    *ld = (d.n_rows + 63) / 64 * 64;
    return SPMV_SUCCESS;
}

extern "C" int spmv_dev_ell_fill(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                                 int32_t K, int64_t ld, int32_t ki, int32_t *col_out, double *val_out)
{
    if ((ki != 1 && ki != 2) || K < 0 || K % ki != 0 || ld < d.n_rows || ld % 64 != 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_ell_fill: bad arguments");
    if (ld == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    const hipStream_t st = (hipStream_t)d.stream;
    hipLaunchKernelGGL(ell_fill_kernel, dim3((unsigned)((ld + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       d.n_rows, row_ptr, col, val, K, ld, ki, col_out, val_out);
    return sync_or_fail(st, "spmv_dev_ell_fill");
}

extern "C" int spmv_dev_sell_plan(spmv_dims d, const int64_t *row_ptr, const int32_t *col, int32_t C,
                                  int32_t sigma, int32_t ki, int64_t n_slices, int32_t *perm, int64_t *slice_ptr,
                                  int32_t *slice_col, int64_t *stored)
{
    if (d.n_rows < 0 || d.n_rows > INT32_MAX || C <= 0 || C > 1024 || (ki != 1 && ki != 2) || !stored)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_sell_plan: bad arguments");
    if (sigma > 1 && sigma % C != 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_sell_plan: sigma must be 1 or a multiple of C");
    if (sigma > kSortMax)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_sell_plan: sigma > 4096 (use the host builder)");
    if (n_slices != (d.n_rows + C - 1) / C)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_sell_plan: n_slices != ceil(N/C)");
    SPMV_GUARD(d);
    const hipStream_t st = (hipStream_t)d.stream;
    const int64_t slots = n_slices * C;
    hipLaunchKernelGGL(sell_perm_init_kernel, dim3(grid_for(slots)), dim3(kBlock), 0, st, slots, d.n_rows, perm);
    if (sigma > 1 && d.n_rows > 0) {
        const int64_t n_win = (d.n_rows + sigma - 1) / sigma;
        hipLaunchKernelGGL(sell_window_sort_kernel, dim3((unsigned)n_win), dim3(1024), 0, st, d.n_rows, sigma,
                           row_ptr, perm);
    }
    Scratch lens, tmp;
    hipError_t e = lens.alloc((size_t)(n_slices + 1) * sizeof(int64_t));
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_dev_sell_plan: scratch", e);
    if (n_slices > 0)
        hipLaunchKernelGGL(sell_slice_kernel, dim3((unsigned)((n_slices + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           st, n_slices, C, ki, row_ptr, col, perm, (int64_t *)lens.p, slice_col);
    // slice_ptr = exclusive scan of the slice lengths (n_slices + 1 entries)
    e = hipMemsetAsync((int64_t *)lens.p + n_slices, 0, sizeof(int64_t), st);
    size_t tbytes = 0;
    if (e == hipSuccess)
        e = hipcub::DeviceScan::ExclusiveSum(nullptr, tbytes, (const int64_t *)lens.p, slice_ptr, n_slices + 1, st);
    if (e == hipSuccess)
        e = tmp.alloc(tbytes);
    if (e == hipSuccess)
        e = hipcub::DeviceScan::ExclusiveSum(tmp.p, tbytes, (const int64_t *)lens.p, slice_ptr, n_slices + 1, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(stored, slice_ptr + n_slices, sizeof(int64_t), hipMemcpyDeviceToHost, st);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_dev_sell_plan: scan", e);
    return sync_or_fail(st, "spmv_dev_sell_plan");
}

extern "C" int spmv_dev_sell_fill(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                                  int32_t C, int32_t ki, int64_t n_slices, const int64_t *slice_ptr,
                                  const int32_t *perm, const int32_t *slice_col, int32_t *col_out,
                                  double *val_out)
{
    if (C <= 0 || C > 1024 || (ki != 1 && ki != 2) || n_slices < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_sell_fill: bad arguments");
    if (n_slices == 0)
        return SPMV_SUCCESS;
    SPMV_GUARD(d);
    const hipStream_t st = (hipStream_t)d.stream;
    const int64_t slots = n_slices * C;
    hipLaunchKernelGGL(sell_fill_kernel, dim3((unsigned)((slots + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       n_slices, C, ki, row_ptr, col, val, slice_ptr, perm, slice_col, col_out, val_out);
    return sync_or_fail(st, "spmv_dev_sell_fill");
}

extern "C" int spmv_dev_cmrs_build(spmv_dims d, const int64_t *row_ptr, int32_t h, int64_t *strip_ptr,
                                   uint8_t *row_in_strip)
{
    if (h < 1 || h > 64 || d.n_rows < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dev_cmrs_build: bad arguments");
    SPMV_GUARD(d);
    const hipStream_t st = (hipStream_t)d.stream;
    const int64_t ns = (d.n_rows + h - 1) / h;
    hipLaunchKernelGGL(cmrs_strip_kernel, dim3((unsigned)((ns + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       d.n_rows, h, ns, row_ptr, strip_ptr);
    if (d.n_rows > 0)
        hipLaunchKernelGGL(cmrs_rin_kernel, dim3((unsigned)((d.n_rows + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           d.n_rows, h, row_ptr, row_in_strip);
    return sync_or_fail(st, "spmv_dev_cmrs_build");
}
