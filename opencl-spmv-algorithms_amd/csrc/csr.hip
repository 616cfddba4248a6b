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

#include "common.h"

namespace spmv {

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

    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if constexpr (PAIR) {
        // 16-byte loads: lane reads the aligned pair (p, p+1); entries of
        // the pair outside [beg, end) are zeroed by value (their column is
        // a valid neighbour column, so the gather stays in bounds).  The
        // last pair of the row is loaded as a scalar when p+1 == end, so
        // nothing past val[nnz-1] is ever read.
        int64_t p = (beg & ~(int64_t)1) + 2 * lane;
        for (; p + 1 + 2 * L < end; p += 4 * L) {
            const double2 va = *reinterpret_cast<const double2 *>(val + p);
            const int2 ca = *reinterpret_cast<const int2 *>(col + p);
            const double2 vb = *reinterpret_cast<const double2 *>(val + p + 2 * L);
            const int2 cb = *reinterpret_cast<const int2 *>(col + p + 2 * L);
            s0 += (p >= beg ? va.x : 0.0) * x[ca.x];
            s1 += va.y * x[ca.y];
            s2 += vb.x * x[cb.x];
            s3 += vb.y * x[cb.y];
        }
        for (; p < end; p += 2 * L) {
            if (p + 1 < end) {
                const double2 va = *reinterpret_cast<const double2 *>(val + p);
                const int2 ca = *reinterpret_cast<const int2 *>(col + p);
                s0 += (p >= beg ? va.x : 0.0) * x[ca.x];
                s1 += va.y * x[ca.y];
            } else if (p >= beg) {
                s0 += val[p] * x[col[p]];
            }
        }
        double sum = group_sum<L>((s0 + s1) + (s2 + s3));
        if (lane == 0 && row < n_rows)
            y[row] = sum;
        return;
    }
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
        y[row] = sum;
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

template <int L>
static void launch_csr(const spmv_dims &d, const int64_t *row_ptr,
                       const int32_t *col, const double *val, const double *x,
                       double *y)
{
    constexpr int RPB = kBlock / L;
    const int64_t blocks = (d.n_rows + RPB - 1) / RPB;
    const int remap = xcd_remap_enabled() ? 1 : 0;
    if (csr_pair_loads())
        hipLaunchKernelGGL((csr_vector_kernel<L, true>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, (hipStream_t)d.stream, d.n_rows,
                           row_ptr, col, val, x, y, remap);
    else
        hipLaunchKernelGGL((csr_vector_kernel<L, false>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, (hipStream_t)d.stream, d.n_rows,
                           row_ptr, col, val, x, y, remap);
}

}  // namespace spmv

using namespace spmv;

extern "C" int spmv_csr_auto_lanes(int64_t n_rows, int64_t nnz)
{
    // About one lane per 8 entries of the mean row: every lane then runs
    // ~2 iterations of its 4-deep unrolled body, and the group is small
    // enough that short rows waste few lanes (mean 64 -> L = 8 measured
    // best on the cant-like batch, profiles/round1_sweep.md); rounded to a
    // power of two in [2, 64].
    double mean = n_rows > 0 ? (double)nnz / (double)n_rows : 0.0;
    int L = 2;
    while (L < 64 && (double)(2 * L) * 8.0 <= mean * 1.5)
        L *= 2;
    return L;
}

extern "C" int spmv_csr_run(spmv_dims d, const int64_t *row_ptr,
                            const int32_t *col, const double *val,
                            const double *x, double *y, int lanes_per_row)
{
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run: negative size");
    if (d.n_rows == 0)
        return SPMV_SUCCESS;
    if ((d.n_rows + 1) / 2 > (int64_t)INT32_MAX * 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_csr_run: too many rows");
    SPMV_GUARD(d);
    int L = lanes_per_row > 0 ? lanes_per_row : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    switch (L) {
    case 2: launch_csr<2>(d, row_ptr, col, val, x, y); break;
    case 4: launch_csr<4>(d, row_ptr, col, val, x, y); break;
    case 8: launch_csr<8>(d, row_ptr, col, val, x, y); break;
    case 16: launch_csr<16>(d, row_ptr, col, val, x, y); break;
    case 32: launch_csr<32>(d, row_ptr, col, val, x, y); break;
    case 64: launch_csr<64>(d, row_ptr, col, val, x, y); break;
    default:
        return fail_msg(SPMV_OTHER_ERROR,
                        "spmv_csr_run: lanes_per_row must be 0 or a power of two in [2,64]");
    }
    SPMV_CHECK_LAUNCH("csr_vector_kernel");
    return SPMV_SUCCESS;
}
