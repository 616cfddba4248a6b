// vec.hip — the fp64 vector kernels of iterated SpMV (SURVEY.md §8f row 3:
// power iteration / CG over row shards, the y all-gather reused as the
// next x).  The reference runs one SpMV and stops (reference csr.c:198-236),
// so these have no reference counterpart; they exist so that an iteration
// never leaves the device: every scalar (norms, dot products, CG's alpha
// and beta) lives in device memory, is all-reduced there over RCCL, and is
// read by the next kernel without a host round trip.
//
// Reductions are deterministic: a fixed two-stage tree whose shape depends
// only on n, so the same data always gives the same bits (no atomics).
// All kernels are HBM-streaming (8-24 B per element, no reuse).
#include "common.h"

namespace spmv {

constexpr int kDotBlocks = 1024;  // stage-1 partials (fixed -> deterministic)

__device__ __forceinline__ double block_sum(double v, double *s_warp)
{
    v = group_sum<kWave>(v);
    const int w = threadIdx.x / kWave;
    if (threadIdx.x % kWave == 0)
        s_warp[w] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x < kWave) {
        const int nw = blockDim.x / kWave;
        t = (int)threadIdx.x < nw ? s_warp[threadIdx.x] : 0.0;
        t = group_sum<kWave>(t);
    }
    return t;  // valid in thread 0
}

// stage 1: block b sums indices b*256 + t + k*G*256 in a fixed order
__global__ __launch_bounds__(kBlock) void dot_partial_kernel(int64_t n, const double *__restrict__ a,
                                                             const double *__restrict__ b,
                                                             double *__restrict__ partial)
{
    __shared__ double s_warp[kBlock / kWave];
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    double s0 = 0.0, s1 = 0.0;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + stride < n; i += 2 * stride) {
        s0 += a[i] * b[i];
        s1 += a[i + stride] * b[i + stride];
    }
    if (i < n)
        s0 += a[i] * b[i];
    const double t = block_sum(s0 + s1, s_warp);
    if (threadIdx.x == 0)
        partial[blockIdx.x] = t;
}

// stage 2: one block folds the G partials in a fixed order
__global__ __launch_bounds__(1024) void dot_final_kernel(int g, const double *__restrict__ partial,
                                                         double *__restrict__ out)
{
    __shared__ double s_warp[1024 / kWave];
    const double v = (int)threadIdx.x < g ? partial[threadIdx.x] : 0.0;
    const double t = block_sum(v, s_warp);
    if (threadIdx.x == 0)
        *out = t;
}

static int dot_blocks(int64_t n)
{
    const int64_t per = (int64_t)kBlock * 8;  // >= 8 elements per thread before splitting further
    int64_t g = (n + per - 1) / per;
    return (int)(g < 1 ? 1 : (g > kDotBlocks ? kDotBlocks : g));
}

// y += sign * (*num / *den) * x
__global__ __launch_bounds__(kBlock) void axpy_ratio_kernel(int64_t n, const double *__restrict__ num,
                                                            const double *__restrict__ den, double sign,
                                                            const double *__restrict__ x,
                                                            double *__restrict__ y)
{
    const double alpha = sign * (*num / *den);
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        y[i] += alpha * x[i];
}

// y = x + (*num / *den) * y
__global__ __launch_bounds__(kBlock) void xpay_ratio_kernel(int64_t n, const double *__restrict__ num,
                                                            const double *__restrict__ den,
                                                            const double *__restrict__ x,
                                                            double *__restrict__ y)
{
    const double beta = *num / *den;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        y[i] = x[i] + beta * y[i];
}

// y = x / sqrt(*s)
__global__ __launch_bounds__(kBlock) void scale_rsqrt_kernel(int64_t n, const double *__restrict__ s,
                                                             const double *__restrict__ x,
                                                             double *__restrict__ y)
{
    const double inv = 1.0 / sqrt(*s);
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        y[i] = x[i] * inv;
}

// out[k] = x[order[k]]: x in the layout of a column-relabelled matrix
// (spmv_column_relabel); the replication step's gather, not the SpMV's
__global__ __launch_bounds__(kBlock) void gather_kernel(int64_t n, const int32_t *__restrict__ order,
                                                        const double *__restrict__ x, double *__restrict__ out)
{
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        out[i] = x[order[i]];
}

static unsigned stream_grid(int64_t n)
{
    // a few waves of workgroups per CU is enough for a pure stream
    int64_t g = (n + kBlock * 4 - 1) / (kBlock * 4);
    return (unsigned)(g < 1 ? 1 : (g > 256 * 16 ? 256 * 16 : g));
}

}  // namespace spmv

using namespace spmv;

extern "C" size_t spmv_dot_ws_bytes(int64_t n)
{
    return (size_t)dot_blocks(n) * sizeof(double);
}

extern "C" int spmv_dot(int64_t n, const double *a, const double *b, double *out, void *ws,
                        size_t ws_bytes, int device, void *stream)
{
    if (n < 0 || !out)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dot: bad arguments");
    const int g = dot_blocks(n);
    if (!ws || ws_bytes < (size_t)g * sizeof(double))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_dot: workspace too small");
    DeviceGuard guard(device);
    if (guard.rc() != SPMV_SUCCESS)
        return guard.rc();
    const hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(dot_partial_kernel, dim3(g), dim3(kBlock), 0, st, n, a, b, (double *)ws);
    hipLaunchKernelGGL(dot_final_kernel, dim3(1), dim3(1024), 0, st, g, (const double *)ws, out);
    SPMV_CHECK_LAUNCH("dot kernels");
    return SPMV_SUCCESS;
}

extern "C" int spmv_axpy_ratio(int64_t n, const double *num, const double *den, double sign,
                               const double *x, double *y, int device, void *stream)
{
    if (n < 0 || !num || !den)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_axpy_ratio: bad arguments");
    if (n == 0)
        return SPMV_SUCCESS;
    DeviceGuard guard(device);
    if (guard.rc() != SPMV_SUCCESS)
        return guard.rc();
    hipLaunchKernelGGL(axpy_ratio_kernel, dim3(stream_grid(n)), dim3(kBlock), 0, (hipStream_t)stream, n, num,
                       den, sign, x, y);
    SPMV_CHECK_LAUNCH("axpy_ratio_kernel");
    return SPMV_SUCCESS;
}

extern "C" int spmv_xpay_ratio(int64_t n, const double *num, const double *den, const double *x, double *y,
                               int device, void *stream)
{
    if (n < 0 || !num || !den)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_xpay_ratio: bad arguments");
    if (n == 0)
        return SPMV_SUCCESS;
    DeviceGuard guard(device);
    if (guard.rc() != SPMV_SUCCESS)
        return guard.rc();
    hipLaunchKernelGGL(xpay_ratio_kernel, dim3(stream_grid(n)), dim3(kBlock), 0, (hipStream_t)stream, n, num,
                       den, x, y);
    SPMV_CHECK_LAUNCH("xpay_ratio_kernel");
    return SPMV_SUCCESS;
}

extern "C" int spmv_scale_rsqrt(int64_t n, const double *s, const double *x, double *y, int device,
                                void *stream)
{
    if (n < 0 || !s)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_scale_rsqrt: bad arguments");
    if (n == 0)
        return SPMV_SUCCESS;
    DeviceGuard guard(device);
    if (guard.rc() != SPMV_SUCCESS)
        return guard.rc();
    hipLaunchKernelGGL(scale_rsqrt_kernel, dim3(stream_grid(n)), dim3(kBlock), 0, (hipStream_t)stream, n, s,
                       x, y);
    SPMV_CHECK_LAUNCH("scale_rsqrt_kernel");
    return SPMV_SUCCESS;
}

extern "C" int spmv_gather(int64_t n, const int32_t *order, const double *x, double *out, int device, void *stream)
{
    if (n < 0 || (n > 0 && (!order || !x || !out)) || (n > 0 && x == out))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_gather: bad arguments");
    if (n == 0)
        return SPMV_SUCCESS;
    DeviceGuard guard(device);
    if (guard.rc() != SPMV_SUCCESS)
        return guard.rc();
    hipLaunchKernelGGL(gather_kernel, dim3(stream_grid(n)), dim3(kBlock), 0, (hipStream_t)stream, n, order, x, out);
    SPMV_CHECK_LAUNCH("gather_kernel");
    return SPMV_SUCCESS;
}
