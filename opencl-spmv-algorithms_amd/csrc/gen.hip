// gen.hip — device-side generator for the banded matrix of BASELINE.json
// configs[4] (10^8 rows, 1.6e9 entries): at that size a host-built CSR
// plus upload (19.6 GB over PCIe) dominates, so each GPU writes its own
// row shard straight into HBM.  Values are bit-identical to the host
// generator spmv_gen_banded_csr (host/gen.c): splitmix64(seed, 16·row+k)
// mapped to [-1, 1), column (row + k - 8) mod n.
#include "common.h"

namespace spmv {

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ double banded_value(uint64_t seed, uint64_t index)
{
    const uint64_t h = mix64(seed * 0xD1B54A32D192ED03ULL + (index + 1) * 0x9E3779B97F4A7C15ULL);
    return (double)(h >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

__device__ __forceinline__ int32_t banded_col(int64_t n, int64_t g, int k)
{
    int64_t c = (g + k - 8) % n;
    return (int32_t)(c < 0 ? c + n : c);
}

// CSR: one thread per (local row, k)
__global__ __launch_bounds__(kBlock) void banded_csr_kernel(int64_t n, uint64_t seed,
                                                            int64_t row_begin, int64_t m,
                                                            int64_t *__restrict__ row_ptr,
                                                            int32_t *__restrict__ col,
                                                            double *__restrict__ val)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t <= m)
        row_ptr[t] = 16 * t;
    if (t >= 16 * m)
        return;
    const int64_t i = t >> 4;
    const int k = (int)(t & 15);
    const int64_t g = row_begin + i;
    col[t] = banded_col(n, g, k);
    val[t] = banded_value(seed, (uint64_t)g * 16 + (uint64_t)k);
}

// SELL-C with k-interleave ki: every row has 16 entries, so the sigma sort
// is the identity and every slice has width 16; slots past the shard's
// last row are padding (perm -1, value 0, column 0).
__global__ __launch_bounds__(kBlock) void banded_sell_kernel(int64_t n, uint64_t seed,
                                                             int64_t row_begin, int64_t m,
                                                             int32_t C, int32_t ki,
                                                             int64_t n_slices,
                                                             int64_t *__restrict__ slice_ptr,
                                                             int32_t *__restrict__ perm,
                                                             int32_t *__restrict__ col,
                                                             double *__restrict__ val)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // (slot, k)
    const int64_t slots = n_slices * C;
    if (t <= n_slices)
        slice_ptr[t] = t * (int64_t)C * 16;
    if (t < slots)
        perm[t] = t < m ? (int32_t)t : -1;
    if (t >= slots * 16)
        return;
    const int64_t slot = t >> 4;
    const int k = (int)(t & 15);
    const int64_t s = slot / C, r = slot - s * C;
    const int64_t pos = s * (int64_t)C * 16 + (k / ki) * (int64_t)C * ki + r * ki + (k % ki);
    if (slot < m) {
        const int64_t g = row_begin + slot;
        col[pos] = banded_col(n, g, k);
        val[pos] = banded_value(seed, (uint64_t)g * 16 + (uint64_t)k);
    } else {
        col[pos] = 0;
        val[pos] = 0.0;
    }
}

}  // namespace spmv

using namespace spmv;

extern "C" int spmv_gen_banded_device(int64_t n, uint64_t seed, int64_t row_begin,
                                      int64_t row_end, int layout, int32_t C, int32_t ki,
                                      int64_t *ptr, int32_t *perm, int32_t *col, double *val,
                                      int device, void *stream)
{
    if (n < 16 || n > INT32_MAX || row_begin < 0 || row_end > n || row_begin > row_end)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_gen_banded_device: bad row range");
    if (layout != 0 && layout != 1)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_gen_banded_device: layout must be 0 (CSR) or 1 (SELL)");
    if (layout == 1 && (C < 1 || C > 1024 || (ki != 1 && ki != 2)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_gen_banded_device: bad C / ki");
    DeviceGuard guard(device);
    if (guard.rc() != SPMV_SUCCESS)
        return guard.rc();
    const int64_t m = row_end - row_begin;
    if (layout == 0) {
        const int64_t work = 16 * m + 1;
        const int64_t blocks = (work + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(banded_csr_kernel, dim3((unsigned)blocks), dim3(kBlock), 0,
                           (hipStream_t)stream, n, seed, row_begin, m, ptr, col, val);
    } else {
        const int64_t ns = (m + C - 1) / C;
        const int64_t work = ns * C * 16 + 1;
        const int64_t blocks = (work + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(banded_sell_kernel, dim3((unsigned)blocks), dim3(kBlock), 0,
                           (hipStream_t)stream, n, seed, row_begin, m, C, ki, ns, ptr, perm, col,
                           val);
    }
    SPMV_CHECK_LAUNCH("banded generator");
    return SPMV_SUCCESS;
}
