// lab_stamps_csr.h — per-wave phase stamps of the CSR x-window kernel, for
// lab builds only: tools/build_variant.sh stamps_csr compiles csrc/csr.hip
// with `-include tools/lab_stamps_csr.h`, which turns the product's no-op
// CSR_STAMP(k) hooks into s_memrealtime stamps (100 MHz) and exports
// spmv_lab_csr_stamps() for tools/sell_stamps.py --kernel csr.
// Phases: 0 start, 1 window and offsets published, 2 chunk 0's products in
// LDS, 3 its barrier, 4 its row sums read, 5 its second barrier, 6 / 7
// chunks 1 / 2's products in LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kCsrStampWaves = 8192, kCsrStamps = 8;
static __device__ uint64_t g_csr_stamps[kCsrStampWaves * kCsrStamps];
#define CSR_STAMP(k)                                                                                   \
    do {                                                                                               \
        const int64_t sw_ = (int64_t)blockIdx.x * (256 / 64) + threadIdx.x / 64;                       \
        if ((threadIdx.x & 63) == 0 && sw_ < kCsrStampWaves && (k) < kCsrStamps)                       \
            g_csr_stamps[sw_ * kCsrStamps + (k)] = __builtin_amdgcn_s_memrealtime();                   \
    } while (0)

extern "C" int spmv_lab_csr_stamps(void *host, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_csr_stamps), bytes);
}
