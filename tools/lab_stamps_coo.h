// lab_stamps_coo.h — per-tile phase stamps of coo_staged_kernel, for lab
// builds only: tools/build_variant.sh stamps_coo compiles csrc/staged.hip
// with `-include tools/lab_stamps_coo.h`, which turns the product's no-op
// COO_STAMP / COO_NOTE / COO_STAMP_END hooks into s_memrealtime stamps
// (100 MHz) of thread 0 and exports spmv_lab_coo_stamps() for
// tools/coo_stamps.py.  Slots: 0 start, 1 products and keys in LDS,
// 2 row starts in LDS, 3 end (after a barrier: the whole tile), 4 the
// tile's row span, 5 its path (0 row starts, 1 bitmap, 2 searches).
// (The plain and accumulate paths that return early stamp nothing in 3.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kCooStampTiles = 16384, kCooStamps = 8;
static __device__ uint64_t g_coo_stamps[kCooStampTiles * kCooStamps];
#define COO_STAMP(k)                                                                     \
    do {                                                                                 \
        if (threadIdx.x == 0 && tile < kCooStampTiles)                                   \
            g_coo_stamps[tile * kCooStamps + (k)] = __builtin_amdgcn_s_memrealtime();     \
    } while (0)
#define COO_NOTE(k, v)                                                                   \
    do {                                                                                 \
        if (threadIdx.x == 0 && tile < kCooStampTiles)                                   \
            g_coo_stamps[tile * kCooStamps + (k)] = (v);                                 \
    } while (0)
#define COO_STAMP_END() \
    do {                \
        __syncthreads(); \
        COO_STAMP(3);   \
    } while (0)

extern "C" int spmv_lab_coo_stamps(void *host, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_coo_stamps), bytes);
}

extern "C" int spmv_lab_coo_stamps_clear()
{
    static uint64_t zero[kCooStampTiles * kCooStamps];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_coo_stamps), zero, sizeof zero);
}
