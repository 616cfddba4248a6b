// lab_stamps_sell.h — per-wave phase stamps of the small-matrix SELL kernel,
// for lab builds only: tools/build_variant.sh stamps_sell compiles
// csrc/sell.hip with `-include tools/lab_stamps_sell.h`, which turns the
// product's no-op SELL_STAMP(k) / SELL_STAMP_HWID() hooks into
// s_memrealtime stamps (100 MHz) and exports spmv_lab_sell_stamps() for
// tools/sell_stamps.py.  Phases: 0 start, 1 x window published (barrier),
// 2 first batch summed, 3 all batches summed, 4 partial sums published,
// 5 y stored; slot 7 = the wave's HW_ID register (CU / SIMD placement).
// The macros expand inside sell_small_kernel (bid, wv, lane, its geometry).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kStampWaves = 8192, kStamps = 8;
static __device__ uint64_t g_sell_stamps[kStampWaves * kStamps];
#define SELL_STAMP(k)                                                                                   \
    do {                                                                                                \
        const int64_t sw_ = bid * (kSellSmallS * kSellSmallP) + wv;                                     \
        if (lane == 0 && sw_ < kStampWaves)                                                             \
            g_sell_stamps[sw_ * kStamps + (k)] = __builtin_amdgcn_s_memrealtime();                      \
    } while (0)
#define SELL_STAMP_HWID()                                                                               \
    do {                                                                                                \
        uint32_t hid_;                                                                                  \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hid_));                              \
        const int64_t sw_ = bid * (kSellSmallS * kSellSmallP) + wv;                                     \
        if (lane == 0 && sw_ < kStampWaves)                                                             \
            g_sell_stamps[sw_ * kStamps + 7] = hid_;                                                    \
    } while (0)

extern "C" int spmv_lab_sell_stamps(void *host, size_t bytes)
{
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sell_stamps), bytes);
}
