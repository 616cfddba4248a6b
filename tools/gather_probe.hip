// gather_probe.hip — cost of random 8-byte gathers from a vector the size of
// the R-MAT's x (80 MB, inside the 256 MiB Infinity Cache), by memory type
// and load policy.  The R-MAT tiled CSR kernel's cold-column gathers each
// fill a whole 128-B L2 line (profiles/traffic_rmat.json: 37 M 128-B
// requests per launch, 3.46x bytes_alg); this asks whether an allocation or
// load form that the L2 does not line-fill moves fewer bytes per gather and
// finishes sooner.  Diagnostic only (not part of libspmv_hip.so).
//   hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o tools/gather_probe
//   tools/gather_probe [n_gathers] [table_doubles] [reps]
// One JSON line per (memory, policy): median ms, gathers/s, 8-B bytes/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            exit(2);                                                          \
        }                                                                     \
    } while (0)

// POL 0 plain, 1 non-temporal, 2 system-scope relaxed atomic load (sc0 sc1)
template <int POL>
__device__ __forceinline__ double gload(const double *p)
{
    if constexpr (POL == 0)
        return *p;
    else if constexpr (POL == 1)
        return __builtin_nontemporal_load(p);
    else
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Grid-stride: U gathers per thread in flight (index loads coalesced).
template <int POL, int U>
__global__ __launch_bounds__(256) void gather_kernel(const int32_t *__restrict__ idx, int64_t n,
                                                     const double *__restrict__ tbl, double *__restrict__ out)
{
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double s = 0.0;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        int32_t c[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            c[u] = __builtin_nontemporal_load(idx + i + u * stride);
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = gload<POL>(tbl + c[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            s += v[u];
    }
    for (; i < n; i += stride)
        s += gload<POL>(tbl + idx[i]);
    out[(int64_t)blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void flush_kernel(uint4 *p, int64_t n16, uint32_t t)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
        p[i] = make_uint4(t, t, t, t);
}

static uint64_t mix(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

int main(int argc, char **argv)
{
    const int64_t n = argc > 1 ? atoll(argv[1]) : 16000000;
    const int64_t m = argc > 2 ? atoll(argv[2]) : 10000000;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    std::vector<int32_t> h(n);
    for (int64_t i = 0; i < n; ++i)
        h[i] = (int32_t)(mix((uint64_t)i) % (uint64_t)m);
    int32_t *idx;
    double *out;
    uint4 *scratch;
    const int64_t flush = 512ll << 20;
    CHECK(hipMalloc(&idx, n * 4));
    CHECK(hipMalloc(&out, 1 << 24));
    CHECK(hipMalloc(&scratch, flush));
    CHECK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<double> ones(m, 1.0);
    struct Mem { const char *name; unsigned flags; int ext; };
    const Mem mems[] = {{"coarse", 0, 0}, {"uncached", hipDeviceMallocUncached, 1},
                        {"finegrained", hipDeviceMallocFinegrained, 1}};
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned blocks = (unsigned)cus * 8;
    for (const Mem &mm : mems) {
        double *tbl = nullptr;
        hipError_t e = mm.ext ? hipExtMallocWithFlags((void **)&tbl, m * 8, mm.flags) : hipMalloc(&tbl, m * 8);
        if (e != hipSuccess) {
            printf("{\"mem\": \"%s\", \"error\": \"%s\"}\n", mm.name, hipGetErrorString(e));
            continue;
        }
        CHECK(hipMemcpy(tbl, ones.data(), m * 8, hipMemcpyHostToDevice));
        for (int pol = 0; pol < 3; ++pol) {
            for (int cold = 0; cold < 2; ++cold) {
                std::vector<float> ts;
                for (int r = 0; r < reps + 2; ++r) {
                    if (cold)
                        hipLaunchKernelGGL(flush_kernel, dim3(4096), dim3(256), 0, 0, scratch, flush / 16, (uint32_t)r);
                    else  // warm: the table was read by the previous rep; touch it once before the first
                        if (r == 0)
                            hipLaunchKernelGGL((gather_kernel<0, 8>), dim3(blocks), dim3(256), 0, 0, idx, n, tbl, out);
                    CHECK(hipEventRecord(e0, 0));
                    if (pol == 0)
                        hipLaunchKernelGGL((gather_kernel<0, 8>), dim3(blocks), dim3(256), 0, 0, idx, n, tbl, out);
                    else if (pol == 1)
                        hipLaunchKernelGGL((gather_kernel<1, 8>), dim3(blocks), dim3(256), 0, 0, idx, n, tbl, out);
                    else
                        hipLaunchKernelGGL((gather_kernel<2, 8>), dim3(blocks), dim3(256), 0, 0, idx, n, tbl, out);
                    CHECK(hipEventRecord(e1, 0));
                    CHECK(hipEventSynchronize(e1));
                    float ms = 0;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    if (r >= 2)
                        ts.push_back(ms);
                }
                std::sort(ts.begin(), ts.end());
                const double med = ts[ts.size() / 2];
                double chk = 0;
                CHECK(hipMemcpy(&chk, out, 8, hipMemcpyDeviceToHost));
                printf("{\"mem\": \"%s\", \"policy\": \"%s\", \"state\": \"%s\", \"gathers\": %lld, \"table_MB\": %.1f, "
                       "\"ms\": %.4f, \"Ggathers_s\": %.2f, \"GBs_8B\": %.1f, \"GBs_128B_lines\": %.1f}\n",
                       mm.name, pol == 0 ? "plain" : pol == 1 ? "nt" : "sc0sc1", cold ? "cold" : "warm",
                       (long long)n, m * 8e-6, med, n / (med * 1e6), n * 8 / (med * 1e6), n * 128 / (med * 1e6));
                fflush(stdout);
            }
        }
        CHECK(hipFree(tbl));
    }
    return 0;
}
