// bw_probe.hip — achievable HBM bandwidth on this MI355X, for the roofline
// next to the 8 TB/s spec (MI355X_MICROARCH.md quotes 6.29 TB/s for a
// float4 copy).  Streams a 2 GiB buffer (8x the Infinity Cache) with the
// access widths the SpMV kernels use and prints one JSON line per kernel.
// Also the calibration workload for FETCH_SIZE (known bytes per launch).
//   hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            exit(2);                                                          \
        }                                                                     \
    } while (0)

template <typename T>
__device__ __forceinline__ double fold(T v);
template <>
__device__ __forceinline__ double fold(double v) { return v; }
template <>
__device__ __forceinline__ double fold(double2 v) { return v.x + v.y; }

// Grid-stride read; one store per thread keeps the loads alive.
template <typename T, int UNROLL>
__global__ __launch_bounds__(256) void read_kernel(const T *__restrict__ a, size_t n,
                                                   double *__restrict__ out)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    double s = 0.0;
    for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
        T v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            v[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            s += fold(v[u]);
    }
    for (; i < n; i += stride)
        s += fold(a[i]);
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = s;
}

// One-shot grid, each workgroup reads U·4 KiB contiguous (the SpMV
// kernels' shape: no grid stride, every block streams its own tile).
// NT = non-temporal loads.  The store never happens; it keeps the loads.
template <bool NT, int U>
__global__ __launch_bounds__(256) void tile_read_kernel(const double2 *__restrict__ a, size_t n,
                                                        double *__restrict__ out)
{
    typedef double v2 __attribute__((ext_vector_type(2)));
    const size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x;
    double s = 0.0;
    v2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t i = base + (size_t)u * 256;
        const v2 *p = reinterpret_cast<const v2 *>(a + (i < n ? i : 0));
        if constexpr (NT)
            v[u] = __builtin_nontemporal_load(p);
        else
            v[u] = *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        s += v[u].x + v[u].y;
    if (s == 123.456)
        out[0] = s;
}

// The CSR kernels' stream without their LDS work: each workgroup reads the
// values (16-B pairs) and columns (8-B pairs) of CH-entry chunks of its
// E-entry tile, R pairs per lane per chunk, nt, and folds them (the
// ceiling of the csr_xwin_kernel access pattern: two arrays, 24 B per pair).
template <int R>
__global__ __launch_bounds__(256) void csr_stream_kernel(const double *__restrict__ val,
                                                         const int *__restrict__ col, size_t nnz, size_t tile,
                                                         double *__restrict__ out)
{
    typedef double v2 __attribute__((ext_vector_type(2)));
    typedef int i2 __attribute__((ext_vector_type(2)));
    constexpr size_t CH = 2 * 256 * R;
    const size_t t0 = (size_t)blockIdx.x * tile;
    const size_t t1 = t0 + tile < nnz ? t0 + tile : nnz;
    double s = 0.0;
    for (size_t cb = t0; cb < t1; cb += CH) {
        v2 v[R];
        i2 c[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const size_t p = cb + 2 * (threadIdx.x + (size_t)k * 256);
            const size_t q = p + 1 < t1 ? p : t0;
            v[k] = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(val + q));
            c[k] = __builtin_nontemporal_load(reinterpret_cast<const i2 *>(col + q));
        }
#pragma unroll
        for (int k = 0; k < R; ++k)
            s += v[k].x * (double)c[k].x + v[k].y * (double)c[k].y;
    }
    if (s == 123.456)
        out[0] = s;
}

// The stream above plus the staged kernels' per-chunk LDS work, to price
// it apart from everything else (x windows, offsets, reductions):
// SYNC 0 = products stored to LDS only; SYNC 1 = products stored to LDS, barrier, each lane reads 2R products back
// (a row slice), barrier; SYNC 2 = as 1, software-pipelined (the next chunk's
// loads issued before the barrier, as csr_xwin_kernel MODE 3).
template <int R, int SYNC>
__global__ __launch_bounds__(256) void csr_stage_probe_kernel(const double *__restrict__ val,
                                                              const int *__restrict__ col, size_t nnz, size_t tile,
                                                              double *__restrict__ out)
{
    typedef double v2 __attribute__((ext_vector_type(2)));
    typedef int i2 __attribute__((ext_vector_type(2)));
    constexpr size_t CH = 2 * 256 * R;
    __shared__ v2 s_prod[256 * R];
    const double *prod = reinterpret_cast<const double *>(s_prod);
    const size_t t0 = (size_t)blockIdx.x * tile;
    const size_t t1 = t0 + tile < nnz ? t0 + tile : nnz;
    double s = 0.0;
    v2 v[R];
    i2 c[R];
    auto issue = [&](size_t cb) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const size_t p = cb + 2 * (threadIdx.x + (size_t)k * 256);
            const size_t q = p + 1 < t1 ? p : t0;
            v[k] = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(val + q));
            c[k] = __builtin_nontemporal_load(reinterpret_cast<const i2 *>(col + q));
        }
    };
    issue(t0);
    for (size_t cb = t0; cb < t1; cb += CH) {
#pragma unroll
        for (int k = 0; k < R; ++k)
            s_prod[threadIdx.x + k * 256] = v2{v[k].x * (double)c[k].x, v[k].y * (double)c[k].y};
        if constexpr (SYNC == 2) {
            if (cb + CH < t1)
                issue(cb + CH);
        }
        if constexpr (SYNC > 0) {
            __syncthreads();
            // lane group of 4 sums a 2R·4-entry slice (stride 4), as slice_sum<4>
            const int g = threadIdx.x / 4, lane = threadIdx.x % 4;
#pragma unroll
            for (int k = 0; k < 2 * R; ++k)
                s += prod[g * 8 * R + lane + 4 * k];
            __syncthreads();
        } else {
            s += prod[threadIdx.x];  // SYNC 0: own product back, no barrier
        }
        if constexpr (SYNC != 2) {
            if (cb + CH < t1)
                issue(cb + CH);
        }
    }
    if (s == 123.456)
        out[0] = s;
}

// csr_stage_probe_kernel<R, 1> with the x-window kernel's per-window
// prologue: DEP dependent round trips before the first chunk (DEP >= 1: the
// tile's start is read from `starts`; DEP >= 2: then 768 doubles of `xs` at
// an address from that read are copied to LDS behind a barrier).
template <int R, int DEP>
__global__ __launch_bounds__(256) void csr_prologue_probe_kernel(const double *__restrict__ val,
                                                                 const int *__restrict__ col, size_t nnz, size_t tile,
                                                                 const long long *__restrict__ starts,
                                                                 const double *__restrict__ xs,
                                                                 double *__restrict__ out)
{
    typedef double v2 __attribute__((ext_vector_type(2)));
    typedef int i2 __attribute__((ext_vector_type(2)));
    constexpr size_t CH = 2 * 256 * R;
    __shared__ v2 s_prod[256 * R];
    __shared__ double s_x[768];
    const double *prod = reinterpret_cast<const double *>(s_prod);
    size_t t0 = (size_t)blockIdx.x * tile;
    double s = 0.0;
    if constexpr (DEP >= 1)
        t0 = (size_t)starts[blockIdx.x];
    if constexpr (DEP >= 2) {
        const size_t xo = (t0 / 16) & ((1u << 20) - 1);
        for (int i = threadIdx.x; i < 768; i += 256)
            s_x[i] = xs[xo + i];
        __syncthreads();
        s += s_x[(threadIdx.x * 3) % 768];
    }
    const size_t t1 = t0 + tile < nnz ? t0 + tile : nnz;
    for (size_t cb = t0; cb < t1; cb += CH) {
        v2 v[R];
        i2 c[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const size_t p = cb + 2 * (threadIdx.x + (size_t)k * 256);
            const size_t q = p + 1 < t1 ? p : t0;
            v[k] = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(val + q));
            c[k] = __builtin_nontemporal_load(reinterpret_cast<const i2 *>(col + q));
        }
#pragma unroll
        for (int k = 0; k < R; ++k)
            s_prod[threadIdx.x + k * 256] = v2{v[k].x * (double)c[k].x, v[k].y * (double)c[k].y};
        __syncthreads();
        const int g = threadIdx.x / 4, lane = threadIdx.x % 4;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k)
            s += prod[g * 8 * R + lane + 4 * k];
        __syncthreads();
    }
    if (s == 123.456)
        out[0] = s;
}

// Persistent form: gridDim.x resident workgroups, workgroup b streams the
// contiguous range [b·nnz/G, (b+1)·nnz/G) (the static split of
// csr_xstream_kernel), or with DYN the tiles are handed out by an atomic
// counter (`ctr`, zeroed before the launch).
template <int R, bool DYN>
__global__ __launch_bounds__(256) void csr_persistent_probe_kernel(const double *__restrict__ val,
                                                                   const int *__restrict__ col, size_t nnz,
                                                                   size_t tile, unsigned *ctr,
                                                                   double *__restrict__ out)
{
    typedef double v2 __attribute__((ext_vector_type(2)));
    typedef int i2 __attribute__((ext_vector_type(2)));
    constexpr size_t CH = 2 * 256 * R;
    __shared__ v2 s_prod[256 * R];
    __shared__ unsigned s_next;
    const double *prod = reinterpret_cast<const double *>(s_prod);
    double s = 0.0;
    const size_t ntiles = (nnz + tile - 1) / tile;
    size_t a0, a1;
    if constexpr (DYN) {
        a0 = blockIdx.x;
        a1 = a0 + 1;
    } else {
        a0 = (size_t)blockIdx.x * nnz / gridDim.x;
        a1 = ((size_t)blockIdx.x + 1) * nnz / gridDim.x;
        a0 &= ~(size_t)1;
        a1 = blockIdx.x + 1 == gridDim.x ? nnz : a1 & ~(size_t)1;
    }
    while (true) {
        size_t t0, t1;
        if constexpr (DYN) {
            if (a0 >= ntiles)
                break;
            t0 = a0 * tile;
            t1 = t0 + tile < nnz ? t0 + tile : nnz;
            if (threadIdx.x == 0)
                s_next = atomicAdd(ctr, 1u) + gridDim.x;
        } else {
            t0 = a0;
            t1 = a1;
        }
        for (size_t cb = t0; cb < t1; cb += CH) {
            v2 v[R];
            i2 c[R];
#pragma unroll
            for (int k = 0; k < R; ++k) {
                const size_t p = cb + 2 * (threadIdx.x + (size_t)k * 256);
                const size_t q = p + 1 < t1 ? p : t0;
                v[k] = __builtin_nontemporal_load(reinterpret_cast<const v2 *>(val + q));
                c[k] = __builtin_nontemporal_load(reinterpret_cast<const i2 *>(col + q));
            }
#pragma unroll
            for (int k = 0; k < R; ++k)
                s_prod[threadIdx.x + k * 256] = v2{v[k].x * (double)c[k].x, v[k].y * (double)c[k].y};
            __syncthreads();
            const int g = threadIdx.x / 4, lane = threadIdx.x % 4;
#pragma unroll
            for (int k = 0; k < 2 * R; ++k)
                s += prod[g * 8 * R + lane + 4 * k];
            __syncthreads();
        }
        if constexpr (DYN) {
            a0 = s_next;
            __syncthreads();
        } else {
            break;
        }
    }
    if (s == 123.456)
        out[0] = s;
}

__global__ __launch_bounds__(256) void copy_kernel(const double2 *__restrict__ a,
                                                   double2 *__restrict__ b, size_t n)
{
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    for (; i < n; i += stride)
        b[i] = a[i];
}

template <typename K>
static double time_ms(K launch, int reps)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i)
        launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv)
{
    const size_t bytes = (argc > 1 ? (size_t)atoll(argv[1]) : (size_t)2 << 30);
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    void *a, *b;
    double *out;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMemset(a, 1, bytes));
    const int grid = 256 * 16;  // 16 workgroups per CU, grid-stride
    CHECK(hipMalloc(&out, (size_t)grid * 256 * sizeof(double)));
    const size_t n8 = bytes / 8, n16 = bytes / 16;

    double t;
    t = time_ms([&] { hipLaunchKernelGGL((read_kernel<double2, 4>), dim3(grid), dim3(256), 0, 0,
                                         (const double2 *)a, n16, out); }, reps);
    printf("{\"probe\": \"read_dwordx4\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", bytes, t,
           bytes / t * 1e-6);
    t = time_ms([&] { hipLaunchKernelGGL((read_kernel<double, 4>), dim3(grid), dim3(256), 0, 0,
                                         (const double *)a, n8, out); }, reps);
    printf("{\"probe\": \"read_dwordx2\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", bytes, t,
           bytes / t * 1e-6);
    const unsigned g4 = (unsigned)((n16 + 4 * 256 - 1) / (4 * 256));
    const unsigned g8 = (unsigned)((n16 + 8 * 256 - 1) / (8 * 256));
    const unsigned g16 = (unsigned)((n16 + 16 * 256 - 1) / (16 * 256));
    t = time_ms([&] { hipLaunchKernelGGL((tile_read_kernel<false, 4>), dim3(g4), dim3(256), 0, 0,
                                         (const double2 *)a, n16, out); }, reps);
    printf("{\"probe\": \"tile_read_dwordx4_u4\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", bytes, t,
           bytes / t * 1e-6);
    t = time_ms([&] { hipLaunchKernelGGL((tile_read_kernel<false, 8>), dim3(g8), dim3(256), 0, 0,
                                         (const double2 *)a, n16, out); }, reps);
    printf("{\"probe\": \"tile_read_dwordx4_u8\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", bytes, t,
           bytes / t * 1e-6);
    t = time_ms([&] { hipLaunchKernelGGL((tile_read_kernel<false, 16>), dim3(g16), dim3(256), 0, 0,
                                         (const double2 *)a, n16, out); }, reps);
    printf("{\"probe\": \"tile_read_dwordx4_u16\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", bytes, t,
           bytes / t * 1e-6);
    t = time_ms([&] { hipLaunchKernelGGL((tile_read_kernel<true, 8>), dim3(g8), dim3(256), 0, 0,
                                         (const double2 *)a, n16, out); }, reps);
    printf("{\"probe\": \"tile_read_dwordx4_u8_nt\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", bytes, t,
           bytes / t * 1e-6);
    t = time_ms([&] { hipLaunchKernelGGL((tile_read_kernel<true, 16>), dim3(g16), dim3(256), 0, 0,
                                         (const double2 *)a, n16, out); }, reps);
    printf("{\"probe\": \"tile_read_dwordx4_u16_nt\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", bytes, t,
           bytes / t * 1e-6);
    {   // CSR-shaped stream: 128M entries (the cant-like batch), 8-B values + 4-B columns
        const size_t nnz = (size_t)128 << 20;
        double *val;
        int *col;
        CHECK(hipMalloc(&val, nnz * 8));
        CHECK(hipMalloc(&col, nnz * 4));
        CHECK(hipMemset(val, 0, nnz * 8));
        CHECK(hipMemset(col, 0, nnz * 4));
        const size_t tiles[] = {2048, 8192, 32768};
        for (size_t tile : tiles) {
            const unsigned g = (unsigned)((nnz + tile - 1) / tile);
            t = time_ms([&] { hipLaunchKernelGGL((csr_stream_kernel<4>), dim3(g), dim3(256), 0, 0, val, col, nnz,
                                                 tile, out); }, reps);
            printf("{\"probe\": \"csr_stream_r4_tile%zu_nt\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
                   tile, nnz * 12, t, nnz * 12 / t * 1e-6);
        }
        t = time_ms([&] { hipLaunchKernelGGL((csr_stream_kernel<8>), dim3((unsigned)(nnz / 8192)), dim3(256), 0,
                                             0, val, col, nnz, (size_t)8192, out); }, reps);
        printf("{\"probe\": \"csr_stream_r8_tile8192_nt\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
               nnz * 12, t, nnz * 12 / t * 1e-6);
        // the same stream with dynamic LDS reserved per workgroup, so only
        // 160 KiB / lds workgroups fit a CU (occupancy of the LDS-staged kernels)
        const size_t ldss[] = {20 << 10, 26 << 10, 32 << 10, 40 << 10};
        for (size_t lds : ldss) {
            t = time_ms([&] { hipLaunchKernelGGL((csr_stream_kernel<4>), dim3((unsigned)(nnz / 8192)), dim3(256), lds,
                                                 0, val, col, nnz, (size_t)8192, out); }, reps);
            printf("{\"probe\": \"csr_stream_r4_tile8192_nt_lds%zuk\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
                   lds >> 10, nnz * 12, t, nnz * 12 / t * 1e-6);
        }
        // the per-chunk LDS work and barriers on top of the stream (tile 8192
        // entries ~ one 128-row window of the cant batch), at the default
        // occupancy and with LDS reserved down to 6 / 5 workgroups per CU
        const size_t pads[] = {0, 14 << 10, 20 << 10};
        for (size_t lds : pads) {
            const unsigned g = (unsigned)(nnz / 8192);
            t = time_ms([&] { hipLaunchKernelGGL((csr_stage_probe_kernel<3, 1>), dim3(g), dim3(256), lds, 0, val, col,
                                                 nnz, (size_t)8192, out); }, reps);
            printf("{\"probe\": \"csr_stage_r3_sync_lds%zuk\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
                   lds >> 10, nnz * 12, t, nnz * 12 / t * 1e-6);
            t = time_ms([&] { hipLaunchKernelGGL((csr_stage_probe_kernel<3, 2>), dim3(g), dim3(256), lds, 0, val, col,
                                                 nnz, (size_t)8192, out); }, reps);
            printf("{\"probe\": \"csr_stage_r3_pipe_lds%zuk\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
                   lds >> 10, nnz * 12, t, nnz * 12 / t * 1e-6);
            t = time_ms([&] { hipLaunchKernelGGL((csr_stage_probe_kernel<3, 0>), dim3(g), dim3(256), lds, 0, val, col,
                                                 nnz, (size_t)8192, out); }, reps);
            printf("{\"probe\": \"csr_stage_r3_nosync_lds%zuk\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
                   lds >> 10, nnz * 12, t, nnz * 12 / t * 1e-6);
        }
        {   // prologue round trips per 8192-entry tile (one x window of the kernel)
            const unsigned g = (unsigned)(nnz / 8192);
            long long *starts;
            double *xs;
            CHECK(hipMalloc(&starts, g * sizeof(long long)));
            CHECK(hipMalloc(&xs, (2u << 20) * sizeof(double)));
            CHECK(hipMemset(xs, 0, (2u << 20) * sizeof(double)));
            long long *h = (long long *)malloc(g * sizeof(long long));
            for (unsigned i = 0; i < g; ++i)
                h[i] = (long long)i * 8192;  // 64-entry aligned
            CHECK(hipMemcpy(starts, h, g * sizeof(long long), hipMemcpyHostToDevice));
            free(h);
            t = time_ms([&] { hipLaunchKernelGGL((csr_prologue_probe_kernel<3, 0>), dim3(g), dim3(256), 0, 0, val, col,
                                                 nnz, (size_t)8192, starts, xs, out); }, reps);
            printf("{\"probe\": \"csr_prologue_dep0\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", nnz * 12, t,
                   nnz * 12 / t * 1e-6);
            t = time_ms([&] { hipLaunchKernelGGL((csr_prologue_probe_kernel<3, 1>), dim3(g), dim3(256), 0, 0, val, col,
                                                 nnz, (size_t)8192, starts, xs, out); }, reps);
            printf("{\"probe\": \"csr_prologue_dep1\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", nnz * 12, t,
                   nnz * 12 / t * 1e-6);
            t = time_ms([&] { hipLaunchKernelGGL((csr_prologue_probe_kernel<3, 2>), dim3(g), dim3(256), 0, 0, val, col,
                                                 nnz, (size_t)8192, starts, xs, out); }, reps);
            printf("{\"probe\": \"csr_prologue_dep2\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", nnz * 12, t,
                   nnz * 12 / t * 1e-6);
            // the same with each tile starting on an even entry that is not
            // 64-entry aligned (row groups start anywhere): 16-B value pairs,
            // but a wave's 1 KiB of values spans 9 cache lines instead of 8
            h = (long long *)malloc(g * sizeof(long long));
            for (unsigned i = 0; i < g; ++i)
                h[i] = (long long)i * 8192 + 2 * ((i * 37) % 32);
            CHECK(hipMemcpy(starts, h, g * sizeof(long long), hipMemcpyHostToDevice));
            free(h);
            t = time_ms([&] { hipLaunchKernelGGL((csr_prologue_probe_kernel<3, 1>), dim3(g), dim3(256), 0, 0, val, col,
                                                 nnz, (size_t)8192, starts, xs, out); }, reps);
            printf("{\"probe\": \"csr_prologue_dep1_unaligned\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", nnz * 12,
                   t, nnz * 12 / t * 1e-6);
            CHECK(hipFree(starts));
            CHECK(hipFree(xs));
        }
        {   // persistent workgroups: static contiguous split vs tiles from a counter
            unsigned *ctr;
            CHECK(hipMalloc(&ctr, sizeof(unsigned)));
            int per = 0;
            CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, csr_persistent_probe_kernel<3, false>, 256, 0));
            int dev = 0, cus = 0;
            CHECK(hipGetDevice(&dev));
            CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            const int pers[] = {per, 6, 5};
            for (int pc : pers) {
                const unsigned G = (unsigned)(cus * pc);
                t = time_ms([&] { hipLaunchKernelGGL((csr_persistent_probe_kernel<3, false>), dim3(G), dim3(256), 0, 0,
                                                     val, col, nnz, (size_t)8192, ctr, out); }, reps);
                printf("{\"probe\": \"csr_persistent_static_%dpercu\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
                       pc, nnz * 12, t, nnz * 12 / t * 1e-6);
                const size_t dtiles[] = {8192, 32768};
                for (size_t dt : dtiles) {
                    t = time_ms([&] {
                        (void)hipMemsetAsync(ctr, 0, sizeof(unsigned), 0);
                        hipLaunchKernelGGL((csr_persistent_probe_kernel<3, true>), dim3(G), dim3(256), 0, 0, val, col,
                                           nnz, dt, ctr, out);
                    }, reps);
                    printf("{\"probe\": \"csr_persistent_dyn%zu_%dpercu\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n",
                           dt, pc, nnz * 12, t, nnz * 12 / t * 1e-6);
                }
            }
            CHECK(hipFree(ctr));
        }
        CHECK(hipFree(val));
        CHECK(hipFree(col));
    }
    t = time_ms([&] { hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, 0,
                                         (const double2 *)a, (double2 *)b, n16); }, reps);
    printf("{\"probe\": \"copy_dwordx4\", \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", 2 * bytes, t,
           2 * bytes / t * 1e-6);
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(out));
    return 0;
}
