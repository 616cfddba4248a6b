// rmat_exp.hip — experiment kernels for the R-MAT x-gather problem
// (not part of the product library; tools/rmat_exp.py drives them).
//
// Entry-balanced tiled CSR (as csr_tiled_kernel in csrc/staged.hip) with
// knobs: NT stream loads, a hot-column table (columns >= n_cols index
// xh[c - n_cols]), stream-only (gathers from a tiny table: lower bound).
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kBlock = 256;

template <int W>
__device__ __forceinline__ double group_sum(double v)
{
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1)
        v += __shfl_xor(v, off, W);
    return v;
}

typedef double v2f64 __attribute__((ext_vector_type(2)));
typedef int32_t v2i32 __attribute__((ext_vector_type(2)));

template <bool NT, typename T>
__device__ __forceinline__ T ld(const T *p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// MODE 0: x[c]; 1: hot table (c >= M -> xh[c-M]); 2: stream-only xh[c & 4095]
template <int MODE>
__device__ __forceinline__ double gx(const double *__restrict__ x, const double *__restrict__ xh, int64_t M,
                                     int32_t c)
{
    if constexpr (MODE == 0)
        return x[c];
    else if constexpr (MODE == 1) {
        const double *b = c >= M ? xh - M : x;
        return b[c];
    } else
        return xh[c & 4095];
}

__global__ void tile_rows_kernel(int64_t n_rows, int64_t nnz, int64_t tiles, int64_t ch,
                                 const int64_t *__restrict__ row_ptr, int32_t *__restrict__ own_lo)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t > tiles)
        return;
    const int64_t off = t * ch < nnz ? t * ch : nnz + 1;
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

template <int L, int R, bool NT, int MODE>
__global__ __launch_bounds__(kBlock) void tiled_kernel(
    int64_t n_rows, int64_t nnz, int64_t M, const int64_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const double *__restrict__ val, const double *__restrict__ x,
    const double *__restrict__ xh, double *__restrict__ y, const int32_t *__restrict__ own_lo,
    int32_t *__restrict__ carry_row, double *__restrict__ carry_val)
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
    // all loads first, then the gathers
    v2f64 v[R];
    v2i32 c[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int64_t p = t0 + 2 * (int64_t)(threadIdx.x + k * kBlock);
        const int64_t q = p + 1 < t1 ? p : 0;
        v[k] = ld<NT>(reinterpret_cast<const v2f64 *>(val + q));
        c[k] = ld<NT>(reinterpret_cast<const v2i32 *>(col + q));
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int t = threadIdx.x + k * kBlock;
        const int64_t p = t0 + 2 * (int64_t)t;
        double2 pr;
        pr.x = v[k].x * gx<MODE>(x, xh, M, c[k].x);
        pr.y = v[k].y * gx<MODE>(x, xh, M, c[k].y);
        if (p + 1 >= t1) {
            pr = {0.0, 0.0};
            if (p < t1)
                pr.x = val[p] * gx<MODE>(x, xh, M, col[p]);
        }
        s_prod[t] = pr;
    }
    __syncthreads();
    const int g = threadIdx.x / L, lane = threadIdx.x % L;
    if (g == 0) {
        double s = 0.0;
        int32_t cr = -1;
        if (r_lo > 0 && (r_lo == n_rows || row_ptr[r_lo] > t0)) {
            cr = (int32_t)(r_lo - 1);
            const int64_t e = r_lo < n_rows && row_ptr[r_lo] < t1 ? row_ptr[r_lo] : t1;
            for (int64_t j = t0 + lane; j < e; j += L)
                s += prod[j - t0];
        }
        s = group_sum<L>(s);
        if (lane == 0) {
            carry_row[tile] = cr;
            carry_val[tile] = s;
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

__global__ void carry_kernel(int64_t n_tiles, const int32_t *__restrict__ carry_row,
                             const double *__restrict__ carry_val, double *__restrict__ y)
{
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n_tiles)
        return;
    const int32_t r = carry_row[t];
    if (r < 0 || (t > 0 && carry_row[t - 1] == r))
        return;
    double s = 0.0;
    for (int64_t u = t; u < n_tiles && carry_row[u] == r; ++u)
        s += carry_val[u];
    y[r] += s;
}

__global__ void hot_gather_kernel(int64_t H, const int32_t *__restrict__ hot, const double *__restrict__ x,
                                  double *__restrict__ xh)
{
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < H)
        xh[i] = x[hot[i]];
}

template <int L, int R, bool NT, int MODE>
static void run(int64_t n, int64_t nnz, int64_t M, const int64_t *ptr, const int32_t *col, const double *val,
                const double *x, const double *xh, double *y, int32_t *own, int32_t *crow, double *cval,
                hipStream_t st)
{
    constexpr int64_t CH = 2 * kBlock * R;
    const int64_t tiles = (nnz + CH - 1) / CH;
    hipLaunchKernelGGL(tile_rows_kernel, dim3((unsigned)((tiles + kBlock) / kBlock)), dim3(kBlock), 0, st, n, nnz,
                       tiles, CH, ptr, own);
    hipLaunchKernelGGL((tiled_kernel<L, R, NT, MODE>), dim3((unsigned)tiles), dim3(kBlock), 0, st, n, nnz, M, ptr,
                       col, val, x, xh, y, own, crow, cval);
    hipLaunchKernelGGL(carry_kernel, dim3((unsigned)((tiles + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, tiles,
                       crow, cval, y);
}

// variant = R*100 + NT*10 + MODE ; L fixed 4 (mean row 10)
extern "C" int rmat_exp_run(int variant, int64_t n, int64_t nnz, int64_t M, const int64_t *ptr,
                            const int32_t *col, const double *val, const double *x, const int32_t *hot,
                            int64_t H, double *xh, double *y, int32_t *own, int32_t *crow, double *cval,
                            void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(0) != hipSuccess)
        return -2;
    (void)hipGetLastError();
    const int mode = variant % 10, nt = (variant / 10) % 10, R = variant / 100;
    if (mode == 1 && H > 0)
        hipLaunchKernelGGL(hot_gather_kernel, dim3((unsigned)((H + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, H,
                           hot, x, xh);
#define V(RR, NN, MM)                                                                    \
    if (R == RR && nt == NN && mode == MM) {                                             \
        run<4, RR, NN, MM>(n, nnz, M, ptr, col, val, x, xh, y, own, crow, cval, st);     \
        return (int)hipGetLastError();                                                   \
    }
    V(3, 0, 0) V(3, 1, 0) V(3, 0, 1) V(3, 1, 1) V(3, 0, 2) V(3, 1, 2)
    V(6, 0, 0) V(6, 1, 0) V(6, 0, 1) V(6, 1, 1) V(6, 1, 2)
    V(2, 1, 1) V(4, 1, 1) V(8, 1, 1)
#undef V
    return -1;
}

extern "C" int64_t rmat_exp_ws(int R, int64_t nnz) { return (nnz + 2 * kBlock * R - 1) / (2 * kBlock * R) + 1; }
