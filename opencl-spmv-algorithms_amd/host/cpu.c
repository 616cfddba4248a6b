/*
 * cpu.c — OpenMP CPU SpMV loops printed by the drivers as the CPU figure.
 *
 * Same loop structure as the reference's compute_using_cpu functions
 * (reference coo.c:280-300 omp atomic scatter; csr.c:285-309 row-parallel;
 * ell.c:357-383 row-parallel; cmrs.c:319-345 strip-parallel), run over this
 * suite's layouts, plus a SELL loop the reference does not have.
 * Differences: y is zeroed first (the reference accumulated into
 * malloc'd memory, reference csr.c:102), and the thread count is explicit
 * so the printed core count is the one used.
 * These are a reported baseline only; no device path ever falls back here.
 */
#include <omp.h>
#include <string.h>

#include "spmv_host.h"

static int nthreads(int threads) { return threads > 0 ? threads : omp_get_max_threads(); }

int spmv_cpu_threads(void) { return omp_get_max_threads(); }

int spmv_cpu_coo(int64_t n_rows, int64_t nnz, const int32_t *row,
                 const int32_t *col, const double *val, const double *x,
                 double *y, int threads)
{
    memset(y, 0, (size_t)n_rows * sizeof(double));
#pragma omp parallel for num_threads(nthreads(threads)) schedule(static)
    for (int64_t i = 0; i < nnz; ++i) {
        double p = val[i] * x[col[i]];
#pragma omp atomic
        y[row[i]] += p;
    }
    return SPMV_SUCCESS;
}

int spmv_cpu_csr(int64_t n_rows, const int64_t *row_ptr, const int32_t *col,
                 const double *val, const double *x, double *y, int threads)
{
#pragma omp parallel for num_threads(nthreads(threads)) schedule(static)
    for (int64_t r = 0; r < n_rows; ++r) {
        double s = 0.0;
        for (int64_t j = row_ptr[r]; j < row_ptr[r + 1]; ++j)
            s += val[j] * x[col[j]];
        y[r] = s;
    }
    return SPMV_SUCCESS;
}

int spmv_cpu_ell(int64_t n_rows, int32_t K, int64_t ld, int32_t ki,
                 const int32_t *col, const double *val, const double *x,
                 double *y, int threads)
{
#pragma omp parallel for num_threads(nthreads(threads)) schedule(static)
    for (int64_t r = 0; r < n_rows; ++r) {
        double s = 0.0;
        for (int64_t k = 0; k < K; ++k) {
            int64_t pos = (k / ki) * ld * ki + r * ki + (k % ki);
            s += val[pos] * x[col[pos]];
        }
        y[r] = s;
    }
    return SPMV_SUCCESS;
}

int spmv_cpu_sell(int64_t n_rows, int32_t C, int32_t ki, int64_t n_slices,
                  const int64_t *slice_ptr, const int32_t *perm,
                  const int32_t *col, const double *val, const double *x,
                  double *y, int threads)
{
    (void)n_rows;
#pragma omp parallel for num_threads(nthreads(threads)) schedule(dynamic, 16)
    for (int64_t s = 0; s < n_slices; ++s) {
        int64_t base = slice_ptr[s];
        int64_t w = (slice_ptr[s + 1] - base) / C;
        for (int64_t r = 0; r < C; ++r) {
            int32_t row = perm[s * C + r];
            if (row < 0)
                continue;
            double acc = 0.0;
            for (int64_t k = 0; k < w; ++k) {
                int64_t pos = base + (k / ki) * (int64_t)C * ki + r * ki + (k % ki);
                acc += val[pos] * x[col[pos]];
            }
            y[row] = acc;
        }
    }
    return SPMV_SUCCESS;
}

int spmv_cpu_cmrs(int64_t n_rows, int32_t h, int64_t n_strips,
                  const int64_t *strip_ptr, const uint8_t *row_in_strip,
                  const int32_t *col, const double *val, const double *x,
                  double *y, int threads)
{
    if (h < 1 || h > 64) /* the format's strip height (host/formats.c builds 1..64) */
        return SPMV_OTHER_ERROR;
#pragma omp parallel for num_threads(nthreads(threads)) schedule(static)
    for (int64_t s = 0; s < n_strips; ++s) {
        /* one slot per uint8 row tag: a tag >= h (a malformed strip) lands
         * in a slot that is never stored instead of past the array */
        double acc[256];
        for (int r = 0; r < h; ++r)
            acc[r] = 0.0;
        for (int64_t j = strip_ptr[s]; j < strip_ptr[s + 1]; ++j)
            acc[row_in_strip[j]] += val[j] * x[col[j]];
        for (int r = 0; r < h; ++r) {
            int64_t row = s * h + r;
            if (row < n_rows) /* reference Cmrs.cl:38-42 wrote past y here */
                y[row] = acc[r];
        }
    }
    return SPMV_SUCCESS;
}
