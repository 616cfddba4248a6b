/*
 * gen.c — deterministic synthetic matrices for the BASELINE.json configs.
 *
 * The reference's only inputs are databases/cant.mtx and cant-sorted.mtx
 * (reference csr.c:43, coo.c:43), which are Git-LFS pointers that were
 * never fetched.  These generators provide:
 *   - a cant-like stand-in with the real cant's N and nnz counts,
 *   - R-MAT 10^7 x 10^7 / 10^8 entries (BASELINE.json configs[3]),
 *   - the banded 10^8-row / 1.6e9-entry matrix (configs[4]), per row range,
 *   - small random ragged matrices for tests.
 * Every random draw is splitmix64 of (seed, counter), so a draw depends
 * only on its index: generation is order- and thread-count-independent.
 */
#include <stdlib.h>
#include <string.h>

#include "spmv_host.h"

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t spmv_splitmix64(uint64_t seed, uint64_t index)
{
    return mix64(seed * 0xD1B54A32D192ED03ULL + (index + 1) * 0x9E3779B97F4A7C15ULL);
}

static inline double u_pm1(uint64_t h) /* uniform in [-1, 1) */
{
    return (double)(h >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

/* ------------------------------------------------------------ cant-like */

enum { CL_NX = 9, CL_NY = 9, CL_NZ = 257, CL_DOF = 3 };
#define CL_N ((int64_t)CL_NX * CL_NY * CL_NZ * CL_DOF) /* 62,451 */
#define CL_TARGET_NNZ 4007383LL
#define CL_SEED 0xCA17ULL

static inline uint64_t pair_hash(int64_t r, int64_t c) /* r > c */
{
    return spmv_splitmix64(CL_SEED, (uint64_t)r * (uint64_t)CL_N + (uint64_t)c);
}

static int cmp_u64(const void *a, const void *b)
{
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : (x > y);
}

/* Visits the full 27-neighbourhood pattern of row r in ascending column
 * order; returns the number of columns written to cols[]. */
static int cl_row_cols(int64_t r, int64_t *cols)
{
    int64_t node = r / CL_DOF;
    int ix = (int)(node % CL_NX), iy = (int)((node / CL_NX) % CL_NY),
        iz = (int)(node / (CL_NX * CL_NY));
    int n = 0;
    for (int z = iz - 1; z <= iz + 1; ++z) {
        if (z < 0 || z >= CL_NZ)
            continue;
        for (int y = iy - 1; y <= iy + 1; ++y) {
            if (y < 0 || y >= CL_NY)
                continue;
            for (int x = ix - 1; x <= ix + 1; ++x) {
                if (x < 0 || x >= CL_NX)
                    continue;
                int64_t nb = x + (int64_t)CL_NX * (y + (int64_t)CL_NY * z);
                for (int d = 0; d < CL_DOF; ++d)
                    cols[n++] = nb * CL_DOF + d;
            }
        }
    }
    return n;
}

static uint64_t cl_threshold(void)
{
    static uint64_t thr = 0;
    static int done = 0;
    if (done)
        return thr;
    /* hashes of all strictly-lower pairs of the full pattern */
    int64_t cap = CL_N * 41, n = 0, cols[81];
    uint64_t *h = (uint64_t *)malloc((size_t)cap * sizeof(uint64_t));
    int64_t full = 0;
    for (int64_t r = 0; r < CL_N; ++r) {
        int k = cl_row_cols(r, cols);
        full += k;
        for (int i = 0; i < k; ++i)
            if (cols[i] < r)
                h[n++] = pair_hash(r, cols[i]);
    }
    /* drop (full - target)/2 pairs with the smallest hashes */
    int64_t drop = (full - CL_TARGET_NNZ) / 2;
    qsort(h, (size_t)n, sizeof(uint64_t), cmp_u64);
    thr = drop > 0 ? h[drop] : 0;
    free(h);
    done = 1;
    return thr;
}

static inline int cl_keep(int64_t r, int64_t c, uint64_t thr)
{
    if (r == c)
        return 1;
    return (r > c ? pair_hash(r, c) : pair_hash(c, r)) >= thr;
}

static inline double cl_value(int64_t r, int64_t c)
{
    if (r == c)
        return 16.0 + u_pm1(spmv_splitmix64(CL_SEED + 1, (uint64_t)r));
    int64_t a = r > c ? r : c, b = r > c ? c : r;
    return u_pm1(spmv_splitmix64(CL_SEED + 2, (uint64_t)a * (uint64_t)CL_N + (uint64_t)b));
}

int spmv_gen_cantlike(int mode, int64_t copies, int64_t *n_rows, int64_t *nnz,
                      int32_t *row, int32_t *col, double *val)
{
    if (mode < 0 || mode > 2 || copies < 1 || copies * CL_N > INT32_MAX)
        return SPMV_OTHER_ERROR;
    const uint64_t thr = cl_threshold();
    const int64_t per = mode == 2 ? (CL_TARGET_NNZ + CL_N) / 2 : CL_TARGET_NNZ;
    *n_rows = CL_N * copies;
    *nnz = per * copies;
    if (!row)
        return SPMV_SUCCESS;
    /* Row-major enumeration of the kept pattern (mode 0), or of the upper
     * triangle incl. diagonal (mode 2); modes 1 and 2 then swap (r, c):
     * the pattern and values are symmetric, so the transpose of the
     * row-major list is the column-major list of the same matrix. */
    int64_t n = 0, cols[81];
    for (int64_t r = 0; r < CL_N; ++r) {
        int k = cl_row_cols(r, cols);
        for (int i = 0; i < k; ++i) {
            int64_t c = cols[i];
            if (mode == 2 && c < r)
                continue;
            if (!cl_keep(r, c, thr))
                continue;
            if (n >= per)
                return SPMV_OTHER_ERROR;
            if (mode == 0) {
                row[n] = (int32_t)r;
                col[n] = (int32_t)c;
            } else {
                row[n] = (int32_t)c;
                col[n] = (int32_t)r;
            }
            val[n] = cl_value(r, c);
            ++n;
        }
    }
    if (n != per)
        return SPMV_OTHER_ERROR;
    for (int64_t b = 1; b < copies; ++b) {
        int32_t off = (int32_t)(b * CL_N);
        int32_t *rb = row + b * per, *cb = col + b * per;
        double *vb = val + b * per;
        for (int64_t i = 0; i < per; ++i) {
            rb[i] = row[i] + off;
            cb[i] = col[i] + off;
            vb[i] = val[i];
        }
    }
    return SPMV_SUCCESS;
}

/* ---------------------------------------------------------------- R-MAT */

int spmv_gen_rmat(int64_t n, int64_t nnz, int scale, uint64_t seed,
                  int32_t *row, int32_t *col, double *val)
{
    if (n < 1 || n > INT32_MAX || scale < 1 || scale > 31 || (1LL << scale) < n)
        return SPMV_OTHER_ERROR;
    /* quadrant thresholds on 16-bit draws: a=.57 b=.19 c=.19 d=.05 */
    const uint32_t ta = 37356, tb = 37356 + 12452, tc = 37356 + 2 * 12452;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nnz; ++i) {
        int64_t r = 0, c = 0;
        int ok = 0;
        for (uint64_t attempt = 0; attempt < 64 && !ok; ++attempt) {
            r = 0;
            c = 0;
            uint64_t h = 0;
            for (int lvl = 0; lvl < scale; ++lvl) {
                if (lvl % 4 == 0)
                    h = spmv_splitmix64(seed, ((uint64_t)i << 11) + attempt * 8 + (uint64_t)(lvl / 4));
                uint32_t u = (uint32_t)(h >> (16 * (lvl % 4))) & 0xFFFFu;
                int rb = u >= tb, cb = (u >= ta && u < tb) || u >= tc;
                r = (r << 1) | rb;
                c = (c << 1) | cb;
            }
            ok = r < n && c < n;
        }
        if (!ok) { /* practically unreachable; keep the draw in range */
            r %= n;
            c %= n;
        }
        row[i] = (int32_t)r;
        col[i] = (int32_t)c;
        val[i] = u_pm1(spmv_splitmix64(seed ^ 0x5EEDULL, (uint64_t)i));
    }
    return SPMV_SUCCESS;
}

/* --------------------------------------------------------------- banded */

int spmv_gen_banded_csr(int64_t n, uint64_t seed, int64_t row_begin,
                        int64_t row_end, int64_t *row_ptr, int32_t *col,
                        double *val)
{
    if (n < 16 || n > INT32_MAX || row_begin < 0 || row_end > n || row_begin > row_end)
        return SPMV_OTHER_ERROR;
    int64_t m = row_end - row_begin;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i <= m; ++i)
        row_ptr[i] = i * 16;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < m; ++i) {
        int64_t g = row_begin + i;
        for (int k = 0; k < 16; ++k) {
            int64_t c = (g + k - 8) % n;
            if (c < 0)
                c += n;
            col[i * 16 + k] = (int32_t)c;
            val[i * 16 + k] = u_pm1(spmv_splitmix64(seed, (uint64_t)g * 16 + (uint64_t)k));
        }
    }
    return SPMV_SUCCESS;
}

/* --------------------------------------------------------------- random */

int spmv_gen_random(int64_t n_rows, int64_t n_cols, int64_t min_len,
                    int64_t max_len, uint64_t seed, int64_t *nnz,
                    int32_t *row, int32_t *col, double *val)
{
    if (n_rows < 0 || n_cols < 1 || min_len < 0 || max_len < min_len)
        return SPMV_OTHER_ERROR;
    const uint64_t span = (uint64_t)(max_len - min_len + 1);
    int64_t total = 0;
    for (int64_t r = 0; r < n_rows; ++r)
        total += min_len + (int64_t)(spmv_splitmix64(seed, (uint64_t)r) % span);
    *nnz = total;
    if (!row)
        return SPMV_SUCCESS;
    int64_t p = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        int64_t len = min_len + (int64_t)(spmv_splitmix64(seed, (uint64_t)r) % span);
        for (int64_t k = 0; k < len; ++k, ++p) {
            uint64_t h = spmv_splitmix64(seed + 1, (uint64_t)p);
            row[p] = (int32_t)r;
            col[p] = (int32_t)(h % (uint64_t)n_cols);
            val[p] = u_pm1(spmv_splitmix64(seed + 2, (uint64_t)p));
        }
    }
    return SPMV_SUCCESS;
}
