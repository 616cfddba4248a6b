/*
 * formats.c — host builders for the five storage formats.
 *
 * The reference builds every format inside its fscanf loop and assumes a
 * row-sorted file without empty rows (reference csr.c:68-91 leaves ptr[]
 * slots unset after an empty row; sigma_c.c:93-139 and cmrs.c:84-113
 * count any row change as +1 row; ell.c:73-101 drops the last row from
 * K).  Here every builder starts from a CSR produced by a stable counting
 * sort, so any entry order and any number of empty rows is accepted, and
 * the layouts are the wave64 ones documented in spmv.h:
 *   ELL   column-major, ld = round_up(N,64), k-interleave ki
 *         (reference ell.c:118-164 was row-major N x K)
 *   SELL  C-row slices, rows sorted by length inside sigma windows,
 *         column-major inside a slice with k-interleave ki
 *         (reference sigma_c.c:71-202: C = 32, sigma = 1)
 *   CMRS  strips of h rows over the unchanged CSR arrays, uint8
 *         row_in_strip (reference cmrs.c:72-117: int32)
 * Padding slots carry value 0.0 and a column the row already reads (its
 * last real column), so they add no x traffic; the reference left ELL
 * padding values uninitialised (reference ell.c:119) and relied on
 * x[0] == 0.
 */
#include <stdlib.h>
#include <string.h>

#include "spmv_host.h"

static inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

int spmv_coo_sort_by_row(int64_t n_rows, int64_t nnz, const int32_t *row,
                         const int32_t *col, const double *val,
                         int32_t *row_out, int32_t *col_out, double *val_out)
{
    if (n_rows < 0 || nnz < 0)
        return SPMV_OTHER_ERROR;
    int64_t *cursor = (int64_t *)calloc((size_t)n_rows + 1, sizeof(int64_t));
    if (!cursor)
        return SPMV_OTHER_ERROR;
    for (int64_t i = 0; i < nnz; ++i) {
        if (row[i] < 0 || row[i] >= n_rows) {
            free(cursor);
            return SPMV_OTHER_ERROR;
        }
        cursor[row[i] + 1]++;
    }
    for (int64_t r = 0; r < n_rows; ++r)
        cursor[r + 1] += cursor[r];
    for (int64_t i = 0; i < nnz; ++i) {
        int64_t p = cursor[row[i]]++;
        row_out[p] = row[i];
        col_out[p] = col[i];
        val_out[p] = val[i];
    }
    free(cursor);
    return SPMV_SUCCESS;
}

int spmv_csr_from_coo(int64_t n_rows, int64_t nnz, const int32_t *row,
                      const int32_t *col, const double *val,
                      int64_t *row_ptr, int32_t *col_out, double *val_out)
{
    if (n_rows < 0 || nnz < 0)
        return SPMV_OTHER_ERROR;
    memset(row_ptr, 0, ((size_t)n_rows + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < nnz; ++i) {
        if (row[i] < 0 || row[i] >= n_rows)
            return SPMV_OTHER_ERROR;
        row_ptr[row[i] + 1]++;
    }
    for (int64_t r = 0; r < n_rows; ++r)
        row_ptr[r + 1] += row_ptr[r];
    /* stable scatter: reuse row_ptr[r] as the cursor, then shift back */
    for (int64_t i = 0; i < nnz; ++i) {
        int64_t p = row_ptr[row[i]]++;
        col_out[p] = col[i];
        val_out[p] = val[i];
    }
    for (int64_t r = n_rows; r > 0; --r)
        row_ptr[r] = row_ptr[r - 1];
    row_ptr[0] = 0;
    return SPMV_SUCCESS;
}

int spmv_csr_row_stats(int64_t n_rows, const int64_t *row_ptr,
                       int64_t *min_len, int64_t *max_len, double *mean_len)
{
    int64_t mn = n_rows > 0 ? INT64_MAX : 0, mx = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        int64_t l = row_ptr[r + 1] - row_ptr[r];
        if (l < mn)
            mn = l;
        if (l > mx)
            mx = l;
    }
    if (min_len)
        *min_len = mn;
    if (max_len)
        *max_len = mx;
    if (mean_len)
        *mean_len = n_rows > 0 ? (double)row_ptr[n_rows] / (double)n_rows : 0.0;
    return SPMV_SUCCESS;
}

/* Entries of every row sorted by column, stable (equal columns keep their
 * order): insertion sort below 32 entries, else a merge sort through a
 * per-thread scratch of the longest row. */
typedef struct {
    int32_t c;
    double v;
} cv_t;

static void sort_row(cv_t *a, cv_t *tmp, int64_t n)
{
    if (n < 32) {
        for (int64_t i = 1; i < n; ++i) {
            const cv_t k = a[i];
            int64_t j = i - 1;
            while (j >= 0 && a[j].c > k.c) {
                a[j + 1] = a[j];
                --j;
            }
            a[j + 1] = k;
        }
        return;
    }
    const int64_t h = n / 2;
    sort_row(a, tmp, h);
    sort_row(a + h, tmp, n - h);
    int64_t i = 0, j = h, k = 0;
    while (i < h && j < n)
        tmp[k++] = a[j].c < a[i].c ? a[j++] : a[i++];
    while (i < h)
        tmp[k++] = a[i++];
    while (j < n)
        tmp[k++] = a[j++];
    memcpy(a, tmp, (size_t)n * sizeof(cv_t));
}

int spmv_csr_sort_rows(int64_t n_rows, const int64_t *row_ptr, int32_t *col, double *val)
{
    if (n_rows < 0 || !row_ptr || row_ptr[0] < 0 || (row_ptr[n_rows] > 0 && (!col || !val)))
        return SPMV_OTHER_ERROR;
    int64_t mx = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        if (row_ptr[r + 1] < row_ptr[r]) /* offsets must not decrease */
            return SPMV_OTHER_ERROR;
        mx = row_ptr[r + 1] - row_ptr[r] > mx ? row_ptr[r + 1] - row_ptr[r] : mx;
    }
    int bad = 0;
#pragma omp parallel reduction(| : bad)
    {
        cv_t *a = (cv_t *)malloc((size_t)(mx > 0 ? mx : 1) * sizeof(cv_t));
        cv_t *tmp = (cv_t *)malloc((size_t)(mx > 0 ? mx : 1) * sizeof(cv_t));
        if (!a || !tmp) {
            bad = 1;
        } else {
#pragma omp for schedule(dynamic, 1024)
            for (int64_t r = 0; r < n_rows; ++r) {
                const int64_t b = row_ptr[r], n = row_ptr[r + 1] - b;
                if (n < 2)
                    continue;
                for (int64_t e = 0; e < n; ++e)
                    a[e] = (cv_t){col[b + e], val[b + e]};
                sort_row(a, tmp, n);
                for (int64_t e = 0; e < n; ++e) {
                    col[b + e] = a[e].c;
                    val[b + e] = a[e].v;
                }
            }
        }
        free(a);
        free(tmp);
    }
    return bad ? SPMV_OTHER_ERROR : SPMV_SUCCESS;
}

typedef struct {
    int64_t cnt;
    int32_t col;
} col_count_t;

static int by_count_desc(const void *a, const void *b)
{
    const col_count_t *p = (const col_count_t *)a, *q = (const col_count_t *)b;
    if (p->cnt != q->cnt)
        return p->cnt > q->cnt ? -1 : 1;
    return (p->col > q->col) - (p->col < q->col);
}

int spmv_hot_columns_possible(int64_t n_cols, int64_t H_req)
{
    return H_req > 0 || n_cols > ((int64_t)1 << 21);
}

int64_t spmv_hot_columns(int64_t n_cols, int64_t nnz, const int32_t *col, int64_t H_req, int32_t *hot,
                         int32_t *col_out)
{
    /* auto table: 2^19 columns (4 MiB, one XCD's L2), halved down to 2^16
     * while it exceeds nnz / 32: an eighth of the R-MAT 1e7/1e8 (1.25e7
     * entries, one of 8 row shards) ran 0.1330-0.1345 ms mean per shard with
     * 2^18 columns against 0.1343-0.1355 with 2^19 and 0.138-0.140 with 2^17
     * (profiles/round2/shard_rehearse_tiled_h.log): a smaller matrix reuses
     * each table entry less, so the per-run fill costs more than it saves */
    int64_t kAutoH = (int64_t)1 << 19;
    while (kAutoH > ((int64_t)1 << 16) && kAutoH > nnz / 32)
        kAutoH >>= 1;
    const int64_t cap = H_req > 0 ? H_req : kAutoH;
    if (n_cols <= 0 || nnz < 0 || H_req < 0 || !hot || !col_out || (nnz > 0 && !col) ||
        n_cols + cap > INT32_MAX)
        return -1;
    if (col_out != col)
        memcpy(col_out, col, (size_t)nnz * sizeof(int32_t));
    if (!spmv_hot_columns_possible(n_cols, H_req))
        return 0;
    int64_t *cnt = (int64_t *)calloc((size_t)n_cols, sizeof(int64_t));
    if (!cnt)
        return -1;
    int64_t maxc = 0;
    for (int64_t j = 0; j < nnz; ++j) {
        if (col[j] < 0 || col[j] >= n_cols) {
            free(cnt);
            return -1;
        }
        const int64_t c = ++cnt[col[j]];
        maxc = c > maxc ? c : maxc;
    }
    /* threshold count T: every column above T is hot, then columns equal
     * to T in increasing id until cap */
    int64_t *hist = (int64_t *)calloc((size_t)maxc + 2, sizeof(int64_t));
    if (!hist) {
        free(cnt);
        return -1;
    }
    for (int64_t c = 0; c < n_cols; ++c)
        hist[cnt[c]]++;
    int64_t above = 0, T = maxc;
    for (; T >= 1; --T) {
        if (above + hist[T] >= cap)
            break;
        above += hist[T];
    }
    free(hist);
    col_count_t *sel = (col_count_t *)malloc((size_t)cap * sizeof(col_count_t));
    if (!sel) {
        free(cnt);
        return -1;
    }
    int64_t n = 0, eq = 0, mass = 0;
    const int64_t eq_cap = T >= 1 ? cap - above : 0;
    for (int64_t c = 0; c < n_cols; ++c) {
        const int64_t k = cnt[c];
        if (k <= 0 || (T >= 1 && k < T))
            continue;
        if (T >= 1 && k == T) {
            if (eq >= eq_cap)
                continue;
            ++eq;
        }
        sel[n].cnt = k;
        sel[n].col = (int32_t)c;
        mass += k;
        ++n;
    }
    free(cnt);
    /* the rule: worth a table when the chosen columns take half of the
     * gathers and each is re-read at least 8 times per SpMV (the table
     * fill costs one scattered read per hot column) */
    if (H_req == 0 && (2 * mass < nnz || mass < 8 * n)) {
        free(sel);
        return 0;
    }
    qsort(sel, (size_t)n, sizeof *sel, by_count_desc);
    int32_t *rank = (int32_t *)malloc((size_t)n_cols * sizeof(int32_t));
    if (!rank) {
        free(sel);
        return -1;
    }
    for (int64_t c = 0; c < n_cols; ++c)
        rank[c] = -1;
    for (int64_t i = 0; i < n; ++i) {
        hot[i] = sel[i].col;
        rank[sel[i].col] = (int32_t)i;
    }
    free(sel);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < nnz; ++j) {
        const int32_t r = rank[col_out[j]];
        if (r >= 0)
            col_out[j] = (int32_t)(n_cols + r);
    }
    free(rank);
    return n;
}

/* first row r with row_ptr[r] >= off (row_ptr nondecreasing) */
static int64_t first_row_at(int64_t n_rows, const int64_t *row_ptr, int64_t off)
{
    int64_t lo = 0, hi = n_rows;
    while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (row_ptr[mid] < off)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

int64_t spmv_csr_tiled_bigplan(int64_t n_rows, const int64_t *row_ptr, int64_t tile, int32_t cap,
                               int32_t *plan)
{
    const int64_t kBigCap = 65536;
    if (n_rows < 0 || !row_ptr || tile < 2 || tile > 65535 || cap < 0)
        return -1;
    const int64_t nnz = row_ptr[n_rows];
    const int64_t tiles = nnz > 0 ? (nnz + tile - 1) / tile : 0;
    /* pass 1: the big tiles and their listed rows */
    int64_t nbig = 0, items = 0;
    for (int64_t t = 0; t < tiles; ++t) {
        const int64_t t0 = t * tile, t1 = t0 + tile < nnz ? t0 + tile : nnz;
        const int64_t r_lo = first_row_at(n_rows, row_ptr, t0);
        const int64_t r_hi = t1 == nnz ? n_rows - 1 : first_row_at(n_rows, row_ptr, t1) - 1;
        const int64_t nr = r_hi - r_lo + 1;
        if (nr <= cap || nr > kBigCap)
            continue;
        int64_t k = 0;
        for (int64_t r = r_lo; r <= r_hi; ++r) {
            const int64_t b = row_ptr[r + 1] < t1 ? row_ptr[r + 1] : t1;
            if (row_ptr[r] < b)
                ++k;
        }
        ++nbig;
        items += k;
    }
    const int64_t head = tiles + nbig + 1;
    const int64_t len = head + (head & 1) + 2 * items;
    if (len > INT32_MAX)
        return -1;
    if (!plan)
        return len;
    /* pass 2: fill */
    int64_t kb = 0, pos = head + (head & 1);
    for (int64_t t = 0; t < tiles; ++t) {
        const int64_t t0 = t * tile, t1 = t0 + tile < nnz ? t0 + tile : nnz;
        const int64_t r_lo = first_row_at(n_rows, row_ptr, t0);
        const int64_t r_hi = t1 == nnz ? n_rows - 1 : first_row_at(n_rows, row_ptr, t1) - 1;
        const int64_t nr = r_hi - r_lo + 1;
        plan[t] = -1;
        if (nr <= cap || nr > kBigCap)
            continue;
        plan[t] = (int32_t)kb;
        plan[tiles + kb] = (int32_t)pos;
        for (int64_t r = r_lo; r <= r_hi; ++r) {
            const int64_t b = row_ptr[r + 1] < t1 ? row_ptr[r + 1] : t1;
            if (row_ptr[r] < b) {
                plan[pos] = (int32_t)(r - r_lo);
                plan[pos + 1] = (int32_t)((uint32_t)(row_ptr[r] - t0) | ((uint32_t)(b - t0) << 16));
                pos += 2;
            }
        }
        ++kb;
    }
    plan[tiles + kb] = (int32_t)pos;
    if (head & 1)
        plan[head] = 0;
    return len;
}

/* Counting sort of the columns by entry count: ranks are handed out from
 * the largest count down, and inside one count in increasing column id, so
 * the order is the same whatever the thread count. */
int64_t spmv_column_relabel(int64_t n_cols, int64_t nnz, const int32_t *col, int32_t *order, int32_t *newid,
                            int32_t *col_out)
{
    return spmv_column_relabel_ex(n_cols, nnz, col, order, newid, col_out, 0);
}

int64_t spmv_column_relabel_ex(int64_t n_cols, int64_t nnz, const int32_t *col, int32_t *order, int32_t *newid,
                               int32_t *col_out, int32_t ties)
{
    if (ties != 0 && ties != 1)
        return -1;
    if (n_cols <= 0 || n_cols > INT32_MAX || nnz < 0 || !order || !newid || (nnz > 0 && (!col || !col_out)))
        return -1;
    int64_t *cnt = (int64_t *)calloc((size_t)n_cols, sizeof(int64_t));
    if (!cnt)
        return -1;
    int64_t maxc = 0;
    for (int64_t j = 0; j < nnz; ++j) {
        if (col[j] < 0 || col[j] >= n_cols) {
            free(cnt);
            return -1;
        }
        const int64_t c = ++cnt[col[j]];
        maxc = c > maxc ? c : maxc;
    }
    /* first[k] = first rank of count k: counts above k come first */
    int64_t *first = (int64_t *)calloc((size_t)maxc + 2, sizeof(int64_t));
    if (!first) {
        free(cnt);
        return -1;
    }
    for (int64_t c = 0; c < n_cols; ++c)
        first[cnt[c]]++;
    int64_t acc = 0, nonempty = n_cols - first[0];
    for (int64_t k = maxc; k >= 0; --k) {
        const int64_t h = first[k];
        first[k] = acc;
        acc += h;
    }
    if (ties == 0) {
        for (int64_t c = 0; c < n_cols; ++c) {
            const int64_t r = first[cnt[c]]++;
            order[r] = (int32_t)c;
            newid[c] = (int32_t)r;
        }
    } else {
        /* equal counts in order of first appearance in col (row-major CSR:
         * the first row using the column), unused columns last by id */
        for (int64_t c = 0; c < n_cols; ++c)
            newid[c] = -1;
        for (int64_t j = 0; j < nnz; ++j) {
            const int32_t c = col[j];
            if (newid[c] < 0) {
                const int64_t r = first[cnt[c]]++;
                order[r] = c;
                newid[c] = (int32_t)r;
            }
        }
        for (int64_t c = 0; c < n_cols; ++c)
            if (cnt[c] == 0) {
                const int64_t r = first[0]++;
                order[r] = (int32_t)c;
                newid[c] = (int32_t)r;
            }
    }
    free(first);
    free(cnt);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < nnz; ++j)
        col_out[j] = newid[col[j]];
    return nonempty;
}

int spmv_csr_variant_rule(int64_t n_rows, int64_t nnz, int64_t max_len)
{
    const double mean = n_rows > 0 ? (double)nnz / (double)n_rows : 0.0;
    return (max_len > 4096 && (double)max_len > 64.0 * mean) ? 4 : 0;
}

int spmv_csr_pick_variant(int64_t n_rows, const int64_t *row_ptr)
{
    int64_t mx = 0;
    spmv_csr_row_stats(n_rows, row_ptr, NULL, &mx, NULL);
    return spmv_csr_variant_rule(n_rows, n_rows > 0 ? row_ptr[n_rows] - row_ptr[0] : 0, mx);
}

/* ------------------------------------------------------------------ ELL */

int spmv_ell_plan(int64_t n_rows, const int64_t *row_ptr, int32_t ki,
                  int32_t *K, int64_t *ld)
{
    if (ki != 1 && ki != 2)
        return SPMV_OTHER_ERROR;
    int64_t mx = 0;
    spmv_csr_row_stats(n_rows, row_ptr, NULL, &mx, NULL);
    int64_t k = round_up(mx, ki);
    if (k > INT32_MAX)
        return SPMV_OTHER_ERROR;
    *K = (int32_t)k;
    *ld = round_up(n_rows, 64);
    return SPMV_SUCCESS;
}

int spmv_ell_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col,
                  const double *val, int32_t K, int64_t ld, int32_t ki,
                  int32_t *col_out, double *val_out)
{
    if ((ki != 1 && ki != 2) || K % ki != 0 || ld < n_rows || ld % 64 != 0)
        return SPMV_OTHER_ERROR;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < ld; ++i) {
        int64_t b = 0, e = 0;
        if (i < n_rows) {
            b = row_ptr[i];
            e = row_ptr[i + 1];
        }
        int32_t pad_col = e > b ? col[e - 1] : 0;
        for (int64_t k = 0; k < K; ++k) {
            int64_t pos = (k / ki) * ld * ki + i * ki + (k % ki);
            if (b + k < e) {
                col_out[pos] = col[b + k];
                val_out[pos] = val[b + k];
            } else {
                col_out[pos] = pad_col;
                val_out[pos] = 0.0;
            }
        }
    }
    return SPMV_SUCCESS;
}

/* ------------------------------------------------------------- SELL-C-σ */

typedef struct {
    int64_t len;
    int64_t row;
} len_row_t;

static int cmp_len_desc(const void *a, const void *b)
{
    const len_row_t *x = (const len_row_t *)a, *y = (const len_row_t *)b;
    if (x->len != y->len)
        return x->len > y->len ? -1 : 1;
    return x->row < y->row ? -1 : (x->row > y->row);
}

/* perm over n_slices*C slots; -1 marks padding slots. */
static int sell_perm(int64_t n_rows, const int64_t *row_ptr, int32_t C,
                     int32_t sigma, int64_t n_slices, int32_t *perm)
{
    int64_t slots = n_slices * C;
    for (int64_t i = 0; i < slots; ++i)
        perm[i] = i < n_rows ? (int32_t)i : -1;
    if (sigma <= 1)
        return SPMV_SUCCESS;
    int64_t n_win = (n_rows + sigma - 1) / sigma;
    int fail = 0;
#pragma omp parallel
    {
        len_row_t *tmp = (len_row_t *)malloc((size_t)sigma * sizeof(len_row_t));
        if (!tmp) {
#pragma omp atomic write
            fail = 1;
        }
#pragma omp for schedule(dynamic, 16)
        for (int64_t w = 0; w < n_win; ++w) {
            if (!tmp)
                continue;
            int64_t r0 = w * sigma;
            int64_t r1 = r0 + sigma < n_rows ? r0 + sigma : n_rows;
            int64_t n = r1 - r0;
            for (int64_t i = 0; i < n; ++i) {
                tmp[i].row = r0 + i;
                tmp[i].len = row_ptr[r0 + i + 1] - row_ptr[r0 + i];
            }
            qsort(tmp, (size_t)n, sizeof(len_row_t), cmp_len_desc);
            for (int64_t i = 0; i < n; ++i)
                perm[r0 + i] = (int32_t)tmp[i].row;
        }
        free(tmp);
    }
    return fail ? SPMV_OTHER_ERROR : SPMV_SUCCESS;
}

static int sell_check(int64_t n_rows, int32_t C, int32_t sigma, int32_t ki)
{
    if (n_rows < 0 || n_rows > INT32_MAX || C <= 0 || C > 1024)
        return SPMV_OTHER_ERROR;
    if (ki != 1 && ki != 2)
        return SPMV_OTHER_ERROR;
    if (sigma > 1 && sigma % C != 0)
        return SPMV_OTHER_ERROR;
    return SPMV_SUCCESS;
}

int spmv_sell_plan(int64_t n_rows, const int64_t *row_ptr, int32_t C,
                   int32_t sigma, int32_t ki, int64_t *n_slices,
                   int64_t *stored)
{
    int rc = sell_check(n_rows, C, sigma, ki);
    if (rc)
        return rc;
    int64_t ns = (n_rows + C - 1) / C;
    int32_t *perm = (int32_t *)malloc((size_t)(ns * C > 0 ? ns * C : 1) * sizeof(int32_t));
    if (!perm)
        return SPMV_OTHER_ERROR;
    rc = sell_perm(n_rows, row_ptr, C, sigma, ns, perm);
    int64_t total = 0;
    for (int64_t s = 0; s < ns && rc == 0; ++s) {
        int64_t w = 0;
        for (int64_t r = 0; r < C; ++r) {
            int32_t row = perm[s * C + r];
            if (row >= 0) {
                int64_t l = row_ptr[row + 1] - row_ptr[row];
                if (l > w)
                    w = l;
            }
        }
        total += round_up(w, ki) * C;
    }
    free(perm);
    *n_slices = ns;
    *stored = total;
    return rc;
}

int spmv_sell_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col,
                   const double *val, int32_t C, int32_t sigma, int32_t ki,
                   int64_t n_slices, int64_t *slice_ptr, int32_t *perm,
                   int32_t *col_out, double *val_out)
{
    int rc = sell_check(n_rows, C, sigma, ki);
    if (rc)
        return rc;
    if (n_slices != (n_rows + C - 1) / C)
        return SPMV_OTHER_ERROR;
    rc = sell_perm(n_rows, row_ptr, C, sigma, n_slices, perm);
    if (rc)
        return rc;
    slice_ptr[0] = 0;
    for (int64_t s = 0; s < n_slices; ++s) {
        int64_t w = 0;
        for (int64_t r = 0; r < C; ++r) {
            int32_t row = perm[s * C + r];
            if (row >= 0) {
                int64_t l = row_ptr[row + 1] - row_ptr[row];
                if (l > w)
                    w = l;
            }
        }
        slice_ptr[s + 1] = slice_ptr[s] + round_up(w, ki) * C;
    }
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t s = 0; s < n_slices; ++s) {
        int64_t base = slice_ptr[s];
        int64_t w = (slice_ptr[s + 1] - base) / C;
        /* padding of an empty (or missing) row points at a column some row
         * of this slice really reads, so a slice's columns stay a tight
         * window (the x-window kernels stage that window in LDS) */
        int32_t slice_col = 0;
        for (int64_t r = 0; r < C; ++r) {
            int32_t row = perm[s * C + r];
            if (row >= 0 && row_ptr[row + 1] > row_ptr[row]) {
                slice_col = col[row_ptr[row]];
                break;
            }
        }
        for (int64_t r = 0; r < C; ++r) {
            int32_t row = perm[s * C + r];
            int64_t b = 0, e = 0;
            if (row >= 0) {
                b = row_ptr[row];
                e = row_ptr[row + 1];
            }
            int32_t pad_col = e > b ? col[e - 1] : slice_col;
            for (int64_t k = 0; k < w; ++k) {
                int64_t pos = base + (k / ki) * (int64_t)C * ki + r * ki + (k % ki);
                if (b + k < e) {
                    col_out[pos] = col[b + k];
                    val_out[pos] = val[b + k];
                } else {
                    col_out[pos] = pad_col;
                    val_out[pos] = 0.0;
                }
            }
        }
    }
    return SPMV_SUCCESS;
}

/* ----------------------------------------------------------------- CMRS */

int spmv_cmrs_build(int64_t n_rows, const int64_t *row_ptr, int32_t h,
                    int64_t *strip_ptr, uint8_t *row_in_strip)
{
    if (h < 1 || h > 64 || n_rows < 0)
        return SPMV_OTHER_ERROR;
    int64_t ns = (n_rows + h - 1) / h;
    for (int64_t s = 0; s <= ns; ++s) {
        int64_t r = s * h < n_rows ? s * h : n_rows;
        strip_ptr[s] = row_ptr[r];
    }
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n_rows; ++r)
        for (int64_t j = row_ptr[r]; j < row_ptr[r + 1]; ++j)
            row_in_strip[j] = (uint8_t)(r % h);
    return SPMV_SUCCESS;
}

int spmv_cmrs_variant_rule(int64_t n_strips, int64_t nnz, int64_t max_len)
{
    if (n_strips <= 0)
        return 0;
    const double mean = (double)nnz / (double)n_strips;
    return (max_len > 4096 && (double)max_len > 64.0 * mean) ? 1 : 0;
}

int spmv_cmrs_pick_variant(int64_t n_strips, const int64_t *strip_ptr)
{
    if (n_strips <= 0)
        return 0;
    int64_t mx = 0;
    for (int64_t s = 0; s < n_strips; ++s) {
        const int64_t l = strip_ptr[s + 1] - strip_ptr[s];
        mx = l > mx ? l : mx;
    }
    return spmv_cmrs_variant_rule(n_strips, strip_ptr[n_strips] - strip_ptr[0], mx);
}

/* ------------------------------------------------------------ SELL split */

int32_t spmv_sell_split_auto(int64_t n_slices, const int64_t *slice_ptr, int32_t C, int32_t ki)
{
    if (n_slices <= 0 || C <= 0 || (ki != 1 && ki != 2))
        return 0;
    int64_t mx = 0;
    for (int64_t s = 0; s < n_slices; ++s) {
        const int64_t w = (slice_ptr[s + 1] - slice_ptr[s]) / C;
        mx = w > mx ? w : mx;
    }
    const double mean = (double)(slice_ptr[n_slices] - slice_ptr[0]) / (double)C / (double)n_slices;
    if (mx <= 1024 || (double)mx <= 16.0 * mean)
        return 0;
    /* 256 columns per wave whatever the mean: a mean raised by a few hub
     * slices (an R-MAT shard of low row ids) must not lengthen every chunk */
    return (int32_t)round_up(256, ki);
}

int64_t spmv_sell_split_plan(int64_t n_slices, const int64_t *slice_ptr, int32_t C, int32_t T,
                             int32_t *chunk_slice, int32_t *chunk_k0)
{
    if (n_slices < 0 || C <= 0 || T <= 0 || n_slices > INT32_MAX)
        return -1;
    int64_t n = 0;
    for (int64_t s = 0; s < n_slices; ++s) {
        const int64_t w = (slice_ptr[s + 1] - slice_ptr[s]) / C;
        for (int64_t k0 = T; k0 < w; k0 += T, ++n) {
            if (k0 > INT32_MAX)
                return -1;
            if (chunk_slice) {
                chunk_slice[n] = (int32_t)s;
                chunk_k0[n] = (int32_t)k0;
            }
        }
    }
    return n;
}

/* ------------------------------------------------------------------ HYB */

int spmv_hyb_plan(int64_t n_rows, const int64_t *row_ptr, int32_t ki, int32_t K_req, int32_t *K,
                  int64_t *ld, int64_t *tail_nnz)
{
    if ((ki != 1 && ki != 2) || n_rows < 0 || !K || !ld || !tail_nnz)
        return SPMV_OTHER_ERROR;
    const int64_t ldv = round_up(n_rows, 64);
    int64_t mx = 0, nnz = n_rows > 0 ? row_ptr[n_rows] - row_ptr[0] : 0;
    spmv_csr_row_stats(n_rows, row_ptr, NULL, &mx, NULL);
    int64_t k = K_req;
    if (k <= 0) {
        /* width that minimises stored bytes: 12 per ELL slot (all ld rows),
         * 16 per tail entry (row, col, val), plus kHybTwoKernelBytes when
         * both parts are non-empty (two kernels in sequence).  One cant-like
         * matrix cold (events, profiles/round6/ab_hyb_k.md): bytes alone gave
         * K = 52 (ELL + 866 K-entry tail) 22.2 us; K = 82 (the longest row,
         * ELL only) 15.1 us, 8.6 MB more bytes.  K = 0 (COO only) and K =
         * longest row are one kernel each. */
        const double kHybTwoKernelBytes = 32e6; /* ~4 us of HBM time: a launch gap and a latency ramp */
        const int64_t cap = mx < 65536 ? mx : 65536;
        int64_t *cnt = (int64_t *)calloc((size_t)cap + 2, sizeof(int64_t));
        if (!cnt)
            return SPMV_OTHER_ERROR;
        for (int64_t r = 0; r < n_rows; ++r) {
            const int64_t l = row_ptr[r + 1] - row_ptr[r];
            cnt[l < cap ? l : cap]++;
        }
        int64_t gt = n_rows - cnt[0]; /* rows longer than kk */
        int64_t tail = nnz, best_k = 0;
        double best = 16.0 * (double)tail;
        for (int64_t kk = 1; kk <= cap; ++kk) {
            tail -= gt;           /* every row longer than kk-1 moves one entry */
            gt -= cnt[kk];        /* rows longer than kk */
            const double cost = 12.0 * (double)ldv * (double)kk + 16.0 * (double)tail +
                                (tail > 0 ? kHybTwoKernelBytes : 0.0);
            if (cost < best) {
                best = cost;
                best_k = kk;
            }
        }
        free(cnt);
        k = best_k;
    }
    k = round_up(k, ki);
    if (k > INT32_MAX)
        return SPMV_OTHER_ERROR;
    int64_t tail = 0;
    for (int64_t r = 0; r < n_rows; ++r) {
        const int64_t l = row_ptr[r + 1] - row_ptr[r];
        tail += l > k ? l - k : 0;
    }
    *K = (int32_t)k;
    *ld = ldv;
    *tail_nnz = tail;
    return SPMV_SUCCESS;
}

int spmv_hyb_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col, const double *val,
                  int32_t K, int64_t ld, int32_t ki, int32_t *ell_col, double *ell_val,
                  int32_t *tail_row, int32_t *tail_col, double *tail_val)
{
    if ((ki != 1 && ki != 2) || K < 0 || K % ki != 0 || ld < n_rows || ld % 64 != 0)
        return SPMV_OTHER_ERROR;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < ld; ++i) {
        int64_t b = 0, e = 0;
        if (i < n_rows) {
            b = row_ptr[i];
            e = row_ptr[i + 1];
        }
        /* padding reuses the row's last ELL column (a valid gather); with K = 0
         * there is no ELL part and no column to read (found by `make test-san`:
         * col[b - 1] was read for K = 0) */
        const int32_t pad_col = (K > 0 && e > b) ? col[(e - b > K ? b + K : e) - 1] : 0;
        for (int64_t k = 0; k < K; ++k) {
            const int64_t pos = (k / ki) * ld * ki + i * ki + (k % ki);
            if (b + k < e) {
                ell_col[pos] = col[b + k];
                ell_val[pos] = val[b + k];
            } else {
                ell_col[pos] = pad_col;
                ell_val[pos] = 0.0;
            }
        }
    }
    /* tail: entries past the first K of each row, in CSR (row-sorted) order */
    int64_t t = 0;
    for (int64_t r = 0; r < n_rows; ++r)
        for (int64_t j = row_ptr[r] + K; j < row_ptr[r + 1]; ++j) {
            tail_row[t] = (int32_t)r;
            tail_col[t] = col[j];
            tail_val[t] = val[j];
            ++t;
        }
    return SPMV_SUCCESS;
}

/* ------------------------------------------- CSR, 16-bit column offsets */

/* smallest column of block b and whether the block's span fits 16 bits */
static int csr16_block(int64_t nnz, const int32_t *col, int64_t b, int32_t *lo)
{
    const int64_t p0 = b * 64, p1 = p0 + 64 < nnz ? p0 + 64 : nnz;
    int32_t mn = col[p0], mx = col[p0];
    for (int64_t p = p0 + 1; p < p1; ++p) {
        mn = col[p] < mn ? col[p] : mn;
        mx = col[p] > mx ? col[p] : mx;
    }
    *lo = mn;
    return (int64_t)mx - (int64_t)mn <= 65535;
}

int spmv_csr16_plan(int64_t nnz, const int32_t *col, int64_t *n_blocks, int64_t *n_esc)
{
    if (nnz < 0 || !n_blocks || !n_esc)
        return SPMV_OTHER_ERROR;
    const int64_t nb = (nnz + 63) / 64;
    int64_t esc = 0;
#pragma omp parallel for schedule(static) reduction(+ : esc)
    for (int64_t b = 0; b < nb; ++b) {
        int32_t lo;
        esc += !csr16_block(nnz, col, b, &lo);
    }
    if (esc > (int64_t)INT32_MAX)
        return SPMV_OTHER_ERROR;
    *n_blocks = nb;
    *n_esc = esc;
    return SPMV_SUCCESS;
}

int spmv_csr16_fill(int64_t nnz, const int32_t *col, int32_t *blk_base, uint16_t *col_off,
                    int32_t *col_esc)
{
    if (nnz < 0)
        return SPMV_OTHER_ERROR;
    const int64_t nb = (nnz + 63) / 64;
    int64_t slot = 0;
    /* serial: escape slots are numbered in block order */
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t p0 = b * 64, p1 = p0 + 64 < nnz ? p0 + 64 : nnz;
        int32_t lo;
        if (csr16_block(nnz, col, b, &lo)) {
            blk_base[b] = lo;
            for (int64_t p = p0; p < p1; ++p)
                col_off[p] = (uint16_t)(col[p] - lo);
        } else {
            blk_base[b] = (int32_t)(-1 - slot);
            for (int64_t p = p0; p < p0 + 64; ++p)
                col_esc[slot * 64 + (p - p0)] = col[p < p1 ? p : p1 - 1];
            for (int64_t p = p0; p < p1; ++p)
                col_off[p] = 0;
            ++slot;
        }
    }
    return SPMV_SUCCESS;
}

/* -------------------------------------------------- column-grouped CSR */

int32_t spmv_csrg_group(int32_t col, int32_t groups)
{
    const uint64_t h = ((uint64_t)(uint32_t)col >> 4) * 0x9E3779B97F4A7C15ULL;
    return groups > 1 ? (int32_t)((h >> 40) % (uint64_t)groups) : 0;
}

/* groups present in row r (bit g) */
static uint64_t csrg_mask(const int64_t *row_ptr, const int32_t *col, int64_t r, int32_t groups)
{
    uint64_t m = 0;
    for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; ++e)
        m |= 1ULL << spmv_csrg_group(col[e], groups);
    return m;
}

int32_t spmv_csrg_block_rows(void) { return SPMV_CSRG_ROWS; }

int spmv_csrg_plan(int64_t n_rows, const int64_t *row_ptr, const int32_t *col, int32_t groups,
                   int64_t *n_pairs)
{
    if (n_rows < 0 || groups < 1 || groups > 64 || !row_ptr || !n_pairs || (row_ptr[n_rows] > 0 && !col))
        return SPMV_OTHER_ERROR;
    int64_t np = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : np)
    for (int64_t r = 0; r < n_rows; ++r)
        np += __builtin_popcountll(csrg_mask(row_ptr, col, r, groups));
    if (np > (int64_t)INT32_MAX)
        return SPMV_OTHER_ERROR;
    *n_pairs = np;
    return SPMV_SUCCESS;
}

/* Rows are cut into blocks of SPMV_CSRG_ROWS; pass 1 counts each block's
 * pairs and entries per group, a prefix over (group, block) gives every
 * block its starting pair and entry in every group (the group-major
 * layout, and blk_off), pass 2 writes them.  Same layout for any thread
 * count. */
int spmv_csrg_fill(int64_t n_rows, const int64_t *row_ptr, const int32_t *col, const double *val,
                   int32_t groups, int64_t *pair_ptr, int32_t *col_g, double *val_g,
                   int32_t *blk_off, uint16_t *pair_row)
{
    if (n_rows < 0 || groups < 1 || groups > 64 || !row_ptr || !pair_ptr || !blk_off)
        return SPMV_OTHER_ERROR;
    const int64_t nnz = row_ptr[n_rows];
    if (nnz > 0 && (!col || !val || !col_g || !val_g || !pair_row))
        return SPMV_OTHER_ERROR;
    const int64_t B = SPMV_CSRG_ROWS;
    const int64_t nb = (n_rows + B - 1) / B;
    const int G = groups;
    int64_t *pc = calloc((size_t)((nb + 1) * G), sizeof(int64_t)); /* pairs of block k in group g: [g*(nb+1) + k] */
    int64_t *ec = calloc((size_t)((nb + 1) * G), sizeof(int64_t)); /* entries */
    if (!pc || !ec) {
        free(pc);
        free(ec);
        return SPMV_OTHER_ERROR;
    }
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t k = 0; k < nb; ++k) {
        const int64_t r1 = (k + 1) * B < n_rows ? (k + 1) * B : n_rows;
        for (int64_t r = k * B; r < r1; ++r) {
            uint64_t m = 0;
            for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                const int32_t g = spmv_csrg_group(col[e], groups);
                m |= 1ULL << g;
                ++ec[g * (nb + 1) + k];
            }
            for (; m; m &= m - 1)
                ++pc[__builtin_ctzll(m) * (nb + 1) + k];
        }
    }
    /* exclusive prefix in (group, block) order; entry nb of each group row
     * is the group's end (= the next group's start) */
    int64_t ps = 0, es = 0;
    for (int64_t i = 0; i < (nb + 1) * G; ++i) {
        const int64_t pn = pc[i], en = ec[i];
        pc[i] = ps;
        ec[i] = es;
        ps += pn;
        es += en;
    }
    if (ps > (int64_t)INT32_MAX) {
        free(pc);
        free(ec);
        return SPMV_OTHER_ERROR;
    }
    for (int64_t i = 0; i < (nb + 1) * G; ++i)
        blk_off[i] = (int32_t)pc[i];
    pair_ptr[ps] = es;
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t k = 0; k < nb; ++k) {
        int64_t pn[64], en[64];
        for (int g = 0; g < G; ++g) {
            pn[g] = pc[g * (nb + 1) + k];
            en[g] = ec[g * (nb + 1) + k];
        }
        const int64_t r1 = (k + 1) * B < n_rows ? (k + 1) * B : n_rows;
        for (int64_t r = k * B; r < r1; ++r) {
            const uint64_t m = csrg_mask(row_ptr, col, r, groups);
            for (uint64_t mm = m; mm; mm &= mm - 1) { /* each group of the row: open its pair */
                const int g = __builtin_ctzll(mm);
                pair_ptr[pn[g]] = en[g];
                pair_row[pn[g]] = (uint16_t)(r - k * B);
            }
            for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; ++e) { /* entries in CSR order */
                const int g = spmv_csrg_group(col[e], groups);
                col_g[en[g]] = col[e];
                val_g[en[g]] = val[e];
                ++en[g];
            }
            for (uint64_t mm = m; mm; mm &= mm - 1)
                ++pn[__builtin_ctzll(mm)];
        }
    }
    free(pc);
    free(ec);
    return SPMV_SUCCESS;
}

/* ------------------------------------------------------------ sharding */

int spmv_partition_rows_weighted(int64_t n_rows, const int64_t *row_ptr, int parts, int64_t align,
                                 double row_weight, int64_t *bounds)
{
    if (parts < 1 || n_rows < 0 || align < 1 || !(row_weight >= 0.0))
        return SPMV_OTHER_ERROR;
    const double total = (double)row_ptr[n_rows] + row_weight * (double)n_rows;
    bounds[0] = 0;
    for (int p = 1; p < parts; ++p) {
        /* first row whose cost prefix (entries + row_weight per row)
         * reaches p/parts of the total */
        const double target = total * p / parts;
        int64_t lo = 0, hi = n_rows;
        while (lo < hi) {
            int64_t mid = lo + (hi - lo) / 2;
            if ((double)row_ptr[mid] + row_weight * (double)mid < target)
                lo = mid + 1;
            else
                hi = mid;
        }
        int64_t b = (lo + align / 2) / align * align;
        if (total == 0.0)
            b = (n_rows * p / parts) / align * align;
        if (b < bounds[p - 1])
            b = bounds[p - 1];
        if (b > n_rows)
            b = n_rows;
        bounds[p] = b;
    }
    bounds[parts] = n_rows;
    return SPMV_SUCCESS;
}

/* Cost prefix of rows [0, r) under measured shard times: inside old shard
 * g a row costs rate_g * (entries + row_weight), rate_g = ms_g / (the
 * shard's entries + row_weight * rows). */
static double calibrated_prefix(int64_t r, const int64_t *row_ptr, int old_parts, const int64_t *ob,
                                const double *ms, double w)
{
    double c = 0.0;
    for (int g = 0; g < old_parts; ++g) {
        const int64_t lo = ob[g], hi = ob[g + 1];
        const double W = (double)(row_ptr[hi] - row_ptr[lo]) + w * (double)(hi - lo);
        if (r >= hi) {
            c += ms[g];
            continue;
        }
        if (r > lo && W > 0.0)
            c += ms[g] * ((double)(row_ptr[r] - row_ptr[lo]) + w * (double)(r - lo)) / W;
        break;
    }
    return c;
}

int spmv_partition_rows_calibrated(int64_t n_rows, const int64_t *row_ptr, int parts, int64_t align,
                                   double row_weight, int old_parts, const int64_t *old_bounds,
                                   const double *old_ms, int64_t *bounds)
{
    if (parts < 1 || old_parts < 1 || n_rows < 0 || align < 1 || !(row_weight >= 0.0) || !old_bounds ||
        !old_ms || old_bounds[0] != 0 || old_bounds[old_parts] != n_rows)
        return SPMV_OTHER_ERROR;
    double total = 0.0;
    for (int g = 0; g < old_parts; ++g) {
        if (old_bounds[g + 1] < old_bounds[g] || !(old_ms[g] >= 0.0))
            return SPMV_OTHER_ERROR;
        total += old_ms[g];
    }
    if (!(total > 0.0))
        return spmv_partition_rows_weighted(n_rows, row_ptr, parts, align, row_weight, bounds);
    bounds[0] = 0;
    for (int p = 1; p < parts; ++p) {
        const double target = total * p / parts;
        int64_t lo = 0, hi = n_rows;
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo) / 2;
            if (calibrated_prefix(mid, row_ptr, old_parts, old_bounds, old_ms, row_weight) < target)
                lo = mid + 1;
            else
                hi = mid;
        }
        int64_t b = (lo + align / 2) / align * align;
        if (b < bounds[p - 1])
            b = bounds[p - 1];
        if (b > n_rows)
            b = n_rows;
        bounds[p] = b;
    }
    bounds[parts] = n_rows;
    return SPMV_SUCCESS;
}

int64_t spmv_coo_row_shard(int64_t nnz, const int32_t *row, const int32_t *col, const double *val,
                           int64_t lo, int64_t hi, int32_t *row_out, int32_t *col_out, double *val_out)
{
    if (nnz < 0 || lo < 0 || hi < lo || (nnz > 0 && (!row || !col || !val)) || hi - lo > INT32_MAX)
        return -1;
    int64_t k = 0;
    for (int64_t e = 0; e < nnz; ++e) {
        if (row[e] < lo || row[e] >= hi)
            continue;
        if (row_out) {
            row_out[k] = (int32_t)(row[e] - lo);
            col_out[k] = col[e];
            val_out[k] = val[e];
        }
        ++k;
    }
    return k;
}

int spmv_partition_rows(int64_t n_rows, const int64_t *row_ptr, int parts,
                        int64_t align, int64_t *bounds)
{
    if (parts < 1 || n_rows < 0 || align < 1)
        return SPMV_OTHER_ERROR;
    const int64_t nnz = row_ptr[n_rows];
    bounds[0] = 0;
    for (int p = 1; p < parts; ++p) {
        /* first row whose start offset reaches p/parts of the entries */
        int64_t target = (int64_t)((double)nnz * p / parts);
        int64_t lo = 0, hi = n_rows;
        while (lo < hi) {
            int64_t mid = lo + (hi - lo) / 2;
            if (row_ptr[mid] < target)
                lo = mid + 1;
            else
                hi = mid;
        }
        int64_t b = (lo + align / 2) / align * align;
        if (nnz == 0)
            b = (n_rows * p / parts) / align * align;
        if (b < bounds[p - 1])
            b = bounds[p - 1];
        if (b > n_rows)
            b = n_rows;
        bounds[p] = b;
    }
    bounds[parts] = n_rows;
    return SPMV_SUCCESS;
}
