/*
 * mtx.c — Matrix Market coordinate reader/writer.
 *
 * Acceptance semantics follow the reference:
 *   - banner: 5 whitespace tokens, the first must start with
 *     "%%MatrixMarket", the rest are compared case-insensitively
 *     (reference mmio/mmio.c:96-179);
 *   - comment lines starting with '%' before the size line are skipped,
 *     the size line is "M N nz" (reference mmio/mmio.c:189-217);
 *   - complex matrices are rejected (reference inc/helper_functions.h:151);
 *     symmetric / skew / hermitian banners are accepted and the listed
 *     entries are used literally, never mirrored (reference csr.c:77-91
 *     reads exactly nz lines and nothing else);
 *   - entries are "row col value" tokens in any whitespace layout, the
 *     same tokens fscanf("%d %d %lg\n") consumes (reference csr.c:81),
 *     converted 1-based -> 0-based.
 * Deliberate differences (reference behaviour undefined there):
 *   - dense "array" files are rejected instead of mis-parsed;
 *   - pattern files get value 1.0 (the reference's "%lg" would swallow the
 *     next line's row index);
 *   - out-of-range indices and short files are FILE errors instead of
 *     out-of-bounds writes.
 * The whole file is read once into memory and tokenised in place — one
 * pass instead of the reference's three to four fscanf passes — by all
 * OpenMP threads when the file has one entry per line (parse_parallel),
 * else serially.  spmv_bin_* keep a binary copy next to the text file
 * (the text parse dominated the reference's wall time).
 */
#include <ctype.h>
#include <omp.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "spmv_host.h"

typedef struct {
    char *buf;
    size_t len;
    size_t pos;
} text_t;

static int slurp(const char *path, text_t *t)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return -1;
    if (fseek(f, 0, SEEK_END) != 0) {
        fclose(f);
        return -1;
    }
    long sz = ftell(f);
    if (sz < 0) {
        fclose(f);
        return -1;
    }
    rewind(f);
    t->buf = (char *)malloc((size_t)sz + 1);
    if (!t->buf) {
        fclose(f);
        return -1;
    }
    size_t got = fread(t->buf, 1, (size_t)sz, f);
    fclose(f);
    t->buf[got] = '\0';
    t->len = got;
    t->pos = 0;
    return 0;
}

/* Copies the next line (without '\n') into out; returns 0 at EOF. */
static int next_line(text_t *t, char *out, size_t cap)
{
    if (t->pos >= t->len)
        return 0;
    size_t start = t->pos;
    while (t->pos < t->len && t->buf[t->pos] != '\n')
        t->pos++;
    size_t n = t->pos - start;
    if (t->pos < t->len)
        t->pos++; /* skip '\n' */
    if (n >= cap)
        n = cap - 1;
    memcpy(out, t->buf + start, n);
    out[n] = '\0';
    return 1;
}

static void lower(char *s)
{
    for (; *s; ++s)
        *s = (char)tolower((unsigned char)*s);
}

/* Parses banner + size line, leaves t->pos at the first entry token. */
static int parse_header(text_t *t, spmv_mtx_info *info)
{
    char line[1100];
    char banner[64], mtx[64], crd[64], dtype[64], sym[64];

    memset(info, 0, sizeof(*info));
    if (!next_line(t, line, sizeof line))
        return SPMV_FILE_ERROR;
    if (sscanf(line, "%63s %63s %63s %63s %63s", banner, mtx, crd, dtype,
               sym) != 5)
        return SPMV_FILE_ERROR;
    lower(mtx);
    lower(crd);
    lower(dtype);
    lower(sym);
    if (strncmp(banner, "%%MatrixMarket", 14) != 0)
        return SPMV_FILE_ERROR;
    if (strcmp(mtx, "matrix") != 0)
        return SPMV_FILE_ERROR;
    if (strcmp(crd, "coordinate") != 0)
        return SPMV_FILE_ERROR; /* "array" (dense) is not a sparse input */
    if (strcmp(dtype, "real") == 0) {
    } else if (strcmp(dtype, "integer") == 0) {
        info->integer = 1;
    } else if (strcmp(dtype, "pattern") == 0) {
        info->pattern = 1;
    } else {
        return SPMV_FILE_ERROR; /* complex, or unknown */
    }
    if (strcmp(sym, "general") == 0) {
    } else if (strcmp(sym, "symmetric") == 0 || strcmp(sym, "hermitian") == 0 ||
               strcmp(sym, "skew-symmetric") == 0) {
        info->symmetric = 1;
    } else {
        return SPMV_FILE_ERROR;
    }

    /* size line: skip '%' comment lines (and blank lines, as the
     * reference's fscanf fallback does) */
    for (;;) {
        if (!next_line(t, line, sizeof line))
            return SPMV_FILE_ERROR;
        if (line[0] == '%')
            continue;
        long long m, n, z;
        int k = sscanf(line, "%lld %lld %lld", &m, &n, &z);
        if (k == 3) {
            if (m < 0 || n < 0 || z < 0 || m > INT32_MAX || n > INT32_MAX)
                return SPMV_FILE_ERROR;
            info->n_rows = m;
            info->n_cols = n;
            info->nnz = z;
            return SPMV_SUCCESS;
        }
        /* blank (or whitespace-only) line: keep scanning */
        const char *p = line;
        while (*p && isspace((unsigned char)*p))
            ++p;
        if (*p)
            return SPMV_FILE_ERROR;
    }
}

int spmv_mtx_read_info(const char *path, spmv_mtx_info *info)
{
    /* Only the header is needed: read the first few KB, not the file. */
    FILE *f = fopen(path, "rb");
    if (!f)
        return SPMV_FILE_ERROR;
    text_t t;
    size_t cap = 1 << 16;
    t.buf = (char *)malloc(cap + 1);
    if (!t.buf) {
        fclose(f);
        return SPMV_OTHER_ERROR;
    }
    t.len = fread(t.buf, 1, cap, f);
    t.buf[t.len] = '\0';
    t.pos = 0;
    fclose(f);
    int rc = parse_header(&t, info);
    if (rc != SPMV_SUCCESS && t.len == cap) {
        /* very long comment block: fall back to the whole file */
        free(t.buf);
        if (slurp(path, &t) != 0)
            return SPMV_FILE_ERROR;
        rc = parse_header(&t, info);
    }
    free(t.buf);
    return rc;
}

static inline const char *skip_ws(const char *p)
{
    while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' ||
           *p == '\f' || *p == '\v')
        ++p;
    return p;
}

static inline const char *parse_i64(const char *p, long long *out, int *ok)
{
    p = skip_ws(p);
    int neg = 0;
    if (*p == '+' || *p == '-') {
        neg = (*p == '-');
        ++p;
    }
    if (*p < '0' || *p > '9') {
        *ok = 0;
        return p;
    }
    long long v = 0;
    while (*p >= '0' && *p <= '9') {
        v = v * 10 + (*p - '0');
        if (v > (1LL << 40)) { /* far beyond int32: reject, avoid overflow */
            *ok = 0;
            return p;
        }
        ++p;
    }
    *out = neg ? -v : v;
    *ok = 1;
    return p;
}

/* Parses the entries in [p, e) (whole lines); writes them from index 0 of
 * row/col/val when row != NULL.  Returns the count, or -1 on a malformed
 * or out-of-range entry. */
static int64_t parse_range(const char *p, const char *e, const spmv_mtx_info *info,
                           int32_t *row, int32_t *col, double *val)
{
    int64_t n = 0;
    for (;;) {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' ||
                         *p == '\f' || *p == '\v'))
            ++p;
        if (p >= e)
            return n;
        long long r, c;
        int ok;
        p = parse_i64(p, &r, &ok);
        if (!ok || p > e)
            return -1;
        p = parse_i64(p, &c, &ok);
        if (!ok || p > e)
            return -1;
        if (r < 1 || r > info->n_rows || c < 1 || c > info->n_cols)
            return -1;
        double v = 1.0;
        if (!info->pattern) {
            p = skip_ws(p);
            char *end;
            v = strtod(p, &end);
            if (end == p || end > e)
                return -1;
            p = end;
        }
        if (row) {
            row[n] = (int32_t)(r - 1);
            col[n] = (int32_t)(c - 1);
            val[n] = v;
        }
        ++n;
    }
}

/* Multi-threaded entry parse: the entry text is cut into one chunk per
 * thread at line boundaries, each chunk is counted, then parsed into its
 * place.  Valid only when the chunks hold exactly nnz entries in total
 * (one entry per line, nothing after the last one); otherwise the caller
 * falls back to the serial reader, which follows the reference's fscanf
 * semantics exactly (reads nnz entries, ignores the rest). */
static int parse_parallel(const char *b, const char *e, const spmv_mtx_info *info,
                          int32_t *row, int32_t *col, double *val)
{
    int T = omp_get_max_threads();
    if (T > 64)
        T = 64;
    if (T < 2 || e - b < (4 << 20))
        return -1;
    const char *cut[65];
    int64_t cnt[64], off[65];
    cut[0] = b;
    for (int t = 1; t < T; ++t) {
        const char *q = b + (e - b) * t / T;
        if (q < cut[t - 1])
            q = cut[t - 1];
        while (q < e && *q != '\n')
            ++q;
        cut[t] = q < e ? q + 1 : e;
    }
    cut[T] = e;
    int bad = 0;
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; ++t) {
        cnt[t] = parse_range(cut[t], cut[t + 1], info, NULL, NULL, NULL);
        if (cnt[t] < 0) {
#pragma omp atomic write
            bad = 1;
        }
    }
    if (bad)
        return -1;
    off[0] = 0;
    for (int t = 0; t < T; ++t)
        off[t + 1] = off[t] + cnt[t];
    if (off[T] != info->nnz)
        return -1;
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; ++t)
        parse_range(cut[t], cut[t + 1], info, row + off[t], col + off[t], val + off[t]);
    return 0;
}

int spmv_mtx_read(const char *path, spmv_mtx_info *info, int32_t *row,
                  int32_t *col, double *val)
{
    text_t t;
    if (slurp(path, &t) != 0)
        return SPMV_FILE_ERROR;
    int rc = parse_header(&t, info);
    if (rc != SPMV_SUCCESS) {
        free(t.buf);
        return rc;
    }
    const char *p = t.buf + t.pos;
    if (parse_parallel(p, t.buf + t.len, info, row, col, val) == 0) {
        free(t.buf);
        return SPMV_SUCCESS;
    }
    const int64_t nz = info->nnz;
    const int64_t nr = info->n_rows, nc = info->n_cols;
    for (int64_t i = 0; i < nz; ++i) {
        long long r, c;
        int ok;
        p = parse_i64(p, &r, &ok);
        if (!ok)
            goto bad;
        p = parse_i64(p, &c, &ok);
        if (!ok)
            goto bad;
        if (r < 1 || r > nr || c < 1 || c > nc)
            goto bad;
        double v = 1.0;
        if (!info->pattern) {
            p = skip_ws(p);
            char *end;
            errno = 0;
            v = strtod(p, &end);
            if (end == p)
                goto bad;
            p = end;
        }
        row[i] = (int32_t)(r - 1);
        col[i] = (int32_t)(c - 1);
        val[i] = v;
    }
    free(t.buf);
    return SPMV_SUCCESS;
bad:
    free(t.buf);
    return SPMV_FILE_ERROR;
}

int spmv_mtx_write(const char *path, int64_t n_rows, int64_t n_cols,
                   int64_t nnz, const int32_t *row, const int32_t *col,
                   const double *val, int symmetric)
{
    FILE *f = fopen(path, "w");
    if (!f)
        return SPMV_FILE_ERROR;
    size_t bufsz = 1 << 22;
    char *buf = (char *)malloc(bufsz);
    if (buf)
        setvbuf(f, buf, _IOFBF, bufsz);
    fprintf(f, "%%%%MatrixMarket matrix coordinate real %s\n",
            symmetric ? "symmetric" : "general");
    fprintf(f, "%lld %lld %lld\n", (long long)n_rows, (long long)n_cols,
            (long long)nnz);
    for (int64_t i = 0; i < nnz; ++i)
        fprintf(f, "%d %d %.17g\n", row[i] + 1, col[i] + 1, val[i]);
    int bad = ferror(f);
    fclose(f);
    free(buf);
    return bad ? SPMV_FILE_ERROR : SPMV_SUCCESS;
}

/* ------------------------------------------------------- binary cache */

/* Layout: 64-byte header {magic "SPMVBIN1", n_rows, n_cols, nnz, flags,
 * reserved}, then row[nnz] int32, col[nnz] int32, val[nnz] f64, all in
 * file order.  flags: bit0 symmetric, bit1 pattern, bit2 integer. */
typedef struct {
    char magic[8];
    int64_t n_rows, n_cols, nnz, flags, reserved[3];
} bin_header_t;

int spmv_bin_write(const char *path, const spmv_mtx_info *info, const int32_t *row,
                   const int32_t *col, const double *val)
{
    FILE *f = fopen(path, "wb");
    if (!f)
        return SPMV_FILE_ERROR;
    bin_header_t h;
    memset(&h, 0, sizeof h);
    memcpy(h.magic, "SPMVBIN1", 8);
    h.n_rows = info->n_rows;
    h.n_cols = info->n_cols;
    h.nnz = info->nnz;
    h.flags = (info->symmetric ? 1 : 0) | (info->pattern ? 2 : 0) | (info->integer ? 4 : 0);
    size_t z = (size_t)info->nnz;
    int ok = fwrite(&h, sizeof h, 1, f) == 1 && fwrite(row, 4, z, f) == z &&
             fwrite(col, 4, z, f) == z && fwrite(val, 8, z, f) == z;
    ok &= fclose(f) == 0;
    return ok ? SPMV_SUCCESS : SPMV_FILE_ERROR;
}

static int bin_header(FILE *f, spmv_mtx_info *info)
{
    bin_header_t h;
    if (fread(&h, sizeof h, 1, f) != 1 || memcmp(h.magic, "SPMVBIN1", 8) != 0 || h.n_rows < 0 ||
        h.n_cols < 0 || h.nnz < 0)
        return SPMV_FILE_ERROR;
    memset(info, 0, sizeof *info);
    info->n_rows = h.n_rows;
    info->n_cols = h.n_cols;
    info->nnz = h.nnz;
    info->symmetric = (int)(h.flags & 1);
    info->pattern = (int)((h.flags >> 1) & 1);
    info->integer = (int)((h.flags >> 2) & 1);
    return SPMV_SUCCESS;
}

int spmv_bin_read_info(const char *path, spmv_mtx_info *info)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return SPMV_FILE_ERROR;
    int rc = bin_header(f, info);
    fclose(f);
    return rc;
}

int spmv_bin_read(const char *path, spmv_mtx_info *info, int32_t *row, int32_t *col,
                  double *val)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return SPMV_FILE_ERROR;
    int rc = bin_header(f, info);
    size_t z = (size_t)info->nnz;
    if (rc == SPMV_SUCCESS && (fread(row, 4, z, f) != z || fread(col, 4, z, f) != z ||
                               fread(val, 8, z, f) != z))
        rc = SPMV_FILE_ERROR;
    fclose(f);
    for (size_t i = 0; rc == SPMV_SUCCESS && i < z; ++i)
        if (row[i] < 0 || row[i] >= info->n_rows || col[i] < 0 || col[i] >= info->n_cols)
            rc = SPMV_FILE_ERROR;
    return rc;
}
