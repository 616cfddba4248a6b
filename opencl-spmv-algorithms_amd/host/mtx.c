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
 * pass instead of the reference's three to four fscanf passes.
 */
#include <ctype.h>
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
