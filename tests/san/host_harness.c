/*
 * host_harness.c — drives libspmv_host's code (compiled into this binary
 * with -fsanitize=address,undefined by `make test-san`) over every input
 * the reference's host path had latent UB on (the ELL
 * builder's last-row K and uninitialised padding, reference ell.c:73-164;
 * the CMRS builder's tail strip and empty-row assumption, reference
 * cmrs.c:72-117; the CSR/SELL empty-row assumption, csr.c:68-91,
 * sigma_c.c:93-139) and over malformed Matrix Market files.
 *
 * usage: host_harness TMPDIR FILE.mtx...
 * Every format is built, run by the OpenMP CPU loop and checked against
 * the file-order sum (spmv_check, reference inc/helper_functions.h:184-236);
 * any mismatch, or any sanitizer report, fails the run.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "spmv_host.h"

static int g_fail = 0;

#define CHECK(cond, ...)                                                                 \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                         \
            fprintf(stderr, __VA_ARGS__);                                                \
            fputc('\n', stderr);                                                         \
            g_fail = 1;                                                                  \
        }                                                                                \
    } while (0)

static void *xmalloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p) {
        fprintf(stderr, "out of memory\n");
        exit(2);
    }
    return p;
}

static void check_y(const char *what, int64_t n_rows, int64_t nnz, const int32_t *row, const int32_t *col,
                    const double *val, const double *x, const double *y)
{
    int64_t first = -1;
    double ref = 0.0;
    const int64_t bad = spmv_check(n_rows, nnz, row, col, val, x, y, 0.0, 1e-12, &first, &ref);
    CHECK(bad == 0, "%s: %lld bad rows, first %lld (got %g want %g)", what, (long long)bad, (long long)first,
          first >= 0 ? y[first] : 0.0, ref);
}

/* every builder + CPU loop on one matrix (COO in any order) */
static void all_formats(const char *name, int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t *row,
                        const int32_t *col, const double *val)
{
    char what[256];
    double *x = xmalloc((size_t)n_cols * sizeof(double));
    double *y = xmalloc((size_t)n_rows * sizeof(double));
    for (int64_t j = 0; j < n_cols; ++j)
        x[j] = (double)j; /* reference csr.c:95-99 */

    /* COO sorted by row + CPU COO loop */
    int32_t *sr = xmalloc((size_t)nnz * 4), *sc = xmalloc((size_t)nnz * 4);
    double *sv = xmalloc((size_t)nnz * 8);
    CHECK(spmv_coo_sort_by_row(n_rows, nnz, row, col, val, sr, sc, sv) == SPMV_SUCCESS, "%s sort", name);
    CHECK(spmv_cpu_coo(n_rows, nnz, sr, sc, sv, x, y, 2) == SPMV_SUCCESS, "%s cpu coo", name);
    snprintf(what, sizeof what, "%s coo", name);
    check_y(what, n_rows, nnz, row, col, val, x, y);

    /* CSR */
    int64_t *ptr = xmalloc((size_t)(n_rows + 1) * 8);
    int32_t *cc = xmalloc((size_t)nnz * 4);
    double *cv = xmalloc((size_t)nnz * 8);
    CHECK(spmv_csr_from_coo(n_rows, nnz, row, col, val, ptr, cc, cv) == SPMV_SUCCESS, "%s csr", name);
    CHECK(spmv_cpu_csr(n_rows, ptr, cc, cv, x, y, 3) == SPMV_SUCCESS, "%s cpu csr", name);
    snprintf(what, sizeof what, "%s csr", name);
    check_y(what, n_rows, nnz, row, col, val, x, y);
    int64_t mn, mx;
    double mean;
    spmv_csr_row_stats(n_rows, ptr, &mn, &mx, &mean);
    (void)spmv_csr_pick_variant(n_rows, ptr);

    /* hot columns (explicit H) */
    if (nnz > 0) {
        int32_t *hot = xmalloc((size_t)(1 << 19) * 4), *ch = xmalloc((size_t)nnz * 4);
        const int64_t H = spmv_hot_columns(n_cols, nnz, cc, 7, hot, ch);
        CHECK(H >= 0 && H <= 7, "%s hot H=%lld", name, (long long)H);
        for (int64_t e = 0; e < nnz; ++e) {
            const int32_t c = ch[e] >= n_cols ? hot[ch[e] - n_cols] : ch[e];
            if (c != cc[e]) {
                CHECK(0, "%s hot renumbering at %lld", name, (long long)e);
                break;
            }
        }
        free(hot);
        free(ch);
    }

    /* ELL, ki 1 and 2 */
    for (int ki = 1; ki <= 2; ++ki) {
        int32_t K;
        int64_t ld;
        CHECK(spmv_ell_plan(n_rows, ptr, ki, &K, &ld) == SPMV_SUCCESS, "%s ell plan", name);
        const size_t n = (size_t)K * (size_t)ld;
        int32_t *ec = xmalloc(n * 4);
        double *ev = xmalloc(n * 8);
        CHECK(spmv_ell_fill(n_rows, ptr, cc, cv, K, ld, ki, ec, ev) == SPMV_SUCCESS, "%s ell fill", name);
        CHECK(spmv_cpu_ell(n_rows, K, ld, ki, ec, ev, x, y, 2) == SPMV_SUCCESS, "%s cpu ell", name);
        snprintf(what, sizeof what, "%s ell ki=%d", name, ki);
        check_y(what, n_rows, nnz, row, col, val, x, y);
        free(ec);
        free(ev);
    }

    /* SELL: the configs[2] shape, the reference's sigma = 1 / C = 32, wide C */
    const int32_t shapes[][3] = {{64, 1024, 1}, {64, 1024, 2}, {32, 1, 1}, {128, 256, 2}, {64, 64, 1}};
    for (size_t k = 0; k < sizeof shapes / sizeof shapes[0]; ++k) {
        const int32_t C = shapes[k][0], sigma = shapes[k][1], ki = shapes[k][2];
        int64_t ns, stored;
        CHECK(spmv_sell_plan(n_rows, ptr, C, sigma, ki, &ns, &stored) == SPMV_SUCCESS, "%s sell plan", name);
        int64_t *sp = xmalloc((size_t)(ns + 1) * 8);
        int32_t *perm = xmalloc((size_t)ns * C * 4), *scol = xmalloc((size_t)stored * 4);
        double *sval = xmalloc((size_t)stored * 8);
        CHECK(spmv_sell_fill(n_rows, ptr, cc, cv, C, sigma, ki, ns, sp, perm, scol, sval) == SPMV_SUCCESS,
              "%s sell fill", name);
        CHECK(spmv_cpu_sell(n_rows, C, ki, ns, sp, perm, scol, sval, x, y, 2) == SPMV_SUCCESS, "%s cpu sell",
              name);
        snprintf(what, sizeof what, "%s sell C=%d sigma=%d ki=%d", name, C, sigma, ki);
        check_y(what, n_rows, nnz, row, col, val, x, y);
        const int32_t T = spmv_sell_split_auto(ns, sp, C, ki);
        const int64_t nch = spmv_sell_split_plan(ns, sp, C, 2 * ki, NULL, NULL);
        CHECK(T >= 0 && nch >= 0, "%s split plan", name);
        int32_t *cs = xmalloc((size_t)(nch + 1) * 4), *ck = xmalloc((size_t)(nch + 1) * 4);
        CHECK(spmv_sell_split_plan(ns, sp, C, 2 * ki, cs, ck) == nch, "%s split fill", name);
        free(cs);
        free(ck);
        free(sp);
        free(perm);
        free(scol);
        free(sval);
    }

    /* CMRS: h 1, 8 (the reference), 64; N % h != 0 is the reference's tail overflow */
    const int32_t hs[] = {1, 3, 8, 64};
    for (size_t k = 0; k < sizeof hs / sizeof hs[0]; ++k) {
        const int32_t h = hs[k];
        const int64_t ns = (n_rows + h - 1) / h;
        int64_t *stp = xmalloc((size_t)(ns + 1) * 8);
        uint8_t *rin = xmalloc((size_t)nnz);
        CHECK(spmv_cmrs_build(n_rows, ptr, h, stp, rin) == SPMV_SUCCESS, "%s cmrs", name);
        (void)spmv_cmrs_pick_variant(ns, stp);
        CHECK(spmv_cpu_cmrs(n_rows, h, ns, stp, rin, cc, cv, x, y, 2) == SPMV_SUCCESS, "%s cpu cmrs", name);
        snprintf(what, sizeof what, "%s cmrs h=%d", name, h);
        check_y(what, n_rows, nnz, row, col, val, x, y);
        free(stp);
        free(rin);
    }

    /* HYB: the rule's K and a forced small K (long tail) */
    for (int32_t Kreq = 0; Kreq <= 2; Kreq += 2) {
        int32_t K;
        int64_t ld, tail;
        CHECK(spmv_hyb_plan(n_rows, ptr, 2, Kreq, &K, &ld, &tail) == SPMV_SUCCESS, "%s hyb plan", name);
        int32_t *ec = xmalloc((size_t)K * ld * 4), *tr = xmalloc((size_t)tail * 4), *tc = xmalloc((size_t)tail * 4);
        double *ev = xmalloc((size_t)K * ld * 8), *tv = xmalloc((size_t)tail * 8);
        CHECK(spmv_hyb_fill(n_rows, ptr, cc, cv, K, ld, 2, ec, ev, tr, tc, tv) == SPMV_SUCCESS, "%s hyb fill", name);
        /* ELL part + tail by the CPU loops: y = ell(x) + coo_tail(x) */
        double *y2 = xmalloc((size_t)n_rows * 8);
        CHECK(spmv_cpu_ell(n_rows, K, ld, 2, ec, ev, x, y, 1) == SPMV_SUCCESS, "%s hyb ell", name);
        CHECK(spmv_cpu_coo(n_rows, tail, tr, tc, tv, x, y2, 1) == SPMV_SUCCESS, "%s hyb tail", name);
        for (int64_t i = 0; i < n_rows; ++i)
            y[i] += y2[i];
        snprintf(what, sizeof what, "%s hyb K=%d", name, K);
        check_y(what, n_rows, nnz, row, col, val, x, y);
        free(y2);
        free(ec);
        free(tr);
        free(tc);
        free(ev);
        free(tv);
    }

    /* CSR16 */
    int64_t nb, ne;
    CHECK(spmv_csr16_plan(nnz, cc, &nb, &ne) == SPMV_SUCCESS, "%s csr16 plan", name);
    int32_t *bb = xmalloc((size_t)nb * 4), *esc = xmalloc((size_t)ne * 64 * 4);
    uint16_t *off = xmalloc((size_t)nnz * 2);
    CHECK(spmv_csr16_fill(nnz, cc, bb, off, esc) == SPMV_SUCCESS, "%s csr16 fill", name);
    for (int64_t p = 0; p < nnz; ++p) {
        const int32_t b = bb[p / 64];
        const int32_t c = b >= 0 ? b + off[p] : esc[(int64_t)(-1 - b) * 64 + p % 64];
        if (c != cc[p]) {
            CHECK(0, "%s csr16 decode at %lld", name, (long long)p);
            break;
        }
    }
    free(bb);
    free(esc);
    free(off);

    /* row partitions: plain, weighted, calibrated */
    for (int parts = 1; parts <= 8; parts *= 2) {
        int64_t *bd = xmalloc((size_t)(parts + 1) * 8), *bd2 = xmalloc((size_t)(parts + 1) * 8);
        double *ms = xmalloc((size_t)parts * 8);
        CHECK(spmv_partition_rows(n_rows, ptr, parts, 64, bd) == SPMV_SUCCESS, "%s partition", name);
        CHECK(bd[0] == 0 && bd[parts] == n_rows, "%s partition ends", name);
        for (int p = 0; p < parts; ++p) {
            CHECK(bd[p] <= bd[p + 1], "%s partition order", name);
            ms[p] = 1.0 + p;
        }
        CHECK(spmv_partition_rows_weighted(n_rows, ptr, parts, 64, 2.0, bd2) == SPMV_SUCCESS, "%s weighted", name);
        CHECK(spmv_partition_rows_calibrated(n_rows, ptr, parts, 64, 2.0, parts, bd, ms, bd2) == SPMV_SUCCESS,
              "%s calibrated", name);
        CHECK(bd2[0] == 0 && bd2[parts] == n_rows, "%s calibrated ends", name);
        free(bd);
        free(bd2);
        free(ms);
    }
    free(ptr);
    free(cc);
    free(cv);
    free(sr);
    free(sc);
    free(sv);
    free(x);
    free(y);
}

static void one_file(const char *tmp, const char *path)
{
    spmv_mtx_info info;
    if (spmv_mtx_read_info(path, &info) != SPMV_SUCCESS) {
        fprintf(stderr, "skip %s (not readable)\n", path);
        return;
    }
    int32_t *row = xmalloc((size_t)info.nnz * 4), *col = xmalloc((size_t)info.nnz * 4);
    double *val = xmalloc((size_t)info.nnz * 8);
    CHECK(spmv_mtx_read(path, &info, row, col, val) == SPMV_SUCCESS, "read %s", path);
    /* binary cache and text round trips */
    char bin[512], txt[512];
    snprintf(bin, sizeof bin, "%s/harness.bin", tmp);
    snprintf(txt, sizeof txt, "%s/harness.mtx", tmp);
    CHECK(spmv_bin_write(bin, &info, row, col, val) == SPMV_SUCCESS, "bin write %s", path);
    spmv_mtx_info bi;
    CHECK(spmv_bin_read_info(bin, &bi) == SPMV_SUCCESS && bi.nnz == info.nnz, "bin info %s", path);
    int32_t *r2 = xmalloc((size_t)info.nnz * 4), *c2 = xmalloc((size_t)info.nnz * 4);
    double *v2 = xmalloc((size_t)info.nnz * 8);
    CHECK(spmv_bin_read(bin, &bi, r2, c2, v2) == SPMV_SUCCESS, "bin read %s", path);
    CHECK(memcmp(r2, row, (size_t)info.nnz * 4) == 0 && memcmp(c2, col, (size_t)info.nnz * 4) == 0 &&
              memcmp(v2, val, (size_t)info.nnz * 8) == 0,
          "bin round trip %s", path);
    CHECK(spmv_mtx_write(txt, info.n_rows, info.n_cols, info.nnz, row, col, val, info.symmetric) == SPMV_SUCCESS,
          "mtx write %s", path);
    spmv_mtx_info ti;
    CHECK(spmv_mtx_read_info(txt, &ti) == SPMV_SUCCESS && ti.nnz == info.nnz, "mtx reread %s", path);
    CHECK(spmv_mtx_read(txt, &ti, r2, c2, v2) == SPMV_SUCCESS, "mtx reread entries %s", path);
    CHECK(memcmp(v2, val, (size_t)info.nnz * 8) == 0, "mtx %%.17g round trip %s", path);
    all_formats(path, info.n_rows, info.n_cols, info.nnz, row, col, val);
    free(row);
    free(col);
    free(val);
    free(r2);
    free(c2);
    free(v2);
}

/* malformed files: every one must be refused with SPMV_FILE_ERROR, no crash */
static void malformed(const char *tmp)
{
    static const char *cases[] = {
        "",
        "%%MatrixMarket matrix coordinate real general\n",
        "%%MatrixMarket matrix coordinate real general\n3 3\n",
        "%%MatrixMarket matrix coordinate real general\n3 3 2\n1 1 1.0\n",         /* short */
        "%%MatrixMarket matrix coordinate real general\n3 3 1\n4 1 1.0\n",         /* row out of range */
        "%%MatrixMarket matrix coordinate real general\n3 3 1\n1 0 1.0\n",         /* col 0 */
        "%%MatrixMarket matrix coordinate real general\n3 3 1\n-1 1 1.0\n",        /* negative */
        "%%MatrixMarket matrix coordinate complex general\n3 3 1\n1 1 1.0 0.0\n",  /* complex */
        "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",             /* dense */
        "%%MatrixMarket vector coordinate real general\n3 3 1\n1 1 1.0\n",         /* not a matrix */
        "%%NotMarket matrix coordinate real general\n3 3 1\n1 1 1.0\n",            /* banner */
        "%%MatrixMarket matrix coordinate real general\n-3 3 1\n1 1 1.0\n",        /* negative size */
        "%%MatrixMarket matrix coordinate real general\n3 3 1\n1 1 abc\n",         /* bad value */
        "%%MatrixMarket matrix coordinate real general\n3 3 1\n1 1",               /* truncated line */
        "%%MatrixMarket matrix coordinate real general\n99999999999 3 1\n1 1 1\n", /* > int32 rows */
    };
    char path[512];
    snprintf(path, sizeof path, "%s/bad.mtx", tmp);
    for (size_t k = 0; k < sizeof cases / sizeof cases[0]; ++k) {
        FILE *f = fopen(path, "w");
        if (!f) {
            CHECK(0, "cannot write %s", path);
            return;
        }
        fputs(cases[k], f);
        fclose(f);
        spmv_mtx_info info;
        int rc = spmv_mtx_read_info(path, &info);
        if (rc == SPMV_SUCCESS) {
            if (info.nnz < 0 || info.nnz > 16 || info.n_rows > (1 << 20)) {
                CHECK(0, "case %zu: absurd header accepted", k);
                continue;
            }
            int32_t row[16], col[16];
            double val[16];
            rc = spmv_mtx_read(path, &info, row, col, val);
        }
        CHECK(rc == SPMV_FILE_ERROR, "malformed case %zu accepted (rc %d)", k, rc);
    }
    spmv_mtx_info info;
    CHECK(spmv_mtx_read_info("/nonexistent/x.mtx", &info) == SPMV_FILE_ERROR, "missing file");
    CHECK(spmv_bin_read_info(path, &info) == SPMV_FILE_ERROR, "text file read as bin");
}

static void generators(void)
{
    for (int mode = 0; mode <= 2; ++mode) {
        int64_t n, nnz;
        CHECK(spmv_gen_cantlike(mode, 1, &n, &nnz, NULL, NULL, NULL) == SPMV_SUCCESS, "cantlike size");
        int32_t *r = xmalloc((size_t)nnz * 4), *c = xmalloc((size_t)nnz * 4);
        double *v = xmalloc((size_t)nnz * 8);
        CHECK(spmv_gen_cantlike(mode, 1, &n, &nnz, r, c, v) == SPMV_SUCCESS, "cantlike");
        if (mode == 0) {
            char name[64];
            snprintf(name, sizeof name, "cantlike mode %d", mode);
            all_formats(name, n, n, nnz, r, c, v);
        }
        free(r);
        free(c);
        free(v);
    }
    {   /* R-MAT: skewed rows, empty rows, duplicates */
        const int64_t n = 50000, nnz = 400000;
        int32_t *r = xmalloc(nnz * 4), *c = xmalloc(nnz * 4);
        double *v = xmalloc(nnz * 8);
        CHECK(spmv_gen_rmat(n, nnz, 16, 1, r, c, v) == SPMV_SUCCESS, "rmat");
        all_formats("rmat", n, n, nnz, r, c, v);
        free(r);
        free(c);
        free(v);
    }
    {   /* ragged rows 0..700, N % 64 != 0 */
        const int64_t n = 2011;
        int64_t nnz = 0;
        CHECK(spmv_gen_random(n, 3001, 0, 700, 5, &nnz, NULL, NULL, NULL) == SPMV_SUCCESS, "random size");
        int32_t *r = xmalloc((size_t)nnz * 4), *c = xmalloc((size_t)nnz * 4);
        double *v = xmalloc((size_t)nnz * 8);
        CHECK(spmv_gen_random(n, 3001, 0, 700, 5, &nnz, r, c, v) == SPMV_SUCCESS, "random");
        all_formats("random", n, 3001, nnz, r, c, v);
        free(r);
        free(c);
        free(v);
    }
    {   /* banded, a shard in the middle */
        const int64_t n = 100003, lo = 40000, hi = 60001;
        int64_t *p = xmalloc((size_t)(hi - lo + 1) * 8);
        int32_t *c = xmalloc((size_t)(hi - lo) * 16 * 4);
        double *v = xmalloc((size_t)(hi - lo) * 16 * 8);
        CHECK(spmv_gen_banded_csr(n, 2, lo, hi, p, c, v) == SPMV_SUCCESS, "banded");
        CHECK(p[hi - lo] == 16 * (hi - lo), "banded ptr");
        free(p);
        free(c);
        free(v);
    }
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s TMPDIR FILE.mtx...\n", argv[0]);
        return 2;
    }
    for (int i = 2; i < argc; ++i)
        one_file(argv[1], argv[i]);
    malformed(argv[1]);
    generators();
    if (g_fail) {
        fprintf(stderr, "host_harness: FAILED\n");
        return 1;
    }
    printf("host_harness: ok (%d files, malformed inputs, generators)\n", argc - 2);
    return 0;
}
