/*
 * driver.c — the per-format SpMV programs (./bin/coo, csr, ell, sigma_c,
 * cmrs), drop-in replacements of the reference's drivers
 * (reference coo.c, csr.c, ell.c, sigma_c.c, cmrs.c: main()).
 *
 * With no arguments a program behaves like the reference one: it reads
 * databases/cant.mtx (coo, reference coo.c:43) or
 * databases/cant-sorted.mtx (the others, reference csr.c:43), uses
 * x[j] = j (reference csr.c:95-99), runs the kernel, prints the
 * reference's lines (reference inc/helper_functions.h:167-182, the COO
 * "GPU calculations" line coo.c:201, ELL's row statistics ell.c:104),
 * checks the device result against the file-order sum ("result is ok",
 * reference csr.c:229-236), then times the OpenMP CPU loop and checks it
 * ("cpu result is ok", reference csr.c:244-255; none for sigma_c, like
 * the reference).  Exit codes are the reference's (inc/enums.h).
 *
 * Differences, all deliberate:
 *   - the time is the median of --reps hipEvent-timed launches, each after
 *     a 512 MiB cache flush (cold HBM; --warm skips the flush), instead of
 *     one cold launch under a host wall clock (reference csr.c:198-206);
 *   - extra lines after the reference's: algorithmic bytes, effective GB/s,
 *     fraction of the 8 TB/s HBM3E roofline, stored bytes of the format;
 *   - the check uses the suite's 1e-6 relative criterion and also reports
 *     the reference's absolute 1e-6 rule;
 *   - --strict turns a failed check into exit code 4 (the reference always
 *     returns Success, reference csr.c:282).
 * Options: --matrix PATH  --gen cantlike[0|1|2]|rmat[:ROWS:NNZ]|random
 *          --copies B  --reps N  --warmup W  --warm  --device D
 *          --C C --sigma S --ki K --h H --lanes L  --threads T
 *          --cpu / --no-cpu  --strict  --write-mtx PATH  --cache  --no-xwin  --gpus N
 *          --relabel auto|yes|no  --write-y PATH  --help
 *   --cache keeps a binary copy of the parsed file at PATH.bin (SURVEY.md
 *   §8f row 1) and reads it instead of the text whenever it is at least as
 *   new as PATH; the entries, their order and the result are unchanged.
 *   The kernel path is the library's plan for the matrix (spmv_plan_<fmt>,
 *   include/spmv.h) — the same one the Python binding and bench.py run:
 *   x windows in LDS (CSR, ELL, SELL, CMRS; --no-xwin: global gathers), the
 *   SELL head copy, the single-pass COO, entry-balanced tiles for skewed
 *   rows; the "[plan]" line names the kernel.
 *   --relabel (default auto = when the CSR skew rule picks the tiled kernel,
 *   e.g. R-MAT): the columns renumbered by decreasing degree, ties by first
 *   row (spmv_column_relabel_ex) and every row's entries in new-column
 *   order (spmv_csr_sort_rows), x permuted to match once on the host — the
 *   layout bench.py measures configs[3] on; y keeps the original row order
 *   and is checked against the original file.
 *   --write-y PATH writes the device y (n_rows raw fp64, row order).
 *   Device buffers are released by spmv_release() / process exit.
 *   --gpus N (N >= 1) shards the rows over GPUs 0..N-1 from ONE process
 *   (run_multi below): contiguous row ranges (spmv_partition_rows, aligned
 *   to 1024 rows so SELL windows never straddle two GPUs), x replicated,
 *   every shard's kernel writing its rows of a full-length y on its GPU, and
 *   the y exchange as RCCL broadcasts of the real shard sizes
 *   (spmv_multi_allgatherv).  The reference builds its context over every
 *   GPU but runs on the first only (reference csr.c:30,107,115,279).
 */
#define _POSIX_C_SOURCE 200809L
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>

#include "driver.h"
#include "spmv.h"
#include "spmv_host.h"

#define HBM_PEAK_GBS 8000.0

static int cmp_double(const void *a, const void *b);

typedef struct {
    const char *matrix;
    const char *gen;
    const char *write_mtx;
    const char *write_y;
    int64_t copies;
    int reps, warmup, warm, device, C, sigma, ki, h, lanes, threads, cpu, strict, cache, xwin, gpus, index16, single_pass;
    int relabel; /* -1 auto, 0 no, 1 yes */
} opts_t;

static void usage(const char *prog)
{
    printf("usage: %s [--matrix PATH | --gen cantlike[0|1|2]|rmat[:ROWS:NNZ]|random]\n"
           "          [--copies B] [--reps N] [--warmup W] [--warm] [--device D]\n"
           "          [--C C] [--sigma S] [--ki 1|2] [--h H] [--lanes L]\n"
           "          [--threads T] [--cpu|--no-cpu] [--strict] [--write-mtx PATH] [--cache]\n"
           "          [--no-xwin] [--gpus N] [--index16 (sigma_c: SELL16)]\n"
           "          [--carry-pass (coo: the carry kernel even where rows allow one pass)]\n"
           "          [--relabel auto|yes|no] [--write-y PATH]\n",
           prog);
}

static int parse_opts(int argc, char **argv, spmv_format fmt, opts_t *o)
{
    memset(o, 0, sizeof *o);
    o->matrix = fmt == FMT_COO ? "databases/cant.mtx" : "databases/cant-sorted.mtx";
    o->copies = 1;
    o->reps = 50;
    o->warmup = 5;
    o->C = 64;
    o->sigma = 1024;
    o->ki = 0; /* 0: format default (ELL 2, SELL spmv_sell_auto_ki) */
    o->h = 8;
    o->cpu = fmt != FMT_SELL;
    o->xwin = 1;
    o->single_pass = 1;
    o->relabel = -1;
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
#define NEEDV()                                                               \
    do {                                                                      \
        if (!v) {                                                             \
            fprintf(stderr, "%s needs a value\n", a);                        \
            return SPMV_OTHER_ERROR;                                          \
        }                                                                     \
        ++i;                                                                  \
    } while (0)
        if (!strcmp(a, "--matrix")) { NEEDV(); o->matrix = v; }
        else if (!strcmp(a, "--gen")) { NEEDV(); o->gen = v; }
        else if (!strcmp(a, "--write-mtx")) { NEEDV(); o->write_mtx = v; }
        else if (!strcmp(a, "--write-y")) { NEEDV(); o->write_y = v; }
        else if (!strcmp(a, "--relabel")) {
            NEEDV();
            o->relabel = !strcmp(v, "yes") ? 1 : !strcmp(v, "no") ? 0 : !strcmp(v, "auto") ? -1 : -2;
            if (o->relabel == -2) {
                fprintf(stderr, "--relabel takes auto, yes or no\n");
                return SPMV_OTHER_ERROR;
            }
        }
        else if (!strcmp(a, "--copies")) { NEEDV(); o->copies = atoll(v); }
        else if (!strcmp(a, "--reps")) { NEEDV(); o->reps = atoi(v); }
        else if (!strcmp(a, "--warmup")) { NEEDV(); o->warmup = atoi(v); }
        else if (!strcmp(a, "--device")) { NEEDV(); o->device = atoi(v); }
        else if (!strcmp(a, "--C")) { NEEDV(); o->C = atoi(v); }
        else if (!strcmp(a, "--sigma")) { NEEDV(); o->sigma = atoi(v); }
        else if (!strcmp(a, "--ki")) { NEEDV(); o->ki = atoi(v); }
        else if (!strcmp(a, "--h")) { NEEDV(); o->h = atoi(v); }
        else if (!strcmp(a, "--lanes")) { NEEDV(); o->lanes = atoi(v); }
        else if (!strcmp(a, "--threads")) { NEEDV(); o->threads = atoi(v); }
        else if (!strcmp(a, "--gpus")) { NEEDV(); o->gpus = atoi(v); }
        else if (!strcmp(a, "--warm")) o->warm = 1;
        else if (!strcmp(a, "--cpu")) o->cpu = 1;
        else if (!strcmp(a, "--no-cpu")) o->cpu = 0;
        else if (!strcmp(a, "--strict")) o->strict = 1;
        else if (!strcmp(a, "--cache")) o->cache = 1;
        else if (!strcmp(a, "--no-xwin")) o->xwin = 0;
        else if (!strcmp(a, "--index16")) o->index16 = 1;
        else if (!strcmp(a, "--carry-pass")) o->single_pass = 0;
        else if (!strcmp(a, "--help") || !strcmp(a, "-h")) { usage(argv[0]); exit(0); }
        else {
            fprintf(stderr, "unknown option %s\n", a);
            usage(argv[0]);
            return SPMV_OTHER_ERROR;
        }
#undef NEEDV
    }
    if (o->reps < 1 || o->warmup < 0 || o->copies < 1 || (o->ki < 0 || o->ki > 2) ||
        o->h < 1 || o->h > 64 || o->C < 1 || o->C > 1024 || o->gpus < 0 || o->gpus > 64)
        return SPMV_OTHER_ERROR;
    if (o->index16 && (fmt != FMT_SELL || !o->xwin || o->gpus > 0)) {
        fprintf(stderr, "--index16 is SELL16: sigma_c, one GPU, with x windows\n");
        return SPMV_OTHER_ERROR;
    }
    return SPMV_SUCCESS;
}

/* ------------------------------------------------------------- input */

typedef struct {
    int64_t n_rows, n_cols, nnz;
    int32_t *row, *col;
    double *val;
    const char *label;
} coo_t;

/* PATH.bin when --cache is on and it is at least as new as PATH */
static int cache_fresh(const char *mtx, const char *bin)
{
    struct stat sm, sb;
    return stat(mtx, &sm) == 0 && stat(bin, &sb) == 0 && sb.st_mtime >= sm.st_mtime;
}

static int load_cached(const opts_t *o, const char *bin, coo_t *m)
{
    spmv_mtx_info info;
    if (spmv_bin_read_info(bin, &info) != SPMV_SUCCESS)
        return SPMV_FILE_ERROR;
    m->n_rows = info.n_rows;
    m->n_cols = info.n_cols;
    m->nnz = info.nnz;
    m->row = malloc((size_t)(m->nnz + 1) * sizeof(int32_t));
    m->col = malloc((size_t)(m->nnz + 1) * sizeof(int32_t));
    m->val = malloc((size_t)(m->nnz + 1) * sizeof(double));
    if (!m->row || !m->col || !m->val)
        return SPMV_OTHER_ERROR;
    if (spmv_bin_read(bin, &info, m->row, m->col, m->val) != SPMV_SUCCESS)
        return SPMV_FILE_ERROR;
    m->label = o->matrix;
    return SPMV_SUCCESS;
}

static int load_input(const opts_t *o, spmv_format fmt, coo_t *m)
{
    memset(m, 0, sizeof *m);
    char bin[4096] = "";
    if (!o->gen && o->cache) {
        snprintf(bin, sizeof bin, "%s.bin", o->matrix);
        if (cache_fresh(o->matrix, bin)) {
            if (load_cached(o, bin, m) == SPMV_SUCCESS) {
                printf("  [cache] read %s\n", bin);
                return SPMV_SUCCESS;
            }
            free(m->row);
            free(m->col);
            free(m->val);
            memset(m, 0, sizeof *m);
        }
    }
    if (!o->gen) {
        spmv_mtx_info info;
        int rc = spmv_mtx_read_info(o->matrix, &info);
        if (rc != SPMV_SUCCESS) {
            if (errno)
                perror(o->matrix); /* reference csr.c:56 */
            else
                printf("Could not process Matrix Market file %s.\n", o->matrix);
            return SPMV_FILE_ERROR;
        }
        m->n_rows = info.n_rows;
        m->n_cols = info.n_cols;
        m->nnz = info.nnz;
        m->row = malloc((size_t)(m->nnz + 1) * sizeof(int32_t));
        m->col = malloc((size_t)(m->nnz + 1) * sizeof(int32_t));
        m->val = malloc((size_t)(m->nnz + 1) * sizeof(double));
        if (!m->row || !m->col || !m->val)
            return SPMV_OTHER_ERROR;
        if (spmv_mtx_read(o->matrix, &info, m->row, m->col, m->val) != SPMV_SUCCESS) {
            printf("Could not read the entries of %s.\n", o->matrix);
            return SPMV_FILE_ERROR;
        }
        m->label = o->matrix;
        if (bin[0]) {
            if (spmv_bin_write(bin, &info, m->row, m->col, m->val) == SPMV_SUCCESS)
                printf("  [cache] wrote %s\n", bin);
            else
                printf("  [cache] could not write %s (continuing)\n", bin);
        }
        return SPMV_SUCCESS;
    }
    int rc = SPMV_OTHER_ERROR;
    if (!strncmp(o->gen, "cantlike", 8)) {
        /* coo reads the column-major file, the others the row-sorted one */
        int mode = o->gen[8] ? atoi(o->gen + 8) : (fmt == FMT_COO ? 1 : 0);
        rc = spmv_gen_cantlike(mode, o->copies, &m->n_rows, &m->nnz, NULL, NULL, NULL);
        if (rc)
            return rc;
        m->row = malloc((size_t)m->nnz * sizeof(int32_t));
        m->col = malloc((size_t)m->nnz * sizeof(int32_t));
        m->val = malloc((size_t)m->nnz * sizeof(double));
        rc = spmv_gen_cantlike(mode, o->copies, &m->n_rows, &m->nnz, m->row, m->col, m->val);
        m->n_cols = m->n_rows;
        m->label = "cant-like stand-in (synthetic; real cant.mtx is an LFS pointer)";
    } else if (!strncmp(o->gen, "rmat", 4) && (o->gen[4] == 0 || o->gen[4] == ':')) {
        /* rmat = configs[3] (1e7 rows, 1e8 entries); rmat:ROWS:NNZ a smaller one */
        m->n_rows = m->n_cols = 10000000;
        m->nnz = 100000000;
        if (o->gen[4] == ':') {
            long long r = 0, z = 0;
            if (sscanf(o->gen + 5, "%lld:%lld", &r, &z) != 2 || r < 2 || r > INT32_MAX || z < 0) {
                fprintf(stderr, "--gen rmat:ROWS:NNZ\n");
                return SPMV_OTHER_ERROR;
            }
            m->n_rows = m->n_cols = r;
            m->nnz = z;
        }
        int scale = 1;
        while (((int64_t)1 << scale) < m->n_rows)
            ++scale;
        m->row = malloc((size_t)(m->nnz + 1) * sizeof(int32_t));
        m->col = malloc((size_t)(m->nnz + 1) * sizeof(int32_t));
        m->val = malloc((size_t)(m->nnz + 1) * sizeof(double));
        rc = spmv_gen_rmat(m->n_rows, m->nnz, scale, 1, m->row, m->col, m->val);
        m->label = "R-MAT (a,b,c,d) = (.57,.19,.19,.05), seed 1 (synthetic)";
    } else if (!strcmp(o->gen, "random")) {
        m->n_rows = m->n_cols = 100000;
        rc = spmv_gen_random(m->n_rows, m->n_cols, 0, 64, 3, &m->nnz, NULL, NULL, NULL);
        m->row = malloc((size_t)m->nnz * sizeof(int32_t));
        m->col = malloc((size_t)m->nnz * sizeof(int32_t));
        m->val = malloc((size_t)m->nnz * sizeof(double));
        rc = spmv_gen_random(m->n_rows, m->n_cols, 0, 64, 3, &m->nnz, m->row, m->col, m->val);
        m->label = "random ragged 1e5 x 1e5 (synthetic)";
    } else {
        fprintf(stderr, "unknown generator %s\n", o->gen);
    }
    return rc;
}

/* ----------------------------------------------------- device format */

typedef struct {
    spmv_format fmt;
    spmv_dims d;
    /* device arrays (unused ones stay NULL); the plan points at them */
    int64_t *d_ptr;   /* CSR row_ptr / SELL slice_ptr / CMRS strip_ptr */
    int32_t *d_row, *d_col, *d_perm;
    uint8_t *d_rin;
    double *d_val, *d_x, *d_y;
    spmv_plan *plan; /* the library's kernel path for this matrix (spmv.h) */
    int32_t K, C, sigma, ki, h;
    int64_t ld, n_slices, n_strips;
    /* host copies for the CPU loop */
    int64_t *h_ptr;
    int32_t *h_row, *h_col, *h_perm;
    uint8_t *h_rin;
    double *h_val;
    int64_t stored; /* stored entries (incl. padding) */
    size_t stored_bytes;
} dev_fmt_t;

static int upload(void **dst, const void *src, size_t bytes, void *stream)
{
    int rc = spmv_malloc(dst, bytes);
    if (rc == SPMV_SUCCESS)
        rc = spmv_upload(*dst, src, bytes, stream);
    return rc;
}

/* The plan: every kernel choice (x windows, head copy, single pass, tiles,
 * split, hot-column table, SELL16) is the library's (spmv_plan_<fmt>), so
 * this program runs what bench.py and spmv_amd.to_device run. */
static int make_plan(const opts_t *o, dev_fmt_t *f, int relabelled)
{
    spmv_plan_opts po;
    spmv_plan_opts_init(&po);
    po.lanes = o->lanes;
    po.xwin = o->xwin ? -1 : 0;
    po.index16 = o->index16;
    po.coo_pass = o->single_pass ? -1 : 0;
    if (relabelled)
        po.H = 0; /* hot columns are x'[0..H) already: no per-run table */
    switch (f->fmt) {
    case FMT_COO:
        return spmv_plan_coo(f->d, f->d_row, f->d_col, f->d_val, &po, &f->plan);
    case FMT_CSR:
        return spmv_plan_csr(f->d, f->d_ptr, f->d_col, f->d_val, &po, &f->plan);
    case FMT_ELL:
        return spmv_plan_ell(f->d, f->K, f->ld, f->ki, f->d_col, f->d_val, &po, &f->plan);
    case FMT_SELL:
        return spmv_plan_sell(f->d, f->C, f->sigma, f->ki, f->n_slices, f->d_ptr, f->d_perm, f->d_col, f->d_val, &po,
                              &f->plan);
    case FMT_CMRS:
        return spmv_plan_cmrs(f->d, f->h, f->n_strips, f->d_ptr, f->d_rin, f->d_col, f->d_val, &po, &f->plan);
    }
    return SPMV_OTHER_ERROR;
}

static int build_format(const opts_t *o, spmv_format fmt, const coo_t *m, dev_fmt_t *f, int relabelled)
{
    memset(f, 0, sizeof *f);
    f->fmt = fmt;
    f->d.n_rows = m->n_rows;
    f->d.n_cols = m->n_cols;
    f->d.nnz = m->nnz;
    f->d.device = o->device;
    f->d.stream = NULL;
    const int64_t N = m->n_rows, Z = m->nnz;
    int rc;
    if (fmt == FMT_COO) {
        f->h_row = malloc((size_t)(Z + 1) * sizeof(int32_t));
        f->h_col = malloc((size_t)(Z + 1) * sizeof(int32_t));
        f->h_val = malloc((size_t)(Z + 1) * sizeof(double));
        rc = spmv_coo_sort_by_row(N, Z, m->row, m->col, m->val, f->h_row, f->h_col, f->h_val);
        if (rc)
            return rc;
        f->stored = Z;
        f->stored_bytes = (size_t)Z * 16;
        if ((rc = upload((void **)&f->d_row, f->h_row, (size_t)Z * 4, NULL)) ||
            (rc = upload((void **)&f->d_col, f->h_col, (size_t)Z * 4, NULL)) ||
            (rc = upload((void **)&f->d_val, f->h_val, (size_t)Z * 8, NULL)))
            return rc;
        return make_plan(o, f, relabelled);
    }
    /* every other format starts from CSR */
    int64_t *ptr = malloc((size_t)(N + 1) * sizeof(int64_t));
    int32_t *col = malloc((size_t)(Z + 1) * sizeof(int32_t));
    double *val = malloc((size_t)(Z + 1) * sizeof(double));
    if (!ptr || !col || !val)
        return SPMV_OTHER_ERROR;
    if ((rc = spmv_csr_from_coo(N, Z, m->row, m->col, m->val, ptr, col, val)))
        return rc;
    if (fmt == FMT_CSR || fmt == FMT_CMRS) {
        f->h_ptr = ptr;
        f->h_col = col;
        f->h_val = val;
        f->stored = Z;
        if (fmt == FMT_CSR) {
            f->stored_bytes = (size_t)Z * 12 + (size_t)(N + 1) * 8;
            rc = upload((void **)&f->d_ptr, ptr, (size_t)(N + 1) * 8, NULL);
        } else {
            f->h = o->h;
            f->n_strips = (N + o->h - 1) / o->h;
            int64_t *sp = malloc((size_t)(f->n_strips + 1) * sizeof(int64_t));
            f->h_rin = malloc((size_t)(Z + 1));
            if (!sp || !f->h_rin || (rc = spmv_cmrs_build(N, ptr, o->h, sp, f->h_rin)))
                return rc ? rc : SPMV_OTHER_ERROR;
            free(f->h_ptr);
            f->h_ptr = sp;
            f->stored_bytes = (size_t)Z * 13 + (size_t)(f->n_strips + 1) * 8;
            if ((rc = upload((void **)&f->d_ptr, sp, (size_t)(f->n_strips + 1) * 8, NULL)) == SPMV_SUCCESS)
                rc = upload((void **)&f->d_rin, f->h_rin, (size_t)Z, NULL);
        }
        if (rc || (rc = upload((void **)&f->d_col, col, (size_t)Z * 4, NULL)) ||
            (rc = upload((void **)&f->d_val, val, (size_t)Z * 8, NULL)))
            return rc;
        return make_plan(o, f, relabelled);
    }
    if (fmt == FMT_ELL) {
        int64_t mn, mx;
        double mean;
        spmv_csr_row_stats(N, ptr, &mn, &mx, &mean);
        /* reference ell.c:104 */
        printf("average column length %lf, shortest col %lld, longest col %lld\n", mean,
               (long long)mn, (long long)mx);
        f->ki = o->ki ? o->ki : 2;
        if ((rc = spmv_ell_plan(N, ptr, f->ki, &f->K, &f->ld)))
            return rc;
        f->stored = f->ld * f->K;
        if (Z > 0 && (double)f->stored / (double)Z > 64.0) {
            printf("ELL not applicable: padding factor %.1f (stored %lld / %lld entries)\n",
                   (double)f->stored / (double)Z, (long long)f->stored, (long long)Z);
            return SPMV_OTHER_ERROR;
        }
        f->h_col = malloc((size_t)(f->stored + 1) * sizeof(int32_t));
        f->h_val = malloc((size_t)(f->stored + 1) * sizeof(double));
        if ((rc = spmv_ell_fill(N, ptr, col, val, f->K, f->ld, f->ki, f->h_col, f->h_val)))
            return rc;
        f->stored_bytes = (size_t)f->stored * 12;
    } else { /* SELL */
        f->C = o->C;
        f->sigma = o->sigma;
        f->ki = o->ki ? o->ki : spmv_sell_auto_ki(N, o->C);
        if ((rc = spmv_sell_plan(N, ptr, o->C, o->sigma, f->ki, &f->n_slices, &f->stored)))
            return rc;
        f->h_ptr = malloc((size_t)(f->n_slices + 1) * sizeof(int64_t));
        f->h_perm = malloc((size_t)(f->n_slices * o->C + 1) * sizeof(int32_t));
        f->h_col = malloc((size_t)(f->stored + 1) * sizeof(int32_t));
        f->h_val = malloc((size_t)(f->stored + 1) * sizeof(double));
        if ((rc = spmv_sell_fill(N, ptr, col, val, o->C, o->sigma, f->ki, f->n_slices, f->h_ptr,
                                 f->h_perm, f->h_col, f->h_val)))
            return rc;
        f->stored_bytes = (size_t)f->stored * (o->index16 ? 10 : 12) + (size_t)(f->n_slices + 1) * 8 +
                          (size_t)f->n_slices * o->C * 4;
        if ((rc = upload((void **)&f->d_ptr, f->h_ptr, (size_t)(f->n_slices + 1) * 8, NULL)) ||
            (rc = upload((void **)&f->d_perm, f->h_perm, (size_t)f->n_slices * o->C * 4, NULL)))
            return rc;
    }
    free(ptr);
    free(col);
    free(val);
    if ((rc = upload((void **)&f->d_col, f->h_col, (size_t)f->stored * 4, NULL)) ||
        (rc = upload((void **)&f->d_val, f->h_val, (size_t)f->stored * 8, NULL)))
        return rc;
    return make_plan(o, f, relabelled);
}

static int launch(void *arg)
{
    const dev_fmt_t *f = (const dev_fmt_t *)arg;
    return spmv_plan_run(f->plan, f->d_x, f->d_y, f->d.stream);
}

/* the "[plan]" line: the kernel the library chose and its parameters */
static void print_plan(const dev_fmt_t *f, const char *who)
{
    spmv_plan_info info;
    if (f->plan && spmv_plan_get_info(f->plan, &info) == SPMV_SUCCESS)
        printf("  [plan]%s kernel %s: %s\n", who, info.kernel, info.desc);
}

/* The degree-ordered layout (--relabel; bench.py rmat_layout): the matrix
 * in CSR order with columns renumbered by decreasing degree, ties by first
 * appearance (spmv_column_relabel_ex), every row's entries by new column
 * (spmv_csr_sort_rows), and x' = x[order]: the relabelled matrix on x'
 * gives the original y, row for row (summation order aside). */
static int relabel_layout(const coo_t *m, const double *x, coo_t *r, double **xr)
{
    const int64_t N = m->n_rows, M = m->n_cols, Z = m->nnz;
    int64_t *ptr = malloc((size_t)(N + 1) * sizeof(int64_t));
    int32_t *col = malloc((size_t)(Z + 1) * sizeof(int32_t));
    double *val = malloc((size_t)(Z + 1) * sizeof(double));
    int32_t *order = malloc((size_t)(M + 1) * sizeof(int32_t));
    int32_t *newid = malloc((size_t)(M + 1) * sizeof(int32_t));
    int32_t *row = malloc((size_t)(Z + 1) * sizeof(int32_t));
    *xr = malloc((size_t)(M + 1) * sizeof(double));
    if (!ptr || !col || !val || !order || !newid || !row || !*xr)
        return SPMV_OTHER_ERROR;
    int rc = spmv_csr_from_coo(N, Z, m->row, m->col, m->val, ptr, col, val);
    if (rc == SPMV_SUCCESS && spmv_column_relabel_ex(M, Z, col, order, newid, col, 1) < 0)
        rc = SPMV_OTHER_ERROR;
    if (rc == SPMV_SUCCESS)
        rc = spmv_csr_sort_rows(N, ptr, col, val);
    if (rc != SPMV_SUCCESS)
        return rc;
    for (int64_t i = 0; i < N; ++i)
        for (int64_t e = ptr[i]; e < ptr[i + 1]; ++e)
            row[e] = (int32_t)i;
    for (int64_t k = 0; k < M; ++k)
        (*xr)[k] = x[order[k]];
    *r = *m;
    r->row = row;
    r->col = col;
    r->val = val;
    free(ptr);
    free(order);
    free(newid);
    return SPMV_SUCCESS;
}

/* The SpMV's time over `reps` launches.  cold: (span of reps x (512 MiB
 * read flush + SpMV) - span of reps flushes) / reps, events on the stream,
 * the launches queued back to back (the ~80 us flush hides the host);
 * warm: span of reps back-to-back SpMVs / reps.  *ev_median: the median of
 * per-launch event pairs (the rounds 1-5 figure, launch gaps included). */
static int time_spmv(dev_fmt_t *f, int reps, int cold, double *ms, double *ev_median)
{
    void *st = f->d.stream;
    int rc = spmv_flush_cache_read(st, 0); /* allocates the scratch outside the timed spans */
    double both = 0.0, flush = 0.0;
    if (rc == SPMV_SUCCESS)
        rc = spmv_sync(st);
    void *ev[2] = {NULL, NULL};
    if (rc == SPMV_SUCCESS)
        rc = spmv_event_create(&ev[0]);
    if (rc == SPMV_SUCCESS)
        rc = spmv_event_create(&ev[1]);
    for (int pass = 0; pass < 2 && rc == SPMV_SUCCESS; ++pass) {
        if (!cold && pass == 1)
            break;
        rc = spmv_event_record(ev[0], st);
        for (int i = 0; i < reps && rc == SPMV_SUCCESS; ++i) {
            if (cold)
                rc = spmv_flush_cache_read(st, 0);
            if (rc == SPMV_SUCCESS && pass == 0)
                rc = launch(f);
        }
        if (rc == SPMV_SUCCESS)
            rc = spmv_event_record(ev[1], st);
        if (rc == SPMV_SUCCESS)
            rc = spmv_event_elapsed(ev[0], ev[1], pass == 0 ? &both : &flush);
    }
    spmv_event_destroy(ev[0]);
    spmv_event_destroy(ev[1]);
    if (rc != SPMV_SUCCESS)
        return rc;
    *ms = (both - flush) / reps;
    /* per-launch event pairs beside it */
    double *t = malloc((size_t)reps * sizeof(double));
    if (!t)
        return SPMV_OTHER_ERROR;
    for (int i = 0; i < reps && rc == SPMV_SUCCESS; ++i) {
        if (cold)
            rc = spmv_flush_cache_read(st, 0);
        if (rc == SPMV_SUCCESS)
            rc = spmv_time_launch(launch, f, st, &t[i]);
    }
    if (rc == SPMV_SUCCESS) {
        qsort(t, (size_t)reps, sizeof(double), cmp_double);
        *ev_median = t[reps / 2];
    }
    free(t);
    return rc;
}

static int run_cpu(const dev_fmt_t *f, const double *x, double *y, int threads)
{
    const int64_t N = f->d.n_rows;
    switch (f->fmt) {
    case FMT_COO:
        return spmv_cpu_coo(N, f->d.nnz, f->h_row, f->h_col, f->h_val, x, y, threads);
    case FMT_CSR:
        return spmv_cpu_csr(N, f->h_ptr, f->h_col, f->h_val, x, y, threads);
    case FMT_ELL:
        return spmv_cpu_ell(N, f->K, f->ld, f->ki, f->h_col, f->h_val, x, y, threads);
    case FMT_SELL:
        return spmv_cpu_sell(N, f->C, f->ki, f->n_slices, f->h_ptr, f->h_perm, f->h_col,
                             f->h_val, x, y, threads);
    case FMT_CMRS:
        return spmv_cpu_cmrs(N, f->h, f->n_strips, f->h_ptr, f->h_rin, f->h_col, f->h_val, x,
                             y, threads);
    }
    return SPMV_OTHER_ERROR;
}

/* ------------------------------------------------------------ output */

/* reference inc/helper_functions.h:167-173 (2*nnz widened past int32) */
static void print_performance(double ms, int64_t nnz)
{
    printf("Your calculations took %.2lf ms to run.\n", ms);
    printf("Number of operations %lld, PERFORMANCE %lf GFlops\n", (long long)(2 * nnz),
           (2.0 * (double)nnz) / ms * 1e-6);
}

/* reference inc/helper_functions.h:175-182 */
static void print_speed(double ms, int64_t nnz)
{
    printf("GBytes transferred to processor %lf - %lf, speed %lf - %lf GB/s\n",
           (double)nnz * 8 * 1e-9, (double)(2 * nnz) * 8 * 1e-9, (double)nnz * 8 / ms * 1e-6,
           (double)(2 * nnz) * 8 / ms * 1e-6);
}

static int check_and_report(const coo_t *m, const double *x, const double *y, const char *who)
{
    int64_t first_bad = -1;
    double ref_at_bad = 0.0;
    int64_t bad_rel = spmv_check(m->n_rows, m->nnz, m->row, m->col, m->val, x, y, 0.0, 1e-6,
                                 &first_bad, &ref_at_bad);
    int64_t first_abs = -1;
    int64_t bad_abs = spmv_check(m->n_rows, m->nnz, m->row, m->col, m->val, x, y, 1e-6, 0.0,
                                 &first_abs, NULL);
    if (bad_rel != 0 && first_bad >= 0) /* reference helper_functions.h:225 */
        printf("wrong value at index %lld: expected %f - calculated %f\n", (long long)first_bad,
               ref_at_bad, y[first_bad]);
    printf("%sresult is %s\n", who, bad_rel == 0 ? "ok" : "wrong");
    printf("  [check] rel-1e-6: %lld bad rows; reference abs-1e-6 rule: %s (%lld rows)\n",
           (long long)bad_rel, bad_abs == 0 ? "pass" : "fail", (long long)bad_abs);
    return bad_rel == 0;
}

static int cmp_double(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : (x > y);
}

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static const char *fmt_name(spmv_format f)
{
    static const char *n[] = {"coo", "csr", "ell", "sigma_c", "cmrs"};
    return n[f];
}

/* ------------------------------------------------------------ --gpus N */

typedef struct {
    dev_fmt_t *f;
} multi_arg_t;

static int launch_shard(void *arg, int i)
{
    return launch(&((multi_arg_t *)arg)->f[i]);
}

static double median_of(double *v, int n)
{
    qsort(v, (size_t)n, sizeof(double), cmp_double);
    return v[n / 2];
}

static int run_multi(const opts_t *o, spmv_format fmt, const coo_t *m, const double *x, double *y, double *y_cpu,
                     const coo_t *mr, const double *xr)
{
    /* mr / xr: the relabelled matrix and x' the shards run on (= m / x
     * without --relabel); m / x: the original, for the check */
    const int G = o->gpus;
    const int64_t N = m->n_rows, Z = m->nnz;
    int rc;
    /* contiguous row ranges with ~Z/G entries each, 1024-aligned */
    int64_t *ptr = malloc((size_t)(N + 1) * sizeof(int64_t));
    int32_t *tc = malloc((size_t)(Z + 1) * sizeof(int32_t));
    double *tv = malloc((size_t)(Z + 1) * sizeof(double));
    int64_t *bounds = malloc((size_t)(G + 1) * sizeof(int64_t));
    dev_fmt_t *f = calloc((size_t)G, sizeof(dev_fmt_t));
    double **y_full = calloc((size_t)G, sizeof(double *));
    double *ms = malloc((size_t)G * sizeof(double));
    double *t = malloc((size_t)o->reps * sizeof(double)), *tag = malloc((size_t)o->reps * sizeof(double));
    double *tall = malloc((size_t)o->reps * sizeof(double)), *tdev = malloc((size_t)o->reps * G * sizeof(double));
    if (!ptr || !tc || !tv || !bounds || !f || !y_full || !ms || !t || !tag || !tall || !tdev)
        return SPMV_OTHER_ERROR;
    if ((rc = spmv_csr_from_coo(N, Z, mr->row, mr->col, mr->val, ptr, tc, tv)) ||
        (rc = spmv_partition_rows(N, ptr, G, 1024, bounds)))
        return rc;
    free(tc);
    free(tv);
    spmv_multi *mg = NULL;
    if ((rc = spmv_multi_init(G, NULL, &mg)) != SPMV_SUCCESS) {
        printf("RCCL init over %d GPUs failed: %s\n", G, spmv_last_error());
        return rc;
    }
    for (int g = 0; g < G; ++g) {
        const int64_t lo = bounds[g], hi = bounds[g + 1];
        coo_t s = {hi - lo, m->n_cols, 0, NULL, NULL, NULL, m->label};
        s.nnz = spmv_coo_row_shard(Z, mr->row, mr->col, mr->val, lo, hi, NULL, NULL, NULL);
        s.row = malloc((size_t)(s.nnz + 1) * sizeof(int32_t));
        s.col = malloc((size_t)(s.nnz + 1) * sizeof(int32_t));
        s.val = malloc((size_t)(s.nnz + 1) * sizeof(double));
        if (s.nnz < 0 || !s.row || !s.col || !s.val)
            return SPMV_OTHER_ERROR;
        spmv_coo_row_shard(Z, mr->row, mr->col, mr->val, lo, hi, s.row, s.col, s.val);
        opts_t og = *o;
        og.device = spmv_multi_device(mg, g);
        if ((rc = spmv_set_device(og.device)) != SPMV_SUCCESS)
            return rc;
        rc = build_format(&og, fmt, &s, &f[g], mr != m);
        f[g].d.stream = spmv_multi_stream(mg, g);
        if (rc != SPMV_SUCCESS) {
            printf("shard %d: format build/upload failed: %s %s\n", g, spmv_strerror(rc), spmv_last_error());
            return rc == SPMV_OTHER_ERROR ? SPMV_OTHER_ERROR : SPMV_PROGRAM_ERROR;
        }
        /* x replicated; this shard's kernel writes rows [lo, hi) of y_full */
        if ((rc = upload((void **)&f[g].d_x, xr, (size_t)m->n_cols * 8, NULL)) ||
            (rc = spmv_malloc((void **)&y_full[g], (size_t)(N + 1) * 8)) ||
            /* NaN: every row must arrive; queued on the shard's own stream
             * (non-blocking, not ordered with the null stream) so the fill
             * lands before the warm-up kernel writes its rows */
            (rc = spmv_memset(y_full[g], 0xFF, (size_t)(N + 1) * 8, f[g].d.stream)))
            return SPMV_PROGRAM_ERROR;
        f[g].d_y = y_full[g] + lo;
        free(s.row);
        free(s.col);
        free(s.val);
    }
    multi_arg_t arg = {f};
    for (int i = 0; i < o->warmup; ++i)
        for (int g = 0; g < G; ++g) {
            spmv_set_device(spmv_multi_device(mg, g));
            if ((rc = launch(&f[g])) != SPMV_SUCCESS) {
                printf("kernel launch error: %s\n", spmv_last_error());
                return SPMV_PROGRAM_ERROR;
            }
        }
    if ((rc = spmv_multi_sync(mg)))
        return SPMV_PROGRAM_ERROR;
    /* SpMV alone: every GPU's shard launched together (cold unless --warm),
     * the step's time is the slowest GPU's */
    for (int i = 0; i < o->reps; ++i) {
        if ((rc = spmv_multi_time(mg, launch_shard, &arg, !o->warm, ms)) != SPMV_SUCCESS) {
            printf("kernel launch error: %s\n", spmv_last_error());
            return SPMV_PROGRAM_ERROR;
        }
        t[i] = 0.0;
        for (int g = 0; g < G; ++g) {
            tdev[(size_t)g * o->reps + i] = ms[g];
            t[i] = ms[g] > t[i] ? ms[g] : t[i];
        }
    }
    const double spmv_ms = median_of(t, o->reps); /* sorts t */
    const double t_min = t[0];
    /* the y exchange alone, and SpMV + exchange (host wall, all GPUs synchronised) */
    for (int i = 0; i < o->reps; ++i) {
        double t0 = now_s();
        if ((rc = spmv_multi_allgatherv(mg, y_full, bounds)) || (rc = spmv_multi_sync(mg))) {
            printf("RCCL all-gather failed: %s\n", spmv_last_error());
            return SPMV_PROGRAM_ERROR;
        }
        tag[i] = (now_s() - t0) * 1e3;
        t0 = now_s();
        for (int g = 0; g < G && rc == SPMV_SUCCESS; ++g) {
            spmv_set_device(spmv_multi_device(mg, g));
            rc = launch(&f[g]);
        }
        if (rc || (rc = spmv_multi_allgatherv(mg, y_full, bounds)) || (rc = spmv_multi_sync(mg))) {
            printf("SpMV + all-gather failed: %s\n", spmv_last_error());
            return SPMV_PROGRAM_ERROR;
        }
        tall[i] = (now_s() - t0) * 1e3;
    }
    const double ag_ms = median_of(tag, o->reps), all_ms = median_of(tall, o->reps);

    if (fmt == FMT_COO)
        printf("GPU calculations\n"); /* reference coo.c:201 */
    print_performance(spmv_ms, Z);
    print_speed(spmv_ms, Z);
    const double bytes_alg = 12.0 * (double)Z + 4.0 * (double)(N + 1) + 8.0 * (double)m->n_cols + 8.0 * (double)N;
    printf("  [%s] %s | N=%lld M=%lld Z=%lld | %d GPUs, median of %d %s reps of the slowest GPU (min %.4f ms)\n",
           fmt_name(fmt), m->label, (long long)N, (long long)m->n_cols, (long long)Z, G, o->reps,
           o->warm ? "warm (cache-resident)" : "cold (512 MiB flush on every GPU)", t_min);
    printf("  [%s] aggregate effective %.1f GB/s (bytes_alg %.1f MB) = %.1f%% of %d x %.0f GB/s HBM3E\n",
           fmt_name(fmt), bytes_alg / spmv_ms * 1e-6, bytes_alg * 1e-6,
           100.0 * bytes_alg / spmv_ms * 1e-6 / (HBM_PEAK_GBS * G), G, HBM_PEAK_GBS);
    for (int g = 0; g < G; ++g)
        printf("  [multi] GPU %d: rows [%lld, %lld) %lld entries, median %.4f ms\n", spmv_multi_device(mg, g),
               (long long)bounds[g], (long long)bounds[g + 1], (long long)f[g].d.nnz,
               median_of(tdev + (size_t)g * o->reps, o->reps));
    print_plan(&f[0], " GPU 0");
    printf("  [multi] y all-gather over RCCL (%d broadcasts of the real shard rows, %.1f MB per GPU received): "
           "%.4f ms; SpMV + all-gather %.4f ms = %.1f GB/s aggregate\n",
           G, 8e-6 * (double)N * (G - 1) / G, ag_ms, all_ms, bytes_alg / all_ms * 1e-6);

    /* every GPU must now hold the same, complete y */
    int same = 1;
    double *yg = malloc((size_t)(N + 1) * sizeof(double));
    for (int g = 0; g < G; ++g) {
        spmv_set_device(spmv_multi_device(mg, g));
        if (spmv_download(g == 0 ? y : yg, y_full[g], (size_t)N * 8, NULL) != SPMV_SUCCESS) {
            printf("read back error: %s\n", spmv_last_error());
            return SPMV_PROGRAM_ERROR;
        }
        if (g > 0 && memcmp(y, yg, (size_t)N * 8) != 0)
            same = 0;
    }
    free(yg);
    printf("  [multi] y identical on all %d GPUs: %s\n", G, same ? "yes" : "NO");
    int ok = check_and_report(m, x, y, "") && same;
    if (o->cpu) {
        int threads = o->threads > 0 ? o->threads : spmv_cpu_threads();
        double t0 = now_s();
        for (int g = 0; g < G; ++g) /* each shard's loop into its rows: the same reassembly */
            run_cpu(&f[g], xr, y_cpu + bounds[g], threads);
        double cms = (now_s() - t0) * 1e3;
        printf("\nCPU calculations\n"); /* reference csr.c:306 */
        print_performance(cms, Z);
        printf("  [cpu] %d OpenMP threads, effective %.1f GB/s\n", threads, bytes_alg / cms * 1e-6);
        ok &= check_and_report(m, x, y_cpu, "cpu ");
    }
    spmv_multi_free(mg);
    return (o->strict && !ok) ? SPMV_OTHER_ERROR : SPMV_SUCCESS;
}

int spmv_driver_main(int argc, char **argv, spmv_format fmt)
{
    setvbuf(stdout, NULL, _IOLBF, 0);
    opts_t o;
    if (parse_opts(argc, argv, fmt, &o) != SPMV_SUCCESS)
        return SPMV_OTHER_ERROR;

    int ndev = 0;
    if (spmv_device_count(&ndev) != SPMV_SUCCESS || ndev <= o.device || ndev < o.gpus) {
        printf("No HIP GPU device found (%s)\n", spmv_last_error());
        return SPMV_DEVICE_ERROR; /* reference csr.c:25-28 */
    }
    if (spmv_set_device(o.device) != SPMV_SUCCESS)
        return SPMV_DEVICE_ERROR;

    coo_t m;
    errno = 0;
    int rc = load_input(&o, fmt, &m);
    if (rc != SPMV_SUCCESS)
        return rc;
    if (o.write_mtx)
        spmv_mtx_write(o.write_mtx, m.n_rows, m.n_cols, m.nnz, m.row, m.col, m.val, 0);

    double *x = malloc((size_t)(m.n_cols + 1) * sizeof(double));
    double *y = malloc((size_t)(m.n_rows + 1) * sizeof(double));
    double *y_cpu = malloc((size_t)(m.n_rows + 1) * sizeof(double));
    if (!x || !y || !y_cpu)
        return SPMV_OTHER_ERROR;
    for (int64_t j = 0; j < m.n_cols; ++j)
        x[j] = (double)j; /* reference csr.c:95-99 */

    /* --relabel: the degree-ordered layout bench.py measures configs[3] on */
    coo_t mr = m;
    double *xr = x;
    int relabel = o.relabel;
    if (relabel < 0) { /* auto: when the CSR skew rule picks the entry-balanced kernel */
        int64_t *ptr = malloc((size_t)(m.n_rows + 1) * sizeof(int64_t));
        int32_t *tc = malloc((size_t)(m.nnz + 1) * sizeof(int32_t));
        double *tv = malloc((size_t)(m.nnz + 1) * sizeof(double));
        if (!ptr || !tc || !tv || spmv_csr_from_coo(m.n_rows, m.nnz, m.row, m.col, m.val, ptr, tc, tv))
            return SPMV_OTHER_ERROR;
        relabel = spmv_csr_pick_variant(m.n_rows, ptr) == 4;
        free(ptr);
        free(tc);
        free(tv);
    }
    if (relabel) {
        if ((rc = relabel_layout(&m, x, &mr, &xr)) != SPMV_SUCCESS) {
            printf("relabel failed\n");
            return rc;
        }
        printf("  [relabel] columns by decreasing degree (ties by first row), rows in new-column order; "
               "x permuted to match\n");
    }
    if (o.gpus >= 1)
        return run_multi(&o, fmt, &m, x, y, y_cpu, &mr, xr);

    dev_fmt_t f;
    rc = build_format(&o, fmt, &mr, &f, relabel);
    if (rc != SPMV_SUCCESS) {
        printf("format build/upload failed: %s %s\n", spmv_strerror(rc), spmv_last_error());
        return rc == SPMV_OTHER_ERROR ? SPMV_OTHER_ERROR : SPMV_PROGRAM_ERROR;
    }
    if (fmt == FMT_COO) { /* stderr: stdout keeps the reference's lines, starting with "GPU calculations" */
        spmv_plan_info info;
        if (spmv_plan_get_info(f.plan, &info) == SPMV_SUCCESS)
            fprintf(stderr, "COO single pass: %s\n",
                    info.single_pass ? "no carry kernel"
                    : o.single_pass  ? "refused (a row runs more than 80 entries past a tile), carry pass"
                                     : "off (--carry-pass)");
    }
    if ((rc = upload((void **)&f.d_x, xr, (size_t)m.n_cols * 8, NULL)) ||
        (rc = spmv_malloc((void **)&f.d_y, (size_t)m.n_rows * 8)) ||
        (rc = spmv_memset(f.d_y, 0xFF, (size_t)m.n_rows * 8, NULL))) /* NaN: y must be written */
        return SPMV_PROGRAM_ERROR;

    for (int i = 0; i < o.warmup; ++i)
        if ((rc = launch(&f)) != SPMV_SUCCESS) {
            printf("kernel launch error: %s\n", spmv_last_error());
            return SPMV_PROGRAM_ERROR;
        }
    /* the SpMV's time: a span of reps x (flush + SpMV) minus a span of reps
     * flushes, HIP events on the stream (bench.py's in-process method; the
     * flush reads 512 MiB so nothing the SpMV needs is cached) — or, with
     * --warm, reps back-to-back launches */
    double ms = 0.0, ms_min = 0.0;
    if ((rc = time_spmv(&f, o.reps, !o.warm, &ms, &ms_min)) != SPMV_SUCCESS) {
        printf("kernel launch error: %s\n", spmv_last_error());
        return SPMV_PROGRAM_ERROR;
    }

    if (fmt == FMT_COO)
        printf("GPU calculations\n"); /* reference coo.c:201 */
    print_performance(ms, m.nnz);
    print_speed(ms, m.nnz);

    const double bytes_alg = 12.0 * (double)m.nnz + 4.0 * (double)(m.n_rows + 1) +
                             8.0 * (double)m.n_cols + 8.0 * (double)m.n_rows;
    char dev[128] = "";
    spmv_device_name(o.device, dev, sizeof dev);
    printf("  [%s] %s | N=%lld M=%lld Z=%lld | %s, %d reps (per-launch event median %.4f ms)\n",
           fmt_name(fmt), m.label, (long long)m.n_rows, (long long)m.n_cols, (long long)m.nnz,
           o.warm ? "warm (cache-resident): span of back-to-back launches / reps"
                  : "cold: (span of reps x (512 MiB read flush + SpMV) - span of reps flushes) / reps",
           o.reps, ms_min);
    printf("  [%s] effective %.1f GB/s (bytes_alg %.1f MB) = %.1f%% of %.0f GB/s HBM3E peak; "
           "stored %.1f MB; %s\n",
           fmt_name(fmt), bytes_alg / ms * 1e-6, bytes_alg * 1e-6,
           100.0 * bytes_alg / ms * 1e-6 / HBM_PEAK_GBS, HBM_PEAK_GBS,
           (double)f.stored_bytes * 1e-6, dev);
    print_plan(&f, "");

    if (spmv_download(y, f.d_y, (size_t)m.n_rows * 8, NULL) != SPMV_SUCCESS) {
        printf("read back error: %s\n", spmv_last_error());
        return SPMV_PROGRAM_ERROR;
    }
    if (o.write_y) {
        FILE *fy = fopen(o.write_y, "wb");
        if (!fy || fwrite(y, sizeof(double), (size_t)m.n_rows, fy) != (size_t)m.n_rows) {
            perror(o.write_y);
            if (fy)
                fclose(fy);
            return SPMV_FILE_ERROR;
        }
        fclose(fy);
    }
    int ok = check_and_report(&m, x, y, "");

    if (o.cpu) {
        int threads = o.threads > 0 ? o.threads : spmv_cpu_threads();
        double t0 = now_s();
        run_cpu(&f, xr, y_cpu, threads);
        double cms = (now_s() - t0) * 1e3;
        printf("\nCPU calculations\n"); /* reference csr.c:306 */
        print_performance(cms, m.nnz);
        printf("  [cpu] %d OpenMP threads, effective %.1f GB/s\n", threads,
               bytes_alg / cms * 1e-6);
        ok &= check_and_report(&m, x, y_cpu, "cpu ");
    }
    spmv_plan_destroy(f.plan);
    return (o.strict && !ok) ? SPMV_OTHER_ERROR : SPMV_SUCCESS;
}
