// plan.hip — the per-format SpMV plans of the C-ABI (include/spmv.h):
// spmv_plan_{coo,csr,ell,sell,cmrs} look at a matrix already in HBM ONCE,
// choose the kernel path the measurements picked for it (x windows in LDS,
// the small-matrix SELL kernel's head copy, the single-pass COO tail, the
// entry-balanced CSR/CMRS tiles with their tile and big-tile plans, the
// SELL wide-slice split, SELL16 column offsets) and build everything that
// path needs; spmv_plan_run then launches it with no allocation, no
// synchronisation and no decision left, so it can be captured in a graph.
//
// This replaces the reference's per-driver launch setup
// (reference coo.c:163-194, csr.c:170-201, ell.c:242-273,
// sigma_c.c:280-311, cmrs.c:195-232: clSetKernelArg x k +
// clEnqueueNDRangeKernel with hard-coded work sizes).  The drivers
// (drivers/driver.c) and the Python binding (spmv_amd.to_device) both
// create plans, so ./bin/<fmt> and bench.py run the same kernels.  The
// individual kernel entry points the plans choose between stay exported
// (include/spmv_ext.h) for A/B tools and the tests that pin each
// variant's bits.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "common.h"
#include "spmv_host.h"

namespace spmv {

enum PlanPath {
    P_COO_CARRY,
    P_COO_TAIL,
    P_COO_XWIN,
    P_COO_HOT,
    P_CSR_VARIANT,
    P_CSR_XWIN,
    P_CSR_TILED,
    P_ELL,
    P_ELL_XWIN,
    P_SELL,
    P_SELL_XWIN,
    P_SELL_XWIN_HEAD,
    P_SELL_SPLIT,
    P_SELL_HOT,
    P_SELL16,
    P_CMRS,
    P_CMRS_XWIN,
    P_CMRS_TILED,
};

// Largest difference of consecutive offsets off[1..n] - off[0..n-1] (a row
// or strip length), per workgroup (the host takes the max of the
// workgroups'): the skew rules of the CSR and CMRS plans, computed where
// the offsets are (build time).
__global__ __launch_bounds__(kBlock) void max_len_kernel(int64_t n, const int64_t *__restrict__ off,
                                                         int64_t *__restrict__ out)
{
    __shared__ int64_t s_m[kBlock / kWave];
    int64_t m = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const int64_t l = off[i + 1] - off[i];
        m = l > m ? l : m;
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
        const int64_t t = __shfl_xor(m, o);
        m = t > m ? t : m;
    }
    if ((threadIdx.x & (kWave - 1)) == 0)
        s_m[threadIdx.x / kWave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / kWave; ++w)
            m = s_m[w] > m ? s_m[w] : m;
        out[blockIdx.x] = m;
    }
}

}  // namespace spmv

using namespace spmv;

struct spmv_plan {
    int fmt;  // SPMV_FMT_*
    int path; // PlanPath
    spmv_dims d;
    spmv_plan_opts o;
    // the caller's arrays (device)
    const int64_t *ptr = nullptr;  // CSR row_ptr / SELL slice_ptr / CMRS strip_ptr
    const int32_t *row = nullptr, *col = nullptr, *perm = nullptr;
    const uint8_t *rin = nullptr;
    const double *val = nullptr;
    // geometry
    int32_t K = 0, C = 0, sigma = 0, ki = 0, h = 0, lanes = 0, variant = 0, xwin_rows = 0;
    int64_t ld = 0, n_slices = 0, n_strips = 0;
    // owned by the plan (device)
    void *win = nullptr;
    int32_t xcap = 0;
    void *head = nullptr;
    size_t head_bytes = 0;
    void *tails = nullptr;
    void *ws = nullptr;
    size_t ws_bytes = 0;
    int32_t *own_lo = nullptr;
    int32_t *big = nullptr;
    int64_t big_len = 0, big_tiles = 0, big_tile = 0;
    int32_t split_T = 0;
    bool tiles_planned = false;  // tiled CMRS: the tile -> first-strip table filled at build
    int64_t n_chunks = 0;
    int32_t *chunk_slice = nullptr, *chunk_k0 = nullptr;
    uint16_t *col16 = nullptr;
    int32_t *hcol = nullptr;  // the columns with hot ids (plan-owned), or NULL
    int32_t *hot = nullptr;   // hot[H]: the hot columns in rank order
    int64_t H = 0;
    size_t owned = 0;
    char kernel[64] = "";
    char desc[320] = "";
};

namespace {

int plan_alloc(spmv_plan *p, void **dst, size_t bytes)
{
    *dst = nullptr;
    hipError_t e = hipMalloc(dst, bytes > 0 ? bytes : 16);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_plan: hipMalloc", e);
    p->owned += bytes;
    return SPMV_SUCCESS;
}

int plan_upload(spmv_plan *p, void **dst, const void *src, size_t bytes)
{
    int rc = plan_alloc(p, dst, bytes);
    if (rc != SPMV_SUCCESS || bytes == 0)
        return rc;
    hipError_t e = hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)p->d.stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize((hipStream_t)p->d.stream);
    return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "spmv_plan: upload", e);
}

// host copy of n+1 device offsets (build time)
int download_offsets(const spmv_plan *p, const int64_t *dptr, int64_t n, int64_t **out)
{
    *out = (int64_t *)malloc((size_t)(n + 1) * sizeof(int64_t));
    if (!*out)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan: out of host memory");
    hipError_t e = hipMemcpyAsync(*out, dptr, (size_t)(n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost,
                                  (hipStream_t)p->d.stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize((hipStream_t)p->d.stream);
    if (e != hipSuccess) {
        free(*out);
        *out = nullptr;
        return fail(SPMV_PROGRAM_ERROR, "spmv_plan: copy offsets", e);
    }
    return SPMV_SUCCESS;
}

// max over i < n of off[i+1] - off[i], on the device
int max_len(const spmv_plan *p, const int64_t *off, int64_t n, int64_t *out)
{
    *out = 0;
    if (n <= 0)
        return SPMV_SUCCESS;
    const int64_t blocks = (n + kBlock - 1) / kBlock < 1024 ? (n + kBlock - 1) / kBlock : 1024;
    int64_t *d = nullptr, h[1024];
    hipError_t e = hipMalloc(&d, (size_t)blocks * sizeof(int64_t));
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_plan: hipMalloc", e);
    const hipStream_t st = (hipStream_t)p->d.stream;
    hipLaunchKernelGGL(max_len_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, n, off, d);
    e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(h, d, (size_t)blocks * sizeof(int64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    (void)hipFree(d);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "spmv_plan: row lengths", e);
    for (int64_t b = 0; b < blocks; ++b)
        *out = h[b] > *out ? h[b] : *out;
    return SPMV_SUCCESS;
}

bool xwin_on(const spmv_plan_opts &o, bool dflt) { return o.xwin < 0 ? dflt : o.xwin != 0; }

// The hot-column table (opts.H: -1 rule, 0 none, > 0 that many) over the
// `count` device columns `col` the format stores: the renumbered copy
// (p->hcol) and the table (p->hot) are plan-owned; H = 0 leaves both NULL.
int build_hot(spmv_plan *p, const int32_t *col, int64_t count)
{
    p->H = 0;
    const int64_t req = p->o.H;
    if (req == 0 || count <= 0 || !spmv_hot_columns_possible(p->d.n_cols, req > 0 ? req : 0))
        return SPMV_SUCCESS;
    if (req < -1)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan: opts.H must be -1, 0 or a table size");
    const hipStream_t st = (hipStream_t)p->d.stream;
    int32_t *hc = (int32_t *)malloc((size_t)count * sizeof(int32_t));
    const int64_t cap = req > ((int64_t)1 << 19) ? req : ((int64_t)1 << 19);
    int32_t *ht = (int32_t *)malloc((size_t)cap * sizeof(int32_t));
    int rc = SPMV_SUCCESS;
    if (!hc || !ht) {
        rc = fail_msg(SPMV_OTHER_ERROR, "spmv_plan: out of host memory");
    } else {
        hipError_t e = hipMemcpyAsync(hc, col, (size_t)count * sizeof(int32_t), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess)
            e = hipStreamSynchronize(st);
        if (e != hipSuccess)
            rc = fail(SPMV_PROGRAM_ERROR, "spmv_plan: copy columns", e);
    }
    if (rc == SPMV_SUCCESS) {
        const int64_t H = spmv_hot_columns(p->d.n_cols, count, hc, req > 0 ? req : 0, ht, hc);
        if (H < 0)
            rc = fail_msg(SPMV_OTHER_ERROR, "spmv_plan: hot-column table (column out of range?)");
        else if (H > 0 && (rc = plan_upload(p, (void **)&p->hcol, hc, (size_t)count * sizeof(int32_t))) ==
                              SPMV_SUCCESS &&
                 (rc = plan_upload(p, (void **)&p->hot, ht, (size_t)H * sizeof(int32_t))) == SPMV_SUCCESS)
            p->H = H;
    }
    free(hc);
    free(ht);
    return rc;
}

// the columns a run reads: the renumbered copy with a hot table
const int32_t *run_col(const spmv_plan *p) { return p->hcol ? p->hcol : p->col; }

spmv_plan *new_plan(int fmt, spmv_dims d, const spmv_plan_opts *o)
{
    spmv_plan *p = new (std::nothrow) spmv_plan();
    if (!p)
        return nullptr;
    p->fmt = fmt;
    p->d = d;
    if (o)
        p->o = *o;
    else
        spmv_plan_opts_init(&p->o);
    return p;
}

int finish(spmv_plan *p, int rc, spmv_plan **out)
{
    if (rc != SPMV_SUCCESS) {
        const char *msg = spmv_last_error();
        char keep[512];
        snprintf(keep, sizeof keep, "%s", msg);
        spmv_plan_destroy(p);
        *out = nullptr;
        return fail_msg(rc, keep);
    }
    *out = p;
    return SPMV_SUCCESS;
}

int check_dims(const spmv_dims &d, const char *who)
{
    static thread_local char msg[128];
    if (d.n_rows < 0 || d.n_cols < 0 || d.nnz < 0) {
        snprintf(msg, sizeof msg, "%s: negative sizes", who);
        return fail_msg(SPMV_OTHER_ERROR, msg);
    }
    return SPMV_SUCCESS;
}

}  // namespace

extern "C" {

void spmv_plan_opts_init(spmv_plan_opts *o)
{
    if (!o)
        return;
    memset(o, 0, sizeof *o);
    o->variant = -1;
    o->xwin = -1;
    o->head = -1;
    o->coo_pass = -1;
    o->split = -1;
    o->bigplan = -1;
    o->H = -1;
}

int spmv_plan_destroy(spmv_plan *p)
{
    if (!p)
        return SPMV_SUCCESS;
    void *owned[] = {p->win,    p->head,        p->tails,    p->ws,    p->own_lo, p->big,
                     p->chunk_slice, p->chunk_k0, p->col16, p->hcol, p->hot};
    int dev = -1;
    (void)hipGetDevice(&dev);
    if (dev != p->d.device)
        (void)hipSetDevice(p->d.device);
    for (void *q : owned)
        if (q)
            (void)hipFree(q);
    if (dev >= 0 && dev != p->d.device)
        (void)hipSetDevice(dev);
    delete p;
    return SPMV_SUCCESS;
}

// ------------------------------------------------------------------ COO
int spmv_plan_coo(spmv_dims d, const int32_t *row, const int32_t *col, const double *val, const spmv_plan_opts *o,
                  spmv_plan **out)
{
    if (!out)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_coo: out is NULL");
    *out = nullptr;
    int rc = check_dims(d, "spmv_plan_coo");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (d.nnz > 0 && (!row || !col || !val))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_coo: NULL array");
    spmv_plan *p = new_plan(SPMV_FMT_COO, d, o);
    if (!p)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_coo: out of host memory");
    SPMV_GUARD(d);
    p->row = row;
    p->col = col;
    p->val = val;
    if ((rc = build_hot(p, col, d.nnz)) != SPMV_SUCCESS)
        return finish(p, rc, out);
    const int64_t H = p->H;
    // x windows are off by default for COO: per-tile windows measured slower
    // (0.534 vs 0.491 ms on the cant-like batch, 22.6 vs 16.4 us on one matrix)
    const bool xw = xwin_on(p->o, false);
    if (p->o.coo_pass == 1 && (xw || H > 0))
        return finish(p, fail_msg(SPMV_OTHER_ERROR, "spmv_plan_coo: the single pass (coo_pass = 1) runs without x "
                                                    "windows and hot-column table"), out);
    if (H > 0) {
        p->path = P_COO_HOT;
        p->ws_bytes = spmv_coo_hot_ws_bytes(d.nnz, H);
        rc = plan_alloc(p, &p->ws, p->ws_bytes);
        snprintf(p->kernel, sizeof p->kernel, "coo_staged_kernel");
        snprintf(p->desc, sizeof p->desc, "COO: staged tiles + carry pass, hot-column table H=%lld", (long long)H);
        return finish(p, rc, out);
    }
    p->ws_bytes = spmv_coo_ws_bytes(d.nnz);
    if (xw) {
        p->path = P_COO_XWIN;
        const size_t wb = spmv_coo_xwin_bytes(d.nnz);
        if ((rc = plan_alloc(p, &p->ws, p->ws_bytes)) == SPMV_SUCCESS &&
            (rc = plan_alloc(p, &p->win, wb)) == SPMV_SUCCESS)
            rc = spmv_coo_xwin_build(d, col, p->win, wb, &p->xcap);
        snprintf(p->kernel, sizeof p->kernel, "coo_staged_kernel");
        snprintf(p->desc, sizeof p->desc, "COO: staged tiles with x windows (xcap %d) + carry pass", p->xcap);
        return finish(p, rc, out);
    }
    if (p->o.coo_pass != 0 && d.nnz > 0) {
        // the single pass (no carry kernel) wherever every row ends within
        // 80 entries of its tile: one cant-like matrix cold 18.1 vs 20.6 us
        const size_t tb = spmv_coo_tail_bytes(d.nnz);
        if ((rc = plan_alloc(p, &p->tails, tb)) != SPMV_SUCCESS)
            return finish(p, rc, out);
        rc = spmv_coo_tail_build(d, row, p->tails, tb);
        if (rc == SPMV_SUCCESS) {
            p->path = P_COO_TAIL;
            snprintf(p->kernel, sizeof p->kernel, "coo_staged_kernel");
            snprintf(p->desc, sizeof p->desc, "COO: single pass (each tile finishes its last row, no carry kernel)");
            return finish(p, rc, out);
        }
        if (p->o.coo_pass == 1)
            return finish(p, rc, out);
        (void)hipFree(p->tails);  // refused (a row runs past the tail cap): the carry pass
        p->tails = nullptr;
    }
    p->path = P_COO_CARRY;
    rc = plan_alloc(p, &p->ws, p->ws_bytes);
    snprintf(p->kernel, sizeof p->kernel, "coo_staged_kernel");
    snprintf(p->desc, sizeof p->desc, "COO: staged tiles + deterministic carry pass");
    return finish(p, rc, out);
}

// ------------------------------------------------------------------ CSR
int spmv_plan_csr(spmv_dims d, const int64_t *row_ptr, const int32_t *col, const double *val,
                  const spmv_plan_opts *o, spmv_plan **out)
{
    if (!out)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_csr: out is NULL");
    *out = nullptr;
    int rc = check_dims(d, "spmv_plan_csr");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (!row_ptr || (d.nnz > 0 && (!col || !val)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_csr: NULL array");
    spmv_plan *p = new_plan(SPMV_FMT_CSR, d, o);
    if (!p)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_csr: out of host memory");
    SPMV_GUARD(d);
    p->ptr = row_ptr;
    p->col = col;
    p->val = val;
    p->lanes = p->o.lanes > 0 ? p->o.lanes : spmv_csr_auto_lanes(d.n_rows, d.nnz);
    p->xwin_rows = p->o.xwin_rows;
    int v = p->o.variant;
    if (v < 0 || v > 4)
        v = -1;
    if (v == -1) {  // the skew rule: entry-balanced tiles when the longest row dwarfs the mean
        int64_t mx = 0;
        if ((rc = max_len(p, row_ptr, d.n_rows, &mx)) != SPMV_SUCCESS)
            return finish(p, rc, out);
        v = spmv_csr_variant_rule(d.n_rows, d.nnz, mx);
    }
    p->variant = v;
    if (v == 4) {
        if ((rc = build_hot(p, col, d.nnz)) != SPMV_SUCCESS)
            return finish(p, rc, out);
        const int64_t H = p->H;
        p->path = P_CSR_TILED;
        p->ws_bytes = spmv_csr_hot_ws_bytes(d.n_rows, d.nnz, H);
        if ((rc = plan_alloc(p, &p->ws, p->ws_bytes)) != SPMV_SUCCESS)
            return finish(p, rc, out);
        const int64_t n_plan = spmv_csr_tiled_plan_len(d.nnz);
        if (n_plan > 0) {  // tile -> first owned row, built once from row_ptr
            if ((rc = plan_alloc(p, (void **)&p->own_lo, (size_t)n_plan * sizeof(int32_t))) != SPMV_SUCCESS ||
                (rc = spmv_csr_tiled_plan(d, row_ptr, p->own_lo)) != SPMV_SUCCESS)
                return finish(p, rc, out);
            // tiles owning more than 1,024 rows (runs of empty rows): the
            // list of their rows with entries (same bits)
            p->big_tile = spmv_csr_tiled_tile(d.n_rows, d.nnz);
            if (p->o.bigplan != 0 && p->big_tile > 0) {
                int64_t *hp = nullptr;
                if ((rc = download_offsets(p, row_ptr, d.n_rows, &hp)) != SPMV_SUCCESS)
                    return finish(p, rc, out);
                const int64_t tiles = (d.nnz + p->big_tile - 1) / p->big_tile;
                const int64_t nb = spmv_csr_tiled_bigplan(d.n_rows, hp, p->big_tile, 1024, nullptr);
                if (nb > tiles) {
                    int32_t *bp = (int32_t *)malloc((size_t)nb * sizeof(int32_t));
                    if (!bp) {
                        free(hp);
                        return finish(p, fail_msg(SPMV_OTHER_ERROR, "spmv_plan_csr: out of host memory"), out);
                    }
                    spmv_csr_tiled_bigplan(d.n_rows, hp, p->big_tile, 1024, bp);
                    for (int64_t t = 0; t < tiles; ++t)
                        p->big_tiles += bp[t] >= 0;
                    if (p->big_tiles > 0) {
                        rc = plan_upload(p, (void **)&p->big, bp, (size_t)nb * sizeof(int32_t));
                        p->big_len = nb;
                    }
                    free(bp);
                }
                free(hp);
                if (rc != SPMV_SUCCESS)
                    return finish(p, rc, out);
            }
        }
        snprintf(p->kernel, sizeof p->kernel, "csr_tiled_kernel");
        snprintf(p->desc, sizeof p->desc,
                 "CSR: entry-balanced tiles of %lld entries (skewed rows), tile plan, %lld big tiles listed%s",
                 (long long)p->big_tile, (long long)p->big_tiles, H > 0 ? ", hot-column table" : "");
        return finish(p, rc, out);
    }
    if (xwin_on(p->o, true) && (v == 0 || v == 3)) {
        p->path = P_CSR_XWIN;
        p->variant = 3;
        const size_t wb = spmv_csr_xwin_bytes(d.n_rows, d.nnz, p->lanes, p->xwin_rows);
        if ((rc = plan_alloc(p, &p->win, wb)) == SPMV_SUCCESS)
            rc = spmv_csr_xwin_build(d, row_ptr, col, p->lanes, p->xwin_rows, p->win, wb, &p->xcap);
        snprintf(p->kernel, sizeof p->kernel, "csr_xwin_kernel");
        snprintf(p->desc, sizeof p->desc, "CSR-vector: %d lanes per row, x windows of %d rows in LDS (xcap %d)",
                 p->lanes, p->xwin_rows > 0 ? p->xwin_rows : 128, p->xcap);
        return finish(p, rc, out);
    }
    p->path = P_CSR_VARIANT;
    static const char *names[] = {"csr_staged_persistent_kernel", "csr_vector_kernel", "csr_staged_kernel",
                                  "csr_staged_persistent_kernel"};
    snprintf(p->kernel, sizeof p->kernel, "%s", names[v]);
    snprintf(p->desc, sizeof p->desc, "CSR-vector: %d lanes per row, variant %d, global x gathers", p->lanes,
             v == 0 ? 3 : v);
    return finish(p, SPMV_SUCCESS, out);
}

// ------------------------------------------------------------------ ELL
int spmv_plan_ell(spmv_dims d, int32_t K, int64_t ld, int32_t ki, const int32_t *col, const double *val,
                  const spmv_plan_opts *o, spmv_plan **out)
{
    if (!out)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_ell: out is NULL");
    *out = nullptr;
    int rc = check_dims(d, "spmv_plan_ell");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (K < 0 || ld < d.n_rows || ld % kWave != 0 || (ki != 1 && ki != 2) || K % ki != 0 ||
        (K > 0 && (!col || !val)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_ell: bad ELL geometry (K, ld, ki) or NULL array");
    spmv_plan *p = new_plan(SPMV_FMT_ELL, d, o);
    if (!p)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_ell: out of host memory");
    SPMV_GUARD(d);
    p->K = K;
    p->ld = ld;
    p->ki = ki;
    p->col = col;
    p->val = val;
    if (xwin_on(p->o, true)) {
        p->path = P_ELL_XWIN;
        const size_t wb = spmv_ell_xwin_bytes(d.n_rows);
        if ((rc = plan_alloc(p, &p->win, wb)) == SPMV_SUCCESS)
            rc = spmv_ell_xwin_build(d, K, ld, ki, col, p->win, wb, &p->xcap);
        snprintf(p->kernel, sizeof p->kernel, "ell_xwin_kernel");
        snprintf(p->desc, sizeof p->desc, "ELL: column-major K=%d ld=%lld ki=%d, x windows in LDS (xcap %d)", K,
                 (long long)ld, ki, p->xcap);
        return finish(p, rc, out);
    }
    p->path = P_ELL;
    snprintf(p->kernel, sizeof p->kernel, "ell_kernel");
    snprintf(p->desc, sizeof p->desc, "ELL: column-major K=%d ld=%lld ki=%d, global x gathers", K, (long long)ld, ki);
    return finish(p, SPMV_SUCCESS, out);
}

// ----------------------------------------------------------------- SELL
int spmv_plan_sell(spmv_dims d, int32_t C, int32_t sigma, int32_t ki, int64_t n_slices, const int64_t *slice_ptr,
                   const int32_t *perm, const int32_t *col, const double *val, const spmv_plan_opts *o,
                   spmv_plan **out)
{
    if (!out)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_sell: out is NULL");
    *out = nullptr;
    int rc = check_dims(d, "spmv_plan_sell");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (C <= 0 || C > 1024 || (ki != 1 && ki != 2) || sigma < 1 || (sigma > 1 && sigma % C) || n_slices < 0 ||
        n_slices * C < d.n_rows || (n_slices > 0 && (!slice_ptr || !perm || !col || !val)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_sell: bad SELL geometry (C, sigma, ki, n_slices) or NULL array");
    spmv_plan *p = new_plan(SPMV_FMT_SELL, d, o);
    if (!p)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_sell: out of host memory");
    SPMV_GUARD(d);
    p->C = C;
    p->sigma = sigma;
    p->ki = ki;
    p->n_slices = n_slices;
    p->ptr = slice_ptr;
    p->perm = perm;
    p->col = col;
    p->val = val;
    const bool small = sell_small(C, n_slices);
    if (p->o.H != 0 && !p->o.index16 && n_slices > 0) {  // the table over the stored columns (padding too)
        int64_t stored = 0;
        hipError_t e = hipMemcpyAsync(&stored, slice_ptr + n_slices, sizeof stored, hipMemcpyDeviceToHost,
                                      (hipStream_t)d.stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize((hipStream_t)d.stream);
        if (e != hipSuccess)
            return finish(p, fail(SPMV_PROGRAM_ERROR, "spmv_plan_sell: stored count", e), out);
        if ((rc = build_hot(p, col, stored)) != SPMV_SUCCESS)
            return finish(p, rc, out);
    }
    const int64_t H = p->H;
    const bool xw = xwin_on(p->o, true) && H == 0;
    // wide slices (power-law rows): split into chunks of T slot columns
    if (p->o.split != 0 && n_slices > 0) {
        int64_t *hs = nullptr;
        if ((rc = download_offsets(p, slice_ptr, n_slices, &hs)) != SPMV_SUCCESS)
            return finish(p, rc, out);
        int32_t T = p->o.split > 0 ? p->o.split : spmv_sell_split_auto(n_slices, hs, C, ki);
        if (T > 0 && T % ki) {
            free(hs);
            return finish(p, fail_msg(SPMV_OTHER_ERROR, "spmv_plan_sell: split T must be a multiple of ki"), out);
        }
        if (T > 0) {
            const int64_t n = spmv_sell_split_plan(n_slices, hs, C, T, nullptr, nullptr);
            int32_t *cs = n >= 0 ? (int32_t *)calloc((size_t)n + 1, sizeof(int32_t)) : nullptr;
            int32_t *ck = n >= 0 ? (int32_t *)calloc((size_t)n + 1, sizeof(int32_t)) : nullptr;
            if (!cs || !ck) {
                free(cs);
                free(ck);
                free(hs);
                return finish(p, fail_msg(SPMV_OTHER_ERROR, "spmv_plan_sell: split plan"), out);
            }
            spmv_sell_split_plan(n_slices, hs, C, T, cs, ck);
            p->split_T = T;
            p->n_chunks = n;
            rc = plan_upload(p, (void **)&p->chunk_slice, cs, (size_t)(n + 1) * sizeof(int32_t));
            if (rc == SPMV_SUCCESS)
                rc = plan_upload(p, (void **)&p->chunk_k0, ck, (size_t)(n + 1) * sizeof(int32_t));
            free(cs);
            free(ck);
        }
        free(hs);
        if (rc != SPMV_SUCCESS)
            return finish(p, rc, out);
    }
    if (p->o.index16 && (p->split_T > 0 || H > 0 || C != kWave || !xwin_on(p->o, true)))
        return finish(p, fail_msg(SPMV_OTHER_ERROR, "spmv_plan_sell: SELL16 (index16) needs C = 64, x windows, no "
                                                    "split and no hot-column table"), out);
    if (xw && n_slices > 0) {
        const size_t wb = spmv_sell_xwin_bytes(n_slices, C, sigma);
        if ((rc = plan_alloc(p, &p->win, wb)) != SPMV_SUCCESS ||
            (rc = spmv_sell_xwin_build(d, C, sigma, n_slices, slice_ptr, col, p->win, wb, &p->xcap)) != SPMV_SUCCESS)
            return finish(p, rc, out);
    }
    const char *kern = small ? "sell_small_kernel" : xw ? "sell_xwin_kernel" : "sell_kernel";
    snprintf(p->kernel, sizeof p->kernel, "%s", kern);
    if (H > 0) {
        p->path = P_SELL_HOT;
        p->ws_bytes = spmv_sell_hot_ws_bytes(p->split_T > 0 ? p->n_chunks : 0, C, H);
        rc = plan_alloc(p, &p->ws, p->ws_bytes);
        snprintf(p->kernel, sizeof p->kernel, "%s", small ? "sell_small_kernel" : "sell_kernel");
        snprintf(p->desc, sizeof p->desc, "SELL-C-sigma C=%d sigma=%d ki=%d: hot-column table H=%lld%s", C, sigma, ki,
                 (long long)H, p->split_T > 0 ? ", wide slices split" : "");
        return finish(p, rc, out);
    }
    if (p->split_T > 0) {
        p->path = P_SELL_SPLIT;
        p->ws_bytes = spmv_sell_split_ws_bytes(p->n_chunks, C);
        rc = plan_alloc(p, &p->ws, p->ws_bytes);
        snprintf(p->desc, sizeof p->desc,
                 "SELL-C-sigma C=%d sigma=%d ki=%d: slices wider than %d slot columns split into %lld chunks%s", C,
                 sigma, ki, p->split_T, (long long)p->n_chunks, p->win ? ", x windows" : "");
        return finish(p, rc, out);
    }
    if (p->o.index16) {  // SELL16: 16-bit column offsets from each workgroup's window base (plan-owned)
        p->path = P_SELL16;
        int64_t nst = 0;  // stored slots = slice_ptr[n_slices]
        if (n_slices > 0) {
            int64_t last = 0;
            hipError_t e = hipMemcpyAsync(&last, slice_ptr + n_slices, sizeof last, hipMemcpyDeviceToHost,
                                          (hipStream_t)d.stream);
            if (e == hipSuccess)
                e = hipStreamSynchronize((hipStream_t)d.stream);
            if (e != hipSuccess)
                return finish(p, fail(SPMV_PROGRAM_ERROR, "spmv_plan_sell: stored count", e), out);
            nst = last;
        }
        if ((rc = plan_alloc(p, (void **)&p->col16, (size_t)(nst > 0 ? nst : 1) * sizeof(uint16_t))) !=
                SPMV_SUCCESS ||
            (n_slices > 0 &&
             (rc = spmv_sell16_fill(d, C, sigma, n_slices, slice_ptr, col, p->win, p->col16)) != SPMV_SUCCESS))
            return finish(p, rc, out);
        p->head_bytes = p->o.head != 0 ? spmv_sell16_head_bytes(n_slices, C, ki) : 0;
        if (p->head_bytes > 0 &&
            ((rc = plan_alloc(p, &p->head, p->head_bytes)) != SPMV_SUCCESS ||
             (rc = spmv_sell16_head_fill(d, C, sigma, ki, n_slices, slice_ptr, val, p->col16, p->head,
                                         p->head_bytes)) != SPMV_SUCCESS))
            return finish(p, rc, out);
        snprintf(p->desc, sizeof p->desc, "SELL16 C=%d sigma=%d ki=%d: 16-bit column offsets, x windows (xcap %d)%s",
                 C, sigma, ki, p->xcap, p->head ? ", head copy" : "");
        return finish(p, SPMV_SUCCESS, out);
    }
    if (p->win) {
        // small matrices: the head copy of every wave's first slot groups
        // (one cant-like matrix cold 11.9 -> 11.4 us, same bits)
        p->head_bytes = p->o.head != 0 ? spmv_sell_head_bytes(n_slices, C, ki) : 0;
        if (p->head_bytes > 0) {
            p->path = P_SELL_XWIN_HEAD;
            if ((rc = plan_alloc(p, &p->head, p->head_bytes)) == SPMV_SUCCESS)
                rc = spmv_sell_head_fill(d, C, sigma, ki, n_slices, slice_ptr, val, col, p->head, p->head_bytes);
        } else {
            p->path = P_SELL_XWIN;
        }
        snprintf(p->desc, sizeof p->desc, "SELL-C-sigma C=%d sigma=%d ki=%d: x windows in LDS (xcap %d)%s", C, sigma,
                 ki, p->xcap, p->head ? ", int32 head copy" : "");
        return finish(p, rc, out);
    }
    p->path = P_SELL;
    snprintf(p->desc, sizeof p->desc, "SELL-C-sigma C=%d sigma=%d ki=%d: global x gathers", C, sigma, ki);
    return finish(p, SPMV_SUCCESS, out);
}

// ----------------------------------------------------------------- CMRS
int spmv_plan_cmrs(spmv_dims d, int32_t h, int64_t n_strips, const int64_t *strip_ptr, const uint8_t *row_in_strip,
                   const int32_t *col, const double *val, const spmv_plan_opts *o, spmv_plan **out)
{
    if (!out)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_cmrs: out is NULL");
    *out = nullptr;
    int rc = check_dims(d, "spmv_plan_cmrs");
    if (rc != SPMV_SUCCESS)
        return rc;
    if (h < 1 || h > 64 || n_strips < 0 || n_strips * h < d.n_rows || !strip_ptr ||
        (d.nnz > 0 && (!row_in_strip || !col || !val)))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_cmrs: bad strip geometry (h, n_strips) or NULL array");
    spmv_plan *p = new_plan(SPMV_FMT_CMRS, d, o);
    if (!p)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_cmrs: out of host memory");
    SPMV_GUARD(d);
    p->h = h;
    p->n_strips = n_strips;
    p->ptr = strip_ptr;
    p->rin = row_in_strip;
    p->col = col;
    p->val = val;
    // variant: -1 rule, 0 the rule too (CSR's convention), 1 strip runs, 2 entry-balanced tiles
    int v = p->o.variant;
    if (v == 1 || v == 2) {
        v = v == 2 ? 1 : 0;
    } else {
        int64_t mx = 0;
        if ((rc = max_len(p, strip_ptr, n_strips, &mx)) != SPMV_SUCCESS)
            return finish(p, rc, out);
        v = spmv_cmrs_variant_rule(n_strips, d.nnz, mx);
    }
    p->variant = v;
    if (v == 1) {
        if ((rc = build_hot(p, col, d.nnz)) != SPMV_SUCCESS)
            return finish(p, rc, out);
        p->path = P_CMRS_TILED;
        p->ws_bytes = spmv_cmrs_hot_ws_bytes(n_strips, d.nnz, h, p->H);
        rc = plan_alloc(p, &p->ws, p->ws_bytes);
        // the tile -> first-strip table once, here, instead of every run
        // (csr_tile_rows_kernel, ~8 us on the R-MAT)
        const int64_t ch = cmrs_tiled_tile(d.n_rows, d.nnz);
        if (rc == SPMV_SUCCESS && d.n_rows > 0 && d.nnz > 0 && h >= 1 && h <= 64 && d.n_rows <= INT32_MAX &&
            n_strips == (d.n_rows + h - 1) / h && ((d.nnz + ch - 1) / ch) * h <= INT32_MAX) {
            rc = cmrs_tiled_planned(d, h, n_strips, strip_ptr, row_in_strip, col, val, nullptr, nullptr, p->H,
                                    p->hot, p->ws, true);
            // runs may come on any stream: the table is complete when the plan is returned
            if (rc == SPMV_SUCCESS && hipStreamSynchronize((hipStream_t)d.stream) != hipSuccess)
                rc = fail_msg(SPMV_PROGRAM_ERROR, "spmv_plan_cmrs: tile table");
            p->tiles_planned = rc == SPMV_SUCCESS;
        }
        snprintf(p->kernel, sizeof p->kernel, "cmrs_tiled_kernel");
        snprintf(p->desc, sizeof p->desc, "CMRS h=%d: entry-balanced tiles (skewed strips)%s", h,
                 p->H > 0 ? ", hot-column table" : "");
        return finish(p, rc, out);
    }
    snprintf(p->kernel, sizeof p->kernel, "cmrs_staged_kernel");
    if (xwin_on(p->o, true)) {
        p->path = P_CMRS_XWIN;
        const size_t wb = spmv_cmrs_xwin_bytes(d, h, n_strips);
        if ((rc = plan_alloc(p, &p->win, wb)) == SPMV_SUCCESS)
            rc = spmv_cmrs_xwin_build(d, h, n_strips, strip_ptr, col, p->win, wb, &p->xcap);
        snprintf(p->desc, sizeof p->desc, "CMRS h=%d: staged strip runs, x windows in LDS (xcap %d)", h, p->xcap);
        return finish(p, rc, out);
    }
    p->path = P_CMRS;
    snprintf(p->desc, sizeof p->desc, "CMRS h=%d: staged strip runs, global x gathers", h);
    return finish(p, SPMV_SUCCESS, out);
}

// ------------------------------------------------------------------ run
int spmv_plan_run(const spmv_plan *p, const double *x, double *y, void *stream)
{
    if (!p)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_run: plan is NULL");
    if ((p->d.n_rows > 0 && !y) || (p->d.nnz > 0 && p->d.n_cols > 0 && !x))
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_run: x or y is NULL");
    spmv_dims d = p->d;
    d.stream = stream;
    const int64_t H = p->H;
    const int32_t *col = run_col(p);
    switch (p->path) {
    case P_COO_CARRY:
        return spmv_coo_run(d, p->row, p->col, p->val, x, y, p->ws, p->ws_bytes);
    case P_COO_TAIL:
        return spmv_coo_run_tail(d, p->row, p->col, p->val, x, y, p->tails);
    case P_COO_XWIN:
        return spmv_coo_run_xwin(d, p->row, p->col, p->val, x, y, p->ws, p->ws_bytes, p->win, p->xcap);
    case P_COO_HOT:
        return spmv_coo_run_hot(d, p->row, col, p->val, x, y, H, p->hot, p->ws, p->ws_bytes);
    case P_CSR_VARIANT:
        return spmv_csr_run_variant(d, p->ptr, p->col, p->val, x, y, p->lanes, p->variant);
    case P_CSR_XWIN:
        return spmv_csr_run_xwin(d, p->ptr, p->col, p->val, x, y, p->lanes, p->xwin_rows, p->win, p->xcap);
    case P_CSR_TILED:
        if (p->big)
            return spmv_csr_run_tiled_plan(d, p->ptr, col, p->val, x, y, H, p->hot, p->own_lo, p->big,
                                           p->big_len, p->big_tile, p->ws, p->ws_bytes);
        return spmv_csr_run_tiled_hot(d, p->ptr, col, p->val, x, y, H, p->hot, p->own_lo, p->ws, p->ws_bytes);
    case P_ELL:
        return spmv_ell_run(d, p->K, p->ld, p->ki, p->col, p->val, x, y);
    case P_ELL_XWIN:
        return spmv_ell_run_xwin(d, p->K, p->ld, p->ki, p->col, p->val, x, y, p->win, p->xcap);
    case P_SELL:
        return spmv_sell_run(d, p->C, p->sigma, p->ki, p->n_slices, p->ptr, p->perm, p->col, p->val, x, y);
    case P_SELL_XWIN:
        return spmv_sell_run_xwin(d, p->C, p->sigma, p->ki, p->n_slices, p->ptr, p->perm, p->col, p->val, x, y,
                                  p->win, p->xcap);
    case P_SELL_XWIN_HEAD:
        return spmv_sell_run_xwin_head(d, p->C, p->sigma, p->ki, p->n_slices, p->ptr, p->perm, p->col, p->val, x, y,
                                       p->win, p->xcap, p->head);
    case P_SELL_SPLIT:
        return spmv_sell_run_split(d, p->C, p->sigma, p->ki, p->n_slices, p->ptr, p->perm, p->col, p->val, x, y,
                                   p->win, p->xcap, p->split_T, p->n_chunks, p->chunk_slice, p->chunk_k0, p->ws,
                                   p->ws_bytes);
    case P_SELL_HOT:
        return spmv_sell_run_hot(d, p->C, p->sigma, p->ki, p->n_slices, p->ptr, p->perm, col, p->val, x, y,
                                 p->split_T > 0 ? p->split_T : INT32_MAX, p->split_T > 0 ? p->n_chunks : 0,
                                 p->chunk_slice, p->chunk_k0, H, p->hot, p->ws, p->ws_bytes);
    case P_SELL16:
        return spmv_sell16_run(d, p->C, p->sigma, p->ki, p->n_slices, p->ptr, p->perm, p->col16, p->val, x, y, p->win,
                               p->xcap, p->head);
    case P_CMRS:
        return spmv_cmrs_run(d, p->h, p->n_strips, p->ptr, p->rin, p->col, p->val, x, y);
    case P_CMRS_XWIN:
        return spmv_cmrs_run_xwin(d, p->h, p->n_strips, p->ptr, p->rin, p->col, p->val, x, y, p->win, p->xcap);
    case P_CMRS_TILED:
        if (p->tiles_planned) {
            SPMV_GUARD(d);
            return cmrs_tiled_planned(d, p->h, p->n_strips, p->ptr, p->rin, col, p->val, x, y, H, p->hot, p->ws,
                                      false);
        }
        return spmv_cmrs_run_tiled_hot(d, p->h, p->n_strips, p->ptr, p->rin, col, p->val, x, y, H, p->hot, p->ws,
                                       p->ws_bytes);
    }
    return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_run: corrupt plan");
}

int spmv_plan_get_info(const spmv_plan *p, spmv_plan_info *info)
{
    if (!p || !info)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_plan_get_info: NULL argument");
    memset(info, 0, sizeof *info);
    info->format = p->fmt;
    info->path = p->path;
    info->lanes = p->lanes;
    info->variant = p->variant;
    info->ki = p->ki;
    info->xcap = p->xcap;
    info->xwin = p->win != nullptr;
    info->head = p->head != nullptr;
    info->single_pass = p->path == P_COO_TAIL;
    info->index16 = p->path == P_SELL16;
    info->split_T = p->split_T;
    info->n_chunks = p->n_chunks;
    info->big_tiles = p->big_tiles;
    info->head_bytes = (int64_t)p->head_bytes;
    info->ws_bytes = (int64_t)p->ws_bytes;
    info->owned_bytes = (int64_t)p->owned;
    info->H = p->H;
    snprintf(info->kernel, sizeof info->kernel, "%s", p->kernel);
    snprintf(info->desc, sizeof info->desc, "%s", p->desc);
    return SPMV_SUCCESS;
}

}  // extern "C"
