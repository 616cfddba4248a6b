// multi.hip — single-process multi-GPU layer of the C-ABI (include/spmv.h
// "multi-GPU"): one RCCL communicator and one stream per device, the y
// all-gather of row shards as grouped broadcasts of the real shard sizes,
// and a timer that brackets one launch per device with events.
//
// The reference builds its OpenCL context over every GPU it finds and then
// uses device 0 only (reference csr.c:107,115, the device loop breaks after
// the first device, csr.c:30,279); there is no collective anywhere in it.
// This layer is the suite's own (SURVEY.md §5 "Distributed comm backend",
// §8e): rows shard across the GPUs of one node, x is replicated, and the
// only exchange is y, over xGMI.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>

#include "common.h"

struct spmv_multi {
    int n;
    int dev[64];
    ncclComm_t comm[64];
    hipStream_t stream[64];
    hipEvent_t ev0[64], ev1[64];
};

namespace spmv {

// RCCL is opened on first use (RTLD_LOCAL), not linked: a process that
// already carries another librccl (PyTorch ships its own) would otherwise
// have two copies interposing each other's symbols, and their exit-time
// destructors free the same objects twice.  Programs that never call
// spmv_multi_* never load it.
struct Rccl {
    bool ok = false;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

static const Rccl &rccl()
{
    static const Rccl r = [] {
        Rccl t;
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr)
                break;
        if (!h)
            return t;
        t.comm_init_all = (decltype(t.comm_init_all))dlsym(h, "ncclCommInitAll");
        t.comm_destroy = (decltype(t.comm_destroy))dlsym(h, "ncclCommDestroy");
        t.broadcast = (decltype(t.broadcast))dlsym(h, "ncclBroadcast");
        t.group_start = (decltype(t.group_start))dlsym(h, "ncclGroupStart");
        t.group_end = (decltype(t.group_end))dlsym(h, "ncclGroupEnd");
        t.error_string = (decltype(t.error_string))dlsym(h, "ncclGetErrorString");
        t.ok = t.comm_init_all && t.comm_destroy && t.broadcast && t.group_start && t.group_end && t.error_string;
        return t;
    }();
    return r;
}

static int nccl_fail(const char *where, ncclResult_t r)
{
    static thread_local char msg[256];
    snprintf(msg, sizeof msg, "%s: %s", where, rccl().error_string(r));
    return fail_msg(r == ncclInvalidArgument || r == ncclInvalidUsage ? SPMV_OTHER_ERROR : SPMV_DEVICE_ERROR, msg);
}

}  // namespace spmv

using namespace spmv;

extern "C" {

int spmv_multi_init(int n_gpus, const int *devices, spmv_multi **out)
{
    if (!out || n_gpus < 1 || n_gpus > 64)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_multi_init: 1..64 devices");
    *out = nullptr;
    if (!rccl().ok)
        return fail_msg(SPMV_DEVICE_ERROR, "spmv_multi_init: librccl.so.1 not found");
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess)
        return fail(SPMV_DEVICE_ERROR, "hipGetDeviceCount", e);
    spmv_multi *m = (spmv_multi *)calloc(1, sizeof(spmv_multi));
    if (!m)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_multi_init: out of host memory");
    m->n = n_gpus;
    for (int i = 0; i < n_gpus; ++i) {
        m->dev[i] = devices ? devices[i] : i;
        if (m->dev[i] < 0 || m->dev[i] >= count) {
            free(m);
            return fail_msg(SPMV_DEVICE_ERROR, "spmv_multi_init: no such device");
        }
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    int rc = SPMV_SUCCESS;
    for (int i = 0; i < n_gpus && rc == SPMV_SUCCESS; ++i) {
        if ((e = hipSetDevice(m->dev[i])) != hipSuccess ||
            (e = hipStreamCreateWithFlags(&m->stream[i], hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreate(&m->ev0[i])) != hipSuccess || (e = hipEventCreate(&m->ev1[i])) != hipSuccess)
            rc = fail(SPMV_DEVICE_ERROR, "spmv_multi_init: stream/events", e);
    }
    if (rc == SPMV_SUCCESS) {
        const ncclResult_t r = rccl().comm_init_all(m->comm, n_gpus, m->dev);
        if (r != ncclSuccess)
            rc = nccl_fail("ncclCommInitAll", r);
    }
    (void)hipSetDevice(prev);
    if (rc != SPMV_SUCCESS) {
        spmv_multi_free(m);
        return rc;
    }
    *out = m;
    return SPMV_SUCCESS;
}

int spmv_multi_free(spmv_multi *m)
{
    if (!m)
        return SPMV_SUCCESS;
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (int i = 0; i < m->n; ++i) {
        if (m->comm[i])
            (void)rccl().comm_destroy(m->comm[i]);
        (void)hipSetDevice(m->dev[i]);
        if (m->ev0[i])
            (void)hipEventDestroy(m->ev0[i]);
        if (m->ev1[i])
            (void)hipEventDestroy(m->ev1[i]);
        if (m->stream[i])
            (void)hipStreamDestroy(m->stream[i]);
    }
    (void)hipSetDevice(prev);
    free(m);
    return SPMV_SUCCESS;
}

int spmv_multi_size(const spmv_multi *m) { return m ? m->n : 0; }
int spmv_multi_device(const spmv_multi *m, int i) { return m && i >= 0 && i < m->n ? m->dev[i] : -1; }
void *spmv_multi_stream(const spmv_multi *m, int i) { return m && i >= 0 && i < m->n ? (void *)m->stream[i] : nullptr; }

int spmv_multi_allgatherv(spmv_multi *m, double *const *y_full, const int64_t *bounds)
{
    if (!m || !y_full || !bounds)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_multi_allgatherv: bad arguments");
    for (int r = 0; r < m->n; ++r)
        if (bounds[r] < 0 || bounds[r + 1] < bounds[r])
            return fail_msg(SPMV_OTHER_ERROR, "spmv_multi_allgatherv: bounds must be non-decreasing");
    ncclResult_t r = rccl().group_start();
    if (r != ncclSuccess)
        return nccl_fail("ncclGroupStart", r);
    // every device takes part in every shard's broadcast: the owner sends
    // y_full[root] + bounds[root] (in place), the others receive into the
    // same rows of their own y_full
    for (int root = 0; root < m->n && r == ncclSuccess; ++root) {
        const size_t count = (size_t)(bounds[root + 1] - bounds[root]);
        if (count == 0)
            continue;
        for (int i = 0; i < m->n && r == ncclSuccess; ++i) {
            double *p = y_full[i] + bounds[root];
            r = rccl().broadcast(p, p, count, ncclDouble, root, m->comm[i], m->stream[i]);
        }
    }
    const ncclResult_t r2 = rccl().group_end();
    if (r != ncclSuccess)
        return nccl_fail("ncclBroadcast", r);
    if (r2 != ncclSuccess)
        return nccl_fail("ncclGroupEnd", r2);
    return SPMV_SUCCESS;
}

int spmv_multi_sync(spmv_multi *m)
{
    if (!m)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_multi_sync: NULL");
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (int i = 0; i < m->n; ++i) {
        hipError_t e = hipSetDevice(m->dev[i]);
        if (e == hipSuccess)
            e = hipStreamSynchronize(m->stream[i]);
        if (e != hipSuccess) {
            (void)hipSetDevice(prev);
            return fail(SPMV_PROGRAM_ERROR, "spmv_multi_sync", e);
        }
    }
    (void)hipSetDevice(prev);
    return SPMV_SUCCESS;
}

int spmv_multi_time(spmv_multi *m, spmv_multi_launch_fn launch, void *arg, int flush, double *ms)
{
    if (!m || !launch || !ms)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_multi_time: bad arguments");
    int prev = 0;
    (void)hipGetDevice(&prev);
    int rc = SPMV_SUCCESS;
    for (int i = 0; i < m->n && rc == SPMV_SUCCESS; ++i) {
        hipError_t e = hipSetDevice(m->dev[i]);
        if (e != hipSuccess) {
            rc = fail(SPMV_DEVICE_ERROR, "spmv_multi_time: hipSetDevice", e);
            break;
        }
        if (flush && (rc = spmv_flush_cache(m->stream[i], 0)) != SPMV_SUCCESS)
            break;
        if ((e = hipEventRecord(m->ev0[i], m->stream[i])) != hipSuccess) {
            rc = fail(SPMV_PROGRAM_ERROR, "spmv_multi_time: event", e);
            break;
        }
    }
    // every device's flush is queued before the first launch, so the
    // launches start together
    for (int i = 0; i < m->n && rc == SPMV_SUCCESS; ++i) {
        (void)hipSetDevice(m->dev[i]);
        rc = launch(arg, i);
        const hipError_t e = hipEventRecord(m->ev1[i], m->stream[i]);
        if (rc == SPMV_SUCCESS && e != hipSuccess)
            rc = fail(SPMV_PROGRAM_ERROR, "spmv_multi_time: event", e);
    }
    for (int i = 0; i < m->n && rc == SPMV_SUCCESS; ++i) {
        (void)hipSetDevice(m->dev[i]);
        float f = 0.f;
        hipError_t e = hipEventSynchronize(m->ev1[i]);
        if (e == hipSuccess)
            e = hipEventElapsedTime(&f, m->ev0[i], m->ev1[i]);
        if (e != hipSuccess)
            rc = fail(SPMV_PROGRAM_ERROR, "spmv_multi_time: elapsed", e);
        ms[i] = (double)f;
    }
    (void)hipSetDevice(prev);
    return rc;
}

}  // extern "C"
