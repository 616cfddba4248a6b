// runtime.hip — device discovery, memory, timing and error plumbing of the
// C-ABI (include/spmv.h).  Replaces the reference's OpenCL platform/device
// discovery (reference inc/helper_functions.h:76-129), buffer creation and
// transfers (reference csr.c:107-133,183-193,220) and its host wall clock
// around one launch (reference csr.c:198-206).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "common.h"

namespace spmv {

static thread_local char g_last_error[512] = "";

int fail(int rc, const char *where, hipError_t e)
{
    snprintf(g_last_error, sizeof g_last_error, "%s: %s (%d)", where,
             hipGetErrorString(e), (int)e);
    return rc;
}

int fail_msg(int rc, const char *msg)
{
    snprintf(g_last_error, sizeof g_last_error, "%s", msg);
    return rc;
}

DeviceGuard::DeviceGuard(int dev)
{
    hipError_t e = hipGetDevice(&prev_);
    if (e != hipSuccess) {
        rc_ = fail(SPMV_DEVICE_ERROR, "hipGetDevice", e);
        prev_ = -1;
        return;
    }
    if (prev_ != dev) {
        e = hipSetDevice(dev);
        if (e != hipSuccess)
            rc_ = fail(SPMV_DEVICE_ERROR, "hipSetDevice", e);
    }
}

DeviceGuard::~DeviceGuard()
{
    int cur = -1;
    if (prev_ >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev_)
        (void)hipSetDevice(prev_);
}

// The A/B switches (spmv_ext.h spmv_set_option): read from the
// environment ONCE, when the library is loaded, then only through
// spmv_set_option; the launch path reads one int, never getenv (VERDICT r5:
// hidden global configuration behind a C-ABI).  -1 = each kernel's default.
static int env_switch(const char *name)
{
    const char *s = getenv(name);
    return (s && (s[0] == '0' || s[0] == '1') && s[1] == 0) ? s[0] - '0' : -1;
}
static std::atomic<int> g_opt_xwin_remap{env_switch("SPMV_XWIN_REMAP")};
static std::atomic<int> g_opt_xcd_remap{env_switch("SPMV_XCD_REMAP")};
static std::atomic<int> g_opt_stream_nt{env_switch("SPMV_STREAM_NT")};
static std::atomic<int> g_opt_csr_prefetch{env_switch("SPMV_CSR_PREFETCH")};

static std::atomic<int> *option_slot(int option)
{
    switch (option) {
    case SPMV_OPT_XWIN_REMAP:
        return &g_opt_xwin_remap;
    case SPMV_OPT_XCD_REMAP:
        return &g_opt_xcd_remap;
    case SPMV_OPT_STREAM_NT:
        return &g_opt_stream_nt;
    case SPMV_OPT_CSR_PREFETCH:
        return &g_opt_csr_prefetch;
    default:
        return nullptr;
    }
}

bool xwin_remap(bool dflt)
{
    const int v = g_opt_xwin_remap.load(std::memory_order_relaxed);
    return v < 0 ? dflt : v == 1;
}

// Off by default: on the cant-like batch the round-robin placement
// measured 1-2 % faster than the contiguous-per-XCD remap
// (profiles/round1/sweeps.md).
bool xcd_remap_enabled() { return g_opt_xcd_remap.load(std::memory_order_relaxed) == 1; }

bool csr_prefetch(bool dflt)
{
    const int v = g_opt_csr_prefetch.load(std::memory_order_relaxed);
    return v < 0 ? dflt : v == 1;
}

bool stream_nt(bool dflt)
{
    const int v = g_opt_stream_nt.load(std::memory_order_relaxed);
    return v < 0 ? dflt : v == 1;
}

// One flush buffer per device, allocated on first use, freed by
// spmv_release().
static void *g_flush[64];
static size_t g_flush_bytes[64];

// evicts by READING the scratch: 16-byte loads, a value that is never true
// keeps them (the caches end up holding clean lines of the scratch)
__global__ __launch_bounds__(kBlock) void flush_read_kernel(const uint4 *__restrict__ p, int64_t n16,
                                                            uint32_t *__restrict__ sink)
{
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += (int64_t)gridDim.x * kBlock) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u && sink)
        sink[threadIdx.x] = acc;
}

// the device's scratch of at least `bytes` (allocated / grown on demand)
static int flush_scratch(size_t bytes, void **buf)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess)
        return fail(SPMV_DEVICE_ERROR, "hipGetDevice", e);
    if (dev < 0 || dev >= 64)
        return fail_msg(SPMV_DEVICE_ERROR, "device ordinal out of range");
    if (g_flush_bytes[dev] < bytes) {
        if (g_flush[dev])
            (void)hipFree(g_flush[dev]);
        g_flush[dev] = nullptr;
        g_flush_bytes[dev] = 0;
        e = hipMalloc(&g_flush[dev], bytes);
        if (e != hipSuccess)
            return fail(SPMV_PROGRAM_ERROR, "hipMalloc(flush)", e);
        g_flush_bytes[dev] = bytes;
    }
    *buf = g_flush[dev];
    return SPMV_SUCCESS;
}

}  // namespace spmv

using namespace spmv;

extern "C" {

const char *spmv_last_error(void) { return g_last_error; }

const char *spmv_strerror(int rc)
{
    switch (rc) {
    case SPMV_SUCCESS:
        return "success";
    case SPMV_DEVICE_ERROR:
        return "device error";
    case SPMV_PROGRAM_ERROR:
        return "launch/copy error";
    case SPMV_FILE_ERROR:
        return "file error";
    case SPMV_OTHER_ERROR:
        return "invalid argument";
    default:
        return "unknown error";
    }
}

const char *spmv_version(void) { return "spmv-hip 0.2 gfx950"; }

int spmv_set_option(int option, int value)
{
    std::atomic<int> *o = option_slot(option);
    if (!o || value < -1 || value > 1)
        return fail_msg(SPMV_OTHER_ERROR, "spmv_set_option: unknown option or value (-1, 0, 1)");
    o->store(value, std::memory_order_relaxed);
    return SPMV_SUCCESS;
}

int spmv_get_option(int option)
{
    std::atomic<int> *o = option_slot(option);
    return o ? o->load(std::memory_order_relaxed) : -2;
}

int spmv_device_count(int *count)
{
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return fail(SPMV_DEVICE_ERROR, "hipGetDeviceCount", e);
    }
    return *count > 0 ? SPMV_SUCCESS
                      : fail_msg(SPMV_DEVICE_ERROR, "no HIP device found");
}

int spmv_set_device(int device)
{
    hipError_t e = hipSetDevice(device);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_DEVICE_ERROR, "hipSetDevice", e);
}

int spmv_device_name(int device, char *buf, size_t len)
{
    hipDeviceProp_t p;
    hipError_t e = hipGetDeviceProperties(&p, device);
    if (e != hipSuccess)
        return fail(SPMV_DEVICE_ERROR, "hipGetDeviceProperties", e);
    snprintf(buf, len, "%s (%s, %d CUs)", p.name, p.gcnArchName,
             p.multiProcessorCount);
    return SPMV_SUCCESS;
}

int spmv_malloc(void **dptr, size_t bytes)
{
    *dptr = nullptr;
    if (bytes == 0)
        bytes = 16;  // keep a valid, distinct pointer for empty arrays
    hipError_t e = hipMalloc(dptr, bytes);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "hipMalloc", e);
}

int spmv_free(void *dptr)
{
    if (!dptr)
        return SPMV_SUCCESS;
    hipError_t e = hipFree(dptr);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "hipFree", e);
}

int spmv_memset(void *dptr, int value, size_t bytes, void *stream)
{
    if (bytes == 0)
        return SPMV_SUCCESS;
    hipError_t e = hipMemsetAsync(dptr, value, bytes, (hipStream_t)stream);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "hipMemsetAsync", e);
}

int spmv_upload(void *dptr, const void *host, size_t bytes, void *stream)
{
    if (bytes == 0)
        return SPMV_SUCCESS;
    hipError_t e = hipMemcpyAsync(dptr, host, bytes, hipMemcpyHostToDevice,
                                  (hipStream_t)stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "upload", e);
}

int spmv_download(void *host, const void *dptr, size_t bytes, void *stream)
{
    if (bytes == 0)
        return SPMV_SUCCESS;
    hipError_t e = hipMemcpyAsync(host, dptr, bytes, hipMemcpyDeviceToHost,
                                  (hipStream_t)stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "download", e);
}

int spmv_stream_create(void **stream)
{
    hipStream_t s;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    *stream = (void *)s;
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "hipStreamCreate", e);
}

int spmv_stream_destroy(void *stream)
{
    hipError_t e = hipStreamDestroy((hipStream_t)stream);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "hipStreamDestroy", e);
}

int spmv_sync(void *stream)
{
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "hipStreamSynchronize", e);
}

int spmv_flush_cache(void *stream, size_t bytes)
{
    if (bytes == 0)
        bytes = (size_t)512 << 20;
    void *buf = nullptr;
    int rc = flush_scratch(bytes, &buf);
    if (rc != SPMV_SUCCESS)
        return rc;
    static unsigned char tick = 0;
    hipError_t e = hipMemsetAsync(buf, ++tick, bytes, (hipStream_t)stream);
    return e == hipSuccess ? SPMV_SUCCESS
                           : fail(SPMV_PROGRAM_ERROR, "flush", e);
}

int spmv_flush_cache_read(void *stream, size_t bytes)
{
    if (bytes == 0)
        bytes = (size_t)512 << 20;
    void *buf = nullptr;
    int rc = flush_scratch(bytes, &buf);
    if (rc != SPMV_SUCCESS)
        return rc;
    hipLaunchKernelGGL(flush_read_kernel, dim3(2048), dim3(kBlock), 0, (hipStream_t)stream, (const uint4 *)buf,
                       (int64_t)(bytes / 16), (uint32_t *)nullptr);
    SPMV_CHECK_LAUNCH("flush_read_kernel");
    return SPMV_SUCCESS;
}

int spmv_event_create(void **ev)
{
    hipEvent_t e0;
    hipError_t e = hipEventCreate(&e0);
    *ev = e == hipSuccess ? (void *)e0 : nullptr;
    return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "hipEventCreate", e);
}

int spmv_event_destroy(void *ev)
{
    if (!ev)
        return SPMV_SUCCESS;
    hipError_t e = hipEventDestroy((hipEvent_t)ev);
    return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "hipEventDestroy", e);
}

int spmv_event_record(void *ev, void *stream)
{
    hipError_t e = hipEventRecord((hipEvent_t)ev, (hipStream_t)stream);
    return e == hipSuccess ? SPMV_SUCCESS : fail(SPMV_PROGRAM_ERROR, "hipEventRecord", e);
}

int spmv_event_elapsed(void *start, void *end, double *ms)
{
    hipError_t e = hipEventSynchronize((hipEvent_t)end);
    float f = 0.f;
    if (e == hipSuccess)
        e = hipEventElapsedTime(&f, (hipEvent_t)start, (hipEvent_t)end);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "event timing", e);
    *ms = (double)f;
    return SPMV_SUCCESS;
}

int spmv_time_launch(spmv_launch_fn launch, void *arg, void *stream, double *ms)
{
    hipEvent_t a, b;
    hipError_t e = hipEventCreate(&a);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "hipEventCreate", e);
    e = hipEventCreate(&b);
    if (e != hipSuccess) {
        (void)hipEventDestroy(a);
        return fail(SPMV_PROGRAM_ERROR, "hipEventCreate", e);
    }
    int rc = SPMV_SUCCESS;
    e = hipEventRecord(a, (hipStream_t)stream);
    if (e == hipSuccess) {
        rc = launch(arg);
        e = hipEventRecord(b, (hipStream_t)stream);
    }
    if (e == hipSuccess)
        e = hipEventSynchronize(b);
    float f = 0.f;
    if (e == hipSuccess)
        e = hipEventElapsedTime(&f, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (e != hipSuccess)
        return fail(SPMV_PROGRAM_ERROR, "event timing", e);
    *ms = (double)f;
    return rc;
}

int spmv_release(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return SPMV_DEVICE_ERROR;
    if (g_flush[dev])
        (void)hipFree(g_flush[dev]);
    g_flush[dev] = nullptr;
    g_flush_bytes[dev] = 0;
    return SPMV_SUCCESS;
}

}  // extern "C"
