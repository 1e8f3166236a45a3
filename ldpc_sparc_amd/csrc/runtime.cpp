// Runtime entry points of the C ABI: errors, devices, streams, memory, events.
#include <mutex>
#include <vector>

#include "common.hpp"

namespace sg {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

static std::mutex g_mu;
static std::vector<hipStream_t> g_streams;
static std::vector<int> g_cus;

int ensure_device() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return fail(SG_ERR_NO_DEVICE,
                    "no GPU visible to the HIP runtime (%s); libldpc_sparc_amd has no CPU path",
                    e == hipSuccess ? "0 devices" : hipGetErrorString(e));
    return SG_OK;
}

static int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess)
        return -1;
    return d;
}

hipStream_t lib_stream() {
    int d = current_device();
    if (d < 0)
        return nullptr;
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_streams.size() <= d)
        g_streams.resize(d + 1, nullptr);
    if (!g_streams[d]) {
        hipStream_t s;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
            return nullptr;
        g_streams[d] = s;
    }
    return g_streams[d];
}

int device_cu_count() {
    int d = current_device();
    if (d < 0)
        return 256;
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_cus.size() <= d)
        g_cus.resize(d + 1, 0);
    if (!g_cus[d]) {
        int cu = 0;
        if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || cu <= 0)
            cu = 256;
        g_cus[d] = cu;
    }
    return g_cus[d];
}

// ---------------------------------------------------------------- profiling
struct ProfRec {
    int phase;
    hipEvent_t a, b;
};
static bool g_prof_on = false;
static int g_prof_level = 1;  // 2: the per-iteration scope only (no per-kernel events inside it)
static std::vector<ProfRec> g_prof_pending;
static std::vector<hipEvent_t> g_ev_pool;
static double g_prof_ms[SG_PH_COUNT] = {0};
static int64_t g_prof_n[SG_PH_COUNT] = {0};

static hipEvent_t ev_get() {
    if (!g_ev_pool.empty()) {
        hipEvent_t e = g_ev_pool.back();
        g_ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// the split engine's per-kernel scopes, nested in its per-iteration scope (SG_PH_AMP_CW)
static bool prof_inner(int phase) {
    return phase == SG_PH_CW2_AB || phase == SG_PH_CW2_AZ || phase == SG_PH_CW2_CTRL;
}

int prof_begin(int phase, hipStream_t s) {
    if (!g_prof_on || (g_prof_level >= 2 && prof_inner(phase))) return -1;
    std::lock_guard<std::mutex> lk(g_mu);
    ProfRec r{phase, ev_get(), ev_get()};
    if (!r.a || !r.b) return -1;
    hipEventRecord(r.a, s);
    g_prof_pending.push_back(r);
    return (int)g_prof_pending.size() - 1;
}

void prof_end(int tok, hipStream_t s) {
    if (tok < 0) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (tok < (int)g_prof_pending.size()) hipEventRecord(g_prof_pending[tok].b, s);
}

}  // namespace sg

using namespace sg;

extern "C" {

const char *sg_last_error(void) { return g_err.c_str(); }
const char *sg_version(void) { return "ldpc_sparc_amd 0.1 (gfx950)"; }

int sg_device_count(int *count) {
    SG_CHECK_ARG(count, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = (e == hipSuccess) ? n : 0;
    return SG_OK;
}

int sg_device_cu_count(int *cus) {
    SG_CHECK_ARG(cus, "cus is NULL");
    SG_TRY(sg::ensure_device());
    *cus = sg::device_cu_count();
    return SG_OK;
}

int sg_set_device(int device) {
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(device));
    return SG_OK;
}

int sg_get_stream(void **stream) {
    SG_CHECK_ARG(stream, "stream is NULL");
    SG_TRY(ensure_device());
    *stream = (void *)lib_stream();
    return *stream ? SG_OK : fail(SG_ERR_HIP, "could not create the library stream");
}

int sg_malloc(void **dptr, size_t bytes) {
    SG_CHECK_ARG(dptr, "dptr is NULL");
    SG_TRY(ensure_device());
    *dptr = nullptr;
    SG_HIP(hipMalloc(dptr, bytes ? bytes : 1));
    return SG_OK;
}

int sg_free(void *dptr) {
    if (!dptr)
        return SG_OK;
    SG_HIP(hipFree(dptr));
    return SG_OK;
}

int sg_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    SG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

int sg_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    SG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

int sg_memset(void *dptr, int value, size_t bytes, void *stream) {
    SG_TRY(ensure_device());
    SG_HIP(hipMemsetAsync(dptr, value, bytes, pick_stream(stream)));
    return SG_OK;
}

int sg_stream_synchronize(void *stream) {
    SG_TRY(ensure_device());
    SG_HIP(hipStreamSynchronize(pick_stream(stream)));
    return SG_OK;
}

int sg_stream_create(void **stream) {
    SG_CHECK_ARG(stream, "null argument");
    SG_TRY(ensure_device());
    hipStream_t s = nullptr;
    SG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return SG_OK;
}

int sg_stream_destroy(void *stream) {
    if (stream) SG_HIP(hipStreamDestroy((hipStream_t)stream));
    return SG_OK;
}

int sg_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_prof_on = on != 0;
    g_prof_level = on;
    return SG_OK;
}

int sg_profile_collect(double *total_ms, int64_t *launches) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto &r : g_prof_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess &&
            r.phase >= 0 && r.phase < SG_PH_COUNT) {
            g_prof_ms[r.phase] += ms;
            g_prof_n[r.phase] += 1;
        }
        g_ev_pool.push_back(r.a);
        g_ev_pool.push_back(r.b);
    }
    g_prof_pending.clear();
    for (int i = 0; i < SG_PH_COUNT; ++i) {
        if (total_ms) total_ms[i] = g_prof_ms[i];
        if (launches) launches[i] = g_prof_n[i];
        g_prof_ms[i] = 0.0;
        g_prof_n[i] = 0;
    }
    return SG_OK;
}

const char *sg_phase_name(int phase) {
    static const char *names[SG_PH_COUNT] = {"ab_passA", "ab_passB", "az_passA", "az_passB", "eta",
                                             "control", "bp_flood", "dense_gemm", "amp_iter", "cw2_ab", "cw2_az",
                                             "cw2_ctrl"};
    return (phase >= 0 && phase < SG_PH_COUNT) ? names[phase] : "unknown";
}

int sg_device_synchronize(void) {
    SG_TRY(ensure_device());
    SG_HIP(hipDeviceSynchronize());
    return SG_OK;
}

int sg_event_create(void **ev) {
    SG_CHECK_ARG(ev, "ev is NULL");
    SG_TRY(ensure_device());
    hipEvent_t e;
    SG_HIP(hipEventCreate(&e));
    *ev = (void *)e;
    return SG_OK;
}

int sg_event_destroy(void *ev) {
    if (ev)
        SG_HIP(hipEventDestroy((hipEvent_t)ev));
    return SG_OK;
}

int sg_event_record(void *ev, void *stream) {
    SG_HIP(hipEventRecord((hipEvent_t)ev, pick_stream(stream)));
    return SG_OK;
}

int sg_event_elapsed_ms(void *start, void *stop, float *ms) {
    SG_HIP(hipEventSynchronize((hipEvent_t)stop));
    SG_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return SG_OK;
}

}  // extern "C"
