// Shared host-side plumbing for libldpc_sparc_amd.so: error reporting across
// the C ABI, per-device library streams, checked HIP calls.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/ldpc_sparc_amd.h"

namespace sg {

void set_error(const char *fmt, ...);
int fail(int code, const char *fmt, ...);

// Ensures a device is present and selected; returns SG_OK or SG_ERR_NO_DEVICE.
int ensure_device();
hipStream_t lib_stream();
inline hipStream_t pick_stream(void *s) { return s ? reinterpret_cast<hipStream_t>(s) : lib_stream(); }
int device_cu_count();

// Per-phase device timing (sg_profile_enable): HIP events recorded on the
// stream a phase is launched on, resolved by sg_profile_collect.
int prof_begin(int phase, hipStream_t s);
void prof_end(int token, hipStream_t s);
struct ProfScope {
    int tok;
    hipStream_t s;
    ProfScope(int phase, hipStream_t st) : tok(prof_begin(phase, st)), s(st) {}
    ~ProfScope() { prof_end(tok, s); }
};

struct HipError {
    hipError_t err;
    const char *what;
};

}  // namespace sg

#define SG_HIP(call)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ::sg::fail(e_ == hipErrorOutOfMemory ? SG_ERR_NOMEM : SG_ERR_HIP,        \
                              "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),        \
                              __FILE__, __LINE__);                                          \
    } while (0)

#define SG_CHECK_ARG(cond, ...)                                                             \
    do {                                                                                    \
        if (!(cond))                                                                        \
            return ::sg::fail(SG_ERR_INVALID, __VA_ARGS__);                                 \
    } while (0)

#define SG_TRY(expr)                                                                        \
    do {                                                                                    \
        int r_ = (expr);                                                                    \
        if (r_ != SG_OK)                                                                    \
            return r_;                                                                      \
    } while (0)
