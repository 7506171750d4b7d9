// Shared host/device helpers for libpulsarutils_hip (gfx950).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "pulsarutils_hip.h"

namespace pu {

void set_error(const char *fmt, ...);

// Map a HIP status to PU_EHIP with a message; returns PU_OK on success.
inline int hip_check(hipError_t e, const char *what)
{
    if (e == hipSuccess) return PU_OK;
    set_error("%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? PU_ENOMEM : PU_EHIP;
}

#define PU_TRY_HIP(expr)                                  \
    do {                                                  \
        int _rc = ::pu::hip_check((expr), #expr);         \
        if (_rc != PU_OK) return _rc;                     \
    } while (0)

#define PU_REQUIRE(cond, ...)                             \
    do {                                                  \
        if (!(cond)) {                                    \
            ::pu::set_error(__VA_ARGS__);                 \
            return PU_EINVAL;                             \
        }                                                 \
    } while (0)

// Launch-error check after a kernel launch.
inline int launch_check(const char *name)
{
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) return PU_OK;
    set_error("launch %s: %s", name, hipGetErrorString(e));
    return PU_EHIP;
}

inline size_t elem_size(int dtype)
{
    switch (dtype) {
    case PU_U8: return 1;
    case PU_F32: return 4;
    case PU_F64: return 8;
    case PU_I64: return 8;
    default: return 0;
    }
}

// Tuning knobs for A/B experiments (group size, workgroup shape, batch sizes ...): read
// from the environment ONLY in the diagnostic build (make stamps: -DPU_STAMPS,
// libpulsarutils_hip_stamps.so).  The production library ignores the environment and
// always runs its defaults or the explicit plan-create arguments, so a stray PU_* in a
// user's environment cannot change a kernel (the reference is configured by kwargs only).
inline bool knob_set(const char *name)
{
#ifdef PU_STAMPS
    return getenv(name) != nullptr;
#else
    (void)name;
    return false;
#endif
}

inline int knob(const char *name, int dflt)
{
#ifdef PU_STAMPS
    if (const char *e = getenv(name)) return atoi(e);
#endif
    (void)name;
    return dflt;
}

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical ids land on one XCD (blocks b, b+8 share one).
__device__ __forceinline__ int xcd_remap(int bid, int nblk)
{
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

}  // namespace pu
