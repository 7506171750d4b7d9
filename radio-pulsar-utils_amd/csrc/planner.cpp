// Host planner + error state of libpulsarutils_hip.  Compiled by g++ (not hipcc) with
// -ffp-contract=off so the float64 arithmetic is plain IEEE libm, like CPython.
//
// pu_shift_table restates dedispersion_shifts (pulsarutils/dedispersion.py:125-139)
// with CPython scalar semantics: ``x ** (-2)`` -> libm pow, ``a // b`` -> the
// fmod-based divmod with a snapped quotient (CPython float_floor_div ==
// numpy npy_floor_divide), ``int(np.rint(q))`` -> nearbyint in round-half-even mode.
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "pulsarutils_hip.h"

namespace pu {

static thread_local std::string g_err;

void set_error(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

// keep pow(x, -2) an actual libm call (no x^-2 -> 1/(x*x) rewrite)
static volatile double kMinusTwo = -2.0;

static double py_floordiv(double a, double b)
{
    if (b == 0.0) return a / b;
    double mod = std::fmod(a, b);
    double div = (a - mod) / b;
    if (mod != 0.0 && ((b < 0) != (mod < 0))) div -= 1.0;
    if (div != 0.0) {
        double fl = std::floor(div);
        if (div - fl > 0.5) fl += 1.0;
        return fl;
    }
    return std::copysign(0.0, a / b);
}

}  // namespace pu

extern "C" {

const char *pu_version(void) { return "pulsarutils-hip 0.1.0 gfx950"; }

const char *pu_last_error(void) { return pu::g_err.c_str(); }

int pu_shift_table(int64_t nchan, const double *dms, int64_t ndm, double start_freq,
                   double bandwidth, double sample_time, int64_t *out)
{
    if (nchan <= 0 || ndm < 0 || (!dms && ndm) || (!out && ndm)) {
        pu::set_error("pu_shift_table: invalid arguments");
        return PU_EINVAL;
    }
    const double dfreq = bandwidth / (double)nchan;
    const double stop = start_freq + bandwidth;
    const double center = (stop + start_freq) / 2.0;
    const double pc = std::pow(center, pu::kMinusTwo);
    // chan_freq ** -2 does not depend on the DM: hoist it
    double *pf = new double[(size_t)nchan];
    for (int64_t i = 0; i < nchan; ++i) pf[i] = std::pow(start_freq + (double)i * dfreq, pu::kMinusTwo);
    int rc = PU_OK;
    for (int64_t d = 0; d < ndm && rc == PU_OK; ++d) {
        const double k = 4149.0 * dms[d];
        const double ref = k * pc;
        int64_t *o = out + d * nchan;
        for (int64_t i = 0; i < nchan; ++i) {
            const double q = pu::py_floordiv(k * pf[i] - ref, sample_time);
            if (!std::isfinite(q) || std::fabs(q) > 9.0e18) {
                pu::set_error("pu_shift_table: non-finite or huge delay at trial %lld", (long long)d);
                rc = PU_EINVAL;
                break;
            }
            o[i] = (int64_t)std::nearbyint(q);
        }
    }
    delete[] pf;
    return rc;
}

}  // extern "C"
