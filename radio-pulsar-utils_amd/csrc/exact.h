// Internal helpers of exact.hip used by the search's certification step (dedisperse.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pu {

// flag[0] = 1 if any element of the (nrows, n) float input is NaN or +-inf (0 for
// integer inputs).  Asynchronous on s.
int nonfinite_any_async(const void *data, int dtype, int64_t nrows, int64_t n, int64_t ld, int32_t *flag,
                        hipStream_t s);

// The reference's dedispersed series (float64, channel order: bit-identical) of ``rows``
// trials whose shifts (device, rows x nchan, each reduced to [0, n)) are given, at samples
// [t_begin, t_begin + t_len) (t_len < 0: to n) into out (rows x t_len).  A direct gather: for
// a handful of trials (certification rechecks).
int exact_series(const void *data, int dtype, int64_t nchan, int64_t n, int64_t ld, const int64_t *shifts, int64_t rows,
                 double *out, hipStream_t s, int64_t t_begin = 0, int64_t t_len = -1);

// The reference's result for every trial when the input holds a non-finite value:
// max = std = NaN, snr = 0, rebin = 0 (dedispersion.py:186-201).
int nan_rule(int64_t ndm, double *max_out, double *std_out, double *snr_out, int32_t *win_out, hipStream_t s);

}  // namespace pu
