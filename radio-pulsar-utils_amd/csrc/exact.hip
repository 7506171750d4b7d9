// The reference's per-trial statistics in numpy's exact order (gfx950).
//
// Replaces the statistics half of _dedispersion_search (pulsarutils/dedispersion.py:
// 186-201) on given float64 dedispersed series, bit for bit:
//   dedisp_shift = dedisp - np.mean(dedisp)
//   for window in 1, 2, 4, 8:
//       reb = quick_resample(dedisp_shift, window)      # (0 + s[wi]) + s[wi+1] + ...
//       snr = np.max(reb) / np.std(reb)                  # NaN-propagating max, numpy std
//       if snr > best_snr: best_snr, best_win = snr, window   (best starts at 0, 0)
//   max = np.max(dedisp_shift), std = np.std(dedisp_shift)
// Means and sums of squares go through pu_row_sums (numpy's 8192-element blocks, each
// pairwise-summed; the reductions the cleaning masks are bit-exact with), maxima through
// an order-preserving 64-bit key (NaN above everything, so a NaN anywhere gives NaN).
//
// Used by pu_plan_search for the trials its fast path cannot certify:
// degenerate series (zero or rounding-level std: constant inputs), non-finite values
// and near-ties between windows; and exported as pu_series_stats.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "exact.h"
#include "pu_common.h"

namespace {

// Order-preserving key of a double for an unsigned max: NaN (either sign) -> all ones,
// x >= +0 -> bits | sign, x <= -0 -> ~bits.  +0 sorts above -0.
__device__ __forceinline__ uint64_t max_key(double x)
{
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    if (x != x) return ~0ull;
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ double key_value(uint64_t k)
{
    if (k == ~0ull) return __longlong_as_double(0x7ff8000000000000ll);  // NaN
    const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
}

// Workgroup max of per-thread keys, one vector atomic per workgroup.
__device__ __forceinline__ void block_max_key(uint64_t k, uint64_t *dst)
{
    __shared__ uint64_t red[256];
    red[threadIdx.x] = k;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = std::max(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(reinterpret_cast<unsigned long long *>(dst), (unsigned long long)red[0]);
}

// S[r][t] = plane[r][t] - mean[r] (the reference's dedisp_shift) and its row max key.
__global__ void __launch_bounds__(256)
exact_shift_kernel(const double *__restrict__ plane, int64_t ld, int64_t n, const double *__restrict__ mean,
                   double *__restrict__ S, uint64_t *__restrict__ key)
{
    const int64_t r = blockIdx.y;
    const double m = mean[r];
    uint64_t k = 0;
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
        const double s = plane[r * ld + t] - m;
        S[r * n + t] = s;
        k = std::max(k, max_key(s));
    }
    block_max_key(k, key + r);
}

// quick_resample of S by w (dedispersion.py:53-56): R[r][i] = ((0 + S[wi]) + S[wi+1]) + ...
// and its row max key.
__global__ void __launch_bounds__(256)
exact_rebin_kernel(const double *__restrict__ S, int64_t n, int w, int64_t nb, double *__restrict__ R,
                   uint64_t *__restrict__ key)
{
    const int64_t r = blockIdx.y;
    uint64_t k = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += (int64_t)gridDim.x * 256) {
        const double *p = S + r * n + (int64_t)w * i;
        double acc = 0.0;
        for (int j = 0; j < w; ++j) acc += p[j];
        R[r * nb + i] = acc;
        k = std::max(k, max_key(acc));
    }
    block_max_key(k, key + r);
}

// Per row: snr_w = max_w / sqrt(var_w) and the reference's strict first-best rule.
__global__ void exact_final_kernel(int64_t rows, int64_t n, const uint64_t *__restrict__ keys,
                                   const double *__restrict__ var, const int32_t *__restrict__ idx,
                                   double *max_out, double *std_out, double *snr_out, int32_t *win_out)
{
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    double best = 0.0;
    int bestw = 0;
    for (int w = 0; w < 4; ++w) {
        if (n >> w == 0) continue;  // np.max of an empty array raises in the reference
        const double snr = key_value(keys[w * rows + r]) / sqrt(var[w * rows + r]);
        if (snr > best) {
            best = snr;
            bestw = 1 << w;
        }
    }
    const int64_t o = idx ? idx[r] : r;
    max_out[o] = key_value(keys[r]);
    std_out[o] = sqrt(var[r]);
    snr_out[o] = best;
    win_out[o] = bestw;
}

// The reference's dedispersed series of a few trials, directly: out[r][t] =
// ((0 + x[0][(t + s[r][0]) mod n]) + x[1][...]) + ... in float64, channel order
// (roll_and_sum's order, dedispersion.py:60-98: bit-identical).  The row shifts (in
// [0, n)) go through LDS 1024 channels at a time.  Every trial reads the whole input
// once (17 GB at C3: ~4 ms), which is why only flagged trials take this path.
//   8-bit: a thread owns 8 consecutive samples and reads them as 3 aligned dwords
//   (lanes 32 B apart: coalesced), bytes extracted by funnel shifts;
//   float: a thread owns samples t0 + l + 64 k (k < 8): every load of a wave is 64
//   consecutive elements.
constexpr int kSeriesPer = 8;

template <typename T>
__global__ void __launch_bounds__(256)
exact_series_kernel(const T *__restrict__ x, int64_t ld, int64_t nchan, int64_t n, const int64_t *__restrict__ shifts,
                    double *__restrict__ out)
{
    __shared__ int64_t sh[1024];
    const int64_t r = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // the wave's 512 samples start at w0; this thread's samples
    const int64_t w0 = ((int64_t)blockIdx.x * 4 + wave) * 64 * kSeriesPer;
    const int64_t t0 = sizeof(T) == 1 ? w0 + (int64_t)kSeriesPer * lane : w0 + lane;
    const int64_t dt = sizeof(T) == 1 ? 1 : 64;  // sample step between this thread's samples
    double acc[kSeriesPer];
#pragma unroll
    for (int k = 0; k < kSeriesPer; ++k) acc[k] = 0.0;
    for (int64_t c0 = 0; c0 < nchan; c0 += 1024) {
        const int64_t nc = nchan - c0 < 1024 ? nchan - c0 : 1024;
        __syncthreads();
        for (int64_t i = threadIdx.x; i < nc; i += 256) sh[i] = shifts[r * nchan + c0 + i];
        __syncthreads();
        if (w0 >= n) continue;
        for (int64_t ci = 0; ci < nc; ++ci) {
            const T *row = x + (c0 + ci) * ld;
            int64_t idx = t0 + sh[ci];
            if (idx >= n) idx -= n;
            if constexpr (sizeof(T) == 1) {
                const bool fast = idx + 12 <= n && t0 + kSeriesPer <= n && (reinterpret_cast<uintptr_t>(row) & 3) == 0;
                if (fast) {
                    const int64_t a = idx & ~int64_t(3);
                    const uint32_t *p = reinterpret_cast<const uint32_t *>(row + a);
                    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
                    const uint32_t sft = (uint32_t)(idx - a) * 8u;
                    // bytes idx .. idx + 7 as two dwords (funnel shift across the dwords)
                    const uint32_t lo = sft ? (d0 >> sft) | (d1 << (32u - sft)) : d0;
                    const uint32_t hi = sft ? (d1 >> sft) | (d2 << (32u - sft)) : d1;
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[k] += (double)((lo >> (8 * k)) & 0xffu);
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[4 + k] += (double)((hi >> (8 * k)) & 0xffu);
                    continue;
                }
            }
#pragma unroll
            for (int k = 0; k < kSeriesPer; ++k) {
                if (t0 + k * dt < n) acc[k] += static_cast<double>(row[idx]);
                idx += dt;
                while (idx >= n) idx -= n;  // n < 64 may wrap more than once
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kSeriesPer; ++k)
        if (t0 + k * dt < n) out[r * n + t0 + k * dt] = acc[k];
}

template <typename T>
__global__ void __launch_bounds__(256)
nonfinite_scan_kernel(const T *__restrict__ x, int64_t nrows, int64_t n, int64_t ld, int32_t *flag)
{
    bool bad = false;
    const int64_t total = nrows * n;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const T v = x[(i / n) * ld + i % n];
        bad |= !isfinite(v);
    }
    if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(flag, 1);
}

__global__ void nan_rule_kernel(int64_t ndm, double *max_out, double *std_out, double *snr_out, int32_t *win_out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ndm) return;
    const double qnan = __longlong_as_double(0x7ff8000000000000ll);
    max_out[i] = qnan;
    std_out[i] = qnan;
    snr_out[i] = 0.0;
    win_out[i] = 0;
}

unsigned grid_for(int64_t n, int64_t cap) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cap, (n + 255) / 256)); }

// Workspace carve-up for R rows of n samples.
struct StatsWs {
    double *S, *R, *mean, *mw, *var;
    uint64_t *keys;
    void *rs;
    size_t rs_bytes;
};

size_t stats_bytes(int64_t rows, int64_t n)
{
    const size_t a = 256;
    auto up = [&](size_t b) { return (b + a - 1) / a * a; };
    return up(rows * n * 8) + up(rows * (n / 2) * 8) + up(pu_row_sums_workspace_bytes(rows, n)) +
           up(rows * 8) + 2 * up(4 * rows * 8) + up(4 * rows * 8);
}

StatsWs carve(void *ws, int64_t rows, int64_t n)
{
    const size_t a = 256;
    auto up = [&](size_t b) { return (b + a - 1) / a * a; };
    char *p = reinterpret_cast<char *>(ws);
    StatsWs w;
    w.S = reinterpret_cast<double *>(p);
    p += up(rows * n * 8);
    w.R = reinterpret_cast<double *>(p);
    p += up(rows * (n / 2) * 8);
    w.rs = p;
    w.rs_bytes = pu_row_sums_workspace_bytes(rows, n);
    p += up(w.rs_bytes);
    w.mean = reinterpret_cast<double *>(p);
    p += up(rows * 8);
    w.mw = reinterpret_cast<double *>(p);
    p += up(4 * rows * 8);
    w.var = reinterpret_cast<double *>(p);
    p += up(4 * rows * 8);
    w.keys = reinterpret_cast<uint64_t *>(p);
    return w;
}

int stats_batch(const double *plane, int64_t rows, int64_t n, int64_t ld, const int32_t *idx, double *max_out,
                double *std_out, double *snr_out, int32_t *win_out, void *ws, hipStream_t s)
{
    StatsWs w = carve(ws, rows, n);
    const dim3 blk(256);
    int rc = pu_row_sums(plane, PU_F64, rows, n, ld, 0, nullptr, nullptr, (double)n, w.mean, w.rs, w.rs_bytes, s);
    if (rc) return rc;
    PU_TRY_HIP(hipMemsetAsync(w.keys, 0, 4 * rows * sizeof(uint64_t), s));
    hipLaunchKernelGGL(exact_shift_kernel, dim3(grid_for(n, 64), (unsigned)rows), blk, 0, s, plane, ld, n, w.mean, w.S,
                       w.keys);
    if ((rc = pu::launch_check("exact_shift_kernel"))) return rc;
    for (int k = 0; k < 4; ++k) {
        const int win = 1 << k;
        const int64_t nb = n / win;
        if (nb == 0) break;
        const double *src = w.S;
        if (k > 0) {
            hipLaunchKernelGGL(exact_rebin_kernel, dim3(grid_for(nb, 64), (unsigned)rows), blk, 0, s, w.S, n, win, nb,
                               w.R, w.keys + k * rows);
            if ((rc = pu::launch_check("exact_rebin_kernel"))) return rc;
            src = w.R;
        }
        // np.std(reb): mean, then the sum of squared deviations, both in numpy's order
        rc = pu_row_sums(src, PU_F64, rows, nb, nb, 0, nullptr, nullptr, (double)nb, w.mw + k * rows, w.rs,
                         w.rs_bytes, s);
        if (!rc)
            rc = pu_row_sums(src, PU_F64, rows, nb, nb, 1, w.mw + k * rows, nullptr, (double)nb, w.var + k * rows,
                             w.rs, w.rs_bytes, s);
        if (rc) return rc;
    }
    hipLaunchKernelGGL(exact_final_kernel, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, s, rows, n, w.keys, w.var,
                       idx, max_out, std_out, snr_out, win_out);
    return pu::launch_check("exact_final_kernel");
}

}  // namespace

namespace pu {

int nonfinite_any_async(const void *data, int dtype, int64_t nrows, int64_t n, int64_t ld, int32_t *flag,
                        hipStream_t s)
{
    PU_TRY_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
    const unsigned grid = grid_for(nrows * n, 4096);
    if (dtype == PU_F32)
        hipLaunchKernelGGL(nonfinite_scan_kernel<float>, dim3(grid), dim3(256), 0, s,
                           reinterpret_cast<const float *>(data), nrows, n, ld, flag);
    else if (dtype == PU_F64)
        hipLaunchKernelGGL(nonfinite_scan_kernel<double>, dim3(grid), dim3(256), 0, s,
                           reinterpret_cast<const double *>(data), nrows, n, ld, flag);
    else
        return PU_OK;  // integers are always finite (the flag stays 0)
    return launch_check("nonfinite_scan_kernel");
}

int exact_series(const void *data, int dtype, int64_t nchan, int64_t n, int64_t ld, const int64_t *shifts, int64_t rows,
                 double *out, hipStream_t s)
{
    const dim3 grid((unsigned)((n + 4 * 64 * kSeriesPer - 1) / (4 * 64 * kSeriesPer)), (unsigned)rows), blk(256);
    switch (dtype) {
    case PU_U8:
        hipLaunchKernelGGL(exact_series_kernel<uint8_t>, grid, blk, 0, s, reinterpret_cast<const uint8_t *>(data), ld,
                           nchan, n, shifts, out);
        break;
    case PU_F32:
        hipLaunchKernelGGL(exact_series_kernel<float>, grid, blk, 0, s, reinterpret_cast<const float *>(data), ld,
                           nchan, n, shifts, out);
        break;
    case PU_F64:
        hipLaunchKernelGGL(exact_series_kernel<double>, grid, blk, 0, s, reinterpret_cast<const double *>(data), ld,
                           nchan, n, shifts, out);
        break;
    default: set_error("exact_series: dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return launch_check("exact_series_kernel");
}

int nan_rule(int64_t ndm, double *max_out, double *std_out, double *snr_out, int32_t *win_out, hipStream_t s)
{
    hipLaunchKernelGGL(nan_rule_kernel, dim3((unsigned)((ndm + 255) / 256)), dim3(256), 0, s, ndm, max_out, std_out,
                       snr_out, win_out);
    return launch_check("nan_rule_kernel");
}

}  // namespace pu

extern "C" {

size_t pu_series_stats_workspace_bytes(int64_t rows, int64_t n)
{
    if (rows <= 0 || n <= 0) return 0;
    return stats_bytes(rows, n);
}

int pu_series_stats(const double *series, int64_t rows, int64_t n, int64_t ld, const int32_t *index,
                    double *max_out, double *std_out, double *snr_out, int32_t *rebin_out, void *workspace,
                    size_t workspace_bytes, void *stream)
{
    PU_REQUIRE(series && max_out && std_out && snr_out && rebin_out, "pu_series_stats: NULL pointer");
    PU_REQUIRE(rows > 0 && n > 0 && ld >= n, "pu_series_stats: bad shape");
    PU_REQUIRE(rows < (int64_t(1) << 31) && n < (int64_t(1) << 40), "pu_series_stats: too large");
    PU_REQUIRE(workspace && reinterpret_cast<uintptr_t>(workspace) % 256 == 0,
               "pu_series_stats: workspace NULL or not 256-byte aligned");
    // rows per batch: as many as the workspace holds
    int64_t per = rows;
    while (per > 1 && stats_bytes(per, n) > workspace_bytes) per = (per + 1) / 2;
    PU_REQUIRE(stats_bytes(per, n) <= workspace_bytes, "pu_series_stats: workspace holds no row (%zu bytes)",
               workspace_bytes);
    hipStream_t s = pu::as_stream(stream);
    for (int64_t r0 = 0; r0 < rows; r0 += per) {
        const int64_t m = std::min(per, rows - r0);
        // outputs of row r go to index[r] (or r): offset the pointers of a batch
        const int32_t *idx = index ? index + r0 : nullptr;
        const int64_t off = index ? 0 : r0;
        int rc = stats_batch(series + r0 * ld, m, n, ld, idx, max_out + off, std_out + off, snr_out + off,
                             rebin_out + off, workspace, s);
        if (rc) return rc;
    }
    return PU_OK;
}

}  // extern "C"
