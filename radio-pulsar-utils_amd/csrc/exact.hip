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
// (roll_and_sum's order, dedispersion.py:60-98: bit-identical), for samples t in
// [t_begin, t_begin + t_len) (out rows of t_len).  The row shifts (in [0, n)) go through LDS
// 1024 channels at a time.  Every trial reads its samples' columns of every channel once
// (17 GB at C3 for the whole series), which is why only flagged trials take this path.
//   8-bit: a thread owns 8 consecutive samples and reads them as 3 aligned dwords
//   (lanes 8 B apart: coalesced), bytes extracted by funnel shifts;
//   float: a thread owns samples t0 + l + 64 k (k < 8): every load of a wave is 64
//   consecutive elements.
// The loads of U consecutive channels are issued before their adds (which stay in channel
// order): one channel per iteration waited on its loads every time (13 ms for one trial at
// C3, latency-bound).
constexpr int kSeriesPer = 8;

template <typename T>
__global__ void __launch_bounds__(256)
exact_series_kernel(const T *__restrict__ x, int64_t ld, int64_t nchan, int64_t n, const int64_t *__restrict__ shifts,
                    double *__restrict__ out, int64_t t_begin, int64_t t_len)
{
    constexpr int U = sizeof(T) == 1 ? 8 : sizeof(T) == 4 ? 4 : 2;  // channels in flight
    __shared__ int64_t sh[1024];
    const int64_t r = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t t_end = t_begin + t_len;
    // the wave's 512 samples start at w0; this thread's samples
    const int64_t w0 = t_begin + ((int64_t)blockIdx.x * 4 + wave) * 64 * kSeriesPer;
    const int64_t t0 = sizeof(T) == 1 ? w0 + (int64_t)kSeriesPer * lane : w0 + lane;
    const int64_t dt = sizeof(T) == 1 ? 1 : 64;  // sample step between this thread's samples
    // 8-bit rows read as aligned dwords (x and ld multiples of 4: uniform)
    const bool rows4 = sizeof(T) == 1 && (reinterpret_cast<uintptr_t>(x) & 3) == 0 && (ld & 3) == 0;
    const bool full = t0 + (kSeriesPer - 1) * dt < t_end;  // every sample of this thread in range
    double acc[kSeriesPer];
#pragma unroll
    for (int k = 0; k < kSeriesPer; ++k) acc[k] = 0.0;
    // one channel's adds, the general way (wrapping windows, partial threads)
    auto slow = [&](int64_t c, int64_t s) {
        const T *row = x + c * ld;
        int64_t idx = t0 + s;
        while (idx >= n) idx -= n;
#pragma unroll
        for (int k = 0; k < kSeriesPer; ++k) {
            if (t0 + k * dt < t_end) acc[k] += static_cast<double>(row[idx]);
            idx += dt;
            while (idx >= n) idx -= n;  // n < 64 may wrap more than once
        }
    };
    for (int64_t c0 = 0; c0 < nchan; c0 += 1024) {
        const int64_t nc = nchan - c0 < 1024 ? nchan - c0 : 1024;
        __syncthreads();
        for (int64_t i = threadIdx.x; i < nc; i += 256) sh[i] = shifts[r * nchan + c0 + i];
        __syncthreads();
        if (w0 >= t_end) continue;
        int64_t ci = 0;
        for (; ci + U <= nc; ci += U) {
            int64_t idx[U];
            bool ok = full;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                idx[u] = t0 + sh[ci + u];
                if (idx[u] >= n) idx[u] -= n;
                ok = ok && idx[u] + (sizeof(T) == 1 ? 12 : (kSeriesPer - 1) * 64 + 1) <= n;
            }
            if (sizeof(T) == 1) ok = ok && rows4;
            if (!ok) {
                for (int u = 0; u < U; ++u) slow(c0 + ci + u, sh[ci + u]);
                continue;
            }
            if constexpr (sizeof(T) == 1) {
                uint32_t d[U][3];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t *p = reinterpret_cast<const uint32_t *>(x + (c0 + ci + u) * ld + (idx[u] & ~int64_t(3)));
                    d[u][0] = p[0];
                    d[u][1] = p[1];
                    d[u][2] = p[2];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t sft = (uint32_t)(idx[u] & 3) * 8u;
                    // bytes idx .. idx + 7 as two dwords (funnel shift across the dwords)
                    const uint32_t lo = sft ? (d[u][0] >> sft) | (d[u][1] << (32u - sft)) : d[u][0];
                    const uint32_t hi = sft ? (d[u][1] >> sft) | (d[u][2] << (32u - sft)) : d[u][1];
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[k] += (double)((lo >> (8 * k)) & 0xffu);
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[4 + k] += (double)((hi >> (8 * k)) & 0xffu);
                }
            } else {
                T v[U][kSeriesPer];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const T *row = x + (c0 + ci + u) * ld + idx[u];
#pragma unroll
                    for (int k = 0; k < kSeriesPer; ++k) v[u][k] = row[k * 64];
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int k = 0; k < kSeriesPer; ++k) acc[k] += static_cast<double>(v[u][k]);
            }
        }
        for (; ci < nc; ++ci) slow(c0 + ci, sh[ci]);
    }
#pragma unroll
    for (int k = 0; k < kSeriesPer; ++k)
        if (t0 + k * dt < t_end) out[r * t_len + (t0 + k * dt - t_begin)] = acc[k];
}

// 8-bit input: the same series from channel segments of kSegChans channels (grid.z), each
// summed as integers and added into out with float64 atomics.  Every partial sum is an
// integer below 2^53, so any order of the adds gives the bits of the channel-order float64
// chain (as colsum_u8_seg_kernel argues for the column sums); the segments give one trial
// nchan / kSegChans times the workgroups (one trial at C3: 10.7 ms sequential over channels).
constexpr int kSegChans = 256;

__global__ void __launch_bounds__(256)
exact_series_u8_seg_kernel(const uint8_t *__restrict__ x, int64_t ld, int64_t nchan, int64_t n,
                           const int64_t *__restrict__ shifts, double *__restrict__ out, int64_t t_begin, int64_t t_len)
{
    constexpr int U = 8;
    __shared__ int64_t sh[kSegChans];
    const int64_t r = blockIdx.y;
    const int64_t c0 = (int64_t)blockIdx.z * kSegChans;
    const int64_t nc = nchan - c0 < kSegChans ? nchan - c0 : kSegChans;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t t_end = t_begin + t_len;
    const int64_t w0 = t_begin + ((int64_t)blockIdx.x * 4 + wave) * 64 * kSeriesPer;
    const int64_t t0 = w0 + (int64_t)kSeriesPer * lane;
    for (int64_t i = threadIdx.x; i < nc; i += 256) sh[i] = shifts[r * nchan + c0 + i];
    __syncthreads();
    if (w0 >= t_end) return;
    const bool full = t0 + kSeriesPer - 1 < t_end;
    uint32_t acc[kSeriesPer];  // <= kSegChans x 255 < 2^17
#pragma unroll
    for (int k = 0; k < kSeriesPer; ++k) acc[k] = 0;
    auto slow = [&](int64_t c, int64_t s) {
        const uint8_t *row = x + c * ld;
        int64_t idx = t0 + s;
        while (idx >= n) idx -= n;
#pragma unroll
        for (int k = 0; k < kSeriesPer; ++k) {
            if (t0 + k < t_end) acc[k] += row[idx];
            idx += 1;
            if (idx >= n) idx -= n;
        }
    };
    int64_t ci = 0;
    for (; ci + U <= nc; ci += U) {
        int64_t idx[U];
        bool ok = full;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            idx[u] = t0 + sh[ci + u];
            if (idx[u] >= n) idx[u] -= n;
            ok = ok && idx[u] + 12 <= n;
        }
        if (!ok) {
            for (int u = 0; u < U; ++u) slow(c0 + ci + u, sh[ci + u]);
            continue;
        }
        uint32_t d[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t *p = reinterpret_cast<const uint32_t *>(x + (c0 + ci + u) * ld + (idx[u] & ~int64_t(3)));
            d[u][0] = p[0];
            d[u][1] = p[1];
            d[u][2] = p[2];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t sft = (uint32_t)(idx[u] & 3) * 8u;
            const uint32_t lo = sft ? (d[u][0] >> sft) | (d[u][1] << (32u - sft)) : d[u][0];
            const uint32_t hi = sft ? (d[u][1] >> sft) | (d[u][2] << (32u - sft)) : d[u][1];
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] += (lo >> (8 * k)) & 0xffu;
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[4 + k] += (hi >> (8 * k)) & 0xffu;
        }
    }
    for (; ci < nc; ++ci) slow(c0 + ci, sh[ci]);
#pragma unroll
    for (int k = 0; k < kSeriesPer; ++k)
        if (t0 + k < t_end) unsafeAtomicAdd(out + r * t_len + (t0 + k - t_begin), (double)acc[k]);
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
                 double *out, hipStream_t s, int64_t t_begin, int64_t t_len)
{
    if (t_len < 0) t_len = n - t_begin;
    if (t_len <= 0 || rows <= 0) return PU_OK;
    const dim3 grid((unsigned)((t_len + 4 * 64 * kSeriesPer - 1) / (4 * 64 * kSeriesPer)), (unsigned)rows), blk(256);
    switch (dtype) {
    case PU_U8:
        if ((reinterpret_cast<uintptr_t>(data) & 3) == 0 && (ld & 3) == 0) {
            // integer channel segments, float64 atomics (exact: integer sums < 2^53)
            PU_TRY_HIP(hipMemsetAsync(out, 0, (size_t)rows * (size_t)t_len * sizeof(double), s));
            const dim3 g3(grid.x, grid.y, (unsigned)((nchan + kSegChans - 1) / kSegChans));
            hipLaunchKernelGGL(exact_series_u8_seg_kernel, g3, blk, 0, s, reinterpret_cast<const uint8_t *>(data), ld,
                               nchan, n, shifts, out, t_begin, t_len);
            return launch_check("exact_series_u8_seg_kernel");
        }
        hipLaunchKernelGGL(exact_series_kernel<uint8_t>, grid, blk, 0, s, reinterpret_cast<const uint8_t *>(data), ld,
                           nchan, n, shifts, out, t_begin, t_len);
        break;
    case PU_F32:
        hipLaunchKernelGGL(exact_series_kernel<float>, grid, blk, 0, s, reinterpret_cast<const float *>(data), ld,
                           nchan, n, shifts, out, t_begin, t_len);
        break;
    case PU_F64:
        hipLaunchKernelGGL(exact_series_kernel<double>, grid, blk, 0, s, reinterpret_cast<const double *>(data), ld,
                           nchan, n, shifts, out, t_begin, t_len);
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
