// RFI-cleaning reductions and apply passes for gfx950 (MI355X).
//
// Replaces the 2-D array passes of the reference cleaning path
// (pulsarutils/clean.py:58-111, 114-133) with bit-exact HIP kernels.  The masks the
// reference derives are threshold comparisons on these reductions, so every sum is
// reproduced in numpy's exact order (SURVEY.md §8 a-R; oracle/numpy_order.py):
//
//   add.reduce over a contiguous row  = 0 + pw(block_0) + pw(block_1) + ...,
//       blocks of 8192 elements, pw = numpy pairwise_sum (8 strided accumulators
//       over 128-element leaves, halving splits at n/2 - (n/2)%8)
//   mean(0) / zero-DM light curve      = sequential over rows
//
// Everything is compiled with -ffp-contract=off: a fused multiply-add would change
// the rounding of x*f - mu and of the squared deviations.
//
// Kernels
//   rowsum_chunk_kernel  one workgroup per (row, full 8192 block): LDS-staged leaves,
//                        8-accumulator leaf sums, in-order pairwise tree.
//   rowsum_tail_kernel   one lane per row for the trailing partial block (irregular
//                        pairwise tree; compile-time-bounded recursion).
//   rowsum_combine       sequential 0 + block sums (+ true_divide by the count).
//   colmean_kernel       one lane per column, rows in order (clean.py:77).
//   gauss_kernel         scipy correlate1d symmetric order, mode 'reflect' (:79).
//   apply_kernel         (x*f - mu)/mu, bad rows zeroed, optional column mean (:81-94).
#include <hip/hip_runtime.h>

#include <cmath>

#include "pu_common.h"

namespace {

constexpr int kBlock = 8192;   // numpy ufunc buffer size
constexpr int kLeaf = 128;     // numpy PW_BLOCKSIZE
constexpr int kLeafPad = 8;    // LDS padding per leaf (bank spread)

template <typename Tin, typename Ta, int MODE>
__device__ __forceinline__ Ta load_val(const Tin *row, int64_t t, Ta center, const double *scale)
{
    if constexpr (MODE == 0) {
        return static_cast<Ta>(row[t]);
    } else if constexpr (MODE == 1) {
        const Ta d = static_cast<Ta>(row[t]) - center;
        return d * d;
    } else if constexpr (MODE == 4) {
        const Ta v = static_cast<Ta>(row[t]);
        return v * v;
    } else {
        return static_cast<Ta>(static_cast<double>(row[t]) * scale[t]);
    }
}

// numpy pairwise_sum over [off, off+n) of a row, one lane.  DEPTH bounds the
// recursion at compile time (n <= 8192 needs < 10 levels).
template <typename Tin, typename Ta, int MODE, int DEPTH>
__device__ Ta pairwise_lane(const Tin *row, int64_t off, int64_t n, Ta center, const double *scale)
{
    if (n < 8) {
        Ta r = Ta(0);
        for (int64_t i = 0; i < n; ++i) r += load_val<Tin, Ta, MODE>(row, off + i, center, scale);
        return r;
    }
    if constexpr (DEPTH > 0) {
        if (n > kLeaf) {
            int64_t n2 = n / 2;
            n2 -= n2 % 8;
            const Ta l = pairwise_lane<Tin, Ta, MODE, DEPTH - 1>(row, off, n2, center, scale);
            const Ta r = pairwise_lane<Tin, Ta, MODE, DEPTH - 1>(row, off + n2, n - n2, center, scale);
            return l + r;
        }
    }
    Ta r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = load_val<Tin, Ta, MODE>(row, off + j, center, scale);
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += load_val<Tin, Ta, MODE>(row, off + i + j, center, scale);
    Ta res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += load_val<Tin, Ta, MODE>(row, off + i, center, scale);
    return res;
}

// Full 8192-element blocks: 64 leaves of 128.  Thread (b = tid/4, q = tid%4) owns
// accumulators r[2q], r[2q+1] of leaf b; the leaf total is
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) via two xor-shuffles, then the 64 leaves
// combine as the perfect binary tree pairwise_sum builds for n = 8192.
template <typename Tin, typename Ta, int MODE>
__global__ void __launch_bounds__(256)
rowsum_chunk_kernel(const Tin *__restrict__ x, int64_t ld, int64_t nfull, int64_t nblk_row,
                    const Ta *__restrict__ centers, const double *__restrict__ scale,
                    Ta *__restrict__ block_sums)
{
    __shared__ Ta buf[64 * (kLeaf + kLeafPad)];
    __shared__ Ta leaves[64];
    const int64_t row = blockIdx.x / nfull;
    const int64_t blk = blockIdx.x % nfull;
    const int tid = threadIdx.x;
    const Tin *rp = x + row * ld;
    const Ta center = MODE == 1 ? centers[row] : Ta(0);
    const int64_t off = blk * kBlock;
    for (int e = tid; e < kBlock; e += 256)
        buf[(e >> 7) * (kLeaf + kLeafPad) + (e & 127)] = load_val<Tin, Ta, MODE>(rp, off + e, center, scale);
    __syncthreads();
    const int b = tid >> 2, q = tid & 3;
    const Ta *lp = buf + b * (kLeaf + kLeafPad) + 2 * q;
    Ta r0 = lp[0], r1 = lp[1];
#pragma unroll
    for (int m = 1; m < 16; ++m) {
        r0 += lp[8 * m];
        r1 += lp[8 * m + 1];
    }
    Ta t = r0 + r1;
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    if (q == 0) leaves[b] = t;
    __syncthreads();
    for (int s = 1; s < 64; s <<= 1) {
        if (tid < 64 && (tid % (2 * s)) == 0) leaves[tid] = leaves[tid] + leaves[tid + s];
        __syncthreads();
    }
    if (tid == 0) block_sums[row * nblk_row + blk] = leaves[0];
}

template <typename Tin, typename Ta, int MODE>
__global__ void __launch_bounds__(64)
rowsum_tail_kernel(const Tin *__restrict__ x, int64_t ld, int64_t nrows, int64_t n, int64_t nfull,
                   int64_t nblk_row, const Ta *__restrict__ centers, const double *__restrict__ scale,
                   Ta *__restrict__ block_sums)
{
    const int64_t row = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (row >= nrows) return;
    const Ta center = MODE == 1 ? centers[row] : Ta(0);
    const int64_t off = nfull * kBlock;
    block_sums[row * nblk_row + nfull] =
        pairwise_lane<Tin, Ta, MODE, 10>(x + row * ld, off, n - off, center, scale);
}

template <typename Ta>
__global__ void rowsum_combine(const Ta *__restrict__ block_sums, int64_t nrows, int64_t nblk_row,
                               double divisor, Ta *__restrict__ out)
{
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    Ta acc = Ta(0);
    for (int64_t k = 0; k < nblk_row; ++k) acc += block_sums[row * nblk_row + k];
    if (divisor > 0) acc = static_cast<Ta>(static_cast<double>(acc) / divisor);
    out[row] = acc;
}

template <typename Tin>
__global__ void colmean_kernel(const Tin *__restrict__ x, int64_t nrows, int64_t n, int64_t ld,
                               const uint8_t *__restrict__ skip, double *__restrict__ out)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    double acc = 0.0;
    int64_t ngood = 0;
    for (int64_t r = 0; r < nrows; ++r) {
        if (skip && skip[r]) continue;
        acc += static_cast<double>(x[r * ld + t]);
        ++ngood;
    }
    out[t] = acc / static_cast<double>(ngood);
}

__device__ __forceinline__ int64_t reflect_index(int64_t i, int64_t n)
{
    // scipy 'reflect' (d c b a | a b c d | d c b a): period 2n, half-sample symmetric
    const int64_t p = 2 * n;
    int64_t m = i % p;
    if (m < 0) m += p;
    return m >= n ? p - 1 - m : m;
}

__global__ void gauss_kernel(const double *__restrict__ x, int64_t n, const double *__restrict__ w,
                             int64_t r, double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double acc = x[i] * w[r];
    for (int64_t jj = -r; jj < 0; ++jj)
        acc += (x[reflect_index(i + jj, n)] + x[reflect_index(i - jj, n)]) * w[r + jj];
    out[i] = acc;
}

__global__ void ratio_kernel(double num, const double *__restrict__ x, int64_t n, double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = num / x[i];
}

template <typename Tin>
__global__ void apply_kernel(const Tin *__restrict__ x, int64_t nchan, int64_t n, int64_t ld,
                             const double *__restrict__ factor, const double *__restrict__ spec,
                             const uint8_t *__restrict__ bad, double *__restrict__ out, int64_t ld_out,
                             double *__restrict__ col_means)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double f = factor[t];
    double acc = 0.0;
    for (int64_t c = 0; c < nchan; ++c) {
        double v = static_cast<double>(x[c * ld + t]) * f;
        const double mu = spec[c];
        v = (v - mu) / mu;
        if (bad && bad[c]) v = 0.0;
        out[c * ld_out + t] = v;
        acc += v;
    }
    if (col_means) col_means[t] = acc / static_cast<double>(nchan);
}

__global__ void zero_cols_kernel(double *out, int64_t nrows, int64_t ld, const int64_t *__restrict__ cols,
                                 int64_t ncols)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = blockIdx.y;
    for (int64_t rr = r; rr < nrows; rr += gridDim.y)
        if (k < ncols) out[rr * ld + cols[k]] = 0.0;
}

template <typename Tin, typename Ta, int MODE>
int row_sums_t(const void *x, int64_t nrows, int64_t n, int64_t ld, const void *center, const double *scale,
               double divisor, void *out, void *ws, hipStream_t s)
{
    const int64_t nfull = n / kBlock;
    const int64_t tail = n % kBlock;
    const int64_t nblk_row = nfull + (tail ? 1 : 0);
    Ta *bs = reinterpret_cast<Ta *>(ws);
    const Tin *xp = reinterpret_cast<const Tin *>(x);
    const Ta *cp = reinterpret_cast<const Ta *>(center);
    if (nfull > 0) {
        PU_REQUIRE(nrows * nfull < (int64_t(1) << 31), "pu_row_sums: too many blocks");
        hipLaunchKernelGGL((rowsum_chunk_kernel<Tin, Ta, MODE>), dim3((unsigned)(nrows * nfull)), dim3(256), 0, s,
                           xp, ld, nfull, nblk_row, cp, scale, bs);
        int rc = pu::launch_check("rowsum_chunk_kernel");
        if (rc) return rc;
    }
    if (tail) {
        hipLaunchKernelGGL((rowsum_tail_kernel<Tin, Ta, MODE>), dim3((unsigned)((nrows + 63) / 64)), dim3(64), 0, s,
                           xp, ld, nrows, n, nfull, nblk_row, cp, scale, bs);
        int rc = pu::launch_check("rowsum_tail_kernel");
        if (rc) return rc;
    }
    hipLaunchKernelGGL((rowsum_combine<Ta>), dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, s, bs, nrows,
                       nblk_row, divisor, reinterpret_cast<Ta *>(out));
    return pu::launch_check("rowsum_combine");
}

template <typename Tin>
int row_sums_in(int mode, bool f32acc, const void *x, int64_t nrows, int64_t n, int64_t ld, const void *center,
                const double *scale, double divisor, void *out, void *ws, hipStream_t s)
{
    if (mode == 2) return row_sums_t<Tin, double, 2>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    if (mode == 3) return row_sums_t<Tin, double, 0>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    if (mode == 4) return row_sums_t<Tin, double, 4>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    if (f32acc) {
        if (mode == 0) return row_sums_t<Tin, float, 0>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
        return row_sums_t<Tin, float, 1>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    }
    if (mode == 0) return row_sums_t<Tin, double, 0>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    return row_sums_t<Tin, double, 1>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
}

unsigned blocks_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

}  // namespace

extern "C" {

size_t pu_row_sums_workspace_bytes(int64_t nrows, int64_t n)
{
    const int64_t nblk = (n + kBlock - 1) / kBlock;
    return (size_t)(nrows > 0 ? nrows : 0) * (size_t)(nblk > 0 ? nblk : 1) * sizeof(double);
}

int pu_row_sums(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, int mode, const void *center,
                const double *scale, double divisor, void *out, void *ws, size_t ws_bytes, void *stream)
{
    PU_REQUIRE(x && out, "pu_row_sums: NULL pointer");
    PU_REQUIRE(nrows > 0 && n > 0 && ld >= n, "pu_row_sums: bad shape");
    PU_REQUIRE(mode >= 0 && mode <= 4, "pu_row_sums: bad mode %d", mode);
    PU_REQUIRE(mode != 1 || center, "pu_row_sums: mode 1 needs center");
    PU_REQUIRE(mode != 2 || scale, "pu_row_sums: mode 2 needs scale");
    PU_REQUIRE(ws && ws_bytes >= pu_row_sums_workspace_bytes(nrows, n), "pu_row_sums: workspace too small");
    hipStream_t s = pu::as_stream(stream);
    switch (dtype) {
    case PU_U8: return row_sums_in<uint8_t>(mode, false, x, nrows, n, ld, center, scale, divisor, out, ws, s);
    case PU_F32: return row_sums_in<float>(mode, true, x, nrows, n, ld, center, scale, divisor, out, ws, s);
    case PU_F64: return row_sums_in<double>(mode, false, x, nrows, n, ld, center, scale, divisor, out, ws, s);
    }
    pu::set_error("pu_row_sums: unsupported dtype %d", dtype);
    return PU_EUNSUPPORTED;
}

int pu_col_means(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, const uint8_t *skip, double *out,
                 void *stream)
{
    PU_REQUIRE(x && out, "pu_col_means: NULL pointer");
    PU_REQUIRE(nrows > 0 && n > 0 && ld >= n, "pu_col_means: bad shape");
    hipStream_t s = pu::as_stream(stream);
    const dim3 g(blocks_for(n, 256)), b(256);
    switch (dtype) {
    case PU_U8:
        hipLaunchKernelGGL(colmean_kernel<uint8_t>, g, b, 0, s, (const uint8_t *)x, nrows, n, ld, skip, out);
        break;
    case PU_F32:
        hipLaunchKernelGGL(colmean_kernel<float>, g, b, 0, s, (const float *)x, nrows, n, ld, skip, out);
        break;
    case PU_F64:
        hipLaunchKernelGGL(colmean_kernel<double>, g, b, 0, s, (const double *)x, nrows, n, ld, skip, out);
        break;
    default: pu::set_error("pu_col_means: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("colmean_kernel");
}

int pu_gaussian_filter1d(const double *x, int64_t n, const double *w, int64_t r, double *out, void *stream)
{
    PU_REQUIRE(x && w && out && n > 0 && r >= 0, "pu_gaussian_filter1d: bad arguments");
    hipLaunchKernelGGL(gauss_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, pu::as_stream(stream), x, n, w, r, out);
    return pu::launch_check("gauss_kernel");
}

int pu_ratio(double num, const double *x, int64_t n, double *out, void *stream)
{
    PU_REQUIRE(x && out && n > 0, "pu_ratio: bad arguments");
    hipLaunchKernelGGL(ratio_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, pu::as_stream(stream), num, x, n, out);
    return pu::launch_check("ratio_kernel");
}

int pu_renorm_apply(const void *x, int dtype, int64_t nchan, int64_t n, int64_t ld, const double *factor,
                    const double *spec, const uint8_t *bad, double *out, int64_t ld_out, double *col_means,
                    void *stream)
{
    PU_REQUIRE(x && factor && spec && out, "pu_renorm_apply: NULL pointer");
    PU_REQUIRE(nchan > 0 && n > 0 && ld >= n && ld_out >= n, "pu_renorm_apply: bad shape");
    hipStream_t s = pu::as_stream(stream);
    const dim3 g(blocks_for(n, 256)), b(256);
    switch (dtype) {
    case PU_U8:
        hipLaunchKernelGGL(apply_kernel<uint8_t>, g, b, 0, s, (const uint8_t *)x, nchan, n, ld, factor, spec, bad,
                           out, ld_out, col_means);
        break;
    case PU_F32:
        hipLaunchKernelGGL(apply_kernel<float>, g, b, 0, s, (const float *)x, nchan, n, ld, factor, spec, bad, out,
                           ld_out, col_means);
        break;
    case PU_F64:
        hipLaunchKernelGGL(apply_kernel<double>, g, b, 0, s, (const double *)x, nchan, n, ld, factor, spec, bad,
                           out, ld_out, col_means);
        break;
    default: pu::set_error("pu_renorm_apply: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("apply_kernel");
}

int pu_zero_columns(double *out, int64_t nrows, int64_t ld, const int64_t *cols, int64_t ncols, void *stream)
{
    PU_REQUIRE(out && nrows > 0 && ld > 0, "pu_zero_columns: bad arguments");
    if (ncols <= 0) return PU_OK;
    PU_REQUIRE(cols != nullptr, "pu_zero_columns: cols is NULL");
    const unsigned gy = (unsigned)(nrows < 1024 ? nrows : 1024);
    hipLaunchKernelGGL(zero_cols_kernel, dim3(blocks_for(ncols, 256), gy), dim3(256), 0, pu::as_stream(stream), out,
                       nrows, ld, cols, ncols);
    return pu::launch_check("zero_cols_kernel");
}

}  // extern "C"
