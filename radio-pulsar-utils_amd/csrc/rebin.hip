// Rebinning and roll helpers (HBM-streaming kernels) for gfx950.
//
//   pu_rebin_time   <- quick_resample           pulsarutils/dedispersion.py:38-57
//   pu_rebin_chan   <- quick_chan_rebin         :15-35
//   pu_roll_rows    <- apply_dm_shifts_to_data  :254-258
//   pu_roll_and_sum <- roll_and_sum             :60-83
//   pu_transpose    <- the (nsamps, nchans) -> (nchans, nsamps) transpose sigpyproc's
//                      readBlock performs (clean.py:327, stats.py:45)
// Each output element is produced by one lane in the reference's add order, so
// results are bit-identical to the reference for every supported dtype.
#include <hip/hip_runtime.h>

#include "pu_common.h"

namespace {

unsigned nblocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

template <typename Tin>
__global__ void rebin_time_kernel(const Tin *__restrict__ x, int64_t nrows, int64_t nout, int64_t ld, int64_t w,
                                  double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = blockIdx.y;
    if (i >= nout) return;
    const Tin *p = x + r * ld + i * w;
    double acc = 0.0;
    for (int64_t j = 0; j < w; ++j) acc += static_cast<double>(p[j]);
    out[r * nout + i] = acc;
}

template <typename Tin, typename Tout>
__global__ void rebin_chan_kernel(const Tin *__restrict__ x, int64_t n, int64_t ld, int64_t rb,
                                  Tout *__restrict__ out)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t g = blockIdx.y;
    if (t >= n) return;
    const Tin *p = x + g * rb * ld + t;
    Tout acc = static_cast<Tout>(p[0]);
    for (int64_t j = 1; j < rb; ++j) acc += static_cast<Tout>(p[j * ld]);
    out[g * n + t] = acc;
}

template <typename T>
__global__ void roll_rows_kernel(const T *__restrict__ x, int64_t n, int64_t ld, const int64_t *__restrict__ shifts,
                                 T *__restrict__ out)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = blockIdx.y;
    if (t >= n) return;
    int64_t s = shifts[r] % n;
    if (s < 0) s += n;
    int64_t idx = t + s;
    if (idx >= n) idx -= n;
    out[r * n + t] = x[r * ld + idx];
}

template <typename Tin>
__global__ void roll_and_sum_kernel(const Tin *__restrict__ x, int64_t n, int64_t roll, double *__restrict__ sum)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int64_t idx = t - roll;
    if (idx < 0) idx += n;
    sum[t] += static_cast<double>(x[idx]);
}

// 64x64 tiles through LDS (+1 element pad against bank conflicts); coalesced reads of
// ``src`` rows and coalesced writes of ``dst`` rows.
template <typename T>
__global__ void __launch_bounds__(256) transpose_kernel(const T *__restrict__ src, int64_t rows, int64_t cols,
                                                        int64_t ld_src, T *__restrict__ dst, int64_t ld_dst)
{
    __shared__ T tile[64][65];
    const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int i = ty; i < 64; i += 4) {
        const int64_t r = r0 + i, c = c0 + tx;
        if (r < rows && c < cols) tile[i][tx] = src[r * ld_src + c];
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
        const int64_t c = c0 + i, r = r0 + tx;
        if (r < rows && c < cols) dst[c * ld_dst + r] = tile[tx][i];
    }
}

}  // namespace

extern "C" {

int pu_transpose(const void *src, int elem_bytes, int64_t rows, int64_t cols, int64_t ld_src, void *dst,
                 int64_t ld_dst, void *stream)
{
    PU_REQUIRE(src && dst && rows >= 0 && cols >= 0 && ld_src >= cols && ld_dst >= rows,
               "pu_transpose: bad arguments");
    if (rows == 0 || cols == 0) return PU_OK;
    PU_REQUIRE((rows + 63) / 64 < 65536, "pu_transpose: too many rows");
    const dim3 g((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64)), b(256);
    hipStream_t s = pu::as_stream(stream);
    switch (elem_bytes) {
    case 1: hipLaunchKernelGGL(transpose_kernel<uint8_t>, g, b, 0, s, (const uint8_t *)src, rows, cols, ld_src, (uint8_t *)dst, ld_dst); break;
    case 2: hipLaunchKernelGGL(transpose_kernel<uint16_t>, g, b, 0, s, (const uint16_t *)src, rows, cols, ld_src, (uint16_t *)dst, ld_dst); break;
    case 4: hipLaunchKernelGGL(transpose_kernel<uint32_t>, g, b, 0, s, (const uint32_t *)src, rows, cols, ld_src, (uint32_t *)dst, ld_dst); break;
    case 8: hipLaunchKernelGGL(transpose_kernel<uint64_t>, g, b, 0, s, (const uint64_t *)src, rows, cols, ld_src, (uint64_t *)dst, ld_dst); break;
    default: pu::set_error("pu_transpose: element size %d unsupported", elem_bytes); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("transpose_kernel");
}


int pu_rebin_time(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, int64_t w, double *out,
                  void *stream)
{
    PU_REQUIRE(x && out && nrows > 0 && n > 0 && ld >= n && w > 0, "pu_rebin_time: bad arguments");
    PU_REQUIRE(nrows < 65536, "pu_rebin_time: at most 65535 rows");
    const int64_t nout = n / w;
    if (nout == 0) return PU_OK;
    const dim3 g(nblocks(nout, 256), (unsigned)nrows), b(256);
    hipStream_t s = pu::as_stream(stream);
    switch (dtype) {
    case PU_U8: hipLaunchKernelGGL(rebin_time_kernel<uint8_t>, g, b, 0, s, (const uint8_t *)x, nrows, nout, ld, w, out); break;
    case PU_F32: hipLaunchKernelGGL(rebin_time_kernel<float>, g, b, 0, s, (const float *)x, nrows, nout, ld, w, out); break;
    case PU_F64: hipLaunchKernelGGL(rebin_time_kernel<double>, g, b, 0, s, (const double *)x, nrows, nout, ld, w, out); break;
    case PU_I64: hipLaunchKernelGGL(rebin_time_kernel<int64_t>, g, b, 0, s, (const int64_t *)x, nrows, nout, ld, w, out); break;
    default: pu::set_error("pu_rebin_time: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("rebin_time_kernel");
}

int pu_rebin_chan(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, int64_t rb, void *out, void *stream)
{
    PU_REQUIRE(x && out && nrows > 0 && n > 0 && ld >= n && rb > 0, "pu_rebin_chan: bad arguments");
    const int64_t ng = nrows / rb;
    if (ng == 0) return PU_OK;
    PU_REQUIRE(ng < 65536, "pu_rebin_chan: at most 65535 output rows");
    const dim3 g(nblocks(n, 256), (unsigned)ng), b(256);
    hipStream_t s = pu::as_stream(stream);
    switch (dtype) {
    case PU_U8: hipLaunchKernelGGL((rebin_chan_kernel<uint8_t, uint64_t>), g, b, 0, s, (const uint8_t *)x, n, ld, rb, (uint64_t *)out); break;
    case PU_F32: hipLaunchKernelGGL((rebin_chan_kernel<float, float>), g, b, 0, s, (const float *)x, n, ld, rb, (float *)out); break;
    case PU_F64: hipLaunchKernelGGL((rebin_chan_kernel<double, double>), g, b, 0, s, (const double *)x, n, ld, rb, (double *)out); break;
    case PU_I64: hipLaunchKernelGGL((rebin_chan_kernel<int64_t, int64_t>), g, b, 0, s, (const int64_t *)x, n, ld, rb, (int64_t *)out); break;
    default: pu::set_error("pu_rebin_chan: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("rebin_chan_kernel");
}

int pu_roll_rows(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, const int64_t *shifts, void *out,
                 void *stream)
{
    PU_REQUIRE(x && out && shifts && nrows > 0 && n > 0 && ld >= n, "pu_roll_rows: bad arguments");
    PU_REQUIRE(nrows < 65536, "pu_roll_rows: at most 65535 rows");
    const dim3 g(nblocks(n, 256), (unsigned)nrows), b(256);
    hipStream_t s = pu::as_stream(stream);
    switch (pu::elem_size(dtype)) {
    case 1: hipLaunchKernelGGL(roll_rows_kernel<uint8_t>, g, b, 0, s, (const uint8_t *)x, n, ld, shifts, (uint8_t *)out); break;
    case 4: hipLaunchKernelGGL(roll_rows_kernel<uint32_t>, g, b, 0, s, (const uint32_t *)x, n, ld, shifts, (uint32_t *)out); break;
    case 8: hipLaunchKernelGGL(roll_rows_kernel<uint64_t>, g, b, 0, s, (const uint64_t *)x, n, ld, shifts, (uint64_t *)out); break;
    default: pu::set_error("pu_roll_rows: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("roll_rows_kernel");
}

int pu_roll_and_sum(const void *x, int dtype, int64_t n, int64_t roll, double *sum, void *stream)
{
    PU_REQUIRE(x && sum && n > 0, "pu_roll_and_sum: bad arguments");
    PU_REQUIRE(roll >= 0 && roll < n, "pu_roll_and_sum: roll %lld outside [0, %lld)", (long long)roll, (long long)n);
    const dim3 g(nblocks(n, 256)), b(256);
    hipStream_t s = pu::as_stream(stream);
    switch (dtype) {
    case PU_U8: hipLaunchKernelGGL(roll_and_sum_kernel<uint8_t>, g, b, 0, s, (const uint8_t *)x, n, roll, sum); break;
    case PU_F32: hipLaunchKernelGGL(roll_and_sum_kernel<float>, g, b, 0, s, (const float *)x, n, roll, sum); break;
    case PU_F64: hipLaunchKernelGGL(roll_and_sum_kernel<double>, g, b, 0, s, (const double *)x, n, roll, sum); break;
    case PU_I64: hipLaunchKernelGGL(roll_and_sum_kernel<int64_t>, g, b, 0, s, (const int64_t *)x, n, roll, sum); break;
    default: pu::set_error("pu_roll_and_sum: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("roll_and_sum_kernel");
}

}  // extern "C"
