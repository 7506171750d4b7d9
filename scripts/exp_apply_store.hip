// Experiment (round 5): the stores of the renormalisation apply pass.
//
// The u8 apply pass (256 MiB read, 2 GiB float64 written) runs at ~4.5 TB/s of writes
// against the 6.2 TB/s a float64 fill reaches.  This program times the production column
// walk (lane owns V columns of every row, 16-byte stores) with
//   - the store's cache-policy bits chosen by inline asm (none / nt / sc1 / sc1 nt / sc0 sc1 /
//     sc0 sc1 nt): global_store_dwordx4 with those modifiers;
//   - V = 4 columns per lane as two column PAIRS 128 columns apart (each store instruction
//     still one contiguous 1 KiB span per wave), half the waves;
// and a float64 fill with each policy as the ceiling.  Same arithmetic as apply_kernel
// ((x f - mu) / mu, bad rows 0, column sums in row order); timing only.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o exp_apply_store scripts/exp_apply_store.hip
//   ./exp_apply_store           -> one JSON line per variant
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

typedef double f64x2 __attribute__((ext_vector_type(2)));

// 16-byte store with cache-policy bits P: 0 none, 1 nt, 2 sc1, 3 sc1 nt, 4 sc0 sc1, 5 sc0 sc1 nt
template <int P>
__device__ __forceinline__ void st16(double *p, f64x2 v)
{
    if constexpr (P == 0) asm volatile("global_store_dwordx4 %0, %1, off" : : "v"(p), "v"(v) : "memory");
    else if constexpr (P == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" : : "v"(p), "v"(v) : "memory");
    else if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
    else if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" : : "v"(p), "v"(v) : "memory");
    else if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" : : "v"(p), "v"(v) : "memory");
}

// V = 2: lane owns columns c, c + 1.  V = 4 (split): lane l of wave w owns {b + 2l, b + 2l + 1}
// and {b + 128 + 2l, b + 129 + 2l}, b = 256 w: every store instruction covers 1 KiB.
template <typename Tin, int V, int U, int P>
__global__ void __launch_bounds__(256)
apply_cols(const Tin *__restrict__ x, int64_t nchan, int64_t n, const double *__restrict__ factor,
           const double *__restrict__ spec, const uint8_t *__restrict__ bad, double *__restrict__ out,
           double *__restrict__ colm)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    int64_t cs[V / 2];
    if constexpr (V == 2) {
        cs[0] = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    } else {
        cs[0] = wave * 256 + 2 * lane;
        cs[1] = cs[0] + 128;
    }
    double f[V], acc[V];
#pragma unroll
    for (int h = 0; h < V / 2; ++h)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f[2 * h + j] = factor[cs[h] + j];
            acc[2 * h + j] = 0.0;
        }
    typedef Tin pair_t __attribute__((ext_vector_type(2)));
    for (int64_t i0 = 0; i0 < nchan; i0 += U) {
        pair_t v[U][V / 2];
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int h = 0; h < V / 2; ++h) v[k][h] = *reinterpret_cast<const pair_t *>(x + (i0 + k) * n + cs[h]);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const double mu = spec[i0 + k];
            const bool b = bad[i0 + k] != 0;
#pragma unroll
            for (int h = 0; h < V / 2; ++h) {
                double r[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    double e = static_cast<double>(v[k][h][j]) * f[2 * h + j];
                    e = (e - mu) / mu;
                    r[j] = b ? 0.0 : e;
                    acc[2 * h + j] += r[j];
                }
                st16<P>(out + (i0 + k) * n + cs[h], f64x2{r[0], r[1]});
            }
        }
    }
#pragma unroll
    for (int h = 0; h < V / 2; ++h)
#pragma unroll
        for (int j = 0; j < 2; ++j) colm[cs[h] + j] = acc[2 * h + j] / (double)nchan;
}

template <int P>
__global__ void __launch_bounds__(256) fill_kernel(double *out, int64_t total)
{
    for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2; i < total; i += (int64_t)gridDim.x * 512)
        st16<P>(out + i, f64x2{1.0, 2.0});
}

static const char *pname[] = {"none", "nt", "sc1", "sc1 nt", "sc0 sc1", "sc0 sc1 nt"};

template <typename Tin, int V, int U, int P>
int runc(const char *name, const void *x, int64_t nchan, int64_t n, const double *factor, const double *spec,
         const uint8_t *bad, double *out, double *colm)
{
    dim3 grid((unsigned)(n / (256 * V)));
    auto go = [&] {
        hipLaunchKernelGGL((apply_cols<Tin, V, U, P>), grid, dim3(256), 0, 0, (const Tin *)x, nchan, n, factor, spec,
                           bad, out, colm);
    };
    for (int i = 0; i < 3; ++i) go();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) go();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    const double bytes = (double)nchan * n * (sizeof(Tin) + 8);
    printf("{\"kernel\": \"apply\", \"dtype\": \"%s\", \"V\": %d, \"U\": %d, \"policy\": \"%s\", \"us\": %.1f, \"TBps\": %.3f}\n",
           name, V, U, pname[P], us, bytes / (us * 1e-6) / 1e12);
    fflush(stdout);
    return 0;
}

template <int P>
int runf(double *out, int64_t total)
{
    auto go = [&] { hipLaunchKernelGGL((fill_kernel<P>), dim3(4096), dim3(256), 0, 0, out, total); };
    for (int i = 0; i < 3; ++i) go();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) go();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    printf("{\"kernel\": \"fill\", \"policy\": \"%s\", \"us\": %.1f, \"TBps\": %.3f}\n", pname[P], us,
           total * 8.0 / (us * 1e-6) / 1e12);
    fflush(stdout);
    return 0;
}

int main()
{
    const int64_t nchan = 1024, n = int64_t(1) << 18;
    void *xf, *xu;
    double *factor, *spec, *out, *colm;
    uint8_t *bad;
    CK(hipMalloc(&xf, nchan * n * 4));
    CK(hipMalloc(&xu, nchan * n));
    CK(hipMalloc(&out, nchan * n * 8));
    CK(hipMalloc(&colm, n * 8));
    CK(hipMalloc(&factor, n * 8));
    CK(hipMalloc(&spec, nchan * 8));
    CK(hipMalloc(&bad, nchan));
    {
        std::vector<float> hf(n);
        for (int64_t i = 0; i < n; ++i) hf[i] = 1.0f + (float)(i % 97) * 0.01f;
        for (int64_t r = 0; r < nchan; ++r) CK(hipMemcpy((float *)xf + r * n, hf.data(), n * 4, hipMemcpyHostToDevice));
        std::vector<double> hd(n, 1.0);
        CK(hipMemcpy(factor, hd.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(spec, hd.data(), nchan * 8, hipMemcpyHostToDevice));
        CK(hipMemset(bad, 0, nchan));
        CK(hipMemset(xu, 7, nchan * n));
    }
    int rc = 0;
    rc |= runf<0>(out, nchan * n);
    rc |= runf<1>(out, nchan * n);
    rc |= runf<2>(out, nchan * n);
    rc |= runf<3>(out, nchan * n);
    rc |= runf<4>(out, nchan * n);
    rc |= runf<5>(out, nchan * n);
    rc |= runc<uint8_t, 2, 32, 0>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 2, 32, 1>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 2, 32, 2>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 2, 32, 3>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 2, 32, 4>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 2, 32, 5>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 4, 16, 0>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 4, 16, 1>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<uint8_t, 4, 16, 3>("u8", xu, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<float, 2, 16, 0>("f32", xf, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<float, 2, 16, 1>("f32", xf, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<float, 2, 16, 2>("f32", xf, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<float, 2, 16, 3>("f32", xf, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<float, 4, 8, 0>("f32", xf, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<float, 4, 8, 2>("f32", xf, nchan, n, factor, spec, bad, out, colm);
    rc |= runc<float, 4, 8, 3>("f32", xf, nchan, n, factor, spec, bad, out, colm);
    return rc;
}
