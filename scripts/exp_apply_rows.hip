// Experiment (round 4): the renormalisation apply pass as a row-tiled stream.
//
// The production apply_kernel walks columns (one lane owns V columns for all rows) so
// that its column means come out in numpy's sequential row order; at C4 that is 1024
// (f32, V = 4) or 2048 (u8, V = 2) waves for the whole chip.  This program times the
// same arithmetic, (x f - mu) / mu with bad rows zeroed, as tiles of RB rows x 256 V
// columns (lanes own V columns of RB rows; per-tile column partial sums, max |e|), to
// see what the 1:2 read:write stream costs without the column walk.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o exp_apply_rows scripts/exp_apply_rows.hip
//   ./exp_apply_rows            -> one JSON line per (dtype, V, RB)
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

template <typename T, int V>
struct alignas(sizeof(T) * V) Vec {
    T v[V];
};

template <typename Tin, int V, int RB, int U>
__global__ void __launch_bounds__(256)
apply_rows(const Tin *__restrict__ x, int64_t nchan, int64_t n, int64_t ld, const double *__restrict__ factor,
           const double *__restrict__ spec, const uint8_t *__restrict__ bad, double *__restrict__ out, int64_t ld_out,
           double *__restrict__ part, unsigned long long *emax)
{
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
    const int64_t r0 = (int64_t)blockIdx.y * RB;
    double f[V], acc[V];
    double m = 0.0;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        f[j] = factor[c + j];
        acc[j] = 0.0;
    }
    const int rn = (int)(nchan - r0 < RB ? nchan - r0 : RB);
    for (int i0 = 0; i0 < rn; i0 += U) {
        Vec<Tin, V> v[U];
        double mu[U];
        bool b[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int64_t r = r0 + (i0 + k < rn ? i0 + k : rn - 1);
            v[k] = *reinterpret_cast<const Vec<Tin, V> *>(x + r * ld + c);
            mu[k] = spec[r];
            b[k] = bad[r] != 0;
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (i0 + k >= rn) break;
            Vec<double, V> res;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                double e = static_cast<double>(v[k].v[j]) * f[j];
                e = (e - mu[k]) / mu[k];
                res.v[j] = b[k] ? 0.0 : e;
                acc[j] += res.v[j];
                m = fmax(m, fabs(res.v[j]));
            }
            double *o = out + (r0 + i0 + k) * ld_out + c;
#pragma unroll
            for (int j = 0; j < V; j += 2) *reinterpret_cast<Vec<double, 2> *>(o + j) = Vec<double, 2>{{res.v[j], res.v[j + 1]}};
        }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) part[(int64_t)blockIdx.y * n + c + j] = acc[j];
    unsigned long long bm = (unsigned long long)__double_as_longlong(m);
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(bm, off, 64);
        bm = o > bm ? o : bm;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(emax, bm);
}


// Column walk (the production layout): lane owns V columns for all rows, batches of U rows
// loaded before use.  DIV = 0 replaces the division by a multiply with 1/mu (timing only).
template <typename Tin, int V, int U, int DIV, bool NT>
__global__ void __launch_bounds__(256)
apply_cols(const Tin *__restrict__ x, int64_t nchan, int64_t n, int64_t ld, const double *__restrict__ factor,
           const double *__restrict__ spec, const uint8_t *__restrict__ bad, double *__restrict__ out, int64_t ld_out,
           double *__restrict__ colm)
{
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
    double f[V], acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        f[j] = factor[c + j];
        acc[j] = 0.0;
    }
    for (int64_t i0 = 0; i0 < nchan; i0 += U) {
        Vec<Tin, V> v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = *reinterpret_cast<const Vec<Tin, V> *>(x + (i0 + k) * ld + c);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const double mu = spec[i0 + k];
            const double ri = 1.0 / mu;
            const bool b = bad[i0 + k] != 0;
            double res[V];
#pragma unroll
            for (int j = 0; j < V; ++j) {
                double e = static_cast<double>(v[k].v[j]) * f[j];
                e = DIV ? (e - mu) / mu : (e - mu) * ri;
                res[j] = b ? 0.0 : e;
                acc[j] += res[j];
            }
            double *o = out + (i0 + k) * ld_out + c;
            typedef double f64x2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int j = 0; j < V; j += 2) {
                if (NT) __builtin_nontemporal_store(f64x2{res[j], res[j + 1]}, reinterpret_cast<f64x2 *>(o + j));
                else *reinterpret_cast<f64x2 *>(o + j) = f64x2{res[j], res[j + 1]};
            }
        }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) colm[c + j] = acc[j] / (double)nchan;
}

template <typename Tin, int V, int U, int DIV, bool NT>
int runc(const char *name, const void *x, int64_t nchan, int64_t n, const double *factor, const double *spec,
         const uint8_t *bad, double *out, double *colm)
{
    dim3 grid((unsigned)(n / (256 * V)));
    auto go = [&] {
        hipLaunchKernelGGL((apply_cols<Tin, V, U, DIV, NT>), grid, dim3(256), 0, 0, (const Tin *)x, nchan, n, n,
                           factor, spec, bad, out, n, colm);
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
    printf("{\"kernel\": \"cols\", \"dtype\": \"%s\", \"V\": %d, \"U\": %d, \"div\": %d, \"nt\": %d, \"us\": %.1f, \"TBps\": %.3f}\n",
           name, V, U, DIV, (int)NT, us, bytes / (us * 1e-6) / 1e12);
    fflush(stdout);
    return 0;
}

template <typename Tin, int V, int RB, int U>
int run(const char *name, const void *x, int64_t nchan, int64_t n, const double *factor, const double *spec,
        const uint8_t *bad, double *out, double *part, unsigned long long *emax)
{
    dim3 grid((unsigned)(n / (256 * V)), (unsigned)((nchan + RB - 1) / RB));
    auto go = [&] {
        hipLaunchKernelGGL((apply_rows<Tin, V, RB, U>), grid, dim3(256), 0, 0, (const Tin *)x, nchan, n, n, factor,
                           spec, bad, out, n, part, emax);
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
    const double bytes = (double)nchan * n * (sizeof(Tin) + 8) + (double)grid.y * n * 8;
    printf("{\"dtype\": \"%s\", \"V\": %d, \"RB\": %d, \"U\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", name, V, RB, U, us,
           bytes / (us * 1e-6) / 1e12);
    fflush(stdout);
    return 0;
}

int main()
{
    const int64_t nchan = 1024, n = int64_t(1) << 18;
    void *xf, *xu;
    double *factor, *spec, *out, *part;
    uint8_t *bad;
    unsigned long long *emax;
    CK(hipMalloc(&xf, nchan * n * 4));
    CK(hipMalloc(&xu, nchan * n));
    CK(hipMalloc(&out, nchan * n * 8));
    CK(hipMalloc(&part, (nchan / 16 + 1) * n * 8));
    CK(hipMalloc(&factor, n * 8));
    CK(hipMalloc(&spec, nchan * 8));
    CK(hipMalloc(&bad, nchan));
    CK(hipMalloc(&emax, 8));
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
    rc |= runc<float, 4, 8, 1, false>("f32", xf, nchan, n, factor, spec, bad, out, part);
    rc |= runc<float, 4, 8, 0, false>("f32", xf, nchan, n, factor, spec, bad, out, part);
    rc |= runc<float, 2, 16, 1, false>("f32", xf, nchan, n, factor, spec, bad, out, part);
    rc |= runc<float, 2, 16, 0, false>("f32", xf, nchan, n, factor, spec, bad, out, part);
    rc |= runc<uint8_t, 2, 32, 1, true>("u8", xu, nchan, n, factor, spec, bad, out, part);
    rc |= runc<uint8_t, 2, 32, 0, true>("u8", xu, nchan, n, factor, spec, bad, out, part);
    rc |= runc<uint8_t, 4, 16, 1, true>("u8", xu, nchan, n, factor, spec, bad, out, part);
    rc |= runc<uint8_t, 4, 16, 0, true>("u8", xu, nchan, n, factor, spec, bad, out, part);
    rc |= runc<uint8_t, 2, 32, 1, false>("u8", xu, nchan, n, factor, spec, bad, out, part);
    rc |= run<float, 2, 64, 8>("f32", xf, nchan, n, factor, spec, bad, out, part, emax);
    return rc;
}
