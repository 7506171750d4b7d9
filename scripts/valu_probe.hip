// Issue-rate probes for the dedispersion inner loop on gfx950 (one binary, no inputs):
//   1. v_add_f32 vs v_pk_add_f32 throughput (16 independent chains per lane)
//   2. register-window adds with a per-trial dynamic source offset:
//      (a) s_set_gpr_idx_on/off around 8 v_add_f32 (VGPR-relative src0)
//      (b) a compiler switch over the offset
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/valu_probe scripts/valu_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIters = 2048;

__global__ void __launch_bounds__(256) add_scalar(float *out, float seed, const unsigned *offs)
{
    float a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = seed + threadIdx.x + i;
    const float b = seed * 0.5f;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i];
    if (s == 12345.0f) out[threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) add_packed(float *out, float seed, const unsigned *offs)
{
    f32x2 a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = f32x2{seed + threadIdx.x + i, seed - i};
    const f32x2 b = f32x2{seed * 0.5f, seed * 0.25f};
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i].x + a[i].y;
    if (s == 12345.0f) out[threadIdx.x] = s;
}

// 2 trials x 8 samples of accumulators pinned to v[40:55], a 16-register window pinned
// to v[24:39]; per trial the window offset r (SGPR, 0..7) is applied by gpr_idx(SRC0).
__global__ void __launch_bounds__(256) add_gpr_idx(float *out, float seed, const unsigned *offs)
{
    f32x16 win, acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        win[i] = seed + threadIdx.x + i;
        acc[i] = 0.0f;
    }
    for (int it = 0; it < kIters; ++it) {
        const unsigned rec = __builtin_amdgcn_readfirstlane(offs[it & 255]);
        const unsigned r0 = rec & 7u, r1 = (rec >> 3) & 7u;
        asm volatile(
            "s_set_gpr_idx_on %2, gpr_idx(SRC0)\n\t"
            "v_add_f32 v40, v24, v40\n\tv_add_f32 v41, v25, v41\n\t"
            "v_add_f32 v42, v26, v42\n\tv_add_f32 v43, v27, v43\n\t"
            "v_add_f32 v44, v28, v44\n\tv_add_f32 v45, v29, v45\n\t"
            "v_add_f32 v46, v30, v46\n\tv_add_f32 v47, v31, v47\n\t"
            "s_set_gpr_idx_off\n\t"
            "s_set_gpr_idx_on %3, gpr_idx(SRC0)\n\t"
            "v_add_f32 v48, v24, v48\n\tv_add_f32 v49, v25, v49\n\t"
            "v_add_f32 v50, v26, v50\n\tv_add_f32 v51, v27, v51\n\t"
            "v_add_f32 v52, v28, v52\n\tv_add_f32 v53, v29, v53\n\t"
            "v_add_f32 v54, v30, v54\n\tv_add_f32 v55, v31, v55\n\t"
            "s_set_gpr_idx_off"
            : "+{v[40:55]}"(acc)
            : "{v[24:39]}"(win), "s"(r0), "s"(r1)
            );
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int R>
__device__ __forceinline__ void add8(float (&acc)[8], const float (&w)[16])
{
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += w[k + R];
}

__device__ __forceinline__ void add8_switch(float (&acc)[8], const float (&w)[16], unsigned r)
{
    switch (r) {
    case 0: add8<0>(acc, w); break;
    case 1: add8<1>(acc, w); break;
    case 2: add8<2>(acc, w); break;
    case 3: add8<3>(acc, w); break;
    case 4: add8<4>(acc, w); break;
    case 5: add8<5>(acc, w); break;
    case 6: add8<6>(acc, w); break;
    default: add8<7>(acc, w); break;
    }
}

__global__ void __launch_bounds__(256) add_switch(float *out, float seed, const unsigned *offs)
{
    float win[16], a0[8], a1[8];
#pragma unroll
    for (int i = 0; i < 16; ++i) win[i] = seed + threadIdx.x + i;
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = a1[i] = 0.0f;
    for (int it = 0; it < kIters; ++it) {
        const unsigned rec = __builtin_amdgcn_readfirstlane(offs[it & 255]);
        add8_switch(a0, win, rec & 7u);
        add8_switch(a1, win, (rec >> 3) & 7u);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a0[i] + a1[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}


// (b) idx mode on once per 4 trials; s_set_gpr_idx_idx between trials
__global__ void __launch_bounds__(256) add_gpr_idx2(float *out, float seed, const unsigned *offs)
{
    f32x16 win, acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        win[i] = seed + threadIdx.x + i;
        acc[i] = 0.0f;
    }
    for (int it = 0; it < kIters; it += 2) {
        const unsigned rec = __builtin_amdgcn_readfirstlane(offs[it & 255]);
        const unsigned r0 = rec & 7u, r1 = (rec >> 3) & 7u, r2 = (rec >> 1) & 7u, r3 = (rec >> 2) & 7u;
        asm volatile(
            "s_set_gpr_idx_on %2, gpr_idx(SRC0)\n\t"
            "v_add_f32 v40, v24, v40\n\tv_add_f32 v41, v25, v41\n\t"
            "v_add_f32 v42, v26, v42\n\tv_add_f32 v43, v27, v43\n\t"
            "v_add_f32 v44, v28, v44\n\tv_add_f32 v45, v29, v45\n\t"
            "v_add_f32 v46, v30, v46\n\tv_add_f32 v47, v31, v47\n\t"
            "s_set_gpr_idx_idx %3\n\t"
            "v_add_f32 v48, v24, v48\n\tv_add_f32 v49, v25, v49\n\t"
            "v_add_f32 v50, v26, v50\n\tv_add_f32 v51, v27, v51\n\t"
            "v_add_f32 v52, v28, v52\n\tv_add_f32 v53, v29, v53\n\t"
            "v_add_f32 v54, v30, v54\n\tv_add_f32 v55, v31, v55\n\t"
            "s_set_gpr_idx_idx %4\n\t"
            "v_add_f32 v40, v24, v40\n\tv_add_f32 v41, v25, v41\n\t"
            "v_add_f32 v42, v26, v42\n\tv_add_f32 v43, v27, v43\n\t"
            "v_add_f32 v44, v28, v44\n\tv_add_f32 v45, v29, v45\n\t"
            "v_add_f32 v46, v30, v46\n\tv_add_f32 v47, v31, v47\n\t"
            "s_set_gpr_idx_idx %5\n\t"
            "v_add_f32 v48, v24, v48\n\tv_add_f32 v49, v25, v49\n\t"
            "v_add_f32 v50, v26, v50\n\tv_add_f32 v51, v27, v51\n\t"
            "v_add_f32 v52, v28, v52\n\tv_add_f32 v53, v29, v53\n\t"
            "v_add_f32 v54, v30, v54\n\tv_add_f32 v55, v31, v55\n\t"
            "s_set_gpr_idx_off"
            : "+{v[40:55]}"(acc)
            : "{v[24:39]}"(win), "s"(r0), "s"(r1), "s"(r2), "s"(r3));
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// (e) control: same adds with plain SALU ops (no indexing) in place of the idx changes
__global__ void __launch_bounds__(256) add_salu_ctrl(float *out, float seed, const unsigned *offs)
{
    f32x16 win, acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        win[i] = seed + threadIdx.x + i;
        acc[i] = 0.0f;
    }
    for (int it = 0; it < kIters; ++it) {
        unsigned rec = __builtin_amdgcn_readfirstlane(offs[it & 255]);
        asm volatile(
            "s_add_u32 %1, %1, 1\n\t"
            "v_add_f32 v40, v24, v40\n\tv_add_f32 v41, v25, v41\n\t"
            "v_add_f32 v42, v26, v42\n\tv_add_f32 v43, v27, v43\n\t"
            "v_add_f32 v44, v28, v44\n\tv_add_f32 v45, v29, v45\n\t"
            "v_add_f32 v46, v30, v46\n\tv_add_f32 v47, v31, v47\n\t"
            "s_add_u32 %1, %1, 1\n\t"
            "s_add_u32 %1, %1, 1\n\t"
            "v_add_f32 v48, v24, v48\n\tv_add_f32 v49, v25, v49\n\t"
            "v_add_f32 v50, v26, v50\n\tv_add_f32 v51, v27, v51\n\t"
            "v_add_f32 v52, v28, v52\n\tv_add_f32 v53, v29, v53\n\t"
            "v_add_f32 v54, v30, v54\n\tv_add_f32 v55, v31, v55\n\t"
            "s_add_u32 %1, %1, 1"
            : "+{v[40:55]}"(acc), "+s"(rec)
            : "{v[24:39]}"(win)
            : "scc");
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

using Kern = void (*)(float *, float, const unsigned *);

static double run(Kern k, float *out, const unsigned *offs, int blocks, double adds_per_iter)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0f, offs);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1.0f, offs);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return 5.0 * blocks * 256.0 * kIters * adds_per_iter / (ms * 1e-3);
}

int main()
{
    const int blocks = 256 * 8 * 4;
    float *out;
    unsigned *offs;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    if (hipMalloc(&offs, 256 * 4) != hipSuccess) return 1;
    unsigned h[256];
    unsigned s = 12345;
    for (int i = 0; i < 256; ++i) {
        s = s * 1103515245u + 12345u;
        h[i] = (s >> 8) & 63u;
    }
    (void)hipMemcpy(offs, h, sizeof h, hipMemcpyHostToDevice);
    printf("v_add_f32          %.2f T adds/s\n", run(add_scalar, out, offs, blocks, 16) / 1e12);
    printf("v_pk_add_f32       %.2f T adds/s\n", run(add_packed, out, offs, blocks, 16) / 1e12);
    printf("gpr_idx window     %.2f T adds/s\n", run(add_gpr_idx, out, offs, blocks, 16) / 1e12);
    printf("gpr_idx_idx window %.2f T adds/s\n", run(add_gpr_idx2, out, offs, blocks, 16) / 1e12);
    printf("salu ctrl window   %.2f T adds/s\n", run(add_salu_ctrl, out, offs, blocks, 16) / 1e12);
    printf("switch window      %.2f T adds/s\n", run(add_switch, out, offs, blocks, 16) / 1e12);
    printf("(peak 78.6 T adds/s = 256 CU x 128 lanes x 2.4 GHz)\n");
    (void)hipFree(out);
    (void)hipFree(offs);
    return 0;
}
