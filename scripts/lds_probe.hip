// LDS-rate probes for the subband sum on gfx950 (one binary, no inputs): what does a
// ds_read_b64 issued with EXEC = 0 cost?  16 waves per workgroup, one workgroup per CU
// (64 KiB LDS), each iteration = 3 windows of 4 x ds_read_b64 + 8 adds per window.
//   full   : all 12 reads with every lane on
//   exec0  : the reads of one window in three with EXEC = 0 (a "duplicate" trial)
//   skip   : that window's reads not issued at all (8 reads per iteration)
//   allz   : all 12 reads with EXEC = 0 (pure issue cost)
//   nop    : that window's 4 reads replaced by 4 ds_nop (lgkmcnt-counted placeholders)
//   read2  : each window as 2 x ds_read2_b64 (offsets 0/512 and 1024/1536 B)
//   r2st64 : each window as 2 x ds_read2st64_b64
//   b128   : each window as 2 x ds_read_b128 (16 B per lane, 16-B aligned)
//   b128m8 : the same at addresses 8 B off the 16-B alignment
//   r2b32  : each window as 4 x ds_read2_b32 (8-B aligned), and 4 B off alignment
//   b64m4  : 4 x ds_read_b64 4 B off alignment
// Adds are v_pk_add_f32 (4 per window), as in the kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/lds_probe scripts/lds_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

template <int MODE>  // 0 full, 1 exec0 on window 1, 2 skip window 1, 3 all exec0, 4 ds_nop
__global__ void __launch_bounds__(1024) lds_kernel(float *out, const unsigned *offs)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *s = reinterpret_cast<float *>(smem);
    for (int i = threadIdx.x; i < 16384; i += 1024) s[i] = (float)i;
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;
    const int lane = threadIdx.x & 63;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 acc[4] = {};
    for (int it = 0; it < kIters; ++it) {
        const unsigned o = __builtin_amdgcn_readfirstlane(offs[it & 255]);
        double w[3][4];
        const uint32_t a0 = base + 8u * lane + (o & 0x3ff0u);
        const uint32_t a1 = base + 8u * lane + ((o >> 4) & 0x3ff0u);
        const uint32_t a2 = base + 8u * lane + ((o >> 8) & 0x3ff0u);
#define RD4(W, A)                                                                                      \
    asm volatile("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:512\n\t"                            \
                 "ds_read_b64 %2, %4 offset:1024\n\tds_read_b64 %3, %4 offset:1536"                    \
                 : "=&v"(W[0]), "=&v"(W[1]), "=&v"(W[2]), "=&v"(W[3])                                    \
                 : "v"(A)                                                                              \
                 : "memory");
        if constexpr (MODE >= 9) {
            // 9: ds_read2_b32 pairs at the 8-B aligned window addresses; 10: the same 4 B off
            // (an odd window of a single-copy slot); 11: ds_read_b64 4 B off alignment
            const uint32_t mo = MODE == 9 ? 0u : 4u;
            const uint32_t b0 = a0 + mo, b1 = a1 + mo, b2 = a2 + mo;
#define RD2W(W, A)                                                                                     \
    if constexpr (MODE == 11)                                                                          \
        asm volatile("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:512\n\t"                            \
                     "ds_read_b64 %2, %4 offset:1024\n\tds_read_b64 %3, %4 offset:1536"                    \
                     : "=&v"(W[0]), "=&v"(W[1]), "=&v"(W[2]), "=&v"(W[3]) : "v"(A) : "memory");           \
    else                                                                                               \
        asm volatile("ds_read2_b32 %0, %4 offset1:1\n\tds_read2_b32 %1, %4 offset0:128 offset1:129\n\t"  \
                     "ds_read2_b32 %2, %5 offset1:1\n\tds_read2_b32 %3, %5 offset0:128 offset1:129"        \
                     : "=&v"(W[0]), "=&v"(W[1]), "=&v"(W[2]), "=&v"(W[3]) : "v"(A), "v"(A + 1024u) : "memory");
            RD2W(w[0], b0) RD2W(w[1], b1) RD2W(w[2], b2)
#undef RD2W
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0][0]), "+v"(w[1][0]), "+v"(w[2][0]) : : "memory");
        } else if constexpr (MODE >= 5) {
            const uint32_t mo = MODE == 8 ? 8u : 0u;
            const uint32_t b0 = MODE >= 7 ? a0 + 8u * lane + mo : a0, b1 = MODE >= 7 ? a1 + 8u * lane + mo : a1,
                           b2 = MODE >= 7 ? a2 + 8u * lane + mo : a2;
#define RD2(W, A)                                                                                      \
    if constexpr (MODE == 5)                                                                           \
        asm volatile("ds_read2_b64 %0, %2 offset1:64\n\tds_read2_b64 %1, %2 offset0:128 offset1:192"     \
                     : "=&v"(W[0]), "=&v"(W[1]) : "v"(A) : "memory");                                  \
    else if constexpr (MODE == 6)                                                                      \
        asm volatile("ds_read2st64_b64 %0, %2 offset1:1\n\tds_read2st64_b64 %1, %2 offset0:2 offset1:3" \
                     : "=&v"(W[0]), "=&v"(W[1]) : "v"(A) : "memory");                                  \
    else                                                                                               \
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:1024"                          \
                     : "=&v"(W[0]), "=&v"(W[1]) : "v"(A) : "memory");
            typedef double f64x2 __attribute__((ext_vector_type(2)));
            f64x2 q[3][2];
            RD2(q[0], b0) RD2(q[1], b1) RD2(q[2], b2)
#undef RD2
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(q[0][0]), "+v"(q[1][0]), "+v"(q[2][0]) : : "memory");
            for (int i = 0; i < 3; ++i) {
                w[i][0] = q[i][0].x; w[i][1] = q[i][0].y; w[i][2] = q[i][1].x; w[i][3] = q[i][1].y;
            }
        } else if constexpr (MODE == 3) {
            uint64_t sv;
            asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 0" : "=s"(sv) : : "memory");
            RD4(w[0], a0) RD4(w[1], a1) RD4(w[2], a2)
            asm volatile("s_mov_b64 exec, %0" : : "s"(sv) : "memory");
        } else {
            RD4(w[0], a0)
            if constexpr (MODE == 1) {
                uint64_t sv;
                asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 0" : "=s"(sv) : : "memory");
                RD4(w[1], a1)
                asm volatile("s_mov_b64 exec, %0" : : "s"(sv) : "memory");
            } else if constexpr (MODE == 0) {
                RD4(w[1], a1)
            } else if constexpr (MODE == 4) {
                asm volatile("ds_nop\n\tds_nop\n\tds_nop\n\tds_nop" : : : "memory");
                for (int j = 0; j < 4; ++j) w[1][j] = w[0][j];
            } else {
                for (int j = 0; j < 4; ++j) w[1][j] = w[0][j];
            }
            RD4(w[2], a2)
        }
#undef RD4
        if constexpr (MODE < 5 || MODE >= 9)
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0][0]), "+v"(w[1][0]), "+v"(w[2][0]) : : "memory");
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[k]) : "v"(w[q][k]));
    }
    float t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) t += acc[k].x + acc[k].y;
    out[blockIdx.x * 1024 + threadIdx.x] = t;
}

// Width probes: MODE 0 = 8 x ds_read_b32, 1 = 4 x ds_read_b64 (same bytes), 2 = 8 x
// ds_write_addtid_b32 (M0 set once), 3 = 4 x ds_write_b64 (same bytes), 4 = 8 x ds_write_b32.
template <int MODE>
__global__ void __launch_bounds__(1024) width_kernel(float *out, const unsigned *offs)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float acc = 0.0f;
    const uint32_t wbase = base + (uint32_t)wave * 4096u;  // 4 KiB per wave
    for (int it = 0; it < kIters; ++it) {
        const unsigned o = __builtin_amdgcn_readfirstlane(offs[it & 255]) & 0x3f00u;  // 256-B aligned
        if constexpr (MODE == 0) {
            const uint32_t a = base + o + 4u * lane;
            float v[8];
            asm volatile("ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:256\n\tds_read_b32 %2, %8 offset:512\n\t"
                         "ds_read_b32 %3, %8 offset:768\n\tds_read_b32 %4, %8 offset:1024\n\t"
                         "ds_read_b32 %5, %8 offset:1280\n\tds_read_b32 %6, %8 offset:1536\n\t"
                         "ds_read_b32 %7, %8 offset:1792\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                           "=&v"(v[7]) : "v"(a) : "memory");
            for (int k = 0; k < 8; ++k) acc += v[k];
        } else if constexpr (MODE == 1) {
            const uint32_t a = base + o + 8u * lane;
            double v[4];
            asm volatile("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:512\n\tds_read_b64 %2, %4 offset:1024\n\t"
                         "ds_read_b64 %3, %4 offset:1536\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]) : "v"(a) : "memory");
            for (int k = 0; k < 4; ++k) acc += (float)v[k];
        } else if constexpr (MODE == 2) {
            const float x = (float)it;
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\t"
                         "ds_write_addtid_b32 %0\n\tds_write_addtid_b32 %0 offset:256\n\t"
                         "ds_write_addtid_b32 %0 offset:512\n\tds_write_addtid_b32 %0 offset:768\n\t"
                         "ds_write_addtid_b32 %0 offset:1024\n\tds_write_addtid_b32 %0 offset:1280\n\t"
                         "ds_write_addtid_b32 %0 offset:1536\n\tds_write_addtid_b32 %0 offset:1792\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : : "v"(x), "s"(__builtin_amdgcn_readfirstlane(wbase + (o & 0x300u))) : "memory");
            acc += x;
        } else if constexpr (MODE == 3) {
            const double x = (double)it;
            const uint32_t a = wbase + (o & 0x300u) + 8u * lane;
            asm volatile("ds_write_b64 %1, %0\n\tds_write_b64 %1, %0 offset:512\n\tds_write_b64 %1, %0 offset:1024\n\t"
                         "ds_write_b64 %1, %0 offset:1536\n\ts_waitcnt lgkmcnt(0)"
                         : : "v"(x), "v"(a) : "memory");
            acc += (float)x;
        } else if constexpr (MODE == 5) {
            // 8 x ds_read_u8 (one byte per lane each)
            const uint32_t a = base + o + lane;
            uint32_t v[8];
            asm volatile("ds_read_u8 %0, %8\n\tds_read_u8 %1, %8 offset:64\n\tds_read_u8 %2, %8 offset:128\n\t"
                         "ds_read_u8 %3, %8 offset:192\n\tds_read_u8 %4, %8 offset:256\n\t"
                         "ds_read_u8 %5, %8 offset:320\n\tds_read_u8 %6, %8 offset:384\n\t"
                         "ds_read_u8 %7, %8 offset:448\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                           "=&v"(v[7]) : "v"(a) : "memory");
            for (int k = 0; k < 8; ++k) acc += (float)v[k];
        } else if constexpr (MODE == 6) {
            // 2 x ds_write_b128 (2 KiB per wave)
            typedef float f4 __attribute__((ext_vector_type(4)));
            const f4 x = {(float)it, 1.0f, 2.0f, 3.0f};
            const uint32_t a = wbase + (o & 0x300u) * 0 + 16u * lane;
            asm volatile("ds_write_b128 %1, %0\n\tds_write_b128 %1, %0 offset:1024\n\ts_waitcnt lgkmcnt(0)"
                         : : "v"(x), "v"(a) : "memory");
            acc += x.x;
        } else {
            const float x = (float)it;
            const uint32_t a = wbase + (o & 0x300u) + 4u * lane;
            asm volatile("ds_write_b32 %1, %0\n\tds_write_b32 %1, %0 offset:256\n\tds_write_b32 %1, %0 offset:512\n\t"
                         "ds_write_b32 %1, %0 offset:768\n\tds_write_b32 %1, %0 offset:1024\n\t"
                         "ds_write_b32 %1, %0 offset:1280\n\tds_write_b32 %1, %0 offset:1536\n\t"
                         "ds_write_b32 %1, %0 offset:1792\n\ts_waitcnt lgkmcnt(0)"
                         : : "v"(x), "v"(a) : "memory");
            acc += x;
        }
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

using Kern = void (*)(float *, const unsigned *);

static double run(Kern k, float *out, const unsigned *offs, int blocks, double reads_per_iter)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(1024), 65536, 0, out, offs);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(1024), 65536, 0, out, offs);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double bytes = 5.0 * blocks * 1024.0 * kIters * reads_per_iter * 8.0;
    printf("  %.3f ms/launch, %.1f TB/s of 12-read-equivalent traffic\n", ms / 5, bytes / (ms * 1e-3) / 1e12);
    return ms / 5;
}

int main()
{
    const int blocks = 256 * 4;
    float *out;
    unsigned *offs;
    if (hipMalloc(&out, (size_t)blocks * 1024 * 4) != hipSuccess) return 1;
    if (hipMalloc(&offs, 256 * 4) != hipSuccess) return 1;
    unsigned h[256];
    unsigned s = 12345;
    for (int i = 0; i < 256; ++i) {
        s = s * 1103515245u + 12345u;
        h[i] = s;
    }
    (void)hipMemcpy(offs, h, sizeof h, hipMemcpyHostToDevice);
    if (hipFuncSetAttribute((const void *)lds_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<5>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<6>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<7>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<9>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) ||
        hipFuncSetAttribute((const void *)lds_kernel<11>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536))
        return 2;
    printf("full (12 reads):\n");
    run(lds_kernel<0>, out, offs, blocks, 12);
    printf("exec0 (8 reads + 4 with EXEC=0):\n");
    run(lds_kernel<1>, out, offs, blocks, 12);
    printf("skip (8 reads):\n");
    run(lds_kernel<2>, out, offs, blocks, 12);
    printf("all EXEC=0 (12 issued, none active):\n");
    run(lds_kernel<3>, out, offs, blocks, 12);
    printf("4 x ds_nop in place of one window:\n");
    run(lds_kernel<4>, out, offs, blocks, 12);
    printf("2 x ds_read2_b64 per window:\n");
    run(lds_kernel<5>, out, offs, blocks, 12);
    printf("2 x ds_read2st64_b64 per window:\n");
    run(lds_kernel<6>, out, offs, blocks, 12);
    printf("2 x ds_read_b128 per window:\n");
    run(lds_kernel<7>, out, offs, blocks, 12);
    printf("2 x ds_read_b128 per window, 8 B off alignment:\n");
    run(lds_kernel<8>, out, offs, blocks, 12);
    printf("4 x ds_read2_b32 per window (8-B aligned):\n");
    run(lds_kernel<9>, out, offs, blocks, 12);
    printf("4 x ds_read2_b32 per window, 4 B off alignment:\n");
    run(lds_kernel<10>, out, offs, blocks, 12);
    printf("4 x ds_read_b64 per window, 4 B off alignment:\n");
    run(lds_kernel<11>, out, offs, blocks, 12);
    for (auto k : {width_kernel<0>, width_kernel<1>, width_kernel<2>, width_kernel<3>, width_kernel<4>,
                   width_kernel<5>, width_kernel<6>})
        if (hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536)) return 3;
    printf("width: 8 x ds_read_b32 (2 KiB per wave):\n");
    run(width_kernel<0>, out, offs, blocks, 4);
    printf("width: 4 x ds_read_b64 (2 KiB per wave):\n");
    run(width_kernel<1>, out, offs, blocks, 4);
    printf("width: 8 x ds_write_addtid_b32 (2 KiB per wave):\n");
    run(width_kernel<2>, out, offs, blocks, 4);
    printf("width: 4 x ds_write_b64 (2 KiB per wave):\n");
    run(width_kernel<3>, out, offs, blocks, 4);
    printf("width: 8 x ds_write_b32 (2 KiB per wave):\n");
    run(width_kernel<4>, out, offs, blocks, 4);
    printf("width: 8 x ds_read_u8 (512 B per wave; TB/s column is 4x the bytes moved):\n");
    run(width_kernel<5>, out, offs, blocks, 4);
    printf("width: 2 x ds_write_b128 (2 KiB per wave):\n");
    run(width_kernel<6>, out, offs, blocks, 4);
    printf("(LDS peak 157.3 TB/s = 256 CU x 256 B/clk x 2.4 GHz)\n");
    const hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    (void)hipFree(out);
    (void)hipFree(offs);
    return 0;
}
