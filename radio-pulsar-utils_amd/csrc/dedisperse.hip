// Incoherent (brute-force) shift-and-sum dedispersion for gfx950 (MI355X).
//
// Replaces the reference hot loop (pulsarutils/dedispersion.py):
//   _dedispersion_search :174-202  (prange over trials -> workgroups over DM tiles)
//   dedisperse/_dedisperse/roll_and_sum :60-98 (circular shift-and-sum, channel order)
//
// out_d[t] = sum_c x[c][(t + s[d][c]) mod N]   (s = dedispersion_shifts, any sign)
//
// Mapping:
//   * one workgroup = 8 waves = one DM tile (64 trials) x one time tile; each wave
//     owns D = 8 trials, lane l owns K samples (float: t0 + 2l + 128j + e, j<4, e<2)
//     -> D*K accumulators in VGPRs.
//   * channel rows are staged in LDS, ncc channels per chunk, each row covering
//     [t0 + smin_c, t0 + TT + smax_c) mod N: the tile's modular halo.  Rows arrive by
//     LDS-DMA (global_load_lds, 1 KiB pieces, per-lane modular addresses only for
//     the rare windows that wrap) into a two-buffer ring: chunk k+1 lands while chunk
//     k is summed.  Converting inputs (u8, f64 -> f32 LDS) use register staging.
//   * per (tile, channel, wave) the host precomputes 8 x u16 "window records": the LDS
//     byte offset of each trial's K-sample window (alignment copy included) and, in
//     bit 15, whether it differs from the previous trial's.  One scalar load per
//     channel; per trial one s_bitcmp1 + branch; the window is re-read (in place, 4 x
//     ds_read_b64) only when it changes -- adjacent plan trials differ by <= 1 sample
//     per channel, so most v_add_f32 reuse registers.  The first window of the next
//     channel is prefetched into the other window buffer while this one is summed.
//   * accumulation in channel order 0..nchan-1 (reference order: with a float64
//     accumulator the series is bit-identical).
//   * epilogue: the dedispersed plane, or per-tile partial statistics of the
//     1/2/4/8-sample rebinned series reduced by pu_finalize_kernel in a fixed order.
//   * blockIdx is remapped XCD-aware so all DM tiles of a time tile run on one XCD.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "pu_common.h"

namespace {

constexpr int kWaves = 10;                // waves per workgroup (each owns D trials): 2 WGs = 5 waves/SIMD
constexpr int kThreads = kWaves * 64;
constexpr int kD = 8;                     // trials per wave
constexpr int kTPT = kWaves * kD;         // trials per tile
constexpr int kPartStride = 16;           // doubles per (trial, time tile) partial record
constexpr size_t kLdsBudget = 64 * 1024;  // per workgroup: 2 workgroups / CU
constexpr int kMaxR = 4;                  // pair mode: distinct relative shifts per pair and tile
constexpr int kMaxSpread = 2048;

struct DedispArgs {
    const void *data;
    int64_t ld;
    int32_t nchan;
    int32_t n;
    int32_t ndt;
    int32_t ntt;
    int32_t ncc;
    int32_t row_stride;
    int32_t small_n;
    int32_t pad0;
    void *plane;
    int64_t ld_plane;
    double *partials;
    // pair mode
    int32_t raw_stride;   // bytes per staged raw channel row
    int32_t pair_bytes;   // bytes per pair slot in the pair-row region
    int32_t nrmax;        // pair rows per slot
    int32_t npairs;
};

template <typename T>
__device__ __forceinline__ T shfl_down(T v, int d)
{
    return __shfl_down(v, d, 64);
}

template <typename T>
__device__ __forceinline__ T shfl_xor(T v, int d)
{
    return __shfl_xor(v, d, 64);
}

// Uniform (scalar-cache) load: the constant address space makes hipcc emit s_load.
template <typename T>
__device__ __forceinline__ T ld_uniform(const T *p)
{
    return *(const __attribute__((address_space(4))) T *)(p);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));  // pair metadata {base0, base1, offsets, nr}

// In-place K-sample window read: 4 x ds_read_b64 at 512-byte strides + wait.  One asm
// block that overwrites the window registers, so the register allocator never keeps
// two versions alive.  Outputs are early-clobber: an LDS read can return (and write
// its destination) before the block's later reads have consumed the address VGPR.
__device__ __forceinline__ void read_window(double (&w)[4], uint32_t addr)
{
    asm volatile(
        "ds_read_b64 %0, %4\n\t"
        "ds_read_b64 %1, %4 offset:512\n\t"
        "ds_read_b64 %2, %4 offset:1024\n\t"
        "ds_read_b64 %3, %4 offset:1536\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
        : "v"(addr)
        : "memory");
}

// Same reads without the wait (prefetch of the next channel's first window); the
// registers are only consumed after wait_window() on them.
__device__ __forceinline__ void prefetch_window(double (&w)[4], uint32_t addr)
{
    asm volatile(
        "ds_read_b64 %0, %4\n\t"
        "ds_read_b64 %1, %4 offset:512\n\t"
        "ds_read_b64 %2, %4 offset:1024\n\t"
        "ds_read_b64 %3, %4 offset:1536"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
        : "v"(addr)
        : "memory");
}

__device__ __forceinline__ void wait_window(double (&w)[4])
{
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]) : : "memory");
}

// Empty asm that "uses" one trial's accumulators: keeps each trial's adds ahead of the
// next window reload (otherwise hipcc sinks all adds to the end of the channel and
// keeps every window version alive in separate registers).
template <typename Ta, int K>
__device__ __forceinline__ void pin_accumulators(Ta (&acc)[K])
{
    if constexpr (K == 8)
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
                     "+v"(acc[6]), "+v"(acc[7]));
    else
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
}

template <typename Tl>
__device__ __forceinline__ Tl window_elem(const double (&w)[4], int k)
{
    if constexpr (sizeof(Tl) == 8) {
        return w[k];
    } else {
        const uint64_t b = __builtin_bit_cast(uint64_t, w[k >> 1]);
        return __builtin_bit_cast(float, (uint32_t)((k & 1) ? (b >> 32) : b));
    }
}

// Add one channel's contribution to all D trials of this wave.  ``rec`` = 8 u16
// window records (byte offset | reload flag << 15); ``w`` holds trial 0's window.
template <typename Tl, typename Ta, int K>
__device__ __forceinline__ void channel_trials(Ta (&acc)[kD][K], double (&w)[4], const u32x4 rec, uint32_t cbase)
{
#pragma unroll
    for (int d = 0; d < kD; ++d) {
        if (d > 0) {
            const uint32_t word = rec[d >> 1] >> (16 * (d & 1));
            if (word & 0x8000u) read_window(w, cbase + (word & 0x7fffu));
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] += static_cast<Ta>(window_elem<Tl>(w, k));
        pin_accumulators(acc[d]);
    }
}

// Outputs of one wave: the dedispersed plane rows of its D trials, or their per-tile
// partial statistics (1/2/4/8-sample rebinned sums: max, shifted sum, shifted sum of
// squares; lane-local in the accumulation type, then float64 wave reductions).
template <typename Tl, typename Ta, int K, bool PLANE, bool STATS>
__device__ __forceinline__ void write_outputs(const Ta (&acc)[kD][K], const DedispArgs &a, int first, int slot0,
                                              int cnt, int t0, int tt, int lane)
{
    constexpr int E = 8 / (int)sizeof(Tl);
    constexpr int J = K / E;
    constexpr int D = kD;
    const int n = a.n;
    // sample index of acc[.][k] for this lane
    auto sample = [&](int k) { return t0 + E * lane + 64 * E * (k / E) + (k % E); };

    if constexpr (PLANE) {
        Ta *plane = reinterpret_cast<Ta *>(a.plane);
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (slot0 + d >= cnt) break;
            Ta *orow = plane + (size_t)(first + slot0 + d) * (size_t)a.ld_plane;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int t = sample(k);
                if (t < n) orow[t] = acc[d][k];
            }
        }
    }
    if constexpr (STATS) {
        // Per trial: lane-local stats of the 1/2/4/8-sample rebinned sums in the
        // accumulation type (few terms), then float64 wave reductions.
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (slot0 + d >= cnt) break;
            const Ta kt = __shfl(acc[d][0], 0, 64);
            Ta mx[4], s1[4], s2[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                mx[w] = -INFINITY;
                s1[w] = Ta(0);
                s2[w] = Ta(0);
            }
            auto account = [&](int w, Ta r, int t, bool lane_ok) {
                const int width = 1 << w;
                if (lane_ok && t + width <= n) {
                    const Ta y = r - Ta(width) * kt;
                    mx[w] = fmax(mx[w], r);
                    s1[w] += y;
                    s2[w] += y * y;
                }
            };
#pragma unroll
            for (int j = 0; j < J; ++j) {
                if constexpr (E == 2) {
                    const Ta a0 = acc[d][2 * j], a1 = acc[d][2 * j + 1];
                    const int t = sample(2 * j);
                    account(0, a0, t, true);
                    account(0, a1, t + 1, true);
                    Ta r = a0 + a1;                       // width 2, in-lane
                    account(1, r, t, true);
                    r += shfl_down(r, 1);                 // width 4
                    account(2, r, t, (lane & 1) == 0);
                    r += shfl_down(r, 2);                 // width 8
                    account(3, r, t, (lane & 3) == 0);
                } else {
                    Ta r = acc[d][j];
                    const int t = sample(j);
                    account(0, r, t, true);
#pragma unroll
                    for (int w = 1; w < 4; ++w) {
                        r += shfl_down(r, 1 << (w - 1));
                        account(w, r, t, (lane & ((1 << w) - 1)) == 0);
                    }
                }
            }
            double* p = a.partials + ((size_t)(first + slot0 + d) * a.ntt + tt) * kPartStride;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                Ta m = mx[w];
                double x1 = static_cast<double>(s1[w]), x2 = static_cast<double>(s2[w]);
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) {
                    m = fmax(m, shfl_xor(m, off));
                    x1 += shfl_xor(x1, off);
                    x2 += shfl_xor(x2, off);
                }
                if (lane == 0) {
                    p[1 + 3 * w] = static_cast<double>(m);
                    p[2 + 3 * w] = x1;
                    p[3 + 3 * w] = x2;
                }
            }
            if (lane == 0) p[0] = static_cast<double>(kt);
        }
    }
}

// float32 accumulators: 2 workgroups x 10 waves per CU = 5 waves per SIMD (<= 96 VGPRs);
// float64 accumulators (reference-exact mode, 128 accumulator VGPRs): 1 workgroup.
template <typename Ta>
constexpr int min_waves_per_simd() { return sizeof(Ta) == 8 ? 3 : 5; }

template <typename Tin, typename Tl, typename Ta, bool PLANE, bool STATS>
__global__ void __launch_bounds__(kThreads, min_waves_per_simd<Ta>())
dedisp_kernel(DedispArgs a, const int32_t *__restrict__ tile_first, const int32_t *__restrict__ tile_count,
              const int32_t *__restrict__ tile_rowlen, const int32_t *__restrict__ base_tab,
              const u32x4 *__restrict__ rec_tab)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool kDma = std::is_same<Tin, Tl>::value;
    constexpr int SZ = (int)sizeof(Tl);
    constexpr int E = 8 / SZ;     // samples per 8-byte LDS read
    constexpr int J = 4;          // reads per window
    constexpr int K = E * J;      // samples per lane
    constexpr int TT = 64 * K;    // samples per time tile
    constexpr int D = kD;

    const int wg = pu::xcd_remap(blockIdx.x, gridDim.x);
    const int dt = wg % a.ndt;
    const int tt = wg / a.ndt;
    const int t0 = tt * TT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int first = ld_uniform(tile_first + dt);
    const int cnt = ld_uniform(tile_count + dt);
    const int rowlen = ld_uniform(tile_rowlen + dt);
    const int slot0 = wave * D;
    const bool active = slot0 < cnt;
    const int n = a.n;
    const int stride = a.row_stride;           // elements per row copy
    const int copy_bytes = stride * SZ;
    const int chan_bytes = E * copy_bytes;
    const int buf_bytes = a.ncc * chan_bytes;
    // LDS byte address of the dynamic region (local-address-space pointer -> 32-bit offset)
    const uint32_t smem_addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;

    Ta acc[D][K];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] = Ta(0);

    const int32_t *base = base_tab + (size_t)dt * a.nchan;
    const u32x4 *recs = rec_tab + (size_t)dt * a.nchan * kWaves + wave;
    const Tin *data = reinterpret_cast<const Tin *>(a.data);
    const int nchunks = (a.nchan + a.ncc - 1) / a.ncc;
    // bytes of a row copy actually moved (whole 256-byte pieces)
    const int cover_bytes = (rowlen * SZ + 255) & ~255;
    const int cover = cover_bytes / SZ;

    // ---- LDS-DMA of chunk k into ring buffer b: each wave moves whole row copies
    auto issue_dma = [&](int k, int b) {
        const int c0 = k * a.ncc;
        const int nc = min(a.ncc, a.nchan - c0);
        const uint32_t bufo = (uint32_t)(b * buf_bytes);
        for (int r = wave; r < nc * E; r += kWaves) {
            const int ci = r / E, q = r % E;
            const int c = c0 + ci;
            const char *row = reinterpret_cast<const char *>(data + (size_t)c * (size_t)a.ld);
            int start = ld_uniform(base + c) + t0 + q;
            if (start >= n) start -= n;
            if (start >= n) start -= n;
            unsigned char *dst = smem + bufo + ci * chan_bytes + q * copy_bytes;
            if (!a.small_n && start + cover <= n) {
                // contiguous window: 1 KiB pieces (16 B/lane), then 256 B pieces
                const char *src = row + (size_t)start * SZ;
                int off = 0;
                for (; off + 1024 <= cover_bytes; off += 1024)
                    __builtin_amdgcn_global_load_lds((const void *)(src + off + 16 * lane),
                                                     (__attribute__((address_space(3))) void *)(dst + off), 16, 0, 0);
                for (; off < cover_bytes; off += 256)
                    __builtin_amdgcn_global_load_lds((const void *)(src + off + 4 * lane),
                                                     (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
            } else {
                // wrapping window: per-lane modular element index, 4 B per lane
                for (int off = 0; off < cover_bytes; off += 256) {
                    const int byte = off + 4 * lane;
                    int idx = start + byte / SZ;
                    if (!a.small_n) {
                        idx = idx >= n ? idx - n : idx;
                    } else {
                        idx %= n;
                    }
                    const char *src = row + (size_t)idx * SZ + (byte % SZ);
                    __builtin_amdgcn_global_load_lds((const void *)src,
                                                     (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
                }
            }
        }
    };

    // ---- register staging for converting inputs (u8 -> f32, f64 -> f32)
    auto stage_regs = [&](int k) {
        const int c0 = k * a.ncc;
        const int nc = min(a.ncc, a.nchan - c0);
        for (int ci = 0; ci < nc; ++ci) {
            const int c = c0 + ci;
            const Tin *row = data + (size_t)c * (size_t)a.ld;
            int start = ld_uniform(base + c) + t0;
            if (start >= n) start -= n;
            Tl *dst = reinterpret_cast<Tl *>(smem + ci * chan_bytes);
            const int len = rowlen + E - 1;
            for (int j = tid; j < len; j += kThreads) {
                int idx = start + j;
                if (!a.small_n) {
                    if (idx >= n) idx -= n;
                } else {
                    idx %= n;
                }
                const Tl v = static_cast<Tl>(row[idx]);
                if (j < rowlen) dst[j] = v;
                if constexpr (E == 2) {
                    if (j >= 1) dst[stride + j - 1] = v;
                }
            }
        }
    };

    if constexpr (kDma) issue_dma(0, 0);
    for (int k = 0; k < nchunks; ++k) {
        const int c0 = k * a.ncc;
        const int nc = min(a.ncc, a.nchan - c0);
        const int b = kDma ? (k & 1) : 0;
        __syncthreads();  // this wave's DMA landed (vmcnt) and every wave left the other buffer
        if constexpr (kDma) {
            if (k + 1 < nchunks) issue_dma(k + 1, b ^ 1);
        } else {
            stage_regs(k);
            __syncthreads();
        }
        if (!active) continue;
        // ---- accumulate the chunk: channel pairs alternate window buffers so the next
        // channel's first window is read while this one is summed
        const uint32_t rows_lane = smem_addr + (uint32_t)(b * buf_bytes) + 8u * lane;
        double w0[4], w1[4];
        const u32x4 *rc = recs + (size_t)c0 * kWaves;
        u32x4 rec0 = ld_uniform(rc);
        u32x4 rec1 = nc > 1 ? ld_uniform(rc + kWaves) : rec0;
        read_window(w0, rows_lane + (rec0[0] & 0x7fffu));
        for (int ci = 0; ci < nc; ci += 2) {
            const uint32_t cb0 = rows_lane + (uint32_t)(ci * chan_bytes);
            const bool has1 = ci + 1 < nc, has2 = ci + 2 < nc, has3 = ci + 3 < nc;
            u32x4 rec2 = rec0, rec3 = rec1;
            if (has2) rec2 = ld_uniform(rc + (size_t)(ci + 2) * kWaves);  // two channels ahead
            if (has1) prefetch_window(w1, cb0 + chan_bytes + (rec1[0] & 0x7fffu));
            channel_trials<Tl, Ta, K>(acc, w0, rec0, cb0);
            if (!has1) break;
            wait_window(w1);
            if (has3) rec3 = ld_uniform(rc + (size_t)(ci + 3) * kWaves);
            if (has2) prefetch_window(w0, cb0 + 2 * chan_bytes + (rec2[0] & 0x7fffu));
            channel_trials<Tl, Ta, K>(acc, w1, rec1, cb0 + chan_bytes);
            if (has2) wait_window(w0);
            rec0 = rec2;
            rec1 = rec3;
        }
    }
    if (!active) return;

    write_outputs<Tl, Ta, K, PLANE, STATS>(acc, a, first, slot0, cnt, t0, tt, lane);
}


// ---------------------------------------------------------------------------------
// Pair mode (float32 accumulation of u8 / f32 / f64 inputs).
//
// For adjacent channels (c0, c1) = (2p, 2p+1) and the tile's trials, channel c1's
// shift relative to c0's, r_d = s_d,c1 - s_d,c0, takes nr <= 4 distinct values
// (adjacent channels' delays drift apart by ~1/nchan sample per trial).  Each chunk
// stages the raw channel rows by LDS-DMA, then one combine pass writes, for every
// distinct r, the pair row P_r[j] = x_c0[b0 + j] + x_c1[b0 + r + j] (two alignment
// copies); a trial then adds ONE pair row per pair: half the adds, half the windows,
// half the scalar work of the channel mode, exact shift indexing.  Only the float32
// summation order changes (x_c0 + x_c1 first); uint8 sums stay exact.
//
// Per (tile, pair) metadata int4 {base0, base1 (-1: no partner, odd nchan),
// packed 8-bit row offsets r_i - rmin, nr}; window records index the pair rows.
template <typename Tin>
__device__ __forceinline__ float raw_at(const unsigned char *row, int i)
{
    return static_cast<float>(reinterpret_cast<const Tin *>(row)[i]);
}

// Byte shift between a uint8 raw row's first sample and the dword-aligned address its
// contiguous DMA started from (0 for wrapping rows, which are moved byte by byte).
__device__ __forceinline__ int row_shift(int base, int t0, int n, int raw_elems, int small_n)
{
    int start = base + t0;
    if (start >= n) start -= n;
    const int al = start & ~3;
    return (!small_n && al + raw_elems <= n) ? start - al : 0;
}

template <typename Tin, typename Ta, bool PLANE, bool STATS>
__global__ void __launch_bounds__(kThreads, min_waves_per_simd<Ta>())
dedisp_pair_kernel(DedispArgs a, const int32_t *__restrict__ tile_first, const int32_t *__restrict__ tile_count,
                   const int32_t *__restrict__ tile_rowlen, const i32x4 *__restrict__ pmeta,
                   const u32x4 *__restrict__ rec_tab)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    typedef float Tl;
    constexpr int SZ = (int)sizeof(Tin);
    constexpr int E = 2;
    constexpr int K = 8;
    constexpr int TT = 64 * K;
    constexpr int D = kD;

    const int wg = pu::xcd_remap(blockIdx.x, gridDim.x);
    const int dt = wg % a.ndt;
    const int tt = wg / a.ndt;
    const int t0 = tt * TT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int first = ld_uniform(tile_first + dt);
    const int cnt = ld_uniform(tile_count + dt);
    const int rowlen = ld_uniform(tile_rowlen + dt);
    const int slot0 = wave * D;
    const bool active = slot0 < cnt;
    const int n = a.n;
    const int stride = a.row_stride;            // floats per pair-row copy
    const int raw_stride = a.raw_stride;        // bytes per raw row
    const int raw_elems = raw_stride / SZ;
    const int pair_bytes = a.pair_bytes;
    const int raw_region = a.ncc * 2 * raw_stride;
    const uint32_t smem_addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;

    Ta acc[D][K];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] = Ta(0);

    const i32x4 *pm_tile = pmeta + (size_t)dt * a.npairs;
    const u32x4 *recs = rec_tab + (size_t)dt * a.npairs * kWaves + wave;
    const Tin *data = reinterpret_cast<const Tin *>(a.data);
    const int nchunks = (a.npairs + a.ncc - 1) / a.ncc;

    // ---- raw rows of chunk k by LDS-DMA: row 2*pi + w = channel c0 (w=0) / c1 (w=1)
    auto issue_dma = [&](int k) {
        const int p0 = k * a.ncc;
        const int nc = min(a.ncc, a.npairs - p0);
        for (int r = wave; r < nc * 2; r += kWaves) {
            const int pi = r >> 1, w = r & 1;
            const i32x4 pm = ld_uniform(pm_tile + p0 + pi);
            const int b = w ? pm.y : pm.x;
            if (b < 0) continue;
            const int c = 2 * (p0 + pi) + w;
            const char *row = reinterpret_cast<const char *>(data + (size_t)c * (size_t)a.ld);
            int start = b + t0;
            if (start >= n) start -= n;
            unsigned char *dst = smem + (pi * 2 + w) * raw_stride;
            if (SZ == 1) start &= ~3;  // dword-aligned DMA source; combine() adds the 0-3 byte shift
            if (!a.small_n && start + raw_elems <= n) {
                const char *src = row + (size_t)start * SZ;
                int off = 0;
                for (; off + 1024 <= raw_stride; off += 1024)
                    __builtin_amdgcn_global_load_lds((const void *)(src + off + 16 * lane),
                                                     (__attribute__((address_space(3))) void *)(dst + off), 16, 0, 0);
                for (; off < raw_stride; off += 256)
                    __builtin_amdgcn_global_load_lds((const void *)(src + off + 4 * lane),
                                                     (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
            } else if constexpr (SZ == 1) {
                start = b + t0;  // wrapping row: unaligned start, byte-wise modular DMA
                if (start >= n) start -= n;
                for (int off = 0; off < raw_stride; off += 64) {
                    int idx = start + off + lane;
                    idx = a.small_n ? idx % n : (idx >= n ? idx - n : idx);
                    __builtin_amdgcn_global_load_lds((const void *)(row + idx),
                                                     (__attribute__((address_space(3))) void *)(dst + off), 1, 0, 0);
                }
            } else {
                for (int off = 0; off < raw_stride; off += 256) {
                    const int byte = off + 4 * lane;
                    int idx = start + byte / SZ;
                    idx = a.small_n ? idx % n : (idx >= n ? idx - n : idx);
                    __builtin_amdgcn_global_load_lds((const void *)(row + (size_t)idx * SZ + (byte % SZ)),
                                                     (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
                }
            }
        }
    };

    // ---- combine pass: pair rows (two aligned copies) from the raw rows, 4 samples
    // per work item: copy0[j..j+3] = P[j..j+3], copy1[j..j+3] = P[j+1..j+4]
    // exact division of small non-negative ints by a runtime divisor: x / d ==
    // umulhi(x, ceil(2^32 / d)) for x * d < 2^32 (here x < 2^16)
    const int nq = (rowlen + 3) >> 2;
    const uint32_t magic_nq = 0xffffffffu / (uint32_t)nq + 1u;
    const uint32_t magic_nr = 0xffffffffu / (uint32_t)a.nrmax + 1u;
    auto combine = [&](int k) {
        const int p0 = k * a.ncc;
        const int nc = min(a.ncc, a.npairs - p0);
        const int total = nc * a.nrmax * nq;
        for (int item = tid; item < total; item += kThreads) {
            const int pr = (int)__umulhi((uint32_t)item, magic_nq);   // pair-row slot
            const int j = (item - pr * nq) * 4;
            const int pi = (int)__umulhi((uint32_t)pr, magic_nr);
            const int ri = pr - pi * a.nrmax;
            const i32x4 pm = pm_tile[p0 + pi];
            if (ri >= pm.w) continue;
            int roff = (pm.z >> (8 * ri)) & 0xff;
            const unsigned char *raw0 = smem + pi * 2 * raw_stride;
            const unsigned char *raw1 = raw0 + raw_stride;
            if constexpr (SZ == 1) {  // undo the DMA's dword alignment of contiguous rows
                raw0 += row_shift(pm.x, t0, n, raw_elems, a.small_n);
                if (pm.y >= 0) roff += row_shift(pm.y, t0, n, raw_elems, a.small_n);
            }
            float v[5];
#pragma unroll
            for (int e = 0; e < 5; ++e) v[e] = raw_at<Tin>(raw0, j + e);
            if (pm.y >= 0) {
#pragma unroll
                for (int e = 0; e < 5; ++e) v[e] += raw_at<Tin>(raw1, j + roff + e);
            }
            float *prow = reinterpret_cast<float *>(smem + raw_region + pi * pair_bytes) + ri * 2 * stride + j;
            *reinterpret_cast<float4 *>(prow) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4 *>(prow + stride) = make_float4(v[1], v[2], v[3], v[4]);
        }
    };

    issue_dma(0);
    for (int k = 0; k < nchunks; ++k) {
        const int p0 = k * a.ncc;
        const int nc = min(a.ncc, a.npairs - p0);
        __syncthreads();  // raw(k) landed; every wave left the pair rows of chunk k-1
        combine(k);
        __syncthreads();  // pair rows ready; raw rows free
        if (k + 1 < nchunks) issue_dma(k + 1);
        if (!active) continue;
        const uint32_t rows_lane = smem_addr + (uint32_t)raw_region + 8u * lane;
        double w0[4], w1[4];
        const u32x4 *rc = recs + (size_t)p0 * kWaves;
        u32x4 rec0 = ld_uniform(rc);
        u32x4 rec1 = nc > 1 ? ld_uniform(rc + kWaves) : rec0;
        read_window(w0, rows_lane + (rec0[0] & 0x7fffu));
        for (int ci = 0; ci < nc; ci += 2) {
            const uint32_t cb0 = rows_lane + (uint32_t)(ci * pair_bytes);
            const bool has1 = ci + 1 < nc, has2 = ci + 2 < nc, has3 = ci + 3 < nc;
            u32x4 rec2 = rec0, rec3 = rec1;
            if (has2) rec2 = ld_uniform(rc + (size_t)(ci + 2) * kWaves);
            if (has1) prefetch_window(w1, cb0 + pair_bytes + (rec1[0] & 0x7fffu));
            channel_trials<Tl, Ta, K>(acc, w0, rec0, cb0);
            if (!has1) break;
            wait_window(w1);
            if (has3) rec3 = ld_uniform(rc + (size_t)(ci + 3) * kWaves);
            if (has2) prefetch_window(w0, cb0 + 2 * pair_bytes + (rec2[0] & 0x7fffu));
            channel_trials<Tl, Ta, K>(acc, w1, rec1, cb0 + pair_bytes);
            if (has2) wait_window(w0);
            rec0 = rec2;
            rec1 = rec3;
        }
    }
    if (!active) return;
    write_outputs<Tl, Ta, K, PLANE, STATS>(acc, a, first, slot0, cnt, t0, tt, lane);
}

// One workgroup per trial: combine the per-time-tile partials in a fixed order
// (thread-strided then an LDS tree: deterministic), then the reference's S/N logic
// (dedispersion.py:186-201): snr_w = max(reb_w)/std(reb_w), first strict best.
__global__ void __launch_bounds__(256)
pu_finalize_kernel(const double *__restrict__ part, int ntt, int n, int tt_len,
                   double *max_out, double *std_out, double *snr_out, int32_t *win_out)
{
    __shared__ double red[3][4][256];
    const int trial = blockIdx.x;
    const int tid = threadIdx.x;
    const double *p = part + (size_t)trial * ntt * kPartStride;
    const double mu = p[0];
    double S1[4] = {0, 0, 0, 0}, S2[4] = {0, 0, 0, 0}, MX[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int i = tid; i < ntt; i += 256) {
        const double *q = p + (size_t)i * kPartStride;
        const double dk = q[0] - mu;
        for (int w = 0; w < 4; ++w) {
            const int width = 1 << w;
            const long lo = (long)i * tt_len / width;
            const long hi = min((long)(i + 1) * tt_len / width, (long)(n / width));
            const double cntb = (double)max(0L, hi - lo);
            if (cntb <= 0) continue;
            const double s1 = q[2 + 3 * w], s2 = q[3 + 3 * w];
            const double wd = width * dk;
            S1[w] += s1 + cntb * wd;
            S2[w] += s2 + 2.0 * wd * s1 + cntb * wd * wd;
            MX[w] = fmax(MX[w], q[1 + 3 * w]);
        }
    }
    for (int w = 0; w < 4; ++w) {
        red[0][w][tid] = S1[w];
        red[1][w][tid] = S2[w];
        red[2][w][tid] = MX[w];
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) {
            for (int w = 0; w < 4; ++w) {
                red[0][w][tid] += red[0][w][tid + s];
                red[1][w][tid] += red[1][w][tid + s];
                red[2][w][tid] = fmax(red[2][w][tid], red[2][w][tid + s]);
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        const double mean = mu + red[0][0][0] / n;  // mean of the dedispersed series
        double best = 0.0;
        int bestw = 0;
        double sd1 = 0.0;
        for (int w = 0; w < 4; ++w) {
            const int width = 1 << w;
            const long nb = n / width;
            if (nb <= 0) continue;
            const double m1 = red[0][w][0] / nb;
            const double var = red[1][w][0] / nb - m1 * m1;
            const double sd = sqrt(var > 0 ? var : 0.0);
            if (w == 0) sd1 = sd;
            const double snr = (red[2][w][0] - width * mean) / sd;
            if (snr > best) {
                best = snr;
                bestw = width;
            }
        }
        max_out[trial] = red[2][0][0] - mean;
        std_out[trial] = sd1;
        snr_out[trial] = best;
        win_out[trial] = bestw;
    }
}


enum Variant { V_U8_F32, V_F32_F32, V_F64_F64, V_U8_F64, V_F32_F64, V_F64_F32, V_COUNT };

struct VariantInfo {
    int lds_elem, acc_f64, dma;
};

// K samples per lane = (8 / LDS element size) * 4 reads; D = 8 trials per wave
constexpr VariantInfo kVariants[V_COUNT] = {
    {4, 0, 0},  // u8 in, f32 LDS (register staging), f32 acc (exact: sums < 2^24)
    {4, 0, 1},  // f32 in, f32 LDS (DMA), f32 acc
    {8, 1, 1},  // f64 in, f64 LDS (DMA), f64 acc (bit-exact vs reference)
    {4, 1, 0},  // u8 in, f32 LDS, f64 acc
    {4, 1, 1},  // f32 in, f32 LDS (DMA), f64 acc (bit-exact vs reference)
    {4, 0, 0},  // f64 in, f32 LDS (register staging), f32 acc
};

int pick_variant(int dtype, int acc)
{
    switch (dtype) {
    case PU_U8: return acc == PU_ACC_F64 ? V_U8_F64 : V_U8_F32;
    case PU_F32: return acc == PU_ACC_F64 ? V_F32_F64 : V_F32_F32;
    case PU_F64: return acc == PU_ACC_F32 ? V_F64_F32 : V_F64_F64;
    default: return -1;
    }
}

}  // namespace

struct pu_plan {
    int dtype = 0, acc = 0, variant = 0;
    int64_t nchan = 0, n = 0, ndm = 0;
    int K = 0, TT = 0;
    int ndt = 0, ntt = 0, ncc = 0, row_stride = 0, small_n = 0, max_spread = 0;
    size_t lds_bytes = 0;
    int32_t *d_first = nullptr, *d_count = nullptr, *d_rowlen = nullptr, *d_base = nullptr;
    u32x4 *d_rec = nullptr;
    // pair mode
    bool pair = false;
    int npairs = 0, raw_stride = 0, pair_bytes = 0, nrmax = 0;
    i32x4 *d_pmeta = nullptr;
    // optional kernel timing: event pairs recorded around each dedispersion launch
    std::vector<hipEvent_t> ev_start, ev_stop;
    int64_t launches = 0;
};

namespace {

template <typename Kern>
int ensure_lds(Kern kern, size_t bytes)
{
    if (bytes <= 64 * 1024) return PU_OK;
    return pu::hip_check(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes),
                         "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
}

template <typename Tin, typename Tl, typename Ta>
int launch_variant(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    const dim3 grid((unsigned)((int64_t)p->ndt * p->ntt)), block(kThreads);
    if constexpr (std::is_same<Tl, float>::value && std::is_same<Ta, float>::value) {
        if (p->pair) {
            if (plane) {
                auto kern = dedisp_pair_kernel<Tin, Ta, true, false>;
                int rc = ensure_lds(kern, p->lds_bytes);
                if (rc) return rc;
                hipLaunchKernelGGL(kern, grid, block, p->lds_bytes, s, a, p->d_first, p->d_count, p->d_rowlen,
                                   p->d_pmeta, p->d_rec);
            } else {
                auto kern = dedisp_pair_kernel<Tin, Ta, false, true>;
                int rc = ensure_lds(kern, p->lds_bytes);
                if (rc) return rc;
                hipLaunchKernelGGL(kern, grid, block, p->lds_bytes, s, a, p->d_first, p->d_count, p->d_rowlen,
                                   p->d_pmeta, p->d_rec);
            }
            return pu::launch_check("dedisp_pair_kernel");
        }
    }
    if (plane) {
        auto kern = dedisp_kernel<Tin, Tl, Ta, true, false>;
        int rc = ensure_lds(kern, p->lds_bytes);
        if (rc) return rc;
        hipLaunchKernelGGL(kern, grid, block, p->lds_bytes, s, a, p->d_first, p->d_count, p->d_rowlen, p->d_base,
                           p->d_rec);
    } else {
        auto kern = dedisp_kernel<Tin, Tl, Ta, false, true>;
        int rc = ensure_lds(kern, p->lds_bytes);
        if (rc) return rc;
        hipLaunchKernelGGL(kern, grid, block, p->lds_bytes, s, a, p->d_first, p->d_count, p->d_rowlen, p->d_base,
                           p->d_rec);
    }
    return pu::launch_check("dedisp_kernel");
}

int dispatch_variant(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    switch (p->variant) {
    case V_U8_F32: return launch_variant<uint8_t, float, float>(p, a, plane, s);
    case V_F32_F32: return launch_variant<float, float, float>(p, a, plane, s);
    case V_F64_F64: return launch_variant<double, double, double>(p, a, plane, s);
    case V_U8_F64: return launch_variant<uint8_t, float, double>(p, a, plane, s);
    case V_F32_F64: return launch_variant<float, float, double>(p, a, plane, s);
    case V_F64_F32: return launch_variant<double, float, float>(p, a, plane, s);
    }
    pu::set_error("bad plan variant");
    return PU_EINVAL;
}

int dispatch(pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    const size_t nslot = p->ev_start.size();
    const size_t slot = nslot ? (size_t)(p->launches % (int64_t)nslot) : 0;
    if (nslot) PU_TRY_HIP(hipEventRecord(p->ev_start[slot], s));
    int rc = dispatch_variant(p, a, plane, s);
    if (rc) return rc;
    if (nslot) PU_TRY_HIP(hipEventRecord(p->ev_stop[slot], s));
    ++p->launches;
    return PU_OK;
}

void free_plan(pu_plan *p)
{
    if (!p) return;
    for (auto e : p->ev_start) (void)hipEventDestroy(e);
    for (auto e : p->ev_stop) (void)hipEventDestroy(e);
    (void)hipFree(p->d_first);
    (void)hipFree(p->d_count);
    (void)hipFree(p->d_rowlen);
    (void)hipFree(p->d_base);
    (void)hipFree(p->d_rec);
    (void)hipFree(p->d_pmeta);
    delete p;
}

template <typename T>
int upload(T **dst, const std::vector<T> &vec)
{
    const size_t bytes = vec.size() * sizeof(T);
    int rc = pu::hip_check(hipMalloc((void **)dst, std::max<size_t>(bytes, 16)), "hipMalloc(plan)");
    if (rc) return rc;
    return pu::hip_check(hipMemcpy(*dst, vec.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy(plan)");
}

}  // namespace

extern "C" {

int pu_plan_create(pu_plan **out, int dtype, int acc, int64_t nchan, int64_t n, const int64_t *shifts,
                   int64_t ndm)
{
    PU_REQUIRE(out != nullptr, "pu_plan_create: out is NULL");
    *out = nullptr;
    const int v = pick_variant(dtype, acc);
    PU_REQUIRE(v >= 0, "pu_plan_create: unsupported dtype %d", dtype);
    PU_REQUIRE(acc >= PU_ACC_NATIVE && acc <= PU_ACC_F64, "pu_plan_create: bad acc %d", acc);
    PU_REQUIRE(nchan > 0 && nchan < (1 << 30), "pu_plan_create: nchan %lld out of range", (long long)nchan);
    PU_REQUIRE(n > 0 && n < (int64_t(1) << 31) - 65536, "pu_plan_create: nsamples %lld out of range",
               (long long)n);
    PU_REQUIRE(ndm > 0 && ndm < (1 << 30), "pu_plan_create: ndm %lld out of range", (long long)ndm);
    PU_REQUIRE(shifts != nullptr, "pu_plan_create: shifts is NULL");
    if (dtype == PU_U8 && acc != PU_ACC_F64)
        PU_REQUIRE(nchan <= 65793, "pu_plan_create: u8 f32 accumulation exact only for nchan <= 65793");

    pu_plan *p = new pu_plan();
    p->dtype = dtype;
    p->acc = acc;
    p->variant = v;
    p->nchan = nchan;
    p->n = n;
    p->ndm = ndm;
    const int esz = kVariants[v].lds_elem;
    const int E = 8 / esz;
    p->K = E * 4;
    p->TT = 64 * p->K;

    // LDS budget per workgroup; PU_LDS_BUDGET_KB overrides (tuning)
    size_t budget = kLdsBudget;
    if (const char *env = getenv("PU_LDS_BUDGET_KB")) budget = (size_t)std::max(8, atoi(env)) * 1024;
    // pair mode for float32 accumulation (channel order is not the reference's there anyway)
    bool want_pair = !kVariants[v].acc_f64 && nchan >= 2 && !getenv("PU_NO_PAIR");
    const int npairs = (int)((nchan + 1) / 2);

    for (int attempt = 0; attempt < 2; ++attempt) {
        const bool pair = want_pair && attempt == 0;
        // ---- greedy DM tiles: up to kTPT consecutive trials whose per-channel shift
        // spread stays <= kMaxSpread (pair mode: <= kMaxR distinct relative shifts per
        // pair with span <= 255)
        std::vector<int32_t> first, count;
        {
            std::vector<int64_t> mn((size_t)nchan), mx((size_t)nchan);
            std::vector<int64_t> rv((size_t)npairs * kMaxR);
            std::vector<int> nrv((size_t)npairs);
            int64_t i = 0;
            while (i < ndm) {
                const int64_t *s0 = shifts + i * nchan;
                for (int64_t c = 0; c < nchan; ++c) mn[c] = mx[c] = s0[c];
                if (pair)
                    for (int q = 0; q < npairs; ++q) {
                        nrv[q] = 1;
                        rv[(size_t)q * kMaxR] = 2 * q + 1 < nchan ? s0[2 * q + 1] - s0[2 * q] : 0;
                    }
                int64_t j = i + 1;
                while (j < ndm && j - i < kTPT) {
                    const int64_t *sj = shifts + j * nchan;
                    bool ok = true;
                    for (int64_t c = 0; c < nchan && ok; ++c)
                        ok = std::max(mx[c], sj[c]) - std::min(mn[c], sj[c]) <= kMaxSpread;
                    if (ok && pair) {
                        for (int q = 0; q < npairs && ok; ++q) {
                            if (2 * q + 1 >= nchan) continue;
                            const int64_t r = sj[2 * q + 1] - sj[2 * q];
                            const int64_t *rq = rv.data() + (size_t)q * kMaxR;
                            bool seen = false;
                            int64_t lo = r, hi = r;
                            for (int t = 0; t < nrv[q]; ++t) {
                                seen |= rq[t] == r;
                                lo = std::min(lo, rq[t]);
                                hi = std::max(hi, rq[t]);
                            }
                            if (!seen && (nrv[q] >= kMaxR || hi - lo > 255)) ok = false;
                        }
                    }
                    if (!ok) break;
                    for (int64_t c = 0; c < nchan; ++c) {
                        mn[c] = std::min(mn[c], sj[c]);
                        mx[c] = std::max(mx[c], sj[c]);
                    }
                    if (pair)
                        for (int q = 0; q < npairs; ++q) {
                            if (2 * q + 1 >= nchan) continue;
                            const int64_t r = sj[2 * q + 1] - sj[2 * q];
                            int64_t *rq = rv.data() + (size_t)q * kMaxR;
                            bool seen = false;
                            for (int t = 0; t < nrv[q]; ++t) seen |= rq[t] == r;
                            if (!seen) rq[nrv[q]++] = r;
                        }
                    ++j;
                }
                first.push_back((int32_t)i);
                count.push_back((int32_t)(j - i));
                i = j;
            }
        }
        const int ndt = (int)first.size();
        // ---- per-tile rows: channel mode = every channel; pair mode = every pair (c0 rows)
        const int nrows = pair ? npairs : (int)nchan;
        std::vector<int32_t> rowlen(ndt), base;
        std::vector<i32x4> pmeta;
        std::vector<int32_t> rel((size_t)ndt * nrows * kTPT);     // window shift relative to the row base
        std::vector<int8_t> rowsel((size_t)ndt * nrows * kTPT, 0); // pair row index
        int max_rowlen = 0, rspan_max = 0, nrmax = 1, max_spread = 0;
        for (int t = 0; t < ndt; ++t) {
            const int64_t i0 = first[t];
            const int cntt = count[t];
            int spread = 0;
            for (int q = 0; q < nrows; ++q) {
                const int c0 = pair ? 2 * q : q;
                int64_t m0 = INT64_MAX, m1 = INT64_MIN;
                for (int d = 0; d < cntt; ++d) {
                    m0 = std::min(m0, shifts[(i0 + d) * nchan + c0]);
                    m1 = std::max(m1, shifts[(i0 + d) * nchan + c0]);
                }
                int64_t b0 = m0 % n;
                if (b0 < 0) b0 += n;
                int64_t R[kMaxR];
                int nr = 1;
                R[0] = 0;
                if (pair && c0 + 1 < nchan) {
                    nr = 0;
                    for (int d = 0; d < cntt; ++d) {
                        const int64_t r = shifts[(i0 + d) * nchan + c0 + 1] - shifts[(i0 + d) * nchan + c0];
                        bool seen = false;
                        for (int u = 0; u < nr; ++u) seen |= R[u] == r;
                        if (!seen) R[nr++] = r;
                    }
                    std::sort(R, R + nr);
                }
                for (int d = 0; d < kTPT; ++d) {
                    const int dd = d < cntt ? d : cntt - 1;  // padding slots repeat the last trial
                    const int64_t sc = shifts[(i0 + dd) * nchan + c0];
                    rel[((size_t)t * nrows + q) * kTPT + d] = (int32_t)((sc - m0) % n);
                    if (pair && c0 + 1 < nchan) {
                        const int64_t r = shifts[(i0 + dd) * nchan + c0 + 1] - sc;
                        rowsel[((size_t)t * nrows + q) * kTPT + d] = (int8_t)(std::find(R, R + nr, r) - R);
                    }
                }
                spread = std::max(spread, (int)std::min<int64_t>(m1 - m0, n - 1));
                if (pair) {
                    int32_t packed = 0;
                    for (int u = 0; u < nr; ++u) packed |= (int32_t)((R[u] - R[0]) & 0xff) << (8 * u);
                    int32_t b1 = -1;
                    if (c0 + 1 < nchan) {
                        int64_t bb = (m0 + R[0]) % n;
                        if (bb < 0) bb += n;
                        b1 = (int32_t)bb;
                        rspan_max = std::max(rspan_max, (int)(R[nr - 1] - R[0]));
                    }
                    pmeta.push_back(i32x4{(int32_t)b0, b1, packed, nr});
                    nrmax = std::max(nrmax, nr);
                } else {
                    base.push_back((int32_t)b0);
                }
            }
            max_spread = std::max(max_spread, spread);
            rowlen[t] = p->TT + spread;
            max_rowlen = std::max(max_rowlen, rowlen[t]);
        }
        // ---- LDS layout
        const int epp = 256 / esz;
        int64_t chan_bytes;
        size_t per_unit;
        int nbuf = 1;
        if (pair) {
            p->row_stride = (max_rowlen + 4 + 63) / 64 * 64;  // floats per pair-row copy
            const int in_sz = (int)pu::elem_size(dtype);
            // raw rows: rowlen + 4 (combine reads 4 past the copy) + r span (+3 alignment slack for u8)
            p->raw_stride = (int)(((int64_t)(max_rowlen + 4 + rspan_max + (in_sz == 1 ? 3 : 0)) * in_sz + 255) / 256 * 256);
            p->pair_bytes = nrmax * 2 * p->row_stride * 4;
            p->small_n = (int64_t)p->raw_stride / in_sz + 2 > n ? 1 : 0;
            chan_bytes = p->pair_bytes;
            per_unit = (size_t)p->pair_bytes + 2 * (size_t)p->raw_stride;
            if (p->pair_bytes >= 32768) continue;  // u16 window records cannot address it
        } else {
            p->row_stride = (max_rowlen + E + epp - 1) / epp * epp;
            p->small_n = (int64_t)p->row_stride + 2 > n ? 1 : 0;
            nbuf = kVariants[v].dma ? 2 : 1;
            chan_bytes = (int64_t)E * p->row_stride * esz;
            per_unit = (size_t)nbuf * chan_bytes;
            if (2 * (int64_t)p->row_stride * esz > 32768) {
                free_plan(p);
                pu::set_error("pu_plan_create: LDS row of %d elements does not fit", p->row_stride);
                return PU_EUNSUPPORTED;
            }
        }
        p->pair = pair;
        p->npairs = pair ? npairs : 0;
        p->nrmax = nrmax;
        p->ndt = ndt;
        p->ntt = (int)((n + p->TT - 1) / p->TT);
        p->max_spread = max_spread;
        p->ncc = (int)std::max<int64_t>(1, std::min<int64_t>(nrows, (int64_t)(budget / per_unit)));
        p->lds_bytes = (size_t)p->ncc * per_unit;
        if (p->lds_bytes > 160 * 1024) {
            free_plan(p);
            pu::set_error("pu_plan_create: LDS row of %d elements does not fit", p->row_stride);
            return PU_EUNSUPPORTED;
        }
        // ---- window records: per (tile, row, wave) 8 x u16 = LDS byte offset of each
        // trial's window inside the row slot | (differs from the previous trial) << 15
        const size_t copy_bytes = (size_t)p->row_stride * (pair ? 4 : esz);
        std::vector<u32x4> rec((size_t)ndt * nrows * kWaves);
        for (size_t t = 0; t < (size_t)ndt; ++t)
            for (int q = 0; q < nrows; ++q)
                for (int w = 0; w < kWaves; ++w) {
                    const int32_t *rr = rel.data() + (t * nrows + q) * kTPT + w * kD;
                    const int8_t *rs = rowsel.data() + (t * nrows + q) * kTPT + w * kD;
                    uint32_t words[kD];
                    uint32_t prev = 0xffffffffu;
                    for (int d = 0; d < kD; ++d) {
                        const uint32_t s = (uint32_t)rr[d];
                        uint32_t off = E == 2 ? (uint32_t)((s & 1u) * copy_bytes + (s & ~1u) * 4u) : s * 8u;
                        off += (uint32_t)rs[d] * 2u * (uint32_t)copy_bytes;
                        words[d] = off | (off != prev ? 0x8000u : 0u);
                        prev = off;
                    }
                    u32x4 r;
                    for (int u = 0; u < 4; ++u) r[u] = words[2 * u] | (words[2 * u + 1] << 16);
                    rec[(t * nrows + q) * kWaves + w] = r;
                }
        if ((int64_t)p->ndt * p->ntt >= (int64_t(1) << 31)) {
            free_plan(p);
            pu::set_error("pu_plan_create: grid too large");
            return PU_EINVAL;
        }
        int rc = PU_OK;
        if (!rc) rc = upload(&p->d_first, first);
        if (!rc) rc = upload(&p->d_count, count);
        if (!rc) rc = upload(&p->d_rowlen, rowlen);
        if (!rc && !pair) rc = upload(&p->d_base, base);
        if (!rc && pair) rc = upload(&p->d_pmeta, pmeta);
        if (!rc) rc = upload(&p->d_rec, rec);
        if (rc) {
            free_plan(p);
            return rc;
        }
        break;
    }
    *out = p;
    return PU_OK;
}

void pu_plan_destroy(pu_plan *p) { free_plan(p); }

int pu_plan_enable_timing(pu_plan *p, int nslots)
{
    PU_REQUIRE(p != nullptr && nslots >= 0 && nslots <= 65536, "pu_plan_enable_timing: bad arguments");
    for (auto e : p->ev_start) (void)hipEventDestroy(e);
    for (auto e : p->ev_stop) (void)hipEventDestroy(e);
    p->ev_start.assign((size_t)nslots, nullptr);
    p->ev_stop.assign((size_t)nslots, nullptr);
    for (int i = 0; i < nslots; ++i) {
        PU_TRY_HIP(hipEventCreate(&p->ev_start[i]));
        PU_TRY_HIP(hipEventCreate(&p->ev_stop[i]));
    }
    p->launches = 0;
    return PU_OK;
}

int pu_plan_kernel_times(pu_plan *p, float *ms, int n)
{
    PU_REQUIRE(p != nullptr && ms != nullptr, "pu_plan_kernel_times: bad arguments");
    const int64_t have = std::min<int64_t>(p->launches, (int64_t)p->ev_start.size());
    const int m = (int)std::min<int64_t>(n, have);
    for (int i = 0; i < m; ++i) {
        PU_TRY_HIP(hipEventSynchronize(p->ev_stop[i]));
        PU_TRY_HIP(hipEventElapsedTime(&ms[i], p->ev_start[i], p->ev_stop[i]));
    }
    return m;
}

size_t pu_plan_workspace_bytes(const pu_plan *p)
{
    if (!p) return 0;
    return (size_t)p->ndm * p->ntt * kPartStride * sizeof(double);
}

int pu_plan_info(const pu_plan *p, int64_t *info, int n)
{
    if (!p || !info) return 0;
    const int64_t v[] = {p->ndm, p->ndt, p->ntt, kTPT, p->TT, p->ncc,
                         p->row_stride, (int64_t)p->lds_bytes, kVariants[p->variant].acc_f64, p->max_spread};
    const int m = std::min<int>(n, (int)(sizeof v / sizeof v[0]));
    for (int k = 0; k < m; ++k) info[k] = v[k];
    return m;
}

static int check_data(const pu_plan *p, const void *data, int64_t ld)
{
    PU_REQUIRE(p != nullptr, "plan is NULL");
    PU_REQUIRE(data != nullptr, "data is NULL");
    PU_REQUIRE(ld >= p->n, "ld %lld < nsamples %lld", (long long)ld, (long long)p->n);
    return PU_OK;
}

int pu_plan_search(pu_plan *p, const void *data, int64_t ld, double *max_out, double *std_out,
                   double *snr_out, int32_t *rebin_out, void *workspace, size_t ws_bytes, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    PU_REQUIRE(max_out && std_out && snr_out && rebin_out, "pu_plan_search: NULL output");
    PU_REQUIRE(workspace && ws_bytes >= pu_plan_workspace_bytes(p), "pu_plan_search: workspace too small");
    DedispArgs a{};
    a.data = data;
    a.ld = ld;
    a.nchan = (int32_t)p->nchan;
    a.n = (int32_t)p->n;
    a.ndt = p->ndt;
    a.ntt = p->ntt;
    a.ncc = p->ncc;
    a.row_stride = p->row_stride;
    a.small_n = p->small_n;
    a.raw_stride = p->raw_stride;
    a.pair_bytes = p->pair_bytes;
    a.nrmax = p->nrmax;
    a.npairs = p->npairs;
    a.partials = reinterpret_cast<double *>(workspace);
    hipStream_t s = pu::as_stream(stream);
    rc = dispatch(p, a, false, s);
    if (rc) return rc;
    hipLaunchKernelGGL(pu_finalize_kernel, dim3((unsigned)p->ndm), dim3(256), 0, s, a.partials, p->ntt,
                       (int)p->n, p->TT, max_out, std_out, snr_out, rebin_out);
    return pu::launch_check("pu_finalize_kernel");
}

int pu_plan_dedisperse(pu_plan *p, const void *data, int64_t ld, void *plane, int64_t ld_plane, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    PU_REQUIRE(plane != nullptr, "pu_plan_dedisperse: plane is NULL");
    PU_REQUIRE(ld_plane >= p->n, "pu_plan_dedisperse: ld_plane < nsamples");
    DedispArgs a{};
    a.data = data;
    a.ld = ld;
    a.nchan = (int32_t)p->nchan;
    a.n = (int32_t)p->n;
    a.ndt = p->ndt;
    a.ntt = p->ntt;
    a.ncc = p->ncc;
    a.row_stride = p->row_stride;
    a.small_n = p->small_n;
    a.raw_stride = p->raw_stride;
    a.pair_bytes = p->pair_bytes;
    a.nrmax = p->nrmax;
    a.npairs = p->npairs;
    a.plane = plane;
    a.ld_plane = ld_plane;
    return dispatch(p, a, true, pu::as_stream(stream));
}

}  // extern "C"
