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
typedef int i32x4 __attribute__((ext_vector_type(4)));

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
// Group mode (float32 accumulation of u8 / f32 / f64 inputs) -- DESIGN.md §4.2.
//
// Channels are taken in groups of G adjacent channels.  For trial d and group g the
// shifts are s_d,c = b_d,g + v_c with b = the group's first-channel shift and v the
// relative-shift VECTOR of the group; adjacent plan trials share v (a group's channels
// drift apart by ~G/nchan sample per trial), so a few distinct vectors serve all trials.
//   1. build_rows_kernel: for every distinct (group, vector) -- a "row" -- the exact
//      partial sum  R[i] = sum_{k<G} x[c_k][(lo + i + v_k) mod N]  (modular wrap
//      materialised, so kernel 2 never wraps).  HBM-streaming.
//   2. dedisp_group_kernel: the channel-mode kernel over groups: per DM tile and group
//      the rows its trials use ("slots") are staged in LDS by DMA, and a trial adds ONE
//      window of its slot per group: out_d[t] = sum_g R_{g,v(d,g)}[t + b_d,g - lo].
// Same sums as the reference (circular shift-and-sum; u8 exact), G x fewer adds.
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));

// bytes of one alignment copy of a staged row of ``rowlen`` samples (host and device)
__host__ __device__ constexpr int group_copy_bytes(int rowlen) { return ((rowlen + 2 + 63) & ~63) * 4; }

struct RowsArgs {
    const void *data;
    int64_t ld;
    const int32_t *meta;   // per row: c0, gsize, lo, v_1 .. v_{G-1}   (stride G + 2)
    float *rows;
    int64_t ldr;           // floats per row
    int32_t n, G, nrows, len;  // len = row samples built per segment
    int32_t T0, small_n;
};

template <typename Tin>
__global__ void __launch_bounds__(256) build_rows_kernel(RowsArgs a)
{
    const int w = pu::xcd_remap(blockIdx.x, gridDim.x);
    const int r = w % a.nrows;      // rows of one group are adjacent: same XCD, shared L2 lines
    const int blk = w / a.nrows;
    const int32_t *m = a.meta + (size_t)r * (a.G + 2);
    const int c0 = ld_uniform(m), gs = ld_uniform(m + 1);
    const int n = a.n;
    int base = ld_uniform(m + 2) + a.T0;
    if (base >= n) base -= n;
    const Tin *x = reinterpret_cast<const Tin *>(a.data) + (size_t)c0 * a.ld;
    float *out = a.rows + (size_t)r * a.ldr;
    const int i_end = min(a.len, (blk + 1) * 1024);
    for (int i = blk * 1024 + threadIdx.x; i < i_end; i += 256) {
        int pos = base + i;
        if (a.small_n) {
            pos %= n;
        } else {
            if (pos >= n) pos -= n;
            if (pos >= n) pos -= n;
        }
        float acc = static_cast<float>(x[pos]);
        for (int k = 1; k < gs; ++k) {
            int idx = pos + ld_uniform(m + 2 + k);
            if (idx >= n) idx -= n;
            acc += static_cast<float>(x[(size_t)k * a.ld + idx]);
        }
        out[i] = acc;
    }
}

struct GroupArgs {
    DedispArgs o;          // outputs (plane / partials), n, ndt, ntt
    const float *rows;
    int64_t ldr;
    int32_t ngroups;
    int32_t tt0;           // first time tile of this segment
    int32_t T0;            // first sample of this segment (rows' origin)
    int32_t buf_bytes;     // one ring buffer
};

// One group's contribution to the wave's D trials; u32 records: LDS byte offset in the
// ring buffer | reload flag << 31.
__device__ __forceinline__ void group_trials(float (&acc)[kD][8], double (&w)[4], const u32x8 rec, uint32_t base)
{
#pragma unroll
    for (int d = 0; d < kD; ++d) {
        if (d > 0) {
            const uint32_t word = rec[d];
            if (word & 0x80000000u) read_window(w, base + (word & 0x7fffffffu));
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[d][k] += window_elem<float>(w, k);
        pin_accumulators(acc[d]);
    }
}

template <bool PLANE, bool STATS>
__global__ void __launch_bounds__(kThreads, 5)
dedisp_group_kernel(GroupArgs a, const int32_t *__restrict__ tile_first, const int32_t *__restrict__ tile_count,
                    const int32_t *__restrict__ tile_rowlen, const i32x2 *__restrict__ tile_chunks,
                    const i32x4 *__restrict__ chunks, const i32x2 *__restrict__ slots,
                    const u32x8 *__restrict__ rec_tab)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int K = 8;
    constexpr int TT = 64 * K;
    constexpr int D = kD;
    const int ndt = a.o.ndt;
    const int wg = pu::xcd_remap(blockIdx.x, gridDim.x);
    const int dt = wg % ndt;
    const int tt = a.tt0 + wg / ndt;
    const int t0 = tt * TT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int first = ld_uniform(tile_first + dt);
    const int cnt = ld_uniform(tile_count + dt);
    const int rowlen = ld_uniform(tile_rowlen + dt);
    const i32x2 tc = ld_uniform(tile_chunks + dt);   // {first chunk, chunk count}
    const int slot0 = wave * D;
    const bool active = slot0 < cnt;
    const uint32_t smem_addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;
    const int cover_bytes = (rowlen * 4 + 255) & ~255;
    const int copy_bytes = group_copy_bytes(rowlen);  // per tile: slot = 2 alignment copies
    const int slot_bytes = 2 * copy_bytes;
    const float *rows = a.rows + (t0 - a.T0);

    float acc[D][K];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] = 0.0f;

    const u32x8 *recs = rec_tab + (size_t)dt * a.ngroups * kWaves + wave;

    // ---- LDS-DMA of chunk k's slots into ring buffer b: job j = (slot, copy q)
    auto issue_dma = [&](int k, int b) {
        const i32x4 ch = ld_uniform(chunks + tc.x + k);  // {group begin, group end, slot begin, slot end}
        const int njobs = 2 * (ch.w - ch.z);
        for (int j = wave; j < njobs; j += kWaves) {
            const i32x2 sl = ld_uniform(slots + ch.z + (j >> 1));  // {row id, start}
            const int q = j & 1;
            const char *src = reinterpret_cast<const char *>(rows + (size_t)sl.x * a.ldr + sl.y + q);
            unsigned char *dst = smem + b * a.buf_bytes + (j >> 1) * slot_bytes + q * copy_bytes;
            int off = 0;
            for (; off + 1024 <= cover_bytes; off += 1024)
                __builtin_amdgcn_global_load_lds((const void *)(src + off + 16 * lane),
                                                 (__attribute__((address_space(3))) void *)(dst + off), 16, 0, 0);
            for (; off < cover_bytes; off += 256)
                __builtin_amdgcn_global_load_lds((const void *)(src + off + 4 * lane),
                                                 (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
        }
    };

    issue_dma(0, 0);
    for (int k = 0; k < tc.y; ++k) {
        const int b = k & 1;
        __syncthreads();  // this wave's DMA landed (vmcnt) and every wave left the other buffer
        if (k + 1 < tc.y) issue_dma(k + 1, b ^ 1);
        if (!active) continue;
        const i32x4 ch = ld_uniform(chunks + tc.x + k);
        const int g0 = ch.x, ng = ch.y - ch.x;
        const uint32_t base = smem_addr + (uint32_t)(b * a.buf_bytes) + 8u * lane;
        double w0[4], w1[4];
        const u32x8 *rc = recs + (size_t)g0 * kWaves;
        u32x8 rec0 = ld_uniform(rc);
        u32x8 rec1 = ng > 1 ? ld_uniform(rc + kWaves) : rec0;
        read_window(w0, base + (rec0[0] & 0x7fffffffu));
        for (int gi = 0; gi < ng; gi += 2) {
            const bool has1 = gi + 1 < ng, has2 = gi + 2 < ng, has3 = gi + 3 < ng;
            u32x8 rec2 = rec0, rec3 = rec1;
            if (has2) rec2 = ld_uniform(rc + (size_t)(gi + 2) * kWaves);
            if (has1) prefetch_window(w1, base + (rec1[0] & 0x7fffffffu));
            group_trials(acc, w0, rec0, base);
            if (!has1) break;
            wait_window(w1);
            if (has3) rec3 = ld_uniform(rc + (size_t)(gi + 3) * kWaves);
            if (has2) prefetch_window(w0, base + (rec2[0] & 0x7fffffffu));
            group_trials(acc, w1, rec1, base);
            if (has2) wait_window(w0);
            rec0 = rec2;
            rec1 = rec3;
        }
    }
    if (!active) return;
    write_outputs<float, float, K, PLANE, STATS>(acc, a.o, first, slot0, cnt, t0, tt, lane);
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
    // group mode (group > 1): rows of exact partial sums, built per time segment
    int group = 1, ngroups = 0, nrows = 0, nseg = 1, seg_len = 0, row_len = 0, buf_bytes = 0, max_span = 0;
    int64_t nchunks = 0, nslots = 0;
    float *d_rows = nullptr;
    int32_t *d_rowmeta = nullptr;
    i32x2 *d_tile_chunks = nullptr, *d_slots = nullptr;
    i32x4 *d_chunks = nullptr;
    u32x8 *d_rec8 = nullptr;
    // optional kernel timing: events before the first launch, after the first row
    // build (single-segment plans) and after the last launch of each dispatch
    std::vector<hipEvent_t> ev_start, ev_mid, ev_stop;
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

template <typename Tin>
void launch_rows(const pu_plan *p, const RowsArgs &ra, hipStream_t s)
{
    const int64_t nblk = (int64_t)((ra.len + 1023) / 1024) * ra.nrows;
    hipLaunchKernelGGL(build_rows_kernel<Tin>, dim3((unsigned)nblk), dim3(256), 0, s, ra);
}

// Group mode: per time segment, build the rows then sum them.
int dispatch_group(pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s, hipEvent_t mid)
{
    RowsArgs ra{};
    ra.data = a.data;
    ra.ld = a.ld;
    ra.meta = p->d_rowmeta;
    ra.rows = p->d_rows;
    ra.ldr = p->row_len;
    ra.n = (int32_t)p->n;
    ra.G = p->group;
    ra.nrows = p->nrows;
    ra.len = p->row_len;
    ra.small_n = p->row_len > p->n ? 1 : 0;
    GroupArgs ga{};
    ga.o = a;
    ga.rows = p->d_rows;
    ga.ldr = p->row_len;
    ga.ngroups = p->ngroups;
    ga.buf_bytes = p->buf_bytes;
    const int tps = p->seg_len / p->TT;  // time tiles per segment
    for (int sg = 0; sg < p->nseg; ++sg) {
        ra.T0 = sg * p->seg_len;
        switch (p->dtype) {
        case PU_U8: launch_rows<uint8_t>(p, ra, s); break;
        case PU_F32: launch_rows<float>(p, ra, s); break;
        default: launch_rows<double>(p, ra, s); break;
        }
        int rc = pu::launch_check("build_rows_kernel");
        if (rc) return rc;
        if (mid && sg == 0 && p->nseg == 1) PU_TRY_HIP(hipEventRecord(mid, s));
        ga.T0 = ra.T0;
        ga.tt0 = sg * tps;
        const int ntt_seg = std::min(p->ntt - ga.tt0, tps);
        const dim3 grid((unsigned)((int64_t)p->ndt * ntt_seg)), block(kThreads);
        if (plane) {
            auto kern = dedisp_group_kernel<true, false>;
            rc = ensure_lds(kern, p->lds_bytes);
            if (rc) return rc;
            hipLaunchKernelGGL(kern, grid, block, p->lds_bytes, s, ga, p->d_first, p->d_count, p->d_rowlen,
                               p->d_tile_chunks, p->d_chunks, p->d_slots, p->d_rec8);
        } else {
            auto kern = dedisp_group_kernel<false, true>;
            rc = ensure_lds(kern, p->lds_bytes);
            if (rc) return rc;
            hipLaunchKernelGGL(kern, grid, block, p->lds_bytes, s, ga, p->d_first, p->d_count, p->d_rowlen,
                               p->d_tile_chunks, p->d_chunks, p->d_slots, p->d_rec8);
        }
        rc = pu::launch_check("dedisp_group_kernel");
        if (rc) return rc;
    }
    return PU_OK;
}

int dispatch(pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    const size_t nslot = p->ev_start.size();
    const size_t slot = nslot ? (size_t)(p->launches % (int64_t)nslot) : 0;
    if (nslot) PU_TRY_HIP(hipEventRecord(p->ev_start[slot], s));
    int rc = p->group > 1 ? dispatch_group(p, a, plane, s, nslot ? p->ev_mid[slot] : nullptr)
                          : dispatch_variant(p, a, plane, s);
    if (rc) return rc;
    if (nslot) PU_TRY_HIP(hipEventRecord(p->ev_stop[slot], s));
    ++p->launches;
    return PU_OK;
}

void destroy_events(pu_plan *p)
{
    for (auto *v : {&p->ev_start, &p->ev_mid, &p->ev_stop}) {
        for (auto e : *v) (void)hipEventDestroy(e);
        v->clear();
    }
}

void free_plan(pu_plan *p)
{
    if (!p) return;
    destroy_events(p);
    (void)hipFree(p->d_first);
    (void)hipFree(p->d_count);
    (void)hipFree(p->d_rowlen);
    (void)hipFree(p->d_base);
    (void)hipFree(p->d_rec);
    (void)hipFree(p->d_rows);
    (void)hipFree(p->d_rowmeta);
    (void)hipFree(p->d_tile_chunks);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_chunks);
    (void)hipFree(p->d_rec8);
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

// ---- channel mode (every variant): DM tiles of <= kTPT trials with per-channel shift
// spread <= kMaxSpread; per (tile, channel) the modular row base; u16 window records.
int plan_channels(pu_plan *p, const int64_t *shifts, size_t budget)
{
    const int64_t nchan = p->nchan, n = p->n, ndm = p->ndm;
    const int esz = kVariants[p->variant].lds_elem;
    const int E = 8 / esz;
    std::vector<int32_t> first, count;
    {
        std::vector<int64_t> mn((size_t)nchan), mx((size_t)nchan);
        int64_t i = 0;
        while (i < ndm) {
            const int64_t *s0 = shifts + i * nchan;
            for (int64_t c = 0; c < nchan; ++c) mn[c] = mx[c] = s0[c];
            int64_t j = i + 1;
            while (j < ndm && j - i < kTPT) {
                const int64_t *sj = shifts + j * nchan;
                bool ok = true;
                for (int64_t c = 0; c < nchan && ok; ++c)
                    ok = std::max(mx[c], sj[c]) - std::min(mn[c], sj[c]) <= kMaxSpread;
                if (!ok) break;
                for (int64_t c = 0; c < nchan; ++c) {
                    mn[c] = std::min(mn[c], sj[c]);
                    mx[c] = std::max(mx[c], sj[c]);
                }
                ++j;
            }
            first.push_back((int32_t)i);
            count.push_back((int32_t)(j - i));
            i = j;
        }
    }
    const int ndt = (int)first.size();
    std::vector<int32_t> rowlen(ndt), base((size_t)ndt * nchan);
    std::vector<int32_t> rel((size_t)ndt * nchan * kTPT);  // window shift relative to the row base
    int max_rowlen = 0, max_spread = 0;
    for (int t = 0; t < ndt; ++t) {
        const int64_t i0 = first[t];
        const int cntt = count[t];
        int spread = 0;
        for (int64_t c = 0; c < nchan; ++c) {
            int64_t m0 = INT64_MAX, m1 = INT64_MIN;
            for (int d = 0; d < cntt; ++d) {
                m0 = std::min(m0, shifts[(i0 + d) * nchan + c]);
                m1 = std::max(m1, shifts[(i0 + d) * nchan + c]);
            }
            int64_t b0 = m0 % n;
            if (b0 < 0) b0 += n;
            base[(size_t)t * nchan + c] = (int32_t)b0;
            for (int d = 0; d < kTPT; ++d) {
                const int dd = d < cntt ? d : cntt - 1;  // padding slots repeat the last trial
                rel[((size_t)t * nchan + c) * kTPT + d] = (int32_t)((shifts[(i0 + dd) * nchan + c] - m0) % n);
            }
            spread = std::max(spread, (int)std::min<int64_t>(m1 - m0, n - 1));
        }
        max_spread = std::max(max_spread, spread);
        rowlen[t] = p->TT + spread;
        max_rowlen = std::max(max_rowlen, rowlen[t]);
    }
    const int epp = 256 / esz;
    p->row_stride = (max_rowlen + E + epp - 1) / epp * epp;
    p->small_n = (int64_t)p->row_stride + 2 > n ? 1 : 0;
    const int nbuf = kVariants[p->variant].dma ? 2 : 1;
    const int64_t chan_bytes = (int64_t)E * p->row_stride * esz;
    if (chan_bytes > 32768) {
        pu::set_error("pu_plan_create: LDS row of %d elements does not fit", p->row_stride);
        return PU_EUNSUPPORTED;
    }
    p->ndt = ndt;
    p->max_spread = max_spread;
    p->ncc = (int)std::max<int64_t>(1, std::min<int64_t>(nchan, (int64_t)(budget / (nbuf * chan_bytes))));
    p->lds_bytes = (size_t)p->ncc * nbuf * chan_bytes;
    if (p->lds_bytes > 160 * 1024) {
        pu::set_error("pu_plan_create: LDS row of %d elements does not fit", p->row_stride);
        return PU_EUNSUPPORTED;
    }
    // window records: per (tile, channel, wave) 8 x u16 = LDS byte offset of each
    // trial's window inside the row slot | (differs from the previous trial) << 15
    const size_t copy_bytes = (size_t)p->row_stride * esz;
    std::vector<u32x4> rec((size_t)ndt * nchan * kWaves);
    for (size_t t = 0; t < (size_t)ndt; ++t)
        for (int64_t c = 0; c < nchan; ++c)
            for (int w = 0; w < kWaves; ++w) {
                const int32_t *rr = rel.data() + (t * nchan + c) * kTPT + w * kD;
                uint32_t words[kD];
                uint32_t prev = 0xffffffffu;
                for (int d = 0; d < kD; ++d) {
                    const uint32_t s = (uint32_t)rr[d];
                    const uint32_t off = E == 2 ? (uint32_t)((s & 1u) * copy_bytes + (s & ~1u) * 4u) : s * 8u;
                    words[d] = off | (off != prev ? 0x8000u : 0u);
                    prev = off;
                }
                u32x4 r;
                for (int u = 0; u < 4; ++u) r[u] = words[2 * u] | (words[2 * u + 1] << 16);
                rec[(t * nchan + c) * kWaves + w] = r;
            }
    if ((int64_t)p->ndt * p->ntt >= (int64_t(1) << 31)) {
        pu::set_error("pu_plan_create: grid too large");
        return PU_EINVAL;
    }
    int rc = PU_OK;
    if (!rc) rc = upload(&p->d_first, first);
    if (!rc) rc = upload(&p->d_count, count);
    if (!rc) rc = upload(&p->d_rowlen, rowlen);
    if (!rc) rc = upload(&p->d_base, base);
    if (!rc) rc = upload(&p->d_rec, rec);
    return rc;
}

// ---- group mode planning (float32 accumulation variants).  Returns PU_EUNSUPPORTED
// when the trial grid does not suit grouping (the caller then plans channel mode).
constexpr int kRowSpan = 2048;   // max first-channel shift range served by one row

struct SlotAcc {
    int32_t row, lo, hi;
};

int plan_group(pu_plan *p, const int64_t *shifts, int G, size_t budget, size_t mem_cap)
{
    const int64_t nchan = p->nchan, n = p->n, ndm = p->ndm;
    const int TT = p->TT;
    const int ngroups = (int)((nchan + G - 1) / G);
    const int buf_bytes = (int)(budget / 2) & ~255;
    std::vector<int32_t> sn((size_t)(ndm * nchan));
    for (size_t i = 0; i < sn.size(); ++i) {
        int64_t v = shifts[i] % n;
        sn[i] = (int32_t)(v < 0 ? v + n : v);
    }
    // ---- rows: distinct relative-shift vectors per group, each split into clusters of
    // first-channel shifts (circularly) no wider than kRowSpan
    std::vector<int32_t> rowid((size_t)(ndm * ngroups)), roff((size_t)(ndm * ngroups));
    std::vector<int32_t> meta;
    int nrows = 0, max_span = 0;
    std::vector<int32_t> order((size_t)ndm), bs;
    for (int g = 0; g < ngroups; ++g) {
        const int64_t c0 = (int64_t)g * G;
        const int gs = (int)std::min<int64_t>(G, nchan - c0);
        auto vec = [&](int64_t d, int k) {
            int32_t v = sn[d * nchan + c0 + k] - sn[d * nchan + c0];
            return v < 0 ? v + (int32_t)n : v;
        };
        auto base_of = [&](int64_t d) { return sn[d * nchan + c0]; };
        for (int64_t d = 0; d < ndm; ++d) order[d] = (int32_t)d;
        std::sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
            for (int k = 1; k < gs; ++k) {
                const int32_t a = vec(x, k), b = vec(y, k);
                if (a != b) return a < b;
            }
            if (base_of(x) != base_of(y)) return base_of(x) < base_of(y);
            return x < y;
        });
        for (int64_t a = 0; a < ndm;) {
            int64_t b = a + 1;
            while (b < ndm) {
                bool same = true;
                for (int k = 1; k < gs && same; ++k) same = vec(order[a], k) == vec(order[b], k);
                if (!same) break;
                ++b;
            }
            const int64_t m = b - a;
            // start after the widest circular gap between consecutive (sorted) bases
            int64_t start = 0, gap = base_of(order[a]) + n - base_of(order[b - 1]);
            for (int64_t i = 0; i + 1 < m; ++i) {
                const int64_t gi = base_of(order[a + i + 1]) - base_of(order[a + i]);
                if (gi > gap) {
                    gap = gi;
                    start = i + 1;
                }
            }
            int32_t lo = 0;
            bool open = false;
            for (int64_t i = 0; i < m; ++i) {
                const int32_t d = order[a + (start + i) % m];
                const int32_t bd = base_of(d);
                int64_t rel = open ? (bd - lo + n) % n : 0;
                if (!open || rel > kRowSpan) {
                    lo = bd;
                    rel = 0;
                    open = true;
                    meta.push_back((int32_t)c0);
                    meta.push_back(gs);
                    meta.push_back(lo);
                    for (int k = 1; k < G; ++k) meta.push_back(k < gs ? vec(d, k) : 0);
                    ++nrows;
                }
                rowid[(size_t)d * ngroups + g] = nrows - 1;
                roff[(size_t)d * ngroups + g] = (int32_t)rel;
                max_span = std::max(max_span, (int)rel);
            }
            a = b;
        }
    }
    // ---- DM tiles: <= kTPT consecutive trials; every group's slots (distinct rows of the
    // tile) must fit one ring buffer at the tile's row length
    std::vector<int32_t> first, count, rowlen;
    std::vector<std::vector<SlotAcc>> tslots;  // per tile * ngroups
    {
        std::vector<std::vector<SlotAcc>> cur((size_t)ngroups), nxt((size_t)ngroups);
        int64_t i = 0;
        while (i < ndm) {
            int spread = 0;
            for (int g = 0; g < ngroups; ++g) {
                const size_t k = (size_t)i * ngroups + g;
                cur[g].assign(1, SlotAcc{rowid[k], roff[k], roff[k]});
            }
            int64_t j = i + 1;
            while (j < ndm && j - i < kTPT) {
                int sp = spread;
                size_t maxslots = 0;
                for (int g = 0; g < ngroups; ++g) {
                    const size_t k = (size_t)j * ngroups + g;
                    nxt[g] = cur[g];
                    bool found = false;
                    for (auto &sa : nxt[g])
                        if (sa.row == rowid[k]) {
                            sa.lo = std::min(sa.lo, roff[k]);
                            sa.hi = std::max(sa.hi, roff[k]);
                            sp = std::max(sp, sa.hi - sa.lo);
                            found = true;
                        }
                    if (!found) nxt[g].push_back(SlotAcc{rowid[k], roff[k], roff[k]});
                    maxslots = std::max(maxslots, nxt[g].size());
                }
                if (sp > kMaxSpread || maxslots * 2 * (size_t)group_copy_bytes(TT + sp) > (size_t)buf_bytes) break;
                std::swap(cur, nxt);
                spread = sp;
                ++j;
            }
            size_t maxslots = 0;
            for (int g = 0; g < ngroups; ++g) maxslots = std::max(maxslots, cur[g].size());
            if (maxslots * 2 * (size_t)group_copy_bytes(TT + spread) > (size_t)buf_bytes) {
                pu::set_error("group mode: slots of one trial exceed the LDS buffer");
                return PU_EUNSUPPORTED;
            }
            first.push_back((int32_t)i);
            count.push_back((int32_t)(j - i));
            rowlen.push_back(TT + spread);
            for (int g = 0; g < ngroups; ++g) tslots.push_back(cur[g]);
            p->max_spread = std::max(p->max_spread, spread);
            i = j;
        }
    }
    const int ndt = (int)first.size();
    // ---- chunks (groups whose slots fit one buffer), slots, window records
    std::vector<i32x2> tile_chunks((size_t)ndt), slots;
    std::vector<i32x4> chunks;
    std::vector<u32x8> rec((size_t)ndt * ngroups * kWaves);
    std::vector<int32_t> slot_in_chunk((size_t)ngroups);
    for (int t = 0; t < ndt; ++t) {
        const uint32_t copy_bytes = (uint32_t)group_copy_bytes(rowlen[t]);
        const int cap = (int)((uint32_t)buf_bytes / (2 * copy_bytes));
        tile_chunks[t] = i32x2{(int32_t)chunks.size(), 0};
        int g = 0;
        while (g < ngroups) {
            const int s_begin = (int)slots.size();
            int used = 0, g_end = g;
            while (g_end < ngroups && used + (int)tslots[(size_t)t * ngroups + g_end].size() <= cap) {
                slot_in_chunk[g_end] = used;
                for (const auto &sa : tslots[(size_t)t * ngroups + g_end]) slots.push_back(i32x2{sa.row, sa.lo});
                used += (int)tslots[(size_t)t * ngroups + g_end].size();
                ++g_end;
            }
            chunks.push_back(i32x4{g, g_end, s_begin, (int32_t)slots.size()});
            tile_chunks[t][1]++;
            g = g_end;
        }
        for (g = 0; g < ngroups; ++g) {
            const auto &sl = tslots[(size_t)t * ngroups + g];
            for (int w = 0; w < kWaves; ++w) {
                u32x8 r;
                uint32_t prev = 0xffffffffu;
                for (int d = 0; d < kD; ++d) {
                    const int dd = std::min(w * kD + d, count[t] - 1);  // padding repeats the last trial
                    const size_t k = (size_t)(first[t] + dd) * ngroups + g;
                    int si = 0;
                    while (sl[si].row != rowid[k]) ++si;
                    const uint32_t s = (uint32_t)(roff[k] - sl[si].lo);
                    const uint32_t off = (uint32_t)(slot_in_chunk[g] + si) * 2u * copy_bytes + (s & 1u) * copy_bytes +
                                         (s & ~1u) * 4u;
                    r[d] = off | (off != prev ? 0x80000000u : 0u);
                    prev = off;
                }
                rec[((size_t)t * ngroups + g) * kWaves + w] = r;
            }
        }
    }
    // ---- time segments: the row buffer holds seg_len samples (+ halo) of every row
    const int64_t ntt = (n + TT - 1) / TT;
    const int64_t halo = (int64_t)max_span + p->max_spread + 128;
    int64_t seg_tiles = ntt;
    while (seg_tiles > 16 && (int64_t)nrows * (seg_tiles * TT + halo) * 4 > (int64_t)mem_cap)
        seg_tiles = (seg_tiles + 1) / 2;
    if ((int64_t)nrows * (seg_tiles * TT + halo) * 4 > (int64_t)mem_cap) {
        pu::set_error("group mode: %d rows exceed the row-buffer cap", nrows);
        return PU_EUNSUPPORTED;
    }
    p->group = G;
    p->ngroups = ngroups;
    p->nrows = nrows;
    p->max_span = max_span;
    p->seg_len = (int)(seg_tiles * TT);
    p->nseg = (int)((ntt + seg_tiles - 1) / seg_tiles);
    p->row_len = (int)((p->seg_len + halo + 63) / 64 * 64);
    p->buf_bytes = buf_bytes;
    p->lds_bytes = 2 * (size_t)buf_bytes;
    p->ndt = ndt;
    p->ncc = 0;
    p->row_stride = group_copy_bytes(*std::max_element(rowlen.begin(), rowlen.end())) / 4;
    p->nchunks = (int64_t)chunks.size();
    p->nslots = (int64_t)slots.size();
    if ((int64_t)p->ndt * p->ntt >= (int64_t(1) << 31) || (int64_t)nrows * ((p->row_len + 1023) / 1024) >= (int64_t(1) << 31)) {
        pu::set_error("pu_plan_create: grid too large");
        return PU_EINVAL;
    }
    int rc = PU_OK;
    if (!rc) rc = upload(&p->d_first, first);
    if (!rc) rc = upload(&p->d_count, count);
    if (!rc) rc = upload(&p->d_rowlen, rowlen);
    if (!rc) rc = upload(&p->d_tile_chunks, tile_chunks);
    if (!rc) rc = upload(&p->d_chunks, chunks);
    if (!rc) rc = upload(&p->d_slots, slots);
    if (!rc) rc = upload(&p->d_rec8, rec);
    if (!rc) rc = upload(&p->d_rowmeta, meta);
    if (!rc)
        rc = pu::hip_check(hipMalloc((void **)&p->d_rows, (size_t)nrows * p->row_len * sizeof(float)),
                           "hipMalloc(group rows)");
    return rc;
}

void reset_tables(pu_plan *p)
{
    pu_plan keep;
    keep.dtype = p->dtype;
    keep.acc = p->acc;
    keep.variant = p->variant;
    keep.nchan = p->nchan;
    keep.n = p->n;
    keep.ndm = p->ndm;
    keep.K = p->K;
    keep.TT = p->TT;
    keep.ntt = p->ntt;
    (void)hipFree(p->d_first);
    (void)hipFree(p->d_count);
    (void)hipFree(p->d_rowlen);
    (void)hipFree(p->d_base);
    (void)hipFree(p->d_rec);
    (void)hipFree(p->d_rows);
    (void)hipFree(p->d_rowmeta);
    (void)hipFree(p->d_tile_chunks);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_chunks);
    (void)hipFree(p->d_rec8);
    *p = keep;
}

}  // namespace

extern "C" {

int pu_plan_create_grouped(pu_plan **out, int dtype, int acc, int64_t nchan, int64_t n, const int64_t *shifts,
                           int64_t ndm, int group)
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
    PU_REQUIRE(group == 0 || group == 1 || group == 2 || group == 4 || group == 8 || group == 16,
               "pu_plan_create: group %d not in {0 (auto), 1, 2, 4, 8, 16}", group);
    if (dtype == PU_U8 && acc != PU_ACC_F64)
        PU_REQUIRE(nchan <= 65793, "pu_plan_create: u8 f32 accumulation exact only for nchan <= 65793");

    pu_plan *p = new pu_plan();
    p->dtype = dtype;
    p->acc = acc;
    p->variant = v;
    p->nchan = nchan;
    p->n = n;
    p->ndm = ndm;
    const int E = 8 / kVariants[v].lds_elem;
    p->K = E * 4;
    p->TT = 64 * p->K;
    p->ntt = (int)((n + p->TT - 1) / p->TT);

    // LDS budget per workgroup; PU_LDS_BUDGET_KB overrides (tuning)
    size_t budget = kLdsBudget;
    if (const char *env = getenv("PU_LDS_BUDGET_KB")) budget = (size_t)std::max(8, atoi(env)) * 1024;
    size_t mem_cap = size_t(16) << 30;
    if (const char *env = getenv("PU_ROWS_MB")) mem_cap = (size_t)std::max(1, atoi(env)) << 20;
    // group size: explicit, else PU_GROUP, else 4; float32 accumulation only (the
    // float64 modes keep the reference's sequential channel order)
    int G = group;
    if (G == 0) {
        G = 4;
        if (const char *env = getenv("PU_GROUP")) G = atoi(env);
    }
    if (kVariants[v].acc_f64) G = 1;
    while (G > 1 && G >= nchan) G >>= 1;
    int rc = PU_EUNSUPPORTED;
    for (; G > 1 && rc == PU_EUNSUPPORTED; G >>= 1) {
        rc = plan_group(p, shifts, G, budget, mem_cap);
        if (rc == PU_EUNSUPPORTED) reset_tables(p);
    }
    if (rc == PU_EUNSUPPORTED) rc = plan_channels(p, shifts, budget);
    if (rc) {
        free_plan(p);
        return rc;
    }
    *out = p;
    return PU_OK;
}

int pu_plan_create(pu_plan **out, int dtype, int acc, int64_t nchan, int64_t n, const int64_t *shifts, int64_t ndm)
{
    return pu_plan_create_grouped(out, dtype, acc, nchan, n, shifts, ndm, 0);
}

void pu_plan_destroy(pu_plan *p) { free_plan(p); }

int pu_plan_enable_timing(pu_plan *p, int nslots)
{
    PU_REQUIRE(p != nullptr && nslots >= 0 && nslots <= 65536, "pu_plan_enable_timing: bad arguments");
    destroy_events(p);
    for (auto *v : {&p->ev_start, &p->ev_mid, &p->ev_stop}) {
        v->assign((size_t)nslots, nullptr);
        for (int i = 0; i < nslots; ++i) PU_TRY_HIP(hipEventCreate(&(*v)[i]));
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

int pu_plan_phase_times(pu_plan *p, float *build_ms, float *sum_ms, int n)
{
    PU_REQUIRE(p != nullptr && build_ms != nullptr && sum_ms != nullptr, "pu_plan_phase_times: bad arguments");
    if (p->group <= 1 || p->nseg != 1) return 0;
    const int64_t have = std::min<int64_t>(p->launches, (int64_t)p->ev_start.size());
    const int m = (int)std::min<int64_t>(n, have);
    for (int i = 0; i < m; ++i) {
        PU_TRY_HIP(hipEventSynchronize(p->ev_stop[i]));
        PU_TRY_HIP(hipEventElapsedTime(&build_ms[i], p->ev_start[i], p->ev_mid[i]));
        PU_TRY_HIP(hipEventElapsedTime(&sum_ms[i], p->ev_mid[i], p->ev_stop[i]));
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
                         p->row_stride, (int64_t)p->lds_bytes, kVariants[p->variant].acc_f64, p->max_spread,
                         p->group, p->nrows, p->nseg, (int64_t)p->nrows * p->row_len * 4, p->nslots};
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

static DedispArgs make_args(const pu_plan *p, const void *data, int64_t ld)
{
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
    return a;
}

int pu_plan_search(pu_plan *p, const void *data, int64_t ld, double *max_out, double *std_out,
                   double *snr_out, int32_t *rebin_out, void *workspace, size_t ws_bytes, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    PU_REQUIRE(max_out && std_out && snr_out && rebin_out, "pu_plan_search: NULL output");
    PU_REQUIRE(workspace && ws_bytes >= pu_plan_workspace_bytes(p), "pu_plan_search: workspace too small");
    DedispArgs a = make_args(p, data, ld);
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
    DedispArgs a = make_args(p, data, ld);
    a.plane = plane;
    a.ld_plane = ld_plane;
    return dispatch(p, a, true, pu::as_stream(stream));
}

}  // extern "C"
