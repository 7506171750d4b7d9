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
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "exact.h"
#include "pu_common.h"

#include "dedisp_common.h"

// dedisp_f64.hip (waves: the planner's kF64Waves, checked against the kernel's)
int pu_dd_launch_f64(bool tin_f32, bool plane, const void *args, size_t args_bytes, size_t lds_bytes,
                     const int32_t *first, const int32_t *count, const int32_t *rowlen, const int32_t *base,
                     const void *rec8, const void *first_off, void *stream, int waves);
// dedisp_f64_kernel's workgroup: 16 waves x 4 trials (= kTPT trials per DM tile)
constexpr int kF64Waves = 16, kF64Trials = 4;

namespace {

template <typename Tin, typename Tl, typename Ta, bool PLANE, bool STATS>
// 4 waves per SIMD (2 workgroups per CU): <= 128 VGPRs, enforced (the float64 epilogue
// left alone took 130, i.e. 3 waves per SIMD)
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4)))
dedisp_kernel(DedispArgs a, const int32_t *__restrict__ tile_first, const int32_t *__restrict__ tile_count,
              const int32_t *__restrict__ tile_rowlen, const int32_t *__restrict__ base_tab,
              const u32x4 *__restrict__ rec_tab)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool kDma = std::is_same<Tin, Tl>::value;
    constexpr int SZ = (int)sizeof(Tl);
    constexpr int E = 8 / SZ;     // samples per 8-byte LDS read
    // reads per window: 4, or 2 when float32 rows feed float64 accumulators (8 trials x 8
    // float64 samples per lane would take 164 VGPRs: 3 waves per SIMD)
    constexpr int J = (sizeof(Ta) == 8 && sizeof(Tl) == 4) ? 2 : 4;
    constexpr int K = E * J;      // samples per lane
    constexpr int TT = 64 * K;    // samples per time tile
    constexpr int D = kD;

    const int wg = pu::xcd_remap(blockIdx.x, gridDim.x);
    const int dt = a.dt0 + wg % a.ndt;
    const int tt = a.tt0 + wg / a.ndt;
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
        if constexpr (kDma) asm volatile("s_waitcnt vmcnt(0)" : : : "memory");  // explicit (see dedisp_sub_kernel)
        __syncthreads();  // this wave's DMA landed and every wave left the other buffer
        if constexpr (kDma) {
            if (k + 1 < nchunks) issue_dma(k + 1, b ^ 1);
        } else {
            stage_regs(k);
            __syncthreads();
        }
        if (!active) continue;
        // ---- accumulate the chunk: channel pairs alternate window buffers so the next
        // channel's first window is read while this one is summed.  (Round 4 tried reads
        // one trial ahead of the adds instead, with a copy per changed window: C1 0.076
        // vs 0.068 ms.)
        const uint32_t rows_lane = smem_addr + (uint32_t)(b * buf_bytes) + 8u * lane;
        double w0[4], w1[4];
        const u32x4 *rc = recs + (size_t)c0 * kWaves;
        u32x4 rec0 = ld_uniform(rc);
        u32x4 rec1 = nc > 1 ? ld_uniform(rc + kWaves) : rec0;
        read_window<J>(w0, rows_lane + (rec0[0] & 0x7fffu));
        for (int ci = 0; ci < nc; ci += 2) {
            const uint32_t cb0 = rows_lane + (uint32_t)(ci * chan_bytes);
            const bool has1 = ci + 1 < nc, has2 = ci + 2 < nc, has3 = ci + 3 < nc;
            u32x4 rec2 = rec0, rec3 = rec1;
            if (has2) rec2 = ld_uniform(rc + (size_t)(ci + 2) * kWaves);  // two channels ahead
            if (has1) prefetch_window<J>(w1, cb0 + chan_bytes + (rec1[0] & 0x7fffu));
            channel_trials<Tl, Ta, K, J>(acc, w0, rec0, cb0);
            if (!has1) break;
            wait_window<J>(w1);
            if (has3) rec3 = ld_uniform(rc + (size_t)(ci + 3) * kWaves);
            if (has2) prefetch_window<J>(w0, cb0 + 2 * chan_bytes + (rec2[0] & 0x7fffu));
            channel_trials<Tl, Ta, K, J>(acc, w1, rec1, cb0 + chan_bytes);
            if (has2) wait_window<J>(w0);
            rec0 = rec2;
            rec1 = rec3;
        }
    }
    if (!active) return;

    if constexpr (STATS && !PLANE && sizeof(Ta) == 8) {
        if (t0 + TT <= n) {  // full tile: the permlane epilogue
            stats_full_f64<E, K>(acc, a, first, slot0, cnt, tt, lane);
            return;
        }
    }
    write_outputs<Tl, Ta, K, kD, PLANE, STATS>(acc, a, first, slot0, cnt, t0, tt, lane);
}


// ---------------------------------------------------------------------------------
// Subband mode (float32 accumulation of u8 / f32 / f64 inputs) -- DESIGN.md §4.2.
//
// Channels are taken in groups of G adjacent channels.  For trial d and group g the
// shifts are s_{d,c0+k} = b_d + v_k, with b_d the group's first-channel shift and v the
// group's relative-shift VECTOR.  Plan trials share a handful of vectors per group
// (channels of a group drift apart by ~G/nchan sample per trial; the floor() of each
// channel's delay jitters by one), so a DM tile of 128 trials needs ~4 distinct vectors
// per group.  Per (DM tile, time tile) workgroup, stage by stage (a stage = a few
// consecutive groups):
//   1. build: for every distinct vector v of the tile in the stage's groups -- a "slot"
//      -- the exact partial sum  R[i] = sum_{k<G} x[c0+k][(t0 + lo + v_k + i) mod N]
//      into LDS (two alignment copies: R[i] and R[i+1] at the same offset), from the
//      stage's channel rows staged in LDS by DMA (f32) or straight from global memory
//      (u8 / f64, converted to f32).  One slot per wave at a time, U 64-element chunks
//      per pass with all their reads in flight;
//   2. sum: every trial adds ONE window of its slot per group:
//      out_d[t0 + i] += R_{v(d)}[i + b_d - lo].
// The gathered elements are the reference's (circular shift-and-sum; u8 exact), with
// G x fewer adds than channel mode.
//
// Lane l of a wave owns samples t0 + 2l + 128j + e (j < K/2, e < 2) of D trials.
typedef int i32x2 __attribute__((ext_vector_type(2)));

// Workgroup shapes: W waves x D trials per wave, K samples per lane (time tile 64 K).
template <int W_, int D_, int K_>
struct SubCfg {
    static constexpr int W = W_, D = D_, K = K_, J = K_ / 2, TT = 64 * K_, T = W_ * D_, THREADS = 64 * W_;
};
using SubWide = SubCfg<16, 8, 8>;   // 128 trials x 512 samples, one workgroup per CU (160 KiB LDS)
using SubPair = SubCfg<8, 16, 4>;   // 128 trials x 256 samples, two workgroups per CU (80 KiB each)
using SubTall = SubCfg<16, 16, 4>;  // 256 trials x 256 samples, one workgroup per CU (160 KiB LDS)
enum SubShape { SUB_WIDE = 0, SUB_PAIR = 1, SUB_TALL = 2 };

template <class F>
auto with_shape(int shape, F &&f)
{
    if (shape == SUB_PAIR) return f(SubPair{});
    if (shape == SUB_TALL) return f(SubTall{});
    return f(SubWide{});
}

// Slot record (int32): slot length (elements, <= TT + spread + 1), copy-0 byte offset in
// the slot area, first channel, channels in the group, then the G sources of element
// 0 (raw-row float offsets in LDS, or sample indices mod N before adding t0).  Padded
// to a whole s_load.
__host__ __device__ constexpr int slot_stride(int G) { return G <= 4 ? 8 : 16; }

struct SubArgs {
    DedispArgs o;           // data, ld, nchan, n, ndt, ntt, small_n; plane / partials
    int32_t ngroups;
    int32_t raw_stride;     // elements per staged channel row (DMA mode; bytes for 8-bit rows)
    int32_t zero_len;       // floats of the zero row at LDS offset 0 (DMA mode, partial groups)
    int32_t lds_bytes;      // dynamic LDS size: a stage's raw rows end here
    int32_t skip;           // diagnostic build only (PU_SUB_SKIP; results invalid): 1 build, 2 sum, 4 DMA, 8 epilogue
    int32_t dma_waves;      // waves that issue the LDS-DMA rows (the last ones of the workgroup)
    int32_t nitems;         // work items (DM tiles x time tiles of this launch)
    int32_t base_bits;      // DMA row words: base = word & (2^base_bits - 1), cover = (word >> base_bits) x 256 B
    int32_t dt_major;       // item order: 0 = time tile major (DM tiles of a time tile share L2), 1 = DM tile major
    void *stamps;           // diagnostic build (PU_STAMPS): 8 x u64 phase-cycle totals
};

// Counted LDS wait that also "defines" the J window registers it guards, so the adds
// that read them cannot be hoisted above it.  lgkmcnt counts the inline-asm reads in
// issue order; an LDS op issued earlier or an outstanding scalar load only makes the
// wait longer, never shorter.
#define PU_WAIT_CASE(N)                                                                        \
    if constexpr (J == 4)                                                                      \
        asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]) \
                     : : "memory");                                                            \
    else                                                                                       \
        asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(w[0]), "+v"(w[1]) : : "memory");

template <int J, int N>
__device__ __forceinline__ void wait_window_n(double (&w)[J])
{
    static_assert(J == 2 || J == 4, "window reads");
    static_assert(N % J == 0 && N <= 3 * J, "lgkmcnt");
    if constexpr (N == 12) {
        PU_WAIT_CASE(12)
    } else if constexpr (N == 8) {
        PU_WAIT_CASE(8)
    } else if constexpr (N == 6) {
        PU_WAIT_CASE(6)
    } else if constexpr (N == 4) {
        PU_WAIT_CASE(4)
    } else if constexpr (N == 2) {
        PU_WAIT_CASE(2)
    } else {
        PU_WAIT_CASE(0)
    }
}
#undef PU_WAIT_CASE

// J x ds_read_b64 of one window (no wait).  Inline asm: hipcc would merge pairs into
// ds_read2st64_b64, which runs at half the LDS rate.
template <int J>
__device__ __forceinline__ void issue_window(double (&w)[J], uint32_t addr)
{
    if constexpr (J == 4)
        asm volatile(
            "ds_read_b64 %0, %4\n\t"
            "ds_read_b64 %1, %4 offset:512\n\t"
            "ds_read_b64 %2, %4 offset:1024\n\t"
            "ds_read_b64 %3, %4 offset:1536"
            : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
            : "v"(addr)
            : "memory");
    else
        asm volatile(
            "ds_read_b64 %0, %2\n\t"
            "ds_read_b64 %1, %2 offset:512"
            : "=&v"(w[0]), "=&v"(w[1])
            : "v"(addr)
            : "memory");
}

// One group's contribution to the wave's D trials: rec[d] = LDS byte offset (slot area
// relative) of trial d's window; reads run 3 trials ahead of the adds.  Accumulators are
// float pairs (samples 2l + 128 j + {0, 1}): one window read is one pair, added by one
// v_pk_add_f32 - two IEEE adds, the same bits as two v_add_f32, at half the VALU issue
// (the sum's 8 v_add_f32 per trial took as many CU cycles as its 4 ds_read_b64).
// (Skipping the reads of windows that repeat the previous trial's - a third of them at
// C2 - was tried: 32 compile-time read patterns chosen per (group, wave) spilled at the
// switch's joins; an EXEC = 0 ds_read_b64 or a ds_nop costs about as much as a real
// read, scripts/lds_probe.hip.)

template <class C, typename RecT>
__device__ __forceinline__ void group_trials(f32x2 (&acc)[C::D][C::J], const RecT rec, uint32_t base)
{
    constexpr int D = C::D, J = C::J;
    double w[4][J];
    issue_window<J>(w[0], base + rec[0]);
    issue_window<J>(w[1], base + rec[1]);
    issue_window<J>(w[2], base + rec[2]);
#pragma unroll
    for (int d = 0; d < D; ++d) {
        if (d + 3 < D) issue_window<J>(w[(d + 3) & 3], base + rec[d + 3]);
        double(&wd)[J] = w[d & 3];
        const int ahead = D - 1 - d < 3 ? D - 1 - d : 3;
        if (ahead == 3)
            wait_window_n<J, 3 * J>(wd);
        else if (ahead == 2)
            wait_window_n<J, 2 * J>(wd);
        else if (ahead == 1)
            wait_window_n<J, J>(wd);
        else
            wait_window_n<J, 0>(wd);
#pragma unroll
        for (int m = 0; m < J; ++m) acc[d][m] += __builtin_bit_cast(f32x2, wd[m]);
        pin_accumulators(acc[d]);
    }
}

// ---- 16-bit integer slots (8-bit input, time tile 256: DESIGN.md §4.1b).  A slot of an
// 8-bit group is a sum of <= G bytes, an integer <= G x 255, kept as u16 in four alignment
// copies (copy s holds R[i + s] at element i), so every window - 256 samples, four per
// lane - is ONE ds_read_b64 at an 8-byte-aligned address: half the sum's LDS reads of the
// float32 slots (two ds_read_b64 per window).  Lane l owns samples 4 l .. 4 l + 3 of its D
// trials in packed u16 accumulators `lo` (every add exact while the total since the last
// flush stays < 2^16) and `hi` (units of 256): every <= F groups (F G 255 + 255 < 2^16)
// `hi += lo >> 8, lo &= 255` - then hi 256 + lo is the exact integer sum (< nchan 255 <
// 2^24), converted to float32 once per item.  The u16 pairs are added as plain 32-bit words
// (v_add_u32): each half stays below 2^16, so no carry crosses into the high half.

#define PU_WAIT1_CASE(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(w) : : "memory");
template <int N>
__device__ __forceinline__ void wait_window1(u32x2 &w)
{
    static_assert(N >= 0 && N <= 7, "lgkmcnt");
    if constexpr (N == 7) { PU_WAIT1_CASE(7) }
    else if constexpr (N == 6) { PU_WAIT1_CASE(6) }
    else if constexpr (N == 5) { PU_WAIT1_CASE(5) }
    else if constexpr (N == 4) { PU_WAIT1_CASE(4) }
    else if constexpr (N == 3) { PU_WAIT1_CASE(3) }
    else if constexpr (N == 2) { PU_WAIT1_CASE(2) }
    else if constexpr (N == 1) { PU_WAIT1_CASE(1) }
    else { PU_WAIT1_CASE(0) }
}
#undef PU_WAIT1_CASE

// s_waitcnt lgkmcnt(N) that "defines" v (the value it guards), N in [0, 15]
#define PU_WAITV_CASE(N) else if constexpr (N0 == N) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(v) : : "memory");
template <int N0>
__device__ __forceinline__ void wait_lgkm(uint32_t &v)
{
    static_assert(N0 >= 0 && N0 <= 15, "lgkmcnt");
    if constexpr (N0 == 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v) : : "memory");
    PU_WAITV_CASE(1) PU_WAITV_CASE(2) PU_WAITV_CASE(3) PU_WAITV_CASE(4) PU_WAITV_CASE(5) PU_WAITV_CASE(6)
    PU_WAITV_CASE(7) PU_WAITV_CASE(8) PU_WAITV_CASE(9) PU_WAITV_CASE(10) PU_WAITV_CASE(11) PU_WAITV_CASE(12)
    PU_WAITV_CASE(13) PU_WAITV_CASE(14) PU_WAITV_CASE(15)
}
#undef PU_WAITV_CASE

#define PU_WAIT2_CASE(N) else if constexpr (N0 == N) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(v) : : "memory");
template <int N0>
__device__ __forceinline__ void wait_lgkm2(u32x2 &v)
{
    static_assert(N0 >= 0 && N0 <= 7, "lgkmcnt");
    if constexpr (N0 == 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v) : : "memory");
    PU_WAIT2_CASE(1) PU_WAIT2_CASE(2) PU_WAIT2_CASE(3) PU_WAIT2_CASE(4) PU_WAIT2_CASE(5) PU_WAIT2_CASE(6)
    PU_WAIT2_CASE(7)
}
#undef PU_WAIT2_CASE

// 16-bit slot build, one chunk of 128 elements: lane l's two elements 128 c + 2 l (+ 1) as
// the byte sums of the G channels (addresses ad[q], reads rb in flight).
// 16-bit slot build, P = 8 / G chunks of 128 elements in flight (2 G P = 16 byte reads,
// all the lgkmcnt field can count): register set C % P holds chunk C's reads.
template <int G, int P, int C>
__device__ __forceinline__ void s16_issue(uint32_t (&rb)[P][G][2], const uint32_t (&ad)[G])
{
#pragma unroll
    for (int q = 0; q < G; ++q) {
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(rb[C % P][q][0]) : "v"(ad[q]), "i"(128 * C) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(rb[C % P][q][1]) : "v"(ad[q]), "i"(128 * C + 1) : "memory");
    }
}

template <int G, int Q>
__device__ __forceinline__ void s16_quad_step(u32x2 (&d)[G], const uint32_t (&src)[G], uint32_t &acc02, uint32_t &acc13)
{
    if constexpr (Q < G) {
        wait_lgkm2<G - 1 - Q>(d[Q]);
        const uint32_t t = __builtin_amdgcn_alignbyte(d[Q].y, d[Q].x, src[Q]);  // bytes src .. src + 3
        acc02 += t & 0x00ff00ffu;
        acc13 += (t >> 8) & 0x00ff00ffu;
        s16_quad_step<G, Q + 1>(d, src, acc02, acc13);
    }
}

// 16-bit slot build, the first 256 elements with four per lane: one ds_read2_b32 per
// channel (the lane's two aligned dwords around its 4 bytes: 4 LDS cycles for 256
// positions, where two ds_read_u8 per 128 positions take 8), the 4 bytes by v_alignbyte
// (src mod 4, uniform per channel), even and odd bytes summed as u16 pairs (no carry
// crosses: each half <= G 255).  ea / eb = the lane's (R[4l], R[4l+1]) / (R[4l+2], R[4l+3]).
template <int G>
__device__ __forceinline__ void s16_quad(const uint32_t (&src)[G], uint32_t smem_addr, int lane, uint32_t &ea,
                                         uint32_t &eb)
{
    u32x2 d[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const uint32_t a = smem_addr + (src[q] & ~3u) + 4u * (uint32_t)lane;
        asm volatile("ds_read2_b32 %0, %1 offset1:1" : "=&v"(d[q]) : "v"(a) : "memory");
    }
    uint32_t acc02 = 0, acc13 = 0;
    s16_quad_step<G, 0>(d, src, acc02, acc13);
    ea = __builtin_amdgcn_perm(acc13, acc02, 0x05040100u);
    eb = __builtin_amdgcn_perm(acc13, acc02, 0x07060302u);
}

// chunks C .. CEND - 1 of the 128-element build, issued ahead as s16_run expects
template <int G, int P, int C, int CEND>
__device__ __forceinline__ void s16_issue_range(uint32_t (&rb)[P][G][2], const uint32_t (&ad)[G])
{
    if constexpr (C < CEND) {
        s16_issue<G, P, C>(rb, ad);
        s16_issue_range<G, P, C + 1, CEND>(rb, ad);
    }
}

template <int G, int P, int C, int NCH>
__device__ __forceinline__ void s16_issue_first(uint32_t (&rb)[P][G][2], const uint32_t (&ad)[G])
{
    if constexpr (C < P && C < NCH) {
        s16_issue<G, P, C>(rb, ad);
        s16_issue_first<G, P, C + 1, NCH>(rb, ad);
    }
}

// Read i of chunk C (channel i / 2, byte i % 2): wait until it landed - the reads complete
// in issue order, so the wait allows every read issued after it to be outstanding: the rest
// of chunk C, the chunks after C already issued and (NEXT) the i already re-issued for chunk
// C + P: lgkmcnt(2 G P - 1) in steady state (an outstanding scalar load only lengthens the
// wait) - add it, and (NEXT) re-issue its register for chunk C + P.
template <int G, int P, int C, int NCH, int I>
__device__ __forceinline__ void s16_step(uint32_t (&rb)[P][G][2], const uint32_t (&ad)[G], uint32_t &s0, uint32_t &s1)
{
    if constexpr (I < 2 * G) {
        constexpr int q = I >> 1, e = I & 1;
        constexpr bool NEXT = C + P < NCH;
        constexpr int L = (C + P <= NCH ? P : NCH - C) - 1;  // later chunks already in flight
        constexpr int N = NEXT ? 2 * G * P - 1 : 2 * G - 1 - I + 2 * G * L;
        static_assert(N >= 0 && N <= 15, "lgkmcnt");
        uint32_t &r = rb[C % P][q][e];
        wait_lgkm<N>(r);
        if constexpr (e == 0)
            s0 += r;
        else
            s1 += r;
        if constexpr (NEXT)
            asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(r) : "v"(ad[q]), "i"(128 * (C + P) + e) : "memory");
        s16_step<G, P, C, NCH, I + 1>(rb, ad, s0, s1);
    }
}

// chunks C .. NCH - 1: e[c] = lane l's elements 128 c + 2 l (+ 1) as a u16 pair
template <int G, int P, int C, int NCH>
__device__ __forceinline__ void s16_run(uint32_t (&rb)[P][G][2], const uint32_t (&ad)[G], uint32_t (&e)[4])
{
    if constexpr (C < NCH) {
        uint32_t s0 = 0, s1 = 0;
        s16_step<G, P, C, NCH, 0>(rb, ad, s0, s1);
        e[C] = s0 | (s1 << 16);
        s16_run<G, P, C + 1, NCH>(rb, ad, e);
    }
}


__device__ __forceinline__ void issue_window1(u32x2 &w, uint32_t addr)
{
    asm volatile("ds_read_b64 %0, %1" : "=&v"(w) : "v"(addr) : "memory");
}

// One group's contribution to the wave's D trials from 16-bit slots: one window read per
// trial, issued A trials ahead of its two v_pk_add_u16.
template <int D, int A, int I, typename RecT>
__device__ __forceinline__ void trials16_step(uint32_t (&lo)[D][2], u32x2 (&w)[A + 1], const RecT &rec, uint32_t base)
{
    if constexpr (I < D) {
        if constexpr (I + A < D) issue_window1(w[(I + A) % (A + 1)], base + rec[I + A]);
        constexpr int ahead = D - 1 - I < A ? D - 1 - I : A;
        u32x2 &wd = w[I % (A + 1)];
        wait_window1<ahead>(wd);
        lo[I][0] += wd.x;  // two u16 sums per dword: no carry crosses (each half < 2^16)
        lo[I][1] += wd.y;
        asm volatile("" : "+v"(lo[I][0]), "+v"(lo[I][1]));
        trials16_step<D, A, I + 1>(lo, w, rec, base);
    }
}

template <class C, typename RecT>
__device__ __forceinline__ void group_trials16(uint32_t (&lo)[C::D][2], const RecT rec, uint32_t base)
{
    constexpr int D = C::D, A = 5;
    u32x2 w[A + 1];
#pragma unroll
    for (int d = 0; d < A && d < D; ++d) issue_window1(w[d], base + rec[d]);
    trials16_step<D, A, 0>(lo, w, rec, base);
}

// per 16-bit half: hi += lo >> 8, lo &= 255 (exact: lo < 2^16; hi counts 256s, < nchan < 2^16,
// so neither 32-bit add carries across the halves)
template <int D>
__device__ __forceinline__ void flush16(uint32_t (&lo)[D][2], uint32_t (&hi)[D][2])
{
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            hi[d][k] += (lo[d][k] >> 8) & 0x00ff00ffu;
            lo[d][k] &= 0x00ff00ffu;
        }
}

// The exact sums as float32 in the float slots' lane layout (lane l: samples 128 j + 2 l +
// e), which the epilogues and write_outputs take: sample 128 j + 2 l + e lives in lane
// 32 j + l / 2, element 2 (l & 1) + e - four ds_bpermute per (trial, j) and a select.
template <int D>
__device__ __forceinline__ void s16_to_pairs(const uint32_t (&lo)[D][2], const uint32_t (&hi)[D][2], f32x2 (&acc)[D][2],
                                             int lane)
{
    const bool odd = lane & 1;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            v[2 * k] = (float)((hi[d][k] & 0xffffu) * 256u + (lo[d][k] & 0xffffu));
            v[2 * k + 1] = (float)((hi[d][k] >> 16) * 256u + (lo[d][k] >> 16));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int src = 4 * (32 * j + (lane >> 1));
            float g[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                g[e] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, v[e])));
            acc[d][j] = odd ? f32x2{g[2], g[3]} : f32x2{g[0], g[1]};
        }
    }
}

// LDS-DMA of one 8-bit channel-row window [start, start + cover) mod n into dst, start
// and n multiples of 4 (the planner folds each row's misalignment into the slot
// sources): 1 KiB pieces while contiguous, per-lane modular dwords if it wraps.
__device__ __forceinline__ void dma_row_u8(unsigned char *dst, const unsigned char *row, int start, int cover_bytes,
                                           int n, bool small_n, int lane)
{
    if (!small_n && start + cover_bytes <= n) {
        const unsigned char *src = row + start;
        int off = 0;
        for (; off + 1024 <= cover_bytes; off += 1024)
            __builtin_amdgcn_global_load_lds((const void *)(src + off + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(dst + off), 16, 0, 0);
        if (off < cover_bytes && lane < (cover_bytes - off) / 16)  // tail: one partial piece
            __builtin_amdgcn_global_load_lds((const void *)(src + off + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(dst + off), 16, 0, 0);
    } else {
        const int nd = n >> 2;
        for (int off = 0; off < cover_bytes; off += 256) {
            int idx = (start >> 2) + (off >> 2) + lane;
            if (small_n) {
                idx %= nd;
            } else {
                idx = idx >= nd ? idx - nd : idx;
            }
            __builtin_amdgcn_global_load_lds((const void *)(row + 4 * idx),
                                             (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
        }
    }
}

// DMA8: 8-bit rows staged by LDS-DMA as bytes (plans with n % 4 == 0); otherwise 8-bit
// and float64 builds read global memory.
// One (DM tile, time tile) work item of the subband kernel: logical index wg; first =
// this workgroup's first item (it writes the zero row, which no item overwrites).
template <class C, typename Tin, int G, bool PLANE, bool STATS, bool DMA8, bool S16>
__device__ __forceinline__ void sub_item(SubArgs &a, const i32x4 *__restrict__ tiles,
                                         const i32x2 *__restrict__ tile_stages, const i32x4 *__restrict__ stages,
                                         const int32_t *__restrict__ slots, const int32_t *__restrict__ base_tab,
                                         const uint32_t *__restrict__ rec_tab, const int wg, const bool first_item)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool kDma = std::is_same<Tin, float>::value || (DMA8 && std::is_same<Tin, uint8_t>::value);
    constexpr int EB = std::is_same<Tin, float>::value ? 4 : 1;  // bytes per staged raw element
    constexpr int W = C::W, D = C::D, K = C::K, TT = C::TT;
    constexpr int MS = slot_stride(G);
    // chunks of 64 per build pass: one pass at a plan grid's spread when G x U values fit
    constexpr int U = std::min((TT + 80 + 63) / 64, (sizeof(Tin) == 8 ? 20 : 40) / G);
    typedef int32_t meta_t __attribute__((ext_vector_type(MS)));
    typedef uint32_t rec_t __attribute__((ext_vector_type(D)));
    const DedispArgs &o = a.o;
    const int ndt = o.ndt;
    // Items in dispatch order.  The planner sorts the DM tiles by decreasing cost, so
    // DM-tile-major order dispatches the longest items first (LPT: the short ones fill
    // the tail), for grids of few items per CU; time-tile-major order keeps the DM tiles
    // of one time tile together (one XCD, its L2 serving their overlapping rows).
    const int dt = o.dt0 + (a.dt_major ? wg / o.ntt_run : wg % ndt);
    const int tt = o.tt0 + (a.dt_major ? wg % o.ntt_run : wg / ndt);
    const int t0 = tt * TT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const i32x4 tile = ld_uniform(tiles + dt);        // {first trial, count, raw row length, copy bytes}
    const i32x2 ts = ld_uniform(tile_stages + dt);    // {first stage, stage count}
    const int first = tile.x, cnt = tile.y;
    // alignment-copy bytes: float32 slots share the tile's (its widest span: whole build
    // passes need no store guards, C2's 2560 B at UP = 10); a 16-bit slot's follow from its
    // own length (the planner sizes it by its own span: (len + 2) u16, 64-rounded)
    const int tile_copy_bytes = tile.w;
    auto copy_bytes_of = [&](int len) {
        if constexpr (S16) return ((len + 65) & ~63) * 2;
        // float32: whole build passes (64 U elements: no store guards), at most the tile's
        const int whole = (len + 64 * U) / (64 * U) * (64 * U) * 4;
        return whole < tile_copy_bytes ? whole : tile_copy_bytes;
    };
    const int slot0 = wave * D;
    const bool active = slot0 < cnt;
    const int n = o.n;
    const bool small_n = o.small_n != 0;
    const Tin *data = reinterpret_cast<const Tin *>(o.data);
    const uint32_t smem_addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;
    const uint32_t lds_base = smem_addr;  // slot records hold absolute LDS offsets
    const float *raw_lds = reinterpret_cast<const float *>(smem);
    const unsigned char *raw_lds8 = smem;

    static_assert(!S16 || (kDma && EB == 1 && C::K == 4), "16-bit slots: 8-bit DMA rows, 256-sample tiles");
    f32x2 acc2[D][C::J];
    if constexpr (!S16) {
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int m = 0; m < C::J; ++m) acc2[d][m] = f32x2{0.0f, 0.0f};
    }
    // 16-bit slots: packed u16 accumulators, flushed every <= F16 groups (see flush16)
    constexpr int F16 = (65535 - 255) / (G * 255);
    uint32_t lo16[S16 ? D : 1][2], hi16[S16 ? D : 1][2];  // u16 pairs: (sample 4 l + 2 k, + 1)
    if constexpr (S16) {
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
            for (int k = 0; k < 2; ++k) lo16[d][k] = hi16[d][k] = 0u;
    }
    int gc16 = 0;  // groups added since the last flush

    const rec_t *recs = reinterpret_cast<const rec_t *>(rec_tab) + (size_t)dt * a.ngroups * W + wave;
    if constexpr (kDma) {
        // zero row (partial groups' missing channels) between the raw rows and the slots
        if (first_item) {
            float *zero = reinterpret_cast<float *>(smem);
            for (int i = tid; i < a.zero_len; i += C::THREADS) zero[i] = 0.0f;
        }
    }

    // ---- DMA mode: the channel rows of stage st into the raw area.  vb = this wave's row
    // bases, lane k holding row wave + W k (one vector load per stage, issued a phase
    // ahead: a scalar load per row put its latency in series with every row's DMA issue,
    // ~10 % of the kernel's wave cycles at C2)
    // Only the last NDW waves issue the DMA (rows dw + NDW k, dw = wave - (W - NDW)): the
    // other waves go straight from the barrier to the sum instead of queueing their DMA
    // instructions behind everyone's on the CU's one texture-address path.
    const int32_t *base_t = base_tab + (size_t)dt * o.nchan;
    const int NDW = a.dma_waves;
#ifdef PU_STAMPS
    int skip = a.skip;  // diagnostic build only: PU_SUB_SKIP ablation (results invalid)
#else
    constexpr int skip = 0;  // the production kernel always does all of its work
#endif
    const int dw = wave - (W - NDW);  // < 0: this wave issues no DMA
    auto bases_of = [&](const i32x4 st) -> int {
        const int c = st.x * G + dw + NDW * lane;
        return dw >= 0 && c < min(st.y * G, o.nchan) ? base_t[c] : 0;
    };
    // this wave's rows of stage st: dw + NDW k for k < rows_of(st)
    auto rows_of = [&](const i32x4 st) {
        return dw < 0 ? 0 : (min(st.y * G, o.nchan) - st.x * G - dw + NDW - 1) / NDW;
    };
    // rows k in [kb, ke) of this wave
    auto issue_raw = [&](const i32x4 st, int vb, int kb, int ke) {
        const int c0 = st.x * G;
        const int nc = min(st.y * G, o.nchan) - c0;
        // the stage's rows end at the top of LDS (the host packs stages so that they never
        // overlap the previous stage's slots, which are summed while these rows land)
        unsigned char *raw = smem + a.lds_bytes - ((nc * a.raw_stride * EB + 255) & ~255);
        const int cover_tile = (tile.z * EB + 255) & ~255;
        const uint32_t base_mask = (1u << a.base_bits) - 1u;
        // row pointers by increments (one 64-bit add per row instead of a 64-bit multiply)
        const size_t row_step = (size_t)NDW * (size_t)o.ld;
        const Tin *rowp = data + (size_t)(c0 + dw + NDW * kb) * (size_t)o.ld;
        for (int k = kb; k < ke; ++k, rowp += row_step) {
            const int ci = dw + NDW * k;
            const int c = c0 + ci;
            // the row word: its base mod N and, in the top bits, this channel's own cover
            // (TT + its shift spread over the tile, in 256-B units; 0 = the tile's)
            const uint32_t word = (uint32_t)(k < 64 ? __builtin_amdgcn_readlane(vb, k) : ld_uniform(base_t + c));
            const uint32_t cu = word >> a.base_bits;
            const int cover_bytes = cu ? (int)(cu << 8) : cover_tile;
            int start = (int)(word & base_mask) + t0;
            if (start >= n) start -= n;
            if constexpr (EB == 4)
                dma_row_f32(raw + ci * a.raw_stride * 4, reinterpret_cast<const float *>(rowp), start, cover_bytes, n,
                            small_n, lane);
            else
                dma_row_u8(raw + ci * a.raw_stride, reinterpret_cast<const unsigned char *>(rowp), start, cover_bytes,
                           n, small_n, lane);
        }
    };

    auto load = [&](const meta_t &m, int q, int i) -> float {
        if constexpr (kDma && EB == 1) {
            return static_cast<float>(raw_lds8[m[4 + q] + i]);  // ds_read_u8
        } else if constexpr (kDma) {
            return raw_lds[m[4 + q] + i];  // past the slot only for masked lanes (row padding)
        } else {
            int pos = m[4 + q] + t0 + i;
            if (small_n) {
                pos %= n;
            } else {
                if (pos >= n) pos -= n;
                if (pos >= n) pos -= n;
            }
            const int ch = min(m[2] + q, o.nchan - 1);  // partial groups: in-bounds, discarded
            return static_cast<float>(data[(size_t)ch * (size_t)o.ld + pos]);
        }
    };

    // ---- one build pass: chunks [i0, i0 + 64 UP) of a slot, written while < lim (whole
    // chunks: lanes past len write row padding).  All G x UP reads in flight.  Reads of
    // chunks past lim are not clamped: their results are discarded, and an LDS read past
    // the allocation returns 0 (clamping them costs a VALU add per read - the reads then
    // cannot fold 256 u into the ds_read offset field - and was measured 1.8 ms slower at
    // C2, 20.2 vs 18.4 ms).
    auto build_pass = [&](auto upc, const meta_t &m, int gs, int i0, int lim, bool whole, int copy_bytes) {
        constexpr int UP = decltype(upc)::value;
        auto at = [&](int u) { return i0 + 64 * u + lane; };
        float r[UP];
        if constexpr (kDma && EB == 1) {
            // 8-bit rows: the bytes summed as integers (v_add3_u32), one convert per element
            // - the same float32 value as the float sum (every partial sum < 2^24 is exact),
            // a third of the VALU work of a convert + add per byte
            uint32_t w[UP][G];
#pragma unroll
            for (int u = 0; u < UP; ++u)
#pragma unroll
                for (int q = 0; q < G; ++q) w[u][q] = raw_lds8[m[4 + q] + at(u)];  // ds_read_u8
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                uint32_t s = 0;
#pragma unroll
                for (int q = 0; q < G; ++q) s += w[u][q];
                r[u] = static_cast<float>(s);
            }
        } else {
            float v[UP][G];
            if (kDma || gs == G) {  // branch-free, all G x UP reads in flight (DMA mode: a
                                    // partial group's missing channels read the zero row)
#pragma unroll
                for (int u = 0; u < UP; ++u)
#pragma unroll
                    for (int q = 0; q < G; ++q) v[u][q] = load(m, q, at(u));
            } else {        // the last, partial group of a band
#pragma unroll
                for (int u = 0; u < UP; ++u)
#pragma unroll
                    for (int q = 0; q < G; ++q) v[u][q] = q < gs ? load(m, q, at(u)) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                r[u] = 0.0f;
#pragma unroll
                for (int q = 0; q < G; ++q) r[u] += v[u][q];
            }
        }
        // all sums before the first (chunk-uniform) write branch: keeps every read
        // of the pass in flight together
#pragma unroll
        for (int u = 0; u < UP; ++u) asm volatile("" : "+v"(r[u]));
        // copy 0 at element i, copy 1 at element i - 1: lane-contiguous dwords, so
        // ds_write_addtid_b32 (address = M0 + offset + 4 lane, no address VGPR):
        // twice the LDS store rate of ds_write_b32 (MI355X_MICROARCH.md §LDS)
        const uint32_t w0 = lds_base + (uint32_t)m[1] + 4u * (uint32_t)i0;
        const uint32_t w1 = w0 + (uint32_t)copy_bytes - 4u;
        // M0 set twice per pass (copy 0, then copy 1) and not restored: hipcc sets M0 afresh
        // in the basic block of every LDS-DMA it emits (checked on the generated code by
        // scripts/check_m0.py; an "m0" clobber would be ignored - hipcc treats M0 as
        // reserved); nothing between these volatile statements uses M0.  (Saving and
        // restoring it cost two scalar instructions per pass: C2 15.78 vs 15.65 ms.)  Setting it around every
        // chunk's two stores instead cost ~7 scalar issue slots per chunk on the CU's shared
        // scalar unit (C2 19.97 -> 19.20 ms, C3 625 trials 156.5 -> 150.9 ms).  When a copy
        // spans whole passes (copy_bytes a multiple of 256 UP: C2's 2560 B at UP = 10) the
        // chunks past len only write the slot's own padding, so the stores need no guards;
        // so does any pass whose UP chunks end inside the copy (4 i0 + 256 UP <= copy_bytes:
        // copy 1's stores end 4 bytes earlier than copy 0's) - round 5: C3's single pass per
        // slot (272 elements, UP = 5) no longer guards each store by a scalar compare + branch
        // when its copy is 6 chunks long.  (whole: pass_whole(i0), decided by the caller - for
        // the first pass once per tile.)
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(w0) : "memory");
        if (whole) {
#pragma unroll
            for (int u = 0; u < UP; ++u)
                asm volatile("ds_write_addtid_b32 %0 offset:%1" : : "v"(r[u]), "i"(256 * u) : "memory");
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(w1) : "memory");
#pragma unroll
            for (int u = 0; u < UP; ++u)
                asm volatile("ds_write_addtid_b32 %0 offset:%1" : : "v"(r[u]), "i"(256 * u) : "memory");
        } else {
#pragma unroll
            for (int u = 0; u < UP; ++u)
                if (i0 + 64 * u < lim)
                    asm volatile("ds_write_addtid_b32 %0 offset:%1" : : "v"(r[u]), "i"(256 * u) : "memory");
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(w1) : "memory");
#pragma unroll
            for (int u = 0; u < UP; ++u)
                if (i0 + 64 * u < lim)
                    asm volatile("ds_write_addtid_b32 %0 offset:%1" : : "v"(r[u]), "i"(256 * u) : "memory");
        }
    };

    // ---- 16-bit slots (S16): one slot in chunks of 128 elements, lane l building elements
    // 128 u + 2 l and + 1 of chunk u (two byte reads per channel, summed as integers) packed
    // as one u16 pair E_u; the odd-shifted pair (R[2k + 1], R[2k + 2]) is E_u's high half
    // with the next lane's low half (DPP wave_shl:1; lane 63 takes chunk u + 1's lane 0 by
    // wave_rol:1).  Stores by ds_write_addtid_b32: E_u to copy 0 and, 4 bytes down, copy 2;
    // O_u to copy 1 and, 4 bytes down, copy 3 (element i of copy s is R[i + s]).  Chunks
    // 0-2 always (len <= 512; a chunk past the copy's end stores only its lanes inside it),
    // chunk 3 when len > 384; the reads of the next 8 / G chunks in flight while a chunk is
    // summed.
    auto slot16_pairs = [&](const meta_t &m) {
        const bool four = m[0] > 384;
        const int copy_bytes = copy_bytes_of(m[0]);
        auto odd = [&](uint32_t e, uint32_t enext) {  // (R[2k + 1], R[2k + 2]) of lane k
            const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)enext, 0x134, 0xf, 0xf, false);  // wave_rol:1
            const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)e, 0x130, 0xf, 0xf, false);  // wave_shl:1
            return __builtin_amdgcn_alignbit(y, e, 16);
        };
        // per channel the lane's byte address; 2 G byte reads per chunk (ds_read_u8 in inline
        // asm: the order kept by s16_run holds ~15 in flight in 16 registers - each value is
        // added, then its register takes the read of chunk c + 8 / G, same channel and byte)
        uint32_t ad[G];
#pragma unroll
        for (int q = 0; q < G; ++q) ad[q] = smem_addr + (uint32_t)m[4 + q] + 2u * (uint32_t)lane;
        constexpr int P = 8 / G;
        uint32_t rb[P][G][2];
        uint32_t e[4] = {0u, 0u, 0u, 0u};
        if (four) {
            s16_issue_first<G, P, 0, 4>(rb, ad);
            s16_run<G, P, 0, 4>(rb, ad, e);
        } else {
            s16_issue_first<G, P, 0, 3>(rb, ad);
            s16_run<G, P, 0, 3>(rb, ad, e);
        }
        const uint32_t e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
        uint32_t o0 = odd(e0, e1), o1 = odd(e1, e2), o2 = odd(e2, e3), o3 = four ? odd(e3, e3) : 0u;
        asm volatile("" : "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3));
        const uint32_t c0 = lds_base + (uint32_t)m[1];
        const uint32_t cbu = (uint32_t)copy_bytes;
        // a chunk reaching past its copy (copies hold TT + span + 2 elements rounded to 64)
        // stores only its lanes inside it (elements 128 c + 2 l <= copy - 2; copies 2 / 3 give
        // up their last dword, beyond every window)
        const bool fit2 = 768u <= cbu, fit3 = 1024u <= cbu;
        const bool in2 = 512 + 4 * lane <= (int)cbu - 4, in3 = 768 + 4 * lane <= (int)cbu - 4;
        auto store = [&](uint32_t base, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(base) : "memory");
            asm volatile("ds_write_addtid_b32 %0 offset:0" : : "v"(v0) : "memory");
            asm volatile("ds_write_addtid_b32 %0 offset:256" : : "v"(v1) : "memory");
            if (fit2 || in2) asm volatile("ds_write_addtid_b32 %0 offset:512" : : "v"(v2) : "memory");
            if (four && (fit3 || in3)) asm volatile("ds_write_addtid_b32 %0 offset:768" : : "v"(v3) : "memory");
        };
        store(c0, e0, e1, e2, e3);
        store(c0 + 2u * cbu - 4u, e0, e1, e2, e3);
        store(c0 + cbu, o0, o1, o2, o3);
        store(c0 + 3u * cbu - 4u, o0, o1, o2, o3);
    };

    auto slot16_quad = [&](const meta_t &m) {
        const int len = m[0];  // 256 (= TT) .. 510
        const int copy_bytes = copy_bytes_of(len);
        auto odd = [&](uint32_t e, uint32_t enext) {  // (R[2k + 1], R[2k + 2]) of lane k
            const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)enext, 0x134, 0xf, 0xf, false);  // wave_rol:1
            const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)e, 0x130, 0xf, 0xf, false);  // wave_shl:1
            return __builtin_amdgcn_alignbit(y, e, 16);
        };
        // the next lane's value (lane 63: lane 0 of `next`)
        auto nextlane = [&](uint32_t v, uint32_t next) {
            const uint32_t x = (uint32_t)__builtin_amdgcn_mov_dpp((int)next, 0x134, 0xf, 0xf, false);
            return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)v, 0x130, 0xf, 0xf, false);
        };
        // elements 0 .. 255: four per lane (s16_quad)
        uint32_t src[G];
#pragma unroll
        for (int q = 0; q < G; ++q) src[q] = (uint32_t)m[4 + q];
        uint32_t ea, eb;
        s16_quad<G>(src, smem_addr, lane, ea, eb);
        // elements 256 .. len - 1 (<= 2 chunks of 128): two per lane, as chunks 2 and 3 of the
        // 128-element build (its reads in flight per s16_run)
        uint32_t ad[G];
#pragma unroll
        for (int q = 0; q < G; ++q) ad[q] = smem_addr + src[q] + 2u * (uint32_t)lane;
        constexpr int P = 8 / G;
        uint32_t rb[P][G][2];
        uint32_t e[4] = {0u, 0u, 0u, 0u};
        const bool t2 = len > 256, t3 = len > 384;
        if (t3) {
            s16_issue_range<G, P, 2, (2 + P < 4 ? 2 + P : 4)>(rb, ad);
            s16_run<G, P, 2, 4>(rb, ad, e);
        } else if (t2) {
            s16_issue_range<G, P, 2, 3>(rb, ad);
            s16_run<G, P, 2, 3>(rb, ad, e);
        }
        // dword j of copy s: copy 0 E[j], copy 1 O[j], copy 2 E[j + 1], copy 3 O[j + 1]
        // (E[k] = (R[2k], R[2k+1]), O[k] = (R[2k+1], R[2k+2])); lane l of the first 256
        // elements owns dwords 2l and 2l + 1: E[2l] = ea, E[2l+1] = eb
        const uint32_t nea = nextlane(ea, e[2]);  // E[2l + 2] (lane 63: the tail's first pair)
        const uint32_t neb = nextlane(eb, e[2]);  // E[2l + 3] (lane 63's is rewritten by the tail)
        u32x2 w0 = {ea, eb}, w2 = {eb, nea};
        u32x2 w1 = {__builtin_amdgcn_alignbit(eb, ea, 16), __builtin_amdgcn_alignbit(nea, eb, 16)};
        u32x2 w3 = {w1.y, __builtin_amdgcn_alignbit(neb, nea, 16)};
        const uint32_t c0 = lds_base + (uint32_t)m[1];
        const uint32_t cbu = (uint32_t)copy_bytes;
        const uint32_t a0 = c0 + 8u * (uint32_t)lane;
        asm volatile("ds_write_b64 %0, %1" : : "v"(a0), "v"(w0) : "memory");
        asm volatile("ds_write_b64 %0, %1" : : "v"(a0 + cbu), "v"(w1) : "memory");
        asm volatile("ds_write_b64 %0, %1" : : "v"(a0 + 2u * cbu), "v"(w2) : "memory");
        asm volatile("ds_write_b64 %0, %1" : : "v"(a0 + 3u * cbu), "v"(w3) : "memory");
        if (t2) {
            // the tail chunks by ds_write_addtid_b32 (copies 2 / 3 4 bytes down, after the
            // first part's stores: its copy-3 dword 127 is rewritten here); a chunk reaching
            // past its copy (copies hold TT + span + 2 elements rounded to 64) stores only its
            // lanes inside it (elements 128 c + 2 l <= copy - 2)
            const uint32_t o2 = odd(e[2], e[3]), o3 = odd(e[3], e[3]);
            const bool in2 = 768u <= cbu || 512 + 4 * lane <= (int)cbu - 4;
            const bool in3 = t3 && (1024u <= cbu || 768 + 4 * lane <= (int)cbu - 4);
            auto store = [&](uint32_t base, uint32_t v2, uint32_t v3) {
                asm volatile("s_mov_b32 m0, %0\n\ts_nop 0" : : "s"(base) : "memory");
                if (in2) asm volatile("ds_write_addtid_b32 %0 offset:512" : : "v"(v2) : "memory");
                if (in3) asm volatile("ds_write_addtid_b32 %0 offset:768" : : "v"(v3) : "memory");
            };
            store(c0, e[2], e[3]);
            store(c0 + 2u * cbu - 4u, e[2], e[3]);
            store(c0 + cbu, o2, o3);
            store(c0 + 3u * cbu - 4u, o2, o3);
        }
    };

    // G = 8: the first 256 elements four per lane (s16_quad: half the build's LDS read cycles;
    // round 6 A/B: C3 625 trials 115.5 -> 113.5 ms, 5000 958 -> 936 ms); G <= 4: two per lane
    // throughout, which measured faster there (5000 trials G = 4: 858 vs 901 ms) - with 2 G
    // byte reads per chunk, 8 / G chunks stay in flight
    auto slot16 = [&](const meta_t &m) {
        if constexpr (G == 8)
            slot16_quad(m);
        else
            slot16_pairs(m);
    };

    // ---- build the stage's slots, one per wave at a time: R[i] (i < len) at copy 0 [i]
    // and copy 1 [i - 1] (copy 1's element -1 lands in copy 0's padding).  (Splitting a
    // slot over waves to balance the ~20 slots of a stage over 16 waves was measured
    // slower: 22.1 / 25.6 vs 20.2 ms for halves / thirds - fewer reads in flight per
    // pass, and the extra pass code spilled registers.)
    auto pass_whole = [&](int i0, int copy_bytes) {
        return copy_bytes % (256 * U) == 0 || 4 * i0 + 256 * U <= copy_bytes;
    };
    auto build = [&](const i32x4 st, const meta_t m0) {
        // the next slot's record is loaded a slot ahead (round 5: loaded on demand, its
        // scalar-load latency stood in front of every slot after a wave's first), through a
        // pointer stepped by W records: past the stage's last slot it reads the next stage's
        // records or the table's padding (upload_sub: W records of zeros), never used.
        // Every slot has a first pass (len >= TT): peeled, with the tile's whole0.
        // Two slots per iteration with ping-pong records (rotating one record through a copy
        // cost a dozen scalar moves per slot).
        auto slot = [&](const meta_t &m) {
            const int len = m[0], gs = m[3];
            const int lim = (len + 63) & ~63;
            const int cb = copy_bytes_of(len);
            build_pass(std::integral_constant<int, U>{}, m, gs, 0, lim, pass_whole(0, cb), cb);
            for (int i0 = 64 * U; i0 < len; i0 += 64 * U)
                build_pass(std::integral_constant<int, U>{}, m, gs, i0, lim, pass_whole(i0, cb), cb);
        };
        meta_t ma = m0;
        const meta_t *mp = reinterpret_cast<const meta_t *>(slots) + (size_t)(st.z + wave + W);
        for (int s = st.z + wave; s < st.w; s += 2 * W, mp += 2 * W) {
            meta_t mb = ld_uniform(mp);
            if constexpr (S16)
                slot16(ma);
            else
                slot(ma);
            if (s + W >= st.w) break;
            ma = ld_uniform(mp + W);
            if constexpr (S16)
                slot16(mb);
            else
                slot(mb);
        }
    };

    // ---- stage loop.  Scalar metadata is loaded one step ahead (the stage records of k+1
    // and k+2, this wave's first DMA row base, slot record and window records), so the
    // loads' latency overlaps the barrier waits instead of the phases.
    const int ns = ts.y;
    auto stage_at = [&](int k) { return ld_uniform(stages + ts.x + min(k, ns - 1)); };
    auto meta_of = [&](const i32x4 st) {
        return ld_uniform(reinterpret_cast<const meta_t *>(slots + (size_t)min(st.z + wave, st.w - 1) * MS));
    };
    i32x4 st = stage_at(0), st1 = stage_at(1);
    if constexpr (kDma) issue_raw(st, bases_of(st), 0, rows_of(st));
#ifdef PU_STAMPS
    // diagnostic build only (make stamps): per-wave cycles per phase, summed over stages
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp = stamp(), tq;
#define PU_PHASE(i) (tq = stamp(), ph[i] += tq - tp, tp = tq)
#else
#define PU_PHASE(i) ((void)0)
#endif
    for (int k = 0; k < ns; ++k) {
        const i32x4 st2 = stage_at(k + 2);
        const meta_t m0 = meta_of(st);
        const rec_t rec0 = ld_uniform(recs + (size_t)st.x * W);
        PU_PHASE(0);
        // This wave's LDS-DMA rows have landed before it arrives at the barrier.  Explicit:
        // a workgroup-scope __syncthreads does not wait for vmcnt on gfx950, and the
        // compiler's own LDS-DMA tracking puts its wait before this wave's first LDS read,
        // after the barrier - too late for the other waves that read these rows.
        asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
        PU_PHASE(7);
        __syncthreads();  // raw rows of stage k landed; every wave left the slot area
        PU_PHASE(1);
        const int vb1 = kDma && k + 1 < ns ? bases_of(st1) : 0;  // lands during the build
        if (!(skip & 1)) build(st, m0);
        PU_PHASE(2);
        __syncthreads();  // slots built; every wave left the raw rows
        PU_PHASE(3);
        if constexpr (kDma) {
            // the next stage's rows land while this stage is summed.  (Spreading these DMAs
            // over the sum's groups instead was measured slower, 20.6 vs 18.5 ms at C2: the
            // issue inside the sum breaks its read pipelining.)
            // The row-base load is waited for HERE, on every path, while no DMA is in
            // flight: left to the compiler, the wait for it lands at the head of the sum
            // loop as vmcnt(0) (its register is reused there), which also waits for all
            // the DMAs just issued - every DMA wave then summed only after its rows landed.
            int vb = vb1;
            asm volatile("" : "+v"(vb));
            if (k + 1 < ns && !(skip & 4)) issue_raw(st1, vb, 0, rows_of(st1));
        }
        PU_PHASE(4);
        // The DMA waves start summing last (their LDS-DMA issue holds them ~10 % of the
        // stage), so they sum at raised priority: the other waves fill the LDS queue
        // around them instead of reaching the barrier first and leaving it half idle
        // (C2 17.3 -> 16.9 ms; raising it for the DMA issue too: 17.6).
        if (dw >= 0) __builtin_amdgcn_s_setprio(1);
        if (active && !(skip & 2)) {
            const uint32_t sb = smem_addr + 8u * lane;  // window records: absolute LDS offsets
            // two groups per iteration with ping-pong records (no per-group record copy).
            // A record is consumed only after the previous group's last lgkmcnt(0) (the empty
            // asm): hoisted into the trial loop, its scalar-load wait drained the LDS reads.
            // The row past the stage's last group is a valid record (clamped index): loaded,
            // never used.
            rec_t ra = rec0;
            const int gl = st.y - 1;
            for (int g = st.x; g < st.y; g += 2) {
                rec_t rb = ld_uniform(recs + (size_t)min(g + 1, gl) * W);
                if constexpr (S16) {
                    if (gc16 + 2 > F16) {
                        flush16<D>(lo16, hi16);
                        gc16 = 0;
                    }
                    gc16 += 2;
                    group_trials16<C>(lo16, ra, sb);
                } else {
                    group_trials<C>(acc2, ra, sb);
                }
                asm volatile("" : "+s"(rb));
                if (g + 1 > gl) break;
                ra = ld_uniform(recs + (size_t)min(g + 2, gl) * W);
                if constexpr (S16)
                    group_trials16<C>(lo16, rb, sb);
                else
                    group_trials<C>(acc2, rb, sb);
                asm volatile("" : "+s"(ra));
            }
        }
        if (dw >= 0) __builtin_amdgcn_s_setprio(0);
        PU_PHASE(5);
        st = st1;
        st1 = st2;
    }
    if constexpr (S16) {
        if (active) s16_to_pairs<D>(lo16, hi16, acc2, lane);
    }
    if constexpr (STATS && !PLANE) {
        if (active && !(skip & 8) && t0 + TT <= n) {
            stats_full_pairs<D, C::J>(acc2, o, first, slot0, cnt, tt, lane);
#ifndef PU_STAMPS
            return;
#else
            skip |= 8;  // stamps build: the epilogue is done, only the stamps remain
#endif
        }
    }
    float acc[D][K];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int m = 0; m < C::J; ++m) {
            acc[d][2 * m] = acc2[d][m].x;
            acc[d][2 * m + 1] = acc2[d][m].y;
        }
#ifdef PU_STAMPS
    if (active && !(skip & 8)) write_outputs<float, float, K, D, PLANE, STATS>(acc, o, first, slot0, cnt, t0, tt, lane);
    PU_PHASE(6);
    if (lane == 0 && a.stamps) {
        for (int i = 0; i < 8; ++i) atomicAdd(reinterpret_cast<unsigned long long *>(a.stamps) + i,
                                              (unsigned long long)ph[i]);
    }
#undef PU_PHASE
#else
#undef PU_PHASE
    if (!active || (skip & 8)) return;
    write_outputs<float, float, K, D, PLANE, STATS>(acc, o, first, slot0, cnt, t0, tt, lane);
#endif
}

// One workgroup per work item.  (A persistent grid - one workgroup per CU looping over
// items b, b + grid, ... - measured slower at C2, 16.68 vs 16.19 ms: the hardware's
// dynamic dispatch of the next workgroup to whichever CU frees first beats a static
// round-robin; and its loop state cost the C3 instantiation scratch spills.)
template <class C, typename Tin, int G, bool PLANE, bool STATS, bool DMA8, bool S16 = false>
__global__ void __launch_bounds__(C::THREADS, 4)
dedisp_sub_kernel(SubArgs a, const i32x4 *__restrict__ tiles, const i32x2 *__restrict__ tile_stages,
                  const i32x4 *__restrict__ stages, const int32_t *__restrict__ slots,
                  const int32_t *__restrict__ base_tab, const uint32_t *__restrict__ rec_tab)
{
    sub_item<C, Tin, G, PLANE, STATS, DMA8, S16>(a, tiles, tile_stages, stages, slots, base_tab, rec_tab,
                                            pu::xcd_remap(blockIdx.x, gridDim.x), true);
}

// Certification state at the workspace tail (pu_plan_workspace_bytes), then the list
// of the trials to recompute (int32 each).
struct CertState {
    int32_t nflag;       // trials the fast path could not certify (listed after the state)
    int32_t nnonfinite;  // of which: a non-finite partial (NaN / inf in the series)
    int32_t scan;        // non-finite input scan (pu::nonfinite_any_async)
    int32_t why[3];      // flagged by: std not above its bound, S/N sign, S/N tie
    int32_t pad[58];
};
static_assert(sizeof(CertState) == 256, "CertState");

// Rounding model of one plan's fast statistics.
struct CertModel {
    int32_t tie_check;  // the series is exact (u8 with exact f32 sums, any f64 accumulation)
    double e_rel;       // per-sample series error bound / (|mean| + 4 std + |max|)
    double gamma;       // relative rounding of the epilogue's sums of (shifted) squares
};

// One workgroup per trial: combine the per-time-tile partials in a fixed order
// (thread-strided then an LDS tree: deterministic), then the reference's S/N logic
// (dedispersion.py:186-201): snr_w = max(reb_w)/std(reb_w), first strict best.
// Certification: a trial whose statistics or S/N decisions the fast path's summation
// order could change is appended to the list in ``cert`` (the host recomputes it
// exactly).  Bounds: the epilogue's sums of squares carry relative error gamma of
// Q = their magnitude (tile-local second moments + recentring terms), so
// |d var| <= 4 gamma Q; a per-sample series error E moves a width-w std by <= w E and
// max - w mean by <= 2 w E.  A trial is flagged when a partial is non-finite, when
// std is not > 4 x its bound (zero or rounding-level std: constant inputs), when
// max - w mean is within its bound of 0 (the S/N sign decision), and - for plans whose
// series is exact - when two S/N values of the strict first-best chain are within the
// sum of their bounds (ties).
template <typename PT>
__global__ void __launch_bounds__(256)
pu_finalize_kernel(const PT *__restrict__ part, int ntt, int n, int tt_len,
                   double *max_out, double *std_out, double *snr_out, int32_t *win_out,
                   CertModel cm, CertState *cert, int32_t *list, int first)
{
    __shared__ double red[4][4][256];
    const int trial = first + (int)blockIdx.x;  // trials [first, first + gridDim.x) of the plan
    const int tid = threadIdx.x;
    const PT *p = part + (size_t)trial * ntt * kPartStride;
    const double mu = p[0];
    double S1[4] = {0, 0, 0, 0}, S2[4] = {0, 0, 0, 0}, MX[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    double A2[4] = {0, 0, 0, 0};
    for (int i = tid; i < ntt; i += 256) {
        const PT *q = p + (size_t)i * kPartStride;
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
            // magnitude the rounding bound scales with: the tile's sum of squares (relative
            // error gamma), its recentring term through s1 (|d s1| <= gamma sum|y| <=
            // gamma sqrt(cnt s2)), and 2^-30 of the float64 recentring square
            A2[w] += fabs(s2) + 2.0 * fabs(wd) * sqrt(cntb * fabs(s2)) + 0x1p-30 * cntb * wd * wd;
            // NaN-propagating (a NaN partial max makes the trial non-finite below)
            MX[w] = (q[1 + 3 * w] > MX[w] || q[1 + 3 * w] != q[1 + 3 * w]) ? q[1 + 3 * w] : MX[w];
        }
    }
    for (int w = 0; w < 4; ++w) {
        red[0][w][tid] = S1[w];
        red[1][w][tid] = S2[w];
        red[2][w][tid] = MX[w];
        red[3][w][tid] = A2[w];
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) {
            for (int w = 0; w < 4; ++w) {
                red[0][w][tid] += red[0][w][tid + s];
                red[1][w][tid] += red[1][w][tid + s];
                const double a = red[2][w][tid], b = red[2][w][tid + s];
                red[2][w][tid] = (b > a || b != b) ? b : a;
                red[3][w][tid] += red[3][w][tid + s];
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        const double mean = mu + red[0][0][0] / n;  // mean of the dedispersed series
        double best = 0.0;
        int bestw = 0;
        double sdw[4] = {0, 0, 0, 0}, Qw[4] = {0, 0, 0, 0};
        bool nonfinite = !isfinite(mu) || !isfinite(mean);
        for (int w = 0; w < 4; ++w) {
            const int width = 1 << w;
            const long nb = n / width;
            if (nb <= 0) continue;
            const double m1 = red[0][w][0] / nb;
            const double var = red[1][w][0] / nb - m1 * m1;
            const double sd = sqrt(var > 0 ? var : 0.0);
            sdw[w] = sd;
            Qw[w] = red[3][w][0] / nb;
            nonfinite = nonfinite || !isfinite(red[0][w][0]) || !isfinite(red[1][w][0]) ||
                        !isfinite(red[2][w][0]) || !isfinite(red[3][w][0]);
            const double snr = (red[2][w][0] - width * mean) / sd;
            if (snr > best) {
                best = snr;
                bestw = width;
            }
        }
        bool uncertain = false;
        int why = -1;
        if (!nonfinite) {
            const double E = cm.e_rel * (fabs(mean) + 4.0 * sdw[0] + fabs(red[2][0][0]));
            double b = 0.0, eb = 0.0;  // the reference's (best_snr, its bound) chain
            for (int w = 0; w < 4 && !uncertain; ++w) {
                const int width = 1 << w;
                if (n / width <= 0) continue;
                const double sd = sdw[w], MXw = red[2][w][0];
                const double e_var = 4.0 * cm.gamma * Qw[w];
                const double e_sd = sd > 0 ? e_var / sd + width * E : INFINITY;
                const double num = MXw - width * mean;
                // max - w mean: the series error, the mean's rounding (through S1), the
                // float64 combination, and - unless the rebinned sums are exact (exact-series
                // plans: integers < 2^24 or float64) - their float32 rounding
                const double e_num = 2.0 * width * E + cm.gamma * width * sqrt(Qw[0]) +
                                     (cm.tie_check ? 0.0 : cm.gamma * fabs(MXw)) +
                                     0x1p-50 * (fabs(MXw) + width * fabs(mean));
                if (!(e_sd <= 0.25 * sd) || !(fabs(num) > e_num)) {
                    uncertain = true;
                    why = !(e_sd <= 0.25 * sd) ? 0 : 1;
                    break;
                }
                const double snr = num / sd;
                const double e_snr = (e_num + fabs(snr) * e_sd) / (sd - e_sd) + 0x1p-44 * fabs(snr);
                if (cm.tie_check) {
                    const double d = snr - b;
                    if (!(fabs(d) > e_snr + eb)) {
                        uncertain = true;
                        why = 2;
                    } else if (d > 0) {
                        b = snr;
                        eb = e_snr;
                    }
                }
            }
        }
        if (nonfinite || uncertain) {
            list[atomicAdd(&cert->nflag, 1)] = trial;
            if (nonfinite) atomicAdd(&cert->nnonfinite, 1);
            if (why >= 0) atomicAdd(&cert->why[why], 1);
        }
        max_out[trial] = red[2][0][0] - mean;
        std_out[trial] = sdw[0];
        snr_out[trial] = best;
        win_out[trial] = bestw;
    }
}


enum Variant { V_U8_F32, V_F32_F32, V_F64_F64, V_U8_F64, V_F32_F64, V_F64_F32, V_COUNT };

struct VariantInfo {
    int lds_elem, acc_f64, dma, fsm;  // fsm: dedisp_f64_kernel (prefetched windows, u32x8 records)
};

// K samples per lane = (8 / LDS element size) * 4 reads; D = 8 trials per wave
constexpr VariantInfo kVariants[V_COUNT] = {
    {4, 0, 0, 0},  // u8 in, f32 LDS (register staging), f32 acc (exact: sums < 2^24)
    {4, 0, 1, 0},  // f32 in, f32 LDS (DMA), f32 acc
    {8, 1, 1, 1},  // f64 in, f64 LDS (DMA), f64 acc (bit-exact vs reference)
    {4, 1, 0, 0},  // u8 in, f32 LDS, f64 acc
    {8, 1, 1, 1},  // f32 in, raw f32 DMA converted to f64 LDS rows, f64 acc (bit-exact vs reference)
    {4, 0, 0, 0},  // f64 in, f32 LDS (register staging), f32 acc
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

// Host-side subband tables of a candidate plan (uploaded only for the plan that is kept).
struct SubHost {
    std::vector<i32x4> tiles, stages;
    std::vector<i32x2> tile_stages;
    std::vector<int32_t> slots, base;
    std::vector<uint32_t> recs;
};

}  // namespace

// Per-plan lock: a plan holds mutable per-call state (timing events and the launch
// counter, the pinned certification copy and the last call's certification outcome),
// and cached plans are shared across threads (ctypes releases the GIL).  Every entry
// point that launches or reads that state holds it for the whole call.  Copying a plan
// (reset_tables) keeps the destination's mutex.
struct PlanLock {
    std::mutex m;
    PlanLock() = default;
    PlanLock(const PlanLock &) {}
    PlanLock &operator=(const PlanLock &) { return *this; }
};

struct pu_plan {
    mutable PlanLock lock;
    SubHost host;
    int dtype = 0, acc = 0, variant = 0;
    int64_t nchan = 0, n = 0, ndm = 0;
    int K = 0, TT = 0;
    int ndt = 0, ntt = 0, ncc = 0, row_stride = 0, small_n = 0, max_spread = 0;
    size_t lds_bytes = 0;
    int32_t *d_first = nullptr, *d_count = nullptr, *d_rowlen = nullptr, *d_base = nullptr;
    u32x4 *d_rec = nullptr;
    uint32_t *d_rec8 = nullptr;  // dedisp_f64_kernel's records (kF64Trials words per channel and wave)
    // subband mode (group > 1): per tile {first, count, raw row length, copy bytes},
    // stages {group begin, group end, item begin, item end}, build items, window records
    int group = 1, ngroups = 0, nslots_total = 0, raw_stride = 0, shape = SUB_WIDE;
    int dma8 = 0;  // subband plan stages 8-bit rows by LDS-DMA (rows must be 4-byte aligned)
    int slot16 = 0;  // subband plan with 16-bit integer slots (8-bit rows)
    int base_bits = 31;  // subband DMA row words: base bits (24: per-channel cover above them)
    size_t slot_bytes = 0, zero_len = 0;
    int64_t exec_adds = 0, lds_traffic = 0;  // per launch (measurement: bench.py roofline)
    int64_t cost_windows16 = 0;  // 16-bit-slot windows per launch (the cost model's extra term)
    std::vector<int32_t> tile_first, tile_count;  // DM tiles in launch order (pu_plan_dm_tiles)
    int64_t nstages = 0;
    int dt_major = 0;  // subband item order (SubArgs::dt_major)
    int opt_u8_dma = -1, opt_dt_major = -1, opt_slot16 = -1;  // pu_plan_opts (planner inputs)
    i32x4 *d_tiles = nullptr, *d_stages = nullptr;
    i32x2 *d_tile_stages = nullptr;
    int32_t *d_slots = nullptr;
    uint32_t *d_recs = nullptr;
    // optional kernel timing: events before the first and after the last launch of
    // each dispatch
    std::vector<hipEvent_t> ev_start, ev_stop;
    int64_t launches = 0;
    uint64_t *d_stamps = nullptr;  // diagnostic build (PU_STAMPS): phase-cycle totals
    // certification: the shift table (host) for exact recomputation of
    // flagged trials, a pinned copy of the device CertState, the last call's outcome
    std::vector<int64_t> shifts;
    CertState *h_cert = nullptr;
    int64_t cert_rechecked = 0, cert_nan = 0, cert_why[3] = {0, 0, 0}, cert_us = 0;
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

// dedisp_f64_kernel (dedisp_f64.hip, its own translation unit and code-generation options)
int launch_f64(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s, bool tin_f32)
{
    // records, then the first-window table (planner: one upload)
    const uint32_t *first_off = p->d_rec8 + (size_t)p->ndt * p->nchan * kTPT / 2;
    return pu_dd_launch_f64(tin_f32, plane, &a, sizeof a, p->lds_bytes, p->d_first, p->d_count, p->d_rowlen,
                            p->d_base, p->d_rec8, first_off, s, kF64Waves);
}

template <typename Tin, typename Tl, typename Ta>
int launch_variant(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    const dim3 grid((unsigned)((int64_t)a.ndt * a.ntt_run)), block(kThreads);
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
    case V_F64_F64: return launch_f64(p, a, plane, s, false);
    case V_U8_F64: return launch_variant<uint8_t, float, double>(p, a, plane, s);
    case V_F32_F64: return launch_f64(p, a, plane, s, true);
    case V_F64_F32: return launch_variant<double, float, float>(p, a, plane, s);
    }
    pu::set_error("bad plan variant");
    return PU_EINVAL;
}

template <class C, typename Tin, int G>
int launch_sub(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    SubArgs sa{};
    sa.o = a;
    sa.ngroups = p->ngroups;
    sa.raw_stride = p->raw_stride;
    sa.zero_len = (int32_t)p->zero_len;
    sa.lds_bytes = (int32_t)p->lds_bytes;
    sa.stamps = p->d_stamps;
    sa.dma_waves = std::min<int>(8, C::W);  // C2 17.6 vs 18.95 ms with all 16 waves, C3 141 vs 150 (625 trials)
#ifdef PU_STAMPS
    // diagnostic build only (make stamps): ablation and DMA-wave tuning knobs
    if (const char *env = getenv("PU_SUB_SKIP")) sa.skip = atoi(env);
    if (const char *env = getenv("PU_DMA_WAVES")) sa.dma_waves = std::clamp(atoi(env), 1, (int)C::W);
#endif

    const int64_t nitems = (int64_t)a.ndt * a.ntt_run;
    sa.nitems = (int32_t)nitems;
    sa.base_bits = p->base_bits;
    sa.dt_major = p->dt_major;
    const int64_t nblk = nitems;
    const dim3 grid((unsigned)nblk), block(C::THREADS);
    auto go = [&](auto kern) {
        int rc = ensure_lds(kern, p->lds_bytes);
        if (rc) return rc;
        hipLaunchKernelGGL(kern, grid, block, p->lds_bytes, s, sa, p->d_tiles, p->d_tile_stages, p->d_stages,
                           p->d_slots, p->d_base, p->d_recs);
        return pu::launch_check("dedisp_sub_kernel");
    };
    if constexpr (std::is_same<Tin, uint8_t>::value) {
        if constexpr (C::K == 4) {
            if (p->slot16)
                return plane ? go(dedisp_sub_kernel<C, Tin, G, true, false, true, true>)
                             : go(dedisp_sub_kernel<C, Tin, G, false, true, true, true>);
        }
        if (p->dma8)
            return plane ? go(dedisp_sub_kernel<C, Tin, G, true, false, true>)
                         : go(dedisp_sub_kernel<C, Tin, G, false, true, true>);
    }
    return plane ? go(dedisp_sub_kernel<C, Tin, G, true, false, false>)
                 : go(dedisp_sub_kernel<C, Tin, G, false, true, false>);
}

template <class C, typename Tin>
int launch_sub_g(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    switch (p->group) {
    case 2: return launch_sub<C, Tin, 2>(p, a, plane, s);
    case 4: return launch_sub<C, Tin, 4>(p, a, plane, s);
    case 8: return launch_sub<C, Tin, 8>(p, a, plane, s);
    }
    pu::set_error("bad plan group %d", p->group);
    return PU_EINVAL;
}

template <typename Tin>
int launch_sub_shape(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    return with_shape(p->shape, [&](auto c) { return launch_sub_g<decltype(c), Tin>(p, a, plane, s); });
}

int dispatch_sub(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    switch (p->dtype) {
    case PU_U8: return launch_sub_shape<uint8_t>(p, a, plane, s);
    case PU_F32: return launch_sub_shape<float>(p, a, plane, s);
    case PU_F64: return launch_sub_shape<double>(p, a, plane, s);
    }
    pu::set_error("bad plan dtype");
    return PU_EINVAL;
}

int dispatch(pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    const size_t nslot = p->ev_start.size();
    const size_t slot = nslot ? (size_t)(p->launches % (int64_t)nslot) : 0;
    if (nslot) PU_TRY_HIP(hipEventRecord(p->ev_start[slot], s));
    int rc = p->group > 1 ? dispatch_sub(p, a, plane, s) : dispatch_variant(p, a, plane, s);
    if (rc) return rc;
    if (nslot) PU_TRY_HIP(hipEventRecord(p->ev_stop[slot], s));
    ++p->launches;
    return PU_OK;
}

void destroy_events(pu_plan *p)
{
    for (auto *v : {&p->ev_start, &p->ev_stop}) {
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
    (void)hipFree(p->d_rec8);
    (void)hipFree(p->d_tiles);
    (void)hipFree(p->d_tile_stages);
    (void)hipFree(p->d_stages);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_recs);
    (void)hipFree(p->d_stamps);
    if (p->h_cert) (void)hipHostFree(p->h_cert);
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
    // Balance the tiles: the greedy pass leaves a short last tile (C1: 64 + 36 trials), and
    // a launch of few workgroups per CU runs as long as its busiest CU.  Same tile count,
    // trials dealt in whole waves (kD) as evenly as possible; kept only if every balanced
    // tile still meets the spread limit.
    if (first.size() > 1) {
        const int64_t nt = (int64_t)first.size();
        const int64_t blocks = (ndm + kD - 1) / kD;
        std::vector<int32_t> bf, bc;
        bool ok = true;
        int64_t t0 = 0;
        for (int64_t t = 0; t < nt && ok; ++t) {
            const int64_t nb = blocks / nt + (t < blocks % nt ? 1 : 0);
            const int64_t t1 = std::min<int64_t>(ndm, t0 + nb * kD);
            for (int64_t c = 0; c < nchan && ok; ++c) {
                int64_t m0 = INT64_MAX, m1 = INT64_MIN;
                for (int64_t d = t0; d < t1; ++d) {
                    m0 = std::min(m0, shifts[d * nchan + c]);
                    m1 = std::max(m1, shifts[d * nchan + c]);
                }
                ok = t1 > t0 && m1 - m0 <= kMaxSpread;
            }
            bf.push_back((int32_t)t0);
            bc.push_back((int32_t)(t1 - t0));
            t0 = t1;
        }
        if (ok && t0 == ndm) {
            first.swap(bf);
            count.swap(bc);
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
    const bool fsm = kVariants[p->variant].fsm != 0;
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
    // dedisp_f64_kernel: two float64 row buffers, plus one raw float32 row per channel for
    // float32 inputs (whole 256-byte DMA pieces)
    // (its stride: the row_stride's, as the kernel computes it), and two slots of window
    // records (one 256-byte DMA per channel, + 2 channels of read-ahead each)
    const int64_t raw_bytes = fsm && p->dtype == PU_F32 ? ((int64_t)p->row_stride * 4 + 255) / 256 * 256 : 0;
    constexpr int64_t kRecChan = 2 * kTPT;  // u16 words
    const int64_t per_chan = nbuf * chan_bytes + raw_bytes + (fsm ? 2 * kRecChan : 0);
    const int64_t fixed = fsm ? 2 * 2 * kRecChan : 0;
    p->ncc = (int)std::max<int64_t>(1, std::min<int64_t>(nchan, (int64_t)((budget - fixed) / per_chan)));
    p->lds_bytes = (size_t)p->ncc * per_chan + fixed;
    if (p->lds_bytes > 160 * 1024) {
        pu::set_error("pu_plan_create: LDS row of %d elements does not fit", p->row_stride);
        return PU_EUNSUPPORTED;
    }
    // window records: per (tile, channel, wave) 8 x u16 = LDS byte offset of each
    // trial's window inside the row slot | (differs from the previous trial) << 15
    // (dedisp_kernel); dedisp_f64_kernel: kF64Trials u16 per (tile, channel, wave), word
    // d = 0 if trial d reads the window of trial d - 1, else 1 + the offset in float64
    // elements, from the chunk's row base, of the window to PREFETCH when trial d's becomes
    // current (the next reloading trial's, after the channel's last reload the next
    // channel's first, 0 + 1 past the chunk: a harmless read of the row base); the reload
    // count of every channel pair the kernel walks (see below) is made even (trial 0 always
    // reloads; an odd count gets a non-reloading trial reloaded too, re-reading its
    // predecessor's window) so that each pair starts and ends in the kernel's state 0.
    // After the records: per (tile, channel, wave) the byte offset of the channel's first
    // window (read at chunk starts).
    const size_t copy_bytes = (size_t)p->row_stride * esz;
    std::vector<u32x4> rec(fsm ? 0 : (size_t)ndt * nchan * kWaves);
    std::vector<uint32_t> rec8(fsm ? (size_t)ndt * nchan * kTPT / 2 + (size_t)ndt * nchan * kF64Waves : 0);
    int64_t f64_reads = 0;  // window reads of dedisp_f64_kernel, per launch and time tile
    if (fsm) {
        if (p->ncc * chan_bytes / 8 + 1 >= (int64_t(1) << 16)) {
            pu::set_error("pu_plan_create: float64 window records overflow");
            return PU_EUNSUPPORTED;
        }
        constexpr int FD = kF64Trials;
        uint32_t *first8 = rec8.data() + (size_t)ndt * nchan * kTPT / 2;
        auto reloads = [&](size_t t, int64_t c, int w, bool (&re)[FD]) {
            const int32_t *rr = rel.data() + (t * nchan + c) * kTPT + w * FD;
            int nre = 0;
            for (int d = 0; d < FD; ++d) {
                re[d] = d == 0 || rr[d] != rr[d - 1];
                nre += re[d];
            }
            return nre;
        };
        auto add_reload = [](bool (&re)[FD]) {  // the last non-reloading trial re-reads
            for (int d = FD - 1; d > 0; --d)
                if (!re[d]) {
                    re[d] = true;
                    return true;
                }
            return false;
        };
        auto emit = [&](size_t t, int64_t c, int w, const bool (&re)[FD]) {
            const int32_t *rr = rel.data() + (t * nchan + c) * kTPT + w * FD;
            const uint32_t cb = (uint32_t)((c % p->ncc) * chan_bytes);
            first8[(t * nchan + c) * kF64Waves + w] = cb + 8u * (uint32_t)rr[0];
            const bool nxt_ok = c + 1 < nchan && (c + 1) % p->ncc != 0;
            const uint32_t nxt_off =
                nxt_ok ? (uint32_t)(cb + chan_bytes + 8u * (uint32_t)rel[((t * nchan + c + 1) * kTPT) + w * FD]) : 0u;
            uint32_t *r = rec8.data() + ((t * nchan + c) * kF64Waves + w) * (FD / 2);
            for (int d = 0; d < FD; ++d) {
                int e = d + 1;
                while (e < FD && !re[e]) ++e;
                const uint32_t off = e < FD ? cb + 8u * (uint32_t)rr[e] : nxt_off;
                const uint32_t word = re[d] ? off / 8u + 1u : 0u;
                r[d / 2] = d % 2 ? r[d / 2] | word << 16 : word;
                if (re[d] && w * FD < count[t]) f64_reads += 1;
            }
        };
        // the kernel walks each chunk's channels in pairs (a lone last one when the chunk's
        // count is odd): a pair's reload count - a lone channel's - is made even, so every
        // pair starts and ends in state 0 (the pair's second channel has an entry for each)
        for (size_t t = 0; t < (size_t)ndt; ++t)
            for (int64_t c0 = 0; c0 < nchan; c0 += p->ncc) {
                const int64_t nc = std::min<int64_t>(p->ncc, nchan - c0);
                for (int64_t ci = 0; ci < nc; ci += 2)
                    for (int w = 0; w < kF64Waves; ++w) {
                        bool ra[FD], rb[FD];
                        int tot = reloads(t, c0 + ci, w, ra);
                        const bool pair = ci + 1 < nc;
                        if (pair) tot += reloads(t, c0 + ci + 1, w, rb);
                        if (tot & 1) {
                            const bool ok = (pair && add_reload(rb)) || add_reload(ra);
                            if (!ok) {
                                pu::set_error("pu_plan_create: float64 reload parity");  // unreachable
                                return PU_EINVAL;
                            }
                        }
                        emit(t, c0 + ci, w, ra);
                        if (pair) emit(t, c0 + ci + 1, w, rb);
                    }
            }
    }
    for (size_t t = 0; t < (size_t)(fsm ? 0 : ndt); ++t)
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
    p->exec_adds = ndm * nchan * (int64_t)p->ntt * p->TT;
    // LDS bytes per launch (bench.py roofline): per time tile, the staged rows (E copies of
    // row_stride elements per channel) and, per active wave and channel, one J x 8-byte
    // x 64-lane window read for the first trial and for every trial whose window differs
    // from the previous trial's (the reload flag); J = p->K / E reads per window
    {
        const int J = p->K / E;
        int64_t lds_tile = 0;
        for (size_t t = 0; t < (size_t)ndt; ++t) {
            // staged rows (dedisp_f64_kernel on float32: + the raw row's DMA write and the
            // converting pass's read)
            lds_tile += nchan * (int64_t)E * p->row_stride * esz + (raw_bytes ? nchan * 2 * raw_bytes : 0);
            if (fsm) continue;  // the float64 kernel's reads: f64_reads (records, below)
            for (int w = 0; w < kWaves && w * kD < count[t]; ++w)
                for (int64_t c = 0; c < nchan; ++c) {
                    const int32_t *rr = rel.data() + (t * nchan + c) * kTPT + w * kD;
                    int reads = 1;
                    for (int d = 1; d < kD; ++d) reads += rr[d] != rr[d - 1] ? 1 : 0;
                    lds_tile += (int64_t)reads * J * 64 * 8;
                }
        }
        lds_tile += f64_reads * J * 64 * 8;
        p->lds_traffic = lds_tile * p->ntt;
    }
    p->tile_first = first;
    p->tile_count = count;
    int rc = PU_OK;
    if (!rc) rc = upload(&p->d_first, first);
    if (!rc) rc = upload(&p->d_count, count);
    if (!rc) rc = upload(&p->d_rowlen, rowlen);
    if (!rc) rc = upload(&p->d_base, base);
    if (!rc) rc = fsm ? upload(&p->d_rec8, rec8) : upload(&p->d_rec, rec);
    return rc;
}

// ---- subband mode planning (float32 accumulation).  Returns PU_EUNSUPPORTED when one
// trial's group does not fit the LDS budget (the caller then tries a smaller G, then
// channel mode).
constexpr int64_t kSubMaxSpread = 2048;
constexpr int64_t kS16Span = 254;  // 16-bit slots: TT + span + 2 <= 512 elements (four build chunks)
constexpr int64_t kDtMajorItems = 16 * 256;  // below this many items per launch: DM-tile-major order

struct SubSlot {
    int32_t vid;     // relative-shift vector id (per group)
    int64_t lo, hi;  // first-channel shift range of the tile's trials with this vector
    int64_t d0;      // one trial with this vector
};

int plan_sub(pu_plan *p, const int64_t *shifts, int G, int shape, size_t budget)
{
    const int64_t nchan = p->nchan, n = p->n, ndm = p->ndm;
    const int W = with_shape(shape, [](auto c) { return decltype(c)::W; });
    const int D = with_shape(shape, [](auto c) { return decltype(c)::D; });
    const int64_t TT = with_shape(shape, [](auto c) { return (int64_t)decltype(c)::TT; });
    const int64_t T = (int64_t)W * D;
    const int ngroups = (int)((nchan + G - 1) / G);
    // 8-bit rows are staged as bytes by LDS-DMA when every row window starts on a dword
    // (n % 4 == 0; the row's misalignment base % 4 is folded into the slot sources)
    bool dma8 = p->dtype == PU_U8 && n % 4 == 0;
    dma8 = dma8 && pu::knob("PU_U8_DMA", p->opt_u8_dma) != 0;
    const bool dma = p->dtype == PU_F32 || dma8;
    const int64_t eb = dma8 ? 1 : 4;  // bytes per staged raw element
    // 16-bit integer slots: 8-bit DMA rows in 256-sample time tiles; four
    // alignment copies of >= 384 u16 elements, slots of <= 512 elements (span <= kS16Span)
    // Every G: with the four-per-lane build G = 8 is faster with 16-bit slots too (C3 625
    // trials 113.5 vs 114.3 ms, 5000: 936 vs 957 - DESIGN.md §4.1b, profiles/r06/experiments/
    // slot16/); the per-window cost term below makes the planner pick G per grid
    const int s16opt = pu::knob("PU_SLOT16", p->opt_slot16);  // -1 auto (= on), 0 off, 1 on
    const bool s16 = dma8 && TT == 256 && s16opt != 0;
    const int64_t ncopies = s16 ? 4 : 2;
    const bool pack_cover = n < (int64_t(1) << 24);  // row bases fit 24 bits: covers above them
    // a stage's raw rows (DMA mode) and its slots share the LDS budget; a stage holds
    // whole groups.  The zero row (DMA mode, partial last group) sits at the end.
    const bool partial = dma && nchan % G != 0;
    const int64_t lds_cap = (int64_t)budget;
    auto S = [&](int64_t d, int64_t c) { return shifts[d * nchan + c]; };
    // elements per staged row: whole 256-byte DMA pieces for 8-bit rows (+3 misalignment)
    auto raw_stride_of = [&](int64_t spread) {
        return dma8 ? (TT + spread + 1 + 3 + 255) / 256 * 256 : (TT + spread + 1 + 63) / 64 * 64;
    };
    // slot copy: len = TT + span + 1 elements + 1 padding float (copy 1's element -1);
    // 16-bit slots: TT + span + 2 u16 (copies 2 and 3 are written 4 bytes down), 64-rounded
    auto copy_of = [&](int64_t span) { return (TT + span + 2 + 63) / 64 * 64 * (s16 ? 2 : 4); };
    auto zero_bytes = [&](int64_t stride) { return partial ? ((stride + 64) * eb + 255) / 256 * 256 : 0; };
    auto raw_bytes = [&](int64_t chans, int64_t stride) { return dma ? (chans * stride * eb + 255) / 256 * 256 : 0; };
    // one group's rows, `slots` slots and the zero row fit the budget
    auto group_fits = [&](int64_t spread, int64_t slots, int64_t span) {
        const int64_t rs = raw_stride_of(spread);
        return raw_bytes(G, rs) + slots * ncopies * copy_of(span) + zero_bytes(rs) <= lds_cap;
    };
    if (!group_fits(0, 1, 0)) return PU_EUNSUPPORTED;

    // ---- relative-shift vector id per (trial, group): v_k = s[c0 + k] - s[c0], k < gs
    std::vector<int32_t> vid((size_t)(ndm * ngroups));
    {
        std::vector<int64_t> order((size_t)ndm);
        for (int g = 0; g < ngroups; ++g) {
            const int64_t c0 = (int64_t)g * G;
            const int gs = (int)std::min<int64_t>(G, nchan - c0);
            auto cmp = [&](int64_t x, int64_t y) {
                for (int k = 1; k < gs; ++k) {
                    const int64_t u = S(x, c0 + k) - S(x, c0), v = S(y, c0 + k) - S(y, c0);
                    if (u != v) return u < v ? -1 : 1;
                }
                return 0;
            };
            for (int64_t d = 0; d < ndm; ++d) order[d] = d;
            std::sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
                const int c = cmp(x, y);
                return c != 0 ? c < 0 : x < y;
            });
            int32_t id = -1;
            for (int64_t i = 0; i < ndm; ++i) {
                if (i == 0 || cmp(order[i], order[i - 1]) != 0) ++id;
                vid[(size_t)order[i] * ngroups + g] = id;
            }
        }
    }

    // ---- DM tiles: <= T consecutive trials whose channel rows (one group's worth)
    // fit the raw area and whose slots of any one group fit the slot area
    std::vector<int32_t> first, count;
    std::vector<int64_t> spread_t, span_t, smin_t, smax_t;  // smin_t / smax_t: per tile x channel
    std::vector<std::vector<SubSlot>> tslots;       // per tile x group
    {
        std::vector<int64_t> mn((size_t)nchan), mx((size_t)nchan);
        std::vector<std::vector<SubSlot>> cur((size_t)ngroups), nxt((size_t)ngroups);
        int64_t i = 0;
        while (i < ndm) {
            for (int64_t c = 0; c < nchan; ++c) mn[c] = mx[c] = S(i, c);
            for (int g = 0; g < ngroups; ++g) {
                const int64_t b = S(i, (int64_t)g * G);
                cur[g].assign(1, SubSlot{vid[(size_t)i * ngroups + g], b, b, i});
            }
            int64_t spread = 0, span = 0;
            int64_t j = i + 1;
            while (j < ndm && j - i < T) {
                int64_t sp = spread;
                for (int64_t c = 0; c < nchan; ++c)
                    sp = std::max(sp, std::max(mx[c], S(j, c)) - std::min(mn[c], S(j, c)));
                if (sp > kSubMaxSpread) break;
                if (!group_fits(sp, 1, 0)) break;
                int64_t spn = span;
                size_t maxslots = 0;
                for (int g = 0; g < ngroups; ++g) {
                    nxt[g] = cur[g];
                    const int32_t v = vid[(size_t)j * ngroups + g];
                    const int64_t b = S(j, (int64_t)g * G);
                    bool found = false;
                    for (auto &sl : nxt[g])
                        if (sl.vid == v) {
                            sl.lo = std::min(sl.lo, b);
                            sl.hi = std::max(sl.hi, b);
                            spn = std::max(spn, sl.hi - sl.lo);
                            found = true;
                            break;
                        }
                    if (!found) nxt[g].push_back(SubSlot{v, b, b, j});
                    maxslots = std::max(maxslots, nxt[g].size());
                }
                if (!group_fits(sp, (int64_t)maxslots, spn)) break;
                if (s16 && spn > kS16Span) break;  // a 16-bit slot holds <= 512 elements
                for (int64_t c = 0; c < nchan; ++c) {
                    mn[c] = std::min(mn[c], S(j, c));
                    mx[c] = std::max(mx[c], S(j, c));
                }
                std::swap(cur, nxt);
                spread = sp;
                span = spn;
                ++j;
            }
            first.push_back((int32_t)i);
            count.push_back((int32_t)(j - i));
            spread_t.push_back(spread);
            span_t.push_back(span);
            smin_t.insert(smin_t.end(), mn.begin(), mn.end());
            smax_t.insert(smax_t.end(), mx.begin(), mx.end());
            for (int g = 0; g < ngroups; ++g) tslots.push_back(cur[g]);
            i = j;
        }
    }
    const int ndt = (int)first.size();
    int64_t raw_stride = 64, max_spread = 0;
    for (int t = 0; t < ndt; ++t) {
        raw_stride = std::max(raw_stride, raw_stride_of(spread_t[t]));
        max_spread = std::max(max_spread, spread_t[t]);
    }
    // the plan-wide row stride may exceed a tile's own: every tile's largest group must
    // still fit with it
    const int64_t zr = zero_bytes(raw_stride);
    const int64_t stage_cap = lds_cap - zr;  // raw rows + slots of one stage (and of the
                                             // next stage's rows + this stage's slots)
    for (int t = 0; t < ndt; ++t) {
        size_t maxslots = 0;
        for (int g = 0; g < ngroups; ++g) maxslots = std::max(maxslots, tslots[(size_t)t * ngroups + g].size());
        if (raw_bytes(G, raw_stride) + (int64_t)maxslots * ncopies * copy_of(span_t[t]) > stage_cap) {
            pu::set_error("subband mode: a group does not fit the LDS budget");
            return PU_EUNSUPPORTED;
        }
    }

    // ---- stages, slot records, window records (D per wave and group), DMA row bases.
    // LDS layout (the budget): [zero row | slots of the stage ... | raw rows of the stage],
    // the raw rows ending at the top.  Slot and window records hold absolute LDS byte
    // offsets.  A stage's rows land (DMA) while the previous stage is summed, so they
    // must also clear the previous stage's slots.  DMA mode: the G - gs missing channels
    // of a partial last group read the zero row, so the build never branches on the
    // group size.
    const int ms = slot_stride(G);
    const int64_t zero_row_f = 0;
    std::vector<i32x4> tiles((size_t)ndt), stages;
    std::vector<i32x2> tile_stages((size_t)ndt);
    std::vector<int32_t> slotmeta, base;
    std::vector<uint32_t> rec((size_t)ndt * ngroups * W * D);
    std::vector<int64_t> slot_base((size_t)ngroups);
    std::vector<std::vector<int64_t>> slot_off((size_t)ngroups);  // per group: each slot's byte offset
    // 16-bit slots' alignment copies are sized by their own span (round 6; the tile's widest
    // span sized every slot before): more groups per stage
    // 16-bit slots by their own span; float32 slots by theirs rounded up to whole build passes
    // of 64 U elements (sub_item's U), at most the tile's size (sub_item's copy_bytes_of)
    const int64_t UP64 = 64 * std::min<int64_t>((TT + 80 + 63) / 64, (p->dtype == PU_F64 ? 20 : 40) / G);
    auto slot_copy = [&](size_t t, const SubSlot &sl) {
        if (s16) return copy_of(sl.hi - sl.lo);
        const int64_t whole = (TT + (sl.hi - sl.lo) + 2 + UP64 - 1) / UP64 * UP64 * 4;
        return std::min(whole, copy_of(span_t[t]));
    };
    auto group_slot_bytes = [&](size_t t, int g) {
        int64_t b = 0;
        for (const auto &sl : tslots[t * ngroups + g]) b += ncopies * slot_copy(t, sl);
        return b;
    };
    int64_t prev_slots = 0;
    // element offset of a stage's first raw row: its rows end at the top of LDS
    auto raw_top_f = [&](int g0, int g1) {
        const int64_t nc = std::min<int64_t>((int64_t)g1 * G, nchan) - (int64_t)g0 * G;
        return (lds_cap - raw_bytes(nc, raw_stride)) / eb;
    };
    auto base_of = [&](int64_t smin_c) {
        int64_t b = smin_c % n;
        return b < 0 ? b + n : b;
    };
    int64_t slot_used = 0, max_stage_chans = 0;
    int64_t adds_tile = 0, lds_tile = 0;  // per time tile, summed over DM tiles
    int64_t win16_tile = 0;               // 16-bit-slot windows per time tile
    std::vector<double> tile_cost((size_t)ndt);  // per DM tile: LDS bytes + stage overhead (cost model)
    for (int t = 0; t < ndt; ++t) {
        const int64_t lds_before = lds_tile;
        const int64_t cb = copy_of(span_t[t]);
        const int64_t *smin = smin_t.data() + (size_t)t * nchan;
        const int64_t *smax = smax_t.data() + (size_t)t * nchan;
        const int64_t trials_run = (count[t] + D - 1) / D * D;  // active waves run all D trials
        adds_tile += trials_run * ngroups * TT;
        lds_tile += trials_run * ngroups * TT * (s16 ? 2 : 4);  // sum: one window read per trial and group
        if (s16) win16_tile += trials_run * ngroups;
        const int64_t row_len = TT + spread_t[t] + 1 + (dma8 ? 3 : 0);  // staged elements per row
        tiles[t] = i32x4{first[t], count[t], (int32_t)row_len, (int32_t)cb};
        if (dma)
            for (int64_t c = 0; c < nchan; ++c) {
                int64_t b = dma8 ? base_of(smin[c]) & ~int64_t(3) : base_of(smin[c]);
                if (pack_cover) {
                    // the channel's own DMA cover: its rows need TT + its spread + 1 (+3)
                    // elements, not the tile's widest (C2: 2304 vs 2560 B for most rows)
                    const int64_t len = TT + (smax[c] - smin[c]) + 1 + (dma8 ? 3 : 0);
                    const int64_t cu = (len * eb + 255) / 256;
                    if (cu < 128) b |= cu << 24;
                }
                base.push_back((int32_t)b);
            }
        tile_stages[t] = i32x2{(int32_t)stages.size(), 0};
        prev_slots = 0;
        int g = 0;
        while (g < ngroups) {
            const int32_t s_begin = (int32_t)(slotmeta.size() / ms);
            int64_t used = 0, chans = 0;
            int g_stop = g;  // pass 1: the stage's group range
            {
                int64_t u = 0, ch = 0;
                while (g_stop < ngroups) {
                    const int gs = (int)std::min<int64_t>(G, nchan - (int64_t)g_stop * G);
                    const int64_t nb = group_slot_bytes((size_t)t, g_stop);
                    const int64_t rb = raw_bytes(ch + gs, raw_stride);
                    if (g_stop > g && (rb + u + nb > stage_cap || rb + prev_slots > stage_cap)) break;
                    u += nb;
                    ch += gs;
                    ++g_stop;
                }
                if (raw_bytes(ch, raw_stride) + prev_slots > stage_cap) {
                    pu::set_error("subband mode: consecutive stages do not fit the LDS budget");
                    return PU_EUNSUPPORTED;
                }
                prev_slots = u;
            }
            int g_end = g;
            while (g_end < g_stop) {
                const int64_t c0 = (int64_t)g_end * G;
                const int gs = (int)std::min<int64_t>(G, nchan - c0);
                const auto &sls = tslots[(size_t)t * ngroups + g_end];
                slot_off[g_end].clear();
                for (const auto &sl : sls) {
                    const int64_t cbs = slot_copy((size_t)t, sl);
                    slot_off[g_end].push_back(used);
                    // 16-bit slots: len = the elements the windows read (the build's chunk count)
                    const int64_t len = TT + (sl.hi - sl.lo) + (s16 ? 0 : 1);
                    adds_tile += len * gs;
                    if (s16)  // chunks of 128: 2 G byte reads, 4 copies x 2 B
                        lds_tile += std::max<int64_t>(3, (len + 127) / 128) * 128 * (G + 8);
                    else
                        lds_tile += ((len + 63) / 64 * 64) * (dma ? eb * G + 8 : 8);  // build reads + 2 writes
                    slotmeta.push_back((int32_t)len);
                    slotmeta.push_back((int32_t)(zr + used));
                    slotmeta.push_back((int32_t)c0);
                    slotmeta.push_back(gs);
                    for (int k = 0; k < ms - 4; ++k) {
                        int64_t src = dma && k < G ? zero_row_f : 0;  // missing channel: zero row
                        if (k < gs) {
                            // smallest shift of channel c0+k over the slot's trials
                            const int64_t sk = sl.lo + S(sl.d0, c0 + k) - S(sl.d0, c0);
                            if (dma) {
                                src = raw_top_f(g, g_stop) + (chans + k) * raw_stride + (sk - smin[c0 + k]) +
                                      (dma8 ? (base_of(smin[c0 + k]) & 3) : 0);
                            } else {
                                src = sk % n;
                                if (src < 0) src += n;
                            }
                        }
                        slotmeta.push_back((int32_t)src);
                    }
                    used += ncopies * cbs;
                }
                chans += gs;
                ++g_end;
            }
            stages.push_back(i32x4{g, g_end, s_begin, (int32_t)(slotmeta.size() / ms)});
            tile_stages[t][1]++;
            if (dma) lds_tile += chans * ((row_len * eb + 255) / 256 * 256);  // DMA writes
            slot_used = std::max(slot_used, zr + used);
            for (int gg = g; gg < g_end; ++gg) slot_base[gg] = zr;
            max_stage_chans = std::max(max_stage_chans, chans);
            g = g_end;
        }
        for (int gg = 0; gg < ngroups; ++gg) {
            const auto &sls = tslots[(size_t)t * ngroups + gg];
            for (int w = 0; w < W; ++w) {
                uint32_t *r = rec.data() + (((size_t)t * ngroups + gg) * W + w) * D;
                for (int d = 0; d < D; ++d) {
                    const int64_t tr = first[t] + std::min<int64_t>(w * D + d, count[t] - 1);  // padding repeats the last trial
                    const int32_t v = vid[(size_t)tr * ngroups + gg];
                    size_t si = 0;
                    while (sls[si].vid != v) ++si;
                    const int64_t rr = S(tr, (int64_t)gg * G) - sls[si].lo;
                    const int64_t cbs = slot_copy((size_t)t, sls[si]);
                    // copy rr mod 2 (float32) / rr mod 4 (u16), the aligned element below rr
                    r[d] = (uint32_t)(slot_base[gg] + slot_off[gg][si] +
                                      (s16 ? (rr & 3) * cbs + (rr & ~int64_t(3)) * 2 : (rr & 1) * cbs + (rr & ~int64_t(1)) * 4));
                }
            }
        }
        tile_cost[t] = (double)(lds_tile - lds_before) + 3.0e6 * tile_stages[t][1];
    }
    // Item order: DM-tile major (longest items first) when the launch gives the CUs only
    // a few items each, where the tail of unequal items weighs; time-tile major otherwise
    // (the DM tiles of one time tile together on one XCD, sharing L2).  PU_DT_MAJOR
    // overrides (tuning).  DM-tile major sorts the DM tiles by decreasing cost; a tile's
    // trials are named by its record, so the order changes nothing else.  (Sorting them
    // for the time-tile-major order too cost C3 1.1 % - 1109 vs 1122 ms.)
    const int64_t ntt_plan = (n + TT - 1) / TT;
    bool dt_major = (int64_t)ndt * ntt_plan < kDtMajorItems;
    if (p->opt_dt_major >= 0) dt_major = p->opt_dt_major != 0;
    dt_major = pu::knob("PU_DT_MAJOR", dt_major ? 1 : 0) != 0;
    if (dt_major) {
        std::vector<int> perm((size_t)ndt);
        for (int t = 0; t < ndt; ++t) perm[t] = t;
        std::stable_sort(perm.begin(), perm.end(), [&](int x, int y) { return tile_cost[x] > tile_cost[y]; });
        std::vector<i32x4> tiles2((size_t)ndt);
        std::vector<i32x2> tile_stages2((size_t)ndt);
        std::vector<int32_t> base2(base.size());
        std::vector<uint32_t> rec2(rec.size());
        const size_t rec_block = (size_t)ngroups * W * D;
        for (int i = 0; i < ndt; ++i) {
            const int t = perm[i];
            tiles2[i] = tiles[t];
            tile_stages2[i] = tile_stages[t];
            if (!base.empty())
                std::copy_n(base.begin() + (size_t)t * nchan, nchan, base2.begin() + (size_t)i * nchan);
            std::copy_n(rec.begin() + (size_t)t * rec_block, rec_block, rec2.begin() + (size_t)i * rec_block);
        }
        tiles.swap(tiles2);
        tile_stages.swap(tile_stages2);
        base.swap(base2);
        rec.swap(rec2);
    }
    const int64_t lds_total = lds_cap;
    if (lds_total > 160 * 1024) {
        pu::set_error("subband mode: %lld bytes of LDS", (long long)lds_total);
        return PU_EUNSUPPORTED;
    }
    const int64_t ntt = (n + TT - 1) / TT;
    if ((int64_t)ndt * ntt >= (int64_t(1) << 31) || (int64_t)slotmeta.size() >= (int64_t(1) << 31)) {
        pu::set_error("pu_plan_create: grid too large");
        return PU_EINVAL;
    }
    p->group = G;
    p->ngroups = ngroups;
    p->ndt = ndt;
    p->shape = shape;
    p->K = (int)(TT / 64);
    p->TT = (int)TT;
    p->ntt = (int)ntt;
    p->ncc = (int)max_stage_chans;
    p->raw_stride = (int)raw_stride;
    p->row_stride = (int)raw_stride;
    p->max_spread = (int)max_spread;
    p->small_n = raw_stride + 2 > n ? 1 : 0;
    p->zero_len = zr ? (size_t)(((raw_stride + 64) * eb + 3) / 4) : 0;  // floats
    p->dma8 = dma8 ? 1 : 0;
    p->slot16 = s16 ? 1 : 0;
    p->base_bits = pack_cover ? 24 : 31;
    p->slot_bytes = (size_t)slot_used;
    p->lds_bytes = (size_t)lds_total;
    p->nslots_total = (int)(slotmeta.size() / ms);
    p->nstages = (int64_t)stages.size();
    p->dt_major = dt_major ? 1 : 0;
    p->exec_adds = adds_tile * ntt;
    p->lds_traffic = lds_tile * ntt;
    p->cost_windows16 = win16_tile * ntt;
    // host tables only: the caller uploads the plan it keeps (upload_sub), so comparing
    // candidate group sizes costs no device memory
    p->tile_first.resize((size_t)ndt);
    p->tile_count.resize((size_t)ndt);
    for (int t = 0; t < ndt; ++t) {
        p->tile_first[t] = tiles[t].x;
        p->tile_count[t] = tiles[t].y;
    }
    SubHost &h = p->host;
    h.tiles = std::move(tiles);
    h.tile_stages = std::move(tile_stages);
    h.stages = std::move(stages);
    h.slots = std::move(slotmeta);
    h.recs = std::move(rec);
    h.base = dma ? std::move(base) : std::vector<int32_t>();
    return PU_OK;
}

int upload_sub(pu_plan *p)
{
    SubHost &h = p->host;
    int rc = PU_OK;
    if (!rc) rc = upload(&p->d_tiles, h.tiles);
    if (!rc) rc = upload(&p->d_tile_stages, h.tile_stages);
    if (!rc) rc = upload(&p->d_stages, h.stages);
    // W (<= 16) records of padding: the kernel's build loads each wave's next slot record a
    // slot ahead without clamping the index
    h.slots.resize(h.slots.size() + (size_t)16 * slot_stride(8), 0);
    if (!rc) rc = upload(&p->d_slots, h.slots);
    if (!rc) rc = upload(&p->d_recs, h.recs);
    if (!rc && !h.base.empty()) rc = upload(&p->d_base, h.base);
    h = SubHost{};
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
    keep.opt_u8_dma = p->opt_u8_dma;
    keep.opt_slot16 = p->opt_slot16;
    keep.opt_dt_major = p->opt_dt_major;
    (void)hipFree(p->d_first);
    (void)hipFree(p->d_count);
    (void)hipFree(p->d_rowlen);
    (void)hipFree(p->d_base);
    (void)hipFree(p->d_rec);
    (void)hipFree(p->d_rec8);
    (void)hipFree(p->d_tiles);
    (void)hipFree(p->d_tile_stages);
    (void)hipFree(p->d_stages);
    (void)hipFree(p->d_slots);
    (void)hipFree(p->d_recs);
    *p = keep;
}

// The plan keeps its shift table (host) for the exact recomputation of flagged trials,
// and a pinned copy of the certification state.
int finish_plan(pu_plan *p, const int64_t *shifts)
{
    p->shifts.assign(shifts, shifts + p->ndm * p->nchan);
    return pu::hip_check(hipHostMalloc((void **)&p->h_cert, sizeof(CertState), hipHostMallocDefault),
                         "hipHostMalloc(cert)");
}

// partial records in the plan's accumulation type (the epilogues' sums are float32
// for float32 accumulation: a float record stores them exactly)
size_t part_elem(const pu_plan *p) { return kVariants[p->variant].acc_f64 ? sizeof(double) : sizeof(float); }
size_t part_bytes(const pu_plan *p) { return ((size_t)p->ndm * p->ntt * kPartStride * part_elem(p) + 255) & ~size_t(255); }

// Rounding model of the plan's fast statistics (pu_finalize_kernel).
CertModel cert_model(const pu_plan *p)
{
    CertModel m{};
    if (kVariants[p->variant].acc_f64) {
        m.tie_check = 1;  // float64 channel order: the reference's series bit for bit
        m.e_rel = 0x1p-50;
        m.gamma = 0x1p-44;
    } else if (p->dtype == PU_U8 && 8 * 255 * p->nchan < (int64_t(1) << 24)) {
        // integer sums (and their 8-sample rebins) below 2^24: exact in float32.  The
        // epilogue's sums of squares: <= 14 float32 roundings of nonnegative terms (the
        // shifted value, the square-and-add, 4 lane-local adds, the pair add, 2 permlane
        // and 4 row-reduction adds, the float record) = 14 x 2^-24 < 2^-20
        m.tie_check = 1;
        m.e_rel = 0.0;
        m.gamma = 0x1p-20;
    } else {
        // float32 sums of float data: the typical (random-walk) rounding of nchan terms
        // with an 8x margin, relative to the series' magnitude; S/N ties within the
        // float32 tolerance are not recomputed (the stated tolerance covers them)
        m.tie_check = 0;
        m.e_rel = 8.0 * 0x1p-24 * std::sqrt((double)p->nchan);
        m.gamma = 0x1p-19;
    }
    return m;
}

// cleared: the caller already zeroed the certification state earlier in the stream.
// Trials [first, first + count) (count < 0: every trial); outputs indexed by plan trial.
int launch_finalize(pu_plan *p, const void *part, double *mx, double *sd, double *snr, int32_t *win, char *ws,
                    hipStream_t s, bool cleared = false, int64_t first = 0, int64_t count = -1)
{
    CertState *cert = reinterpret_cast<CertState *>(ws + part_bytes(p));
    int32_t *list = reinterpret_cast<int32_t *>(cert + 1);
    if (!cleared) PU_TRY_HIP(hipMemsetAsync(cert, 0, sizeof(CertState), s));
    if (count < 0) count = p->ndm - first;
    if (count == 0) return PU_OK;
    if (part_elem(p) == sizeof(float))
        hipLaunchKernelGGL(pu_finalize_kernel<float>, dim3((unsigned)count), dim3(256), 0, s,
                           reinterpret_cast<const float *>(part), p->ntt, (int)p->n, p->TT, mx, sd, snr, win, cert_model(p),
                           cert, list, (int)first);
    else
        hipLaunchKernelGGL(pu_finalize_kernel<double>, dim3((unsigned)count), dim3(256), 0, s,
                           reinterpret_cast<const double *>(part), p->ntt, (int)p->n, p->TT, mx, sd, snr, win, cert_model(p),
                           cert, list, (int)first);
    return pu::launch_check("pu_finalize_kernel");
}

// After the finalize kernel: wait for it, then settle the flagged trials.  An input
// holding NaN / inf (found by a scan, run only when some trial saw a non-finite value)
// gives every trial the reference's NaN result; other flagged trials are recomputed
// exactly - their float64 channel-order series (the reference's bit for bit, by a direct
// gather: ~1 ms per trial at C3, far below a channel-mode sub-plan's cost for the
// few trials a search flags) + pu_series_stats - in batches that fit ~1 GiB of
// stream-ordered scratch allocated for the call.
int resolve_flagged(pu_plan *p, const void *data, int64_t ld, double *mx, double *sd, double *snr, int32_t *win,
                    char *ws, hipStream_t s, int64_t first = 0, int64_t count = -1)
{
    if (count < 0) count = p->ndm - first;
    CertState *cert = reinterpret_cast<CertState *>(ws + part_bytes(p));
    const int32_t *list = reinterpret_cast<const int32_t *>(cert + 1);
    p->cert_rechecked = 0;
    p->cert_nan = 0;
    PU_TRY_HIP(hipMemcpyAsync(p->h_cert, cert, sizeof(CertState), hipMemcpyDeviceToHost, s));
    PU_TRY_HIP(hipStreamSynchronize(s));
    const int64_t nflag = p->h_cert->nflag;
    for (int k = 0; k < 3; ++k) p->cert_why[k] = p->h_cert->why[k];
    p->cert_us = 0;
    if (nflag == 0) return PU_OK;
    const auto t_start = std::chrono::steady_clock::now();
    struct Timer {  // host time spent settling the flagged trials (pu_plan_info cert_us)
        pu_plan *p;
        std::chrono::steady_clock::time_point t0;
        ~Timer()
        {
            p->cert_us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0)
                             .count();
        }
    } timer{p, t_start};
    if (p->h_cert->nnonfinite > 0 && p->dtype != PU_U8) {
        int rc = pu::nonfinite_any_async(data, p->dtype, p->nchan, p->n, ld, &cert->scan, s);
        if (rc) return rc;
        PU_TRY_HIP(hipMemcpyAsync(p->h_cert, cert, sizeof(CertState), hipMemcpyDeviceToHost, s));
        PU_TRY_HIP(hipStreamSynchronize(s));
        if (p->h_cert->scan) {
            // every trial's series holds every input sample once (circular shift-and-sum),
            // so a NaN / inf anywhere reaches every trial: np.mean -> NaN or inf, the
            // shifted series -> NaN, max = std = NaN, no S/N beats 0 (dedispersion.py:186-201)
            p->cert_nan = 1;
            int rc2 = pu::nan_rule(count, mx + first, sd + first, snr + first, win + first, s);
            if (rc2) return rc2;
            PU_TRY_HIP(hipStreamSynchronize(s));
            return PU_OK;
        }
    }
    std::vector<int32_t> idx((size_t)nflag);
    PU_TRY_HIP(hipMemcpyAsync(idx.data(), list, (size_t)nflag * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    PU_TRY_HIP(hipStreamSynchronize(s));
    std::sort(idx.begin(), idx.end());
    const int64_t n = p->n, nchan = p->nchan;
    const int64_t per_row = n * 8 + (int64_t)pu_series_stats_workspace_bytes(1, n) + nchan * 8;
    const int64_t B = std::max<int64_t>(1, std::min<int64_t>(nflag, (int64_t(1) << 30) / per_row));
    const size_t plane_b = ((size_t)B * n * sizeof(double) + 255) & ~size_t(255);
    const size_t sws_b = (pu_series_stats_workspace_bytes(B, n) + 255) & ~size_t(255);
    const size_t sh_b = ((size_t)B * nchan * sizeof(int64_t) + 255) & ~size_t(255);
    const size_t need = plane_b + sws_b + sh_b + (size_t)B * sizeof(int32_t);
    // per-call scratch, stream-ordered (no device-wide synchronisation, nothing held
    // with the plan between calls); freed on every return path
    void *rc_buf = nullptr;
    PU_TRY_HIP(hipMallocAsync(&rc_buf, need, s));
    struct Scratch {
        void *b;
        hipStream_t s;
        ~Scratch()
        {
            (void)hipFreeAsync(b, s);
            (void)hipStreamSynchronize(s);
        }
    } scratch{rc_buf, s};
    char *sc = reinterpret_cast<char *>(rc_buf);
    double *plane = reinterpret_cast<double *>(sc);
    void *sws = sc + plane_b;
    int64_t *d_sh = reinterpret_cast<int64_t *>(sc + plane_b + sws_b);
    int32_t *d_idx = reinterpret_cast<int32_t *>(sc + plane_b + sws_b + sh_b);
    std::vector<int64_t> sh;
    int rc = PU_OK;
    for (int64_t i0 = 0; !rc && i0 < nflag; i0 += B) {
        const int64_t m = std::min(B, nflag - i0);
        sh.resize((size_t)(m * nchan));
        for (int64_t k = 0; k < m; ++k)
            std::copy_n(p->shifts.data() + (size_t)idx[(size_t)(i0 + k)] * nchan, nchan, sh.data() + k * nchan);
        for (auto &v : sh) v = ((v % n) + n) % n;  // row index (t + shift) mod n
        rc = pu::hip_check(hipMemcpyAsync(d_sh, sh.data(), sh.size() * sizeof(int64_t), hipMemcpyHostToDevice, s),
                           "hipMemcpyAsync(recheck shifts)");
        if (!rc) rc = pu::exact_series(data, p->dtype, nchan, n, ld, d_sh, m, plane, s);
        if (!rc)
            rc = pu::hip_check(hipMemcpyAsync(d_idx, idx.data() + i0, (size_t)m * sizeof(int32_t),
                                              hipMemcpyHostToDevice, s), "hipMemcpyAsync(recheck index)");
        if (!rc) rc = pu_series_stats(plane, m, n, n, d_idx, mx, sd, snr, win, sws, sws_b, s);
        const int rs = pu::hip_check(hipStreamSynchronize(s), "hipStreamSynchronize(recheck)");
        if (!rc) rc = rs;
    }
    if (!rc) p->cert_rechecked = nflag;
    return rc;
}

}  // namespace

extern "C" {

int pu_plan_create_ex(pu_plan **out, int dtype, int acc, int64_t nchan, int64_t n, const int64_t *shifts,
                      int64_t ndm, const pu_plan_opts *opts)
{
    PU_REQUIRE(out != nullptr, "pu_plan_create: out is NULL");
    PU_REQUIRE(opts != nullptr, "pu_plan_create_ex: opts is NULL");
    const int group = opts->group;
    PU_REQUIRE(opts->shape >= -1 && opts->shape <= 2, "pu_plan_create_ex: shape %d not in {-1, 0, 1, 2}", opts->shape);
    PU_REQUIRE(opts->lds_budget_kb == 0 || (opts->lds_budget_kb >= 8 && opts->lds_budget_kb <= 160),
               "pu_plan_create_ex: lds_budget_kb %d not 0 or in [8, 160]", opts->lds_budget_kb);
    PU_REQUIRE(opts->u8_dma >= -1 && opts->u8_dma <= 1 && opts->dt_major >= -1 && opts->dt_major <= 1 &&
                   opts->slot16 >= -1 && opts->slot16 <= 1,
               "pu_plan_create_ex: u8_dma / dt_major / slot16 must be -1, 0 or 1");
    *out = nullptr;
    const int v = pick_variant(dtype, acc);
    PU_REQUIRE(v >= 0, "pu_plan_create: unsupported dtype %d", dtype);
    PU_REQUIRE(acc >= PU_ACC_NATIVE && acc <= PU_ACC_F64, "pu_plan_create: bad acc %d", acc);
    PU_REQUIRE(nchan > 0 && nchan < (1 << 30), "pu_plan_create: nchan %lld out of range", (long long)nchan);
    PU_REQUIRE(n > 0 && n < (int64_t(1) << 31) - 65536, "pu_plan_create: nsamples %lld out of range",
               (long long)n);
    PU_REQUIRE(ndm > 0 && ndm < (1 << 30), "pu_plan_create: ndm %lld out of range", (long long)ndm);
    PU_REQUIRE(shifts != nullptr, "pu_plan_create: shifts is NULL");
    PU_REQUIRE(group == 0 || group == 1 || group == 2 || group == 4 || group == 8,
               "pu_plan_create: group %d not in {0 (auto), 1, 2, 4, 8}", group);
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
    p->K = E * (kVariants[v].acc_f64 && kVariants[v].lds_elem == 4 ? 2 : 4);  // dedisp_kernel's J
    p->TT = 64 * p->K;
    p->ntt = (int)((n + p->TT - 1) / p->TT);
    p->opt_u8_dma = opts->u8_dma < 0 ? 1 : opts->u8_dma;
    p->opt_dt_major = opts->dt_major;
    p->opt_slot16 = opts->slot16;

    // subband workgroup shape: 0 = wide (1 WG/CU), 1 = pair (2 WGs/CU), 2 = tall (256
    // trials x 256 samples, 1 WG/CU); -1 = the cost model's choice among wide and tall.
    // LDS budget per workgroup (channel / subband mode).  (Diagnostic build: PU_SUB_SHAPE,
    // PU_LDS_BUDGET_KB and PU_GROUP override the options, for A/B sweeps.)
    const int shape_opt = pu::knob("PU_SUB_SHAPE", opts->shape);
    const int budget_kb = pu::knob("PU_LDS_BUDGET_KB", opts->lds_budget_kb);
    int shape = shape_opt < 0 ? SUB_WIDE : std::clamp(shape_opt, 0, 2);
    // dedisp_f64_kernel: 80 KiB (two workgroups per CU); dedisp_kernel: 64 KiB
    size_t budget = kVariants[v].fsm ? 80 * 1024 : kLdsBudget, sub_budget = shape == SUB_PAIR ? 80 * 1024 : 160 * 1024;
    if (budget_kb > 0) budget = sub_budget = (size_t)std::max(8, budget_kb) * 1024;
    // group size: explicit, else the automatic choice (G = 4 where it is not calibrated);
    // float32 accumulation only (the float64 modes keep the reference's sequential
    // channel order)
    int G = pu::knob("PU_GROUP", group);
    bool auto_g = false;
    if (G == 0) {
        G = 4;
        auto_g = !kVariants[v].acc_f64 && nchan > 8;
    }
    G = std::min(G, 8);
    if (kVariants[v].acc_f64) G = 1;
    while (G > 1 && G >= nchan) G >>= 1;
    // The automatic choice is calibrated on the wide shape with DMA-staged rows (f32, or
    // u8 with n % 4 == 0); elsewhere the default stays G = 4.
    const bool dma_rows = dtype == PU_F32 || (dtype == PU_U8 && n % 4 == 0);
    if (auto_g && (shape != SUB_WIDE || !dma_rows || budget_kb > 0)) auto_g = false;
    int rc = PU_EUNSUPPORTED;
    if (auto_g) {
        // Default group size: plan G = 8 and G = 4 on the host and keep the cheaper by the
        // measured cost model: LDS bytes + 3.0e6 B-equivalent per (stage,
        // time tile).  G = 8 halves the LDS traffic at C3 (1240 vs 1328 ms) but its extra
        // stages cost more than that at C2 (22.7 vs 18.4 ms) and C5.  Only the winner's
        // tables are uploaded.  A candidate that does not fit (PU_EUNSUPPORTED) is not
        // viable; any other error is returned as is.
        // Round 6: a 16-bit-slot window costs more than its 512 LDS bytes say (its sum is not
        // LDS-bound: the u16 G = 4 plan lost 6 % to float32 G = 8 at C3's 625-trial shard
        // and won 10 % at its 5000 trials, which the byte model alone ranks the same way at
        // both): + 200 B-equivalent per window, the middle of the (88, 389) the two
        // measurements allow.
        auto cost = [](const pu_plan *q) {
            return (double)q->lds_traffic + 3.0e6 * (double)q->nstages * q->ntt + 200.0 * (double)q->cost_windows16;
        };
        // Round 6, per-slot copy sizes for 16-bit slots: fewer stages for both G, G = 8 most
        // (C3 5000 trials tall G = 4 855.9 -> 847.2 ms, G = 8 936.7 -> 885.3; the 625-trial
        // shard G = 8 114.1 -> 111.9), and the cost above then ranks tall G = 8 first at 5000
        // trials too - wrongly.  Between the two tall 16-bit-slot plans a stage costs 6e6
        // B-equivalents, inside the (4.5e6, 1.0e7) that ranks both measurements right; the
        // winner meets the other shapes under the cost above (6e6 for every plan would pick
        // the wide float32 plan at C3: 1066 vs 847 ms).
        auto cost_tall16 = [](const pu_plan *q) {
            return (double)q->lds_traffic + 6.0e6 * (double)q->nstages * q->ntt + 200.0 * (double)q->cost_windows16;
        };
        auto fresh = [&]() {
            pu_plan *q = new pu_plan();
            q->dtype = p->dtype;
            q->acc = p->acc;
            q->variant = p->variant;
            q->nchan = p->nchan;
            q->n = p->n;
            q->ndm = p->ndm;
            q->K = p->K;
            q->TT = p->TT;
            q->ntt = p->ntt;
            q->opt_u8_dma = p->opt_u8_dma;
            q->opt_slot16 = p->opt_slot16;
            q->opt_dt_major = p->opt_dt_major;
            return q;
        };
        // Round 3: the tall shape (256 trials x 256 samples) competes too, with G = 4 and 8.
        // With the permlane epilogue the same cost model ranks every measured case right:
        // C2 tall G4 14.92 ms (wide G4 15.23, tall G8 20.19), C3 tall G8 1042 ms (wide G8
        // 1114; 625 trials 125.6 vs 132.4, tall G4 135.8), C5 tall G4 0.365 (wide 0.374),
        // C4 wide G4 0.581 (100 trials: tall 0.662).  PU_SUB_SHAPE pins the shape.
        const bool try_tall = shape_opt < 0;
        pu_plan *q = fresh(), *t4 = try_tall ? fresh() : nullptr, *t8 = try_tall ? fresh() : nullptr;
        const int rc8 = plan_sub(q, shifts, 8, shape, sub_budget);
        const int rc4 = plan_sub(p, shifts, 4, shape, sub_budget);
        const int rct4 = t4 ? plan_sub(t4, shifts, 4, SUB_TALL, 160 * 1024) : PU_EUNSUPPORTED;
        const int rct8 = t8 ? plan_sub(t8, shifts, 8, SUB_TALL, 160 * 1024) : PU_EUNSUPPORTED;
        for (int r : {rc8, rc4, rct4, rct8}) {
            if (r != PU_OK && r != PU_EUNSUPPORTED) {
                for (pu_plan *c : {p, q, t4, t8}) free_plan(c);
                return r;
            }
        }
        pu_plan *keep = nullptr, *tall = nullptr;
        if (rct4 == PU_OK && rct8 == PU_OK && t4->slot16 && t8->slot16)
            tall = cost_tall16(t8) < cost_tall16(t4) ? t8 : t4;
        for (auto [cand, ok] : {std::pair<pu_plan *, bool>{p, rc4 == PU_OK}, {q, rc8 == PU_OK},
                                {t4, rct4 == PU_OK && (!tall || tall == t4)}, {t8, rct8 == PU_OK && (!tall || tall == t8)}})
            if (ok && (!keep || cost(cand) < cost(keep))) keep = cand;
        for (pu_plan *cand : {p, q, t4, t8})  // losers (p stays when nothing fits: it is reused below)
            if (cand != keep && (keep || cand != p)) free_plan(cand);
        if (keep) {
            rc = upload_sub(keep);
            if (!rc) rc = finish_plan(keep, shifts);
            if (rc) {
                free_plan(keep);
                return rc;
            }
            *out = keep;
            return PU_OK;
        }
        reset_tables(p);
        G = 2;  // 8 and 4 do not fit: continue with the smaller groups
    }
    for (; G > 1 && rc == PU_EUNSUPPORTED; G >>= 1) {
        rc = plan_sub(p, shifts, G, shape, sub_budget);
        if (rc == PU_OK) rc = upload_sub(p);
        if (rc == PU_EUNSUPPORTED) reset_tables(p);
    }
    if (rc == PU_EUNSUPPORTED) rc = plan_channels(p, shifts, budget);
    if (!rc) rc = finish_plan(p, shifts);
    if (rc) {
        free_plan(p);
        return rc;
    }
    *out = p;
    return PU_OK;
}

int pu_plan_create_grouped(pu_plan **out, int dtype, int acc, int64_t nchan, int64_t n, const int64_t *shifts,
                           int64_t ndm, int group)
{
    pu_plan_opts o{};
    o.group = group;
    o.shape = -1;
    o.u8_dma = -1;
    o.dt_major = -1;
    return pu_plan_create_ex(out, dtype, acc, nchan, n, shifts, ndm, &o);
}

int pu_plan_create(pu_plan **out, int dtype, int acc, int64_t nchan, int64_t n, const int64_t *shifts, int64_t ndm)
{
    return pu_plan_create_grouped(out, dtype, acc, nchan, n, shifts, ndm, 0);
}

void pu_plan_destroy(pu_plan *p) { free_plan(p); }

int pu_plan_enable_timing(pu_plan *p, int nslots)
{
    PU_REQUIRE(p != nullptr && nslots >= 0 && nslots <= 65536, "pu_plan_enable_timing: bad arguments");
    std::lock_guard<std::mutex> guard(p->lock.m);
    destroy_events(p);
    for (auto *v : {&p->ev_start, &p->ev_stop}) {
        v->assign((size_t)nslots, nullptr);
        for (int i = 0; i < nslots; ++i) PU_TRY_HIP(hipEventCreate(&(*v)[i]));
    }
    p->launches = 0;
    return PU_OK;
}

int pu_plan_stamps(pu_plan *p, int64_t *out, int n)
{
    PU_REQUIRE(p != nullptr && out != nullptr, "pu_plan_stamps: bad arguments");
    std::lock_guard<std::mutex> guard(p->lock.m);
#ifdef PU_STAMPS
    if (!p->d_stamps) {
        PU_TRY_HIP(hipMalloc((void **)&p->d_stamps, 8 * sizeof(uint64_t)));
        PU_TRY_HIP(hipMemset(p->d_stamps, 0, 8 * sizeof(uint64_t)));
        return 0;  // armed: the next launches accumulate
    }
    uint64_t h[8];
    PU_TRY_HIP(hipDeviceSynchronize());
    PU_TRY_HIP(hipMemcpy(h, p->d_stamps, sizeof h, hipMemcpyDeviceToHost));
    PU_TRY_HIP(hipMemset(p->d_stamps, 0, 8 * sizeof(uint64_t)));
    const int m = std::min(n, 8);
    for (int i = 0; i < m; ++i) out[i] = (int64_t)h[i];
    return m;
#else
    (void)n;
    return 0;
#endif
}

int pu_plan_kernel_times(pu_plan *p, float *ms, int n)
{
    PU_REQUIRE(p != nullptr && ms != nullptr, "pu_plan_kernel_times: bad arguments");
    std::lock_guard<std::mutex> guard(p->lock.m);
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
    // per-(trial, time tile) partial records | CertState | flagged-trial list
    return part_bytes(p) + sizeof(CertState) + (size_t)p->ndm * sizeof(int32_t);
}

// which kernel a plan's searches launch: 0 dedisp_kernel (channel order), 1 dedisp_f64_kernel,
// 2 dedisp_sub_kernel (float32 slots), 3 dedisp_sub_kernel with 16-bit integer slots
static int64_t plan_kernel(const pu_plan *p)
{
    if (p->group > 1) return p->slot16 ? 3 : 2;
    return kVariants[p->variant].fsm ? 1 : 0;
}

int pu_plan_info(const pu_plan *p, int64_t *info, int n)
{
    if (!p || !info) return 0;
    std::lock_guard<std::mutex> guard(p->lock.m);
    const int64_t v[] = {p->ndm, p->ndt, p->ntt, p->group > 1 ? with_shape(p->shape, [](auto c) { return decltype(c)::T; }) : kTPT, p->TT, p->ncc,
                         p->row_stride, (int64_t)p->lds_bytes, kVariants[p->variant].acc_f64, p->max_spread,
                         p->group, p->nslots_total, p->nstages, (int64_t)p->slot_bytes, p->raw_stride,
                         p->exec_adds, p->lds_traffic, p->cert_rechecked, p->cert_nan, p->cert_why[0],
                         p->cert_why[1], p->cert_why[2], p->cert_us, plan_kernel(p), (int64_t)part_elem(p),
                         kPartStride};
    const int m = std::min<int>(n, (int)(sizeof v / sizeof v[0]));
    for (int k = 0; k < m; ++k) info[k] = v[k];
    return m;
}

static int check_data(const pu_plan *p, const void *data, int64_t ld)
{
    PU_REQUIRE(p != nullptr, "plan is NULL");
    PU_REQUIRE(data != nullptr, "data is NULL");
    PU_REQUIRE(ld >= p->n, "ld %lld < nsamples %lld", (long long)ld, (long long)p->n);
    PU_REQUIRE(!p->dma8 || (reinterpret_cast<uintptr_t>(data) % 4 == 0 && ld % 4 == 0),
               "8-bit subband plan: rows must start on 4-byte boundaries (data %% 4 == 0, ld %% 4 == 0)");
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
    a.tt0 = 0;
    a.ntt_run = p->ntt;
    a.ncc = p->ncc;
    a.row_stride = p->row_stride;
    a.small_n = p->small_n;
    return a;
}

int pu_plan_search_tiles(pu_plan *p, const void *data, int64_t ld, int64_t tt_begin, int64_t tt_end,
                         void *workspace, size_t ws_bytes, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(0 <= tt_begin && tt_begin <= tt_end && tt_end <= p->ntt,
               "pu_plan_search_tiles: tile range [%lld, %lld) outside [0, %d)", (long long)tt_begin,
               (long long)tt_end, p->ntt);
    PU_REQUIRE(workspace && ws_bytes >= pu_plan_workspace_bytes(p), "pu_plan_search_tiles: workspace too small");
    if (tt_begin == tt_end) return PU_OK;
    DedispArgs a = make_args(p, data, ld);
    a.partials = workspace;
    a.tt0 = (int32_t)tt_begin;
    a.ntt_run = (int32_t)(tt_end - tt_begin);
    return dispatch(p, a, false, pu::as_stream(stream));
}

int pu_plan_finalize(pu_plan *p, const void *data, int64_t ld, double *max_out, double *std_out, double *snr_out,
                     int32_t *rebin_out, void *workspace, size_t ws_bytes, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(max_out && std_out && snr_out && rebin_out, "pu_plan_finalize: NULL output");
    PU_REQUIRE(workspace && ws_bytes >= pu_plan_workspace_bytes(p) && reinterpret_cast<uintptr_t>(workspace) % 8 == 0,
               "pu_plan_finalize: workspace too small or not 8-byte aligned");
    hipStream_t s = pu::as_stream(stream);
    char *ws = reinterpret_cast<char *>(workspace);
    rc = launch_finalize(p, ws, max_out, std_out, snr_out, rebin_out, ws, s);
    if (rc) return rc;
    return resolve_flagged(p, data, ld, max_out, std_out, snr_out, rebin_out, ws, s);
}

int pu_plan_finalize_range(pu_plan *p, const void *data, int64_t ld, int64_t trial_begin, int64_t trial_end,
                           double *max_out, double *std_out, double *snr_out, int32_t *rebin_out, void *workspace,
                           size_t ws_bytes, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(0 <= trial_begin && trial_begin <= trial_end && trial_end <= p->ndm,
               "pu_plan_finalize_range: trial range [%lld, %lld) outside [0, %lld)", (long long)trial_begin,
               (long long)trial_end, (long long)p->ndm);
    PU_REQUIRE(max_out && std_out && snr_out && rebin_out, "pu_plan_finalize_range: NULL output");
    PU_REQUIRE(workspace && ws_bytes >= pu_plan_workspace_bytes(p) && reinterpret_cast<uintptr_t>(workspace) % 8 == 0,
               "pu_plan_finalize_range: workspace too small or not 8-byte aligned");
    hipStream_t s = pu::as_stream(stream);
    char *ws = reinterpret_cast<char *>(workspace);
    rc = launch_finalize(p, ws, max_out, std_out, snr_out, rebin_out, ws, s, false, trial_begin,
                         trial_end - trial_begin);
    if (rc) return rc;
    return resolve_flagged(p, data, ld, max_out, std_out, snr_out, rebin_out, ws, s, trial_begin,
                           trial_end - trial_begin);
}

int pu_plan_finalize_range_flagged(pu_plan *p, int64_t trial_begin, int64_t trial_end, double *max_out,
                                   double *std_out, double *snr_out, int32_t *rebin_out, void *workspace,
                                   size_t ws_bytes, int32_t *flagged, int64_t cap, int64_t *counts, void *stream)
{
    PU_REQUIRE(p != nullptr, "plan is NULL");
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(0 <= trial_begin && trial_begin <= trial_end && trial_end <= p->ndm,
               "pu_plan_finalize_range_flagged: trial range [%lld, %lld) outside [0, %lld)", (long long)trial_begin,
               (long long)trial_end, (long long)p->ndm);
    PU_REQUIRE(max_out && std_out && snr_out && rebin_out && counts && (flagged || cap == 0),
               "pu_plan_finalize_range_flagged: NULL output");
    PU_REQUIRE(workspace && ws_bytes >= pu_plan_workspace_bytes(p) && reinterpret_cast<uintptr_t>(workspace) % 8 == 0,
               "pu_plan_finalize_range_flagged: workspace too small or not 8-byte aligned");
    hipStream_t s = pu::as_stream(stream);
    char *ws = reinterpret_cast<char *>(workspace);
    int rc = launch_finalize(p, ws, max_out, std_out, snr_out, rebin_out, ws, s, false, trial_begin,
                             trial_end - trial_begin);
    if (rc) return rc;
    CertState *cert = reinterpret_cast<CertState *>(ws + part_bytes(p));
    const int32_t *list = reinterpret_cast<const int32_t *>(cert + 1);
    PU_TRY_HIP(hipMemcpyAsync(p->h_cert, cert, sizeof(CertState), hipMemcpyDeviceToHost, s));
    PU_TRY_HIP(hipStreamSynchronize(s));
    const int64_t nflag = p->h_cert->nflag;
    counts[0] = nflag;
    counts[1] = p->h_cert->nnonfinite;
    for (int k = 0; k < 3; ++k) p->cert_why[k] = p->h_cert->why[k];
    p->cert_rechecked = 0;
    p->cert_nan = 0;
    p->cert_us = 0;
    const int64_t m = std::min(nflag, cap);
    if (m > 0) {
        PU_TRY_HIP(hipMemcpyAsync(flagged, list, (size_t)m * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        PU_TRY_HIP(hipStreamSynchronize(s));
        std::sort(flagged, flagged + m);
    }
    return PU_OK;
}

int pu_plan_exact_series(pu_plan *p, const void *data, int64_t ld, const int32_t *trials, int64_t m, int64_t t_begin,
                         int64_t t_end, double *out, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(0 <= t_begin && t_begin <= t_end && t_end <= p->n, "pu_plan_exact_series: samples [%lld, %lld) outside [0, %lld)",
               (long long)t_begin, (long long)t_end, (long long)p->n);
    PU_REQUIRE(m >= 0, "pu_plan_exact_series: m < 0");
    if (m == 0 || t_end == t_begin) return PU_OK;
    PU_REQUIRE(trials && out, "pu_plan_exact_series: NULL trials / out");
    const int64_t n = p->n, nchan = p->nchan;
    std::vector<int64_t> sh((size_t)(m * nchan));
    for (int64_t k = 0; k < m; ++k) {
        PU_REQUIRE(0 <= trials[k] && trials[k] < p->ndm, "pu_plan_exact_series: trial %d outside [0, %lld)",
                   trials[k], (long long)p->ndm);
        std::copy_n(p->shifts.data() + (size_t)trials[k] * nchan, nchan, sh.data() + k * nchan);
    }
    for (auto &v : sh) v = ((v % n) + n) % n;
    hipStream_t s = pu::as_stream(stream);
    void *d_sh = nullptr;
    PU_TRY_HIP(hipMallocAsync(&d_sh, sh.size() * sizeof(int64_t), s));
    rc = pu::hip_check(hipMemcpyAsync(d_sh, sh.data(), sh.size() * sizeof(int64_t), hipMemcpyHostToDevice, s),
                       "hipMemcpyAsync(exact series shifts)");
    if (!rc)
        rc = pu::exact_series(data, p->dtype, nchan, n, ld, reinterpret_cast<const int64_t *>(d_sh), m, out, s, t_begin,
                              t_end - t_begin);
    (void)hipFreeAsync(d_sh, s);
    const int rs = pu::hip_check(hipStreamSynchronize(s), "hipStreamSynchronize(exact series)");
    return rc ? rc : rs;
}

int pu_nonfinite_any(const void *data, int dtype, int64_t nrows, int64_t ncols, int64_t ld, int32_t *flag, void *stream)
{
    PU_REQUIRE(data && flag, "pu_nonfinite_any: NULL pointer");
    PU_REQUIRE(nrows >= 0 && ncols >= 0 && ld >= ncols, "pu_nonfinite_any: bad shape");
    hipStream_t s = pu::as_stream(stream);
    if (nrows == 0 || ncols == 0) {
        PU_TRY_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t), s));
        return PU_OK;
    }
    return pu::nonfinite_any_async(data, dtype, nrows, ncols, ld, flag, s);
}

int pu_plan_search(pu_plan *p, const void *data, int64_t ld, double *max_out, double *std_out,
                   double *snr_out, int32_t *rebin_out, void *workspace, size_t ws_bytes, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(max_out && std_out && snr_out && rebin_out, "pu_plan_search: NULL output");
    PU_REQUIRE(workspace && ws_bytes >= pu_plan_workspace_bytes(p) && reinterpret_cast<uintptr_t>(workspace) % 8 == 0,
               "pu_plan_search: workspace too small or not 8-byte aligned");
    DedispArgs a = make_args(p, data, ld);
    a.partials = workspace;
    hipStream_t s = pu::as_stream(stream);
    char *ws = reinterpret_cast<char *>(workspace);
    // the certification state is cleared BEFORE the search kernel: the fill then runs while
    // the stream is idle after the previous call's host read, instead of between the search
    // and finalize kernels (C5: ~10 us of fill + dispatch gap on the step)
    PU_TRY_HIP(hipMemsetAsync(ws + part_bytes(p), 0, sizeof(CertState), s));
    rc = dispatch(p, a, false, s);
    if (rc) return rc;
    rc = launch_finalize(p, a.partials, max_out, std_out, snr_out, rebin_out, ws, s, true);
    if (rc) return rc;
    return resolve_flagged(p, data, ld, max_out, std_out, snr_out, rebin_out, ws, s);
}

int pu_plan_dedisperse(pu_plan *p, const void *data, int64_t ld, void *plane, int64_t ld_plane, void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(plane != nullptr, "pu_plan_dedisperse: plane is NULL");
    PU_REQUIRE(ld_plane >= p->n, "pu_plan_dedisperse: ld_plane < nsamples");
    DedispArgs a = make_args(p, data, ld);
    a.plane = plane;
    a.ld_plane = ld_plane;
    return dispatch(p, a, true, pu::as_stream(stream));
}

int pu_plan_dm_tiles(const pu_plan *p, int32_t *first, int32_t *count, int n)
{
    if (!p) return 0;
    std::lock_guard<std::mutex> guard(p->lock.m);
    const int ndt = (int)p->tile_first.size();
    for (int t = 0; t < std::min(n, ndt); ++t) {
        if (first) first[t] = p->tile_first[t];
        if (count) count[t] = p->tile_count[t];
    }
    return ndt;
}

int pu_plan_dedisperse_dm_tile(pu_plan *p, const void *data, int64_t ld, int64_t dt, void *plane, int64_t ld_plane,
                               void *stream)
{
    int rc = check_data(p, data, ld);
    if (rc) return rc;
    std::lock_guard<std::mutex> guard(p->lock.m);
    PU_REQUIRE(plane != nullptr, "pu_plan_dedisperse_dm_tile: plane is NULL");
    PU_REQUIRE(ld_plane >= p->n, "pu_plan_dedisperse_dm_tile: ld_plane < nsamples");
    PU_REQUIRE(0 <= dt && dt < (int64_t)p->tile_first.size(), "pu_plan_dedisperse_dm_tile: DM tile %lld outside [0, %d)",
               (long long)dt, (int)p->tile_first.size());
    DedispArgs a = make_args(p, data, ld);
    a.dt0 = (int32_t)dt;
    a.ndt = 1;
    // the kernels write trial row (first + i) at plane + (first + i) ld_plane: shift the base
    // so that the tile's rows land at rows 0 .. count - 1 of the caller's plane
    const size_t elem = kVariants[p->variant].acc_f64 ? sizeof(double) : sizeof(float);
    a.plane = reinterpret_cast<void *>(reinterpret_cast<uintptr_t>(plane) -
                                       (uintptr_t)((size_t)p->tile_first[(size_t)dt] * (size_t)ld_plane * elem));
    a.ld_plane = ld_plane;
    return dispatch(p, a, true, pu::as_stream(stream));
}

}  // extern "C"
