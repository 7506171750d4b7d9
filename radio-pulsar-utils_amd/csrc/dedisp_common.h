// Device helpers shared by the dedispersion translation units (dedisperse.hip: the
// float32-accumulation and channel-mode kernels, the planner and the C-ABI;
// dedisp_f64.hip: the float64 prefetching kernel, compiled with its own code-generation
// options).  Everything here is in an anonymous namespace: each translation unit gets its
// own copy of these inline functions and templates.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "pu_common.h"

namespace {

constexpr int kWaves = 8;                 // waves per workgroup (each owns D trials): 2 WGs = 4 waves/SIMD
constexpr int kThreads = kWaves * 64;
constexpr int kD = 8;                     // trials per wave
constexpr int kTPT = kWaves * kD;         // trials per tile
constexpr int kPartStride = 16;           // elements per (trial, time tile) partial record: the
                                          // accumulation type's (float: 64 B, double: 128 B)
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
    int32_t tt0;      // first time tile of this launch (time-tile range launches)
    int32_t ntt_run;  // time tiles this launch covers (grid = ndt x ntt_run)
    int32_t dt0;      // first DM tile of this launch (DM-tile range launches; ndt = their count)
    void *plane;
    int64_t ld_plane;
    void *partials;  // float records for float32 accumulation, double for float64
};

// Uniform (scalar-cache) load: the constant address space makes hipcc emit s_load.
template <typename T>
__device__ __forceinline__ T ld_uniform(const T *p)
{
    return *(const __attribute__((address_space(4))) T *)(p);
}

#ifdef PU_STAMPS
// Diagnostic build only: a shader-clock stamp with the LDS queue drained, fenced
// against scheduling (cdna_hip_programming.md §7, In-kernel stamps).  s_memtime is a
// scalar-cache READ of the clock; the totals leave the kernel through vector atomics.
__device__ __forceinline__ uint64_t stamp()
{
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#endif

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Channel-mode window reads: J x ds_read_b64 at 512-byte strides (inline asm: hipcc
// would merge pairs into ds_read2st64_b64, which runs at half the LDS rate).  Outputs are
// early-clobber: an LDS read can return (and write its destination) before the block's
// later reads have consumed the address VGPR.  prefetch_window issues without a wait; the
// registers are consumed only after wait_window() on them (a counted-free lgkmcnt(0)
// that "defines" them, so no use can be hoisted above it).
template <int J>
__device__ __forceinline__ void prefetch_window(double (&w)[4], uint32_t addr)
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

template <int J>
__device__ __forceinline__ void wait_window(double (&w)[4])
{
    if constexpr (J == 4)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]) : : "memory");
    else
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0]), "+v"(w[1]) : : "memory");
}

template <int J>
__device__ __forceinline__ void read_window(double (&w)[4], uint32_t addr)
{
    prefetch_window<J>(w, addr);
    wait_window<J>(w);
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
    else if constexpr (K == 4)
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
    else
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]));
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

// Add one channel's contribution to all D trials of this wave.  ``rec`` = 8 u16 window
// records (byte offset | reload flag << 15); ``w`` holds trial 0's window (raw LDS
// elements).  The window's K samples are taken into the accumulation type once per
// window (``wv``: a float32 -> float64 conversion per changed window, not per trial and
// sample: round 3 converted on every add, two VALU ops per float64 add at C2 acc='f64');
// a trial whose window differs from the previous trial's re-reads it in place.
template <typename Tl, typename Ta, int K, int J>
__device__ __forceinline__ void channel_trials(Ta (&acc)[kD][K], double (&w)[4], const u32x4 rec, uint32_t cbase)
{
    Ta wv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wv[k] = static_cast<Ta>(window_elem<Tl>(w, k));
#pragma unroll
    for (int d = 0; d < kD; ++d) {
        if (d > 0) {
            const uint32_t word = rec[d >> 1] >> (16 * (d & 1));
            if (word & 0x8000u) {
                read_window<J>(w, cbase + (word & 0x7fffu));
#pragma unroll
                for (int k = 0; k < K; ++k) wv[k] = static_cast<Ta>(window_elem<Tl>(w, k));
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] += wv[k];
        pin_accumulators(acc[d]);
    }
}

// ---- DPP cross-lane helpers (gfx9 DPP: quad_perm / row_shl / row_ror / row_bcast).
// VALU-only: unlike __shfl (ds_bpermute), they use no LDS bandwidth.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xf, false);
}

template <int CTRL, int ROW_MASK = 0xf, typename T>
__device__ __forceinline__ T dpp(T old, T v)
{
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, dpp_u32<CTRL, ROW_MASK>(__builtin_bit_cast(uint32_t, old),
                                                             __builtin_bit_cast(uint32_t, v)));
    } else {
        const uint64_t o = __builtin_bit_cast(uint64_t, old), x = __builtin_bit_cast(uint64_t, v);
        const uint64_t lo = dpp_u32<CTRL, ROW_MASK>((uint32_t)o, (uint32_t)x);
        const uint64_t hi = dpp_u32<CTRL, ROW_MASK>((uint32_t)(o >> 32), (uint32_t)(x >> 32));
        return __builtin_bit_cast(T, lo | (hi << 32));
    }
}

// The DPP-moved value with no "old" operand (v_mov_b32_dpp into a fresh register): lanes
// of rows outside ROW_MASK get an undefined value.  For reductions whose result is read
// from lane 63 only, this drops the zeroing move that update_dpp(0, v) costs per dword.
template <int CTRL, int ROW_MASK = 0xf, typename T>
__device__ __forceinline__ T dpp_undef(T v)
{
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, true));
    } else {
        const uint64_t x = __builtin_bit_cast(uint64_t, v);
        const uint64_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, ROW_MASK, 0xf, true);
        const uint64_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, ROW_MASK, 0xf, true);
        return __builtin_bit_cast(T, lo | (hi << 32));
    }
}

// Value of lane l + S within the lane's row of 16 (row_shl:S); lanes past the row end
// get 0.  Used only where l + S stays in the row.
template <int S, typename T>
__device__ __forceinline__ T row_down(T v)
{
    return dpp<0x100 + S>(T(0), v);
}

// Wave reductions to lane 63: within rows (quad xor 1, 2, row_ror 4, 8), then
// row_bcast15 into rows 1 and 3, row_bcast31 into rows 2 and 3.
// (Only lane 63's result is defined: the row_bcast steps leave rows outside their mask
// with undefined partial sums.)
template <typename T>
__device__ __forceinline__ T wave_sum_to63(T v)
{
    v += dpp_undef<0xB1>(v);
    v += dpp_undef<0x4E>(v);
    v += dpp_undef<0x124>(v);
    v += dpp_undef<0x128>(v);
    v += dpp_undef<0x142, 0xA>(v);
    v += dpp_undef<0x143, 0xC>(v);
    return v;
}

// Sum over the wave to lane 63 of per-lane float64 (or float32) partials.  float32
// partials are summed in float32 within each row of 16 lanes (few terms of one time
// tile), then in float64 across rows.
template <typename Ta>
__device__ __forceinline__ double wave_sum_to63_acc(Ta v)
{
    if constexpr (sizeof(Ta) == 8) {
        return wave_sum_to63(v);
    } else {
        v += dpp_undef<0xB1>(v);
        v += dpp_undef<0x4E>(v);
        v += dpp_undef<0x124>(v);
        v += dpp_undef<0x128>(v);
        double r = static_cast<double>(v);
        r += dpp_undef<0x142, 0xA>(r);
        r += dpp_undef<0x143, 0xC>(r);
        return r;
    }
}

// max for values that are never NaN on the left (running maxima start at -inf and a NaN
// candidate is skipped, as fmax skips it): a compare and a select, where fmax in IEEE
// mode costs two canonicalising maxes on top
template <typename T>
__device__ __forceinline__ T max_nn(T a, T b)
{
    return b > a ? b : a;
}

template <typename T>
__device__ __forceinline__ T wave_max_to63(T v)
{
    const T lo = -INFINITY;
    v = max_nn(v, dpp<0xB1>(lo, v));
    v = max_nn(v, dpp<0x4E>(lo, v));
    v = max_nn(v, dpp<0x124>(lo, v));
    v = max_nn(v, dpp<0x128>(lo, v));
    v = max_nn(v, dpp<0x142, 0xA>(lo, v));
    v = max_nn(v, dpp<0x143, 0xC>(lo, v));
    return v;
}

// max(v, v of the DPP source lane) in one v_max_f32_dpp (rows outside ROW_MASK keep v).
// IEEE-mode v_max_f32 returns the non-NaN operand, as fmax does; hipcc's fmax would
// add canonicalising maxes and could not fold the DPP move.
#define PU_MAX_DPP(NAME, CTRL)                                                                  \
    __device__ __forceinline__ float NAME(float v)                                              \
    {                                                                                           \
        float r = v;                                                                            \
        asm volatile("v_max_f32_dpp %0, %1, %0 " CTRL " bank_mask:0xf" : "+v"(r) : "v"(v));     \
        return r;                                                                               \
    }
PU_MAX_DPP(max_qp1032, "quad_perm:[1,0,3,2] row_mask:0xf")
PU_MAX_DPP(max_qp2301, "quad_perm:[2,3,0,1] row_mask:0xf")
PU_MAX_DPP(max_ror4, "row_ror:4 row_mask:0xf")
PU_MAX_DPP(max_ror8, "row_ror:8 row_mask:0xf")
#undef PU_MAX_DPP

__device__ __forceinline__ float vmax(float a, float b)
{
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));  // pure: may be computed unconditionally
    return r;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// v_max3_f32 (IEEE mode: a NaN operand is skipped, as by v_max_f32)
__device__ __forceinline__ float vmax3(float a, float b, float c)
{
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Cross-lane combines by the gfx950 permlane swaps (VALU, no LDS): one instruction
// exchanges half of two registers, so one swap + one op reduces TWO values by a factor
// of two in lanes.  swap32: lanes 0-31 of the result = op(a[l], a[l + 32]), lanes 32-63
// = op(b[l - 32], b[l]).  swap16 (rows of 16 lanes): [op(a.r0, a.r1), op(b.r0, b.r1),
// op(a.r2, a.r3), op(b.r2, b.r3)].
template <class Op>
__device__ __forceinline__ float swap32_combine(float a, float b, Op op)
{
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                    false, false);
    return op(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
template <class Op>
__device__ __forceinline__ float swap16_combine(float a, float b, Op op)
{
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                    false, false);
    return op(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}

// Row of 16 lanes: every lane gets the row's sum / max (fused DPP ops).
__device__ __forceinline__ float row_allsum(float v)
{
    v += dpp_undef<0xB1>(v);
    v += dpp_undef<0x4E>(v);
    v += dpp_undef<0x124>(v);
    v += dpp_undef<0x128>(v);
    return v;
}
__device__ __forceinline__ float row_allmax(float v)
{
    v = max_qp1032(v);
    v = max_qp2301(v);
    v = max_ror4(v);
    return max_ror8(v);
}

// Search-mode outputs of a wave of the subband kernel for a FULL time tile (every width's
// windows inside the series): the statistics of write_outputs (same partial record) from
// the packed accumulator pairs, without per-sample bounds tests.
//  * Per lane and trial: width 1 on the pairs (v_pk_*), widths 2/4/8 on scalars (the 4-
//    and 8-sample sums are fused v_add_f32_dpp row shifts) accumulated on every lane and
//    kept only on lanes where they are aligned windows, by one select after the loop (a
//    conditional v_max in inline asm became an EXEC-mask branch); squares accumulated by
//    FMA (one rounding), maxima by v_max3_f32 / v_max_f32.
//  * Across the wave, 8 trials at once: permlane32 swaps pair trial k with k + 4 (half
//    the lanes each), permlane16 swaps pair those with k + 2, so each of 2 registers
//    holds 4 trials' partials in its 4 rows; 4 DPP steps finish every row.
//    Per 8 trials and statistic: 6 swaps, 6 ops and 8 DPP steps instead of 6 DPP steps
//    per trial (the previous epilogue: ~10 % of the kernel's wave cycles at C2).
//  * Sums in float32 throughout: <= 14 float32 roundings per term (the shifted value, the
//    4-term lane chain, the pair, 2 swaps, 4 row steps, the square), within the gamma =
//    2^-20 the finalize kernel's certification assumes.
//  * Stores: lane 16 r + i writes field i (< 13) of the record of row r's trial - one
//    store instruction per 4 trials' records instead of one per field and trial.
template <int D, int J>
__device__ __forceinline__ void stats_full_pairs(const f32x2 (&acc)[D][J], const DedispArgs &a, int first, int slot0,
                                                 int cnt, int tt, int lane)
{
    static_assert(D % 8 == 0, "trials per wave");
    constexpr int NV = 9;  // per trial: sum y, sum of squares w = 1,2,4,8, max w = 1,2,4,8
    const bool even = (lane & 1) == 0;
    // The shift (recorded as the partial's center): the tile mean of the wave's first
    // trial.  The wave's D trials are a few DM steps apart, so their tile means differ by
    // a small fraction of the std: the shifted squares stay near the variance and their
    // float32 sums stay accurate, which keeps the finalize's certification bound tight
    // (lane 0's first sample as the shift inflated them by w^2 var).
    float kt;
    {
        f32x2 s0 = acc[0][0];
#pragma unroll
        for (int j = 1; j < J; ++j) s0 += acc[0][j];
        const float v = wave_sum_to63(s0.x + s0.y);
        kt = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63)) *
             (1.0f / (128.0f * J));
    }
    const f32x2 k1 = {kt, kt};
    const float k2 = 2.0f * kt, k4 = 4.0f * kt, k8 = 8.0f * kt;
    static_assert(J % 2 == 0, "sample pairs are taken two blocks at a time");
    const bool lo2 = (lane & 2) == 0;
    auto lane_stats = [&](int d, float (&v)[NV]) {
        f32x2 s1 = {0.0f, 0.0f}, q1 = s1;
        float q2 = 0.0f, q4 = 0.0f, q8 = 0.0f;
        float m1 = -INFINITY, m2 = -INFINITY, m4 = -INFINITY, m8 = -INFINITY;
#pragma unroll
        for (int j = 0; j < J; j += 2) {
            float r2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f32x2 x = acc[d][j + h];
                const f32x2 y = x - k1;
                s1 += y;
                q1 = __builtin_elementwise_fma(y, y, q1);
                m1 = vmax3(m1, x.x, x.y);
                r2[h] = x.x + x.y;  // width 2 (every lane)
                const float y2 = r2[h] - k2;
                q2 = __builtin_fmaf(y2, y2, q2);
                m2 = vmax(m2, r2[h]);
            }
            // widths 4 and 8 of the two blocks j, j + 1 packed into one register (every
            // lane useful, round 4): even lanes hold block j's width-4 sums (r2 of lanes l,
            // l + 1), odd lanes block j + 1's (lanes l - 1, l) - one quad_perm [1,0,3,2] add
            // of the parity-swapped r2; then quad_perm [2,3,0,1] pairs them into width 8 on
            // lanes 4k (block j) and 4k + 1 (block j + 1), the other two lanes of each quad
            // holding copies (dropped after the loop).  (Round 3: both widths on every lane
            // of every block, half / three quarters of them dropped.)
            const float a4 = even ? r2[0] : r2[1];
            const float c4 = even ? r2[1] : r2[0];
            const float r4 = a4 + dpp<0xB1>(0.0f, c4);
            const float y4 = r4 - k4;
            q4 = __builtin_fmaf(y4, y4, q4);
            m4 = vmax(m4, r4);
            const float r8 = r4 + dpp<0x4E>(0.0f, r4);
            const float y8 = r8 - k8;
            q8 = __builtin_fmaf(y8, y8, q8);
            m8 = vmax(m8, r8);
        }
        v[0] = s1.x + s1.y;
        v[1] = q1.x + q1.y;
        v[2] = q2;
        v[3] = q4;
        v[4] = lo2 ? q8 : 0.0f;
        v[5] = m1;
        v[6] = m2;
        v[7] = m4;
        v[8] = lo2 ? m8 : -INFINITY;
    };
    auto add = [](float x, float y) { return x + y; };
    auto mx = [](float x, float y) { return vmax(x, y); };
    // record field f = lane & 15 (< 13): kt | max w, sum, sum of squares w (w = 1, 2, 4, 8)
    const int f = lane & 15, row = lane >> 4;
    const int fw = (f - 1) / 3, fk = (f - 1) % 3;  // f >= 1: width index, 0 max / 1 sum / 2 squares
    // 8 trials at a time (b0 .. b0 + 7): the register footprint of the 16-trial shapes'
    // two passes is that of one
#pragma unroll
    for (int b0 = 0; b0 < D; b0 += 8) {
        // trials k and k + 4 -> U[k] (lanes 0-31: k, 32-63: k + 4)
        float U[4][NV];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float va[NV], vb[NV];
            lane_stats(b0 + k, va);
            lane_stats(b0 + k + 4, vb);
#pragma unroll
            for (int i = 0; i < NV; ++i)
                U[k][i] = i < 5 ? swap32_combine(va[i], vb[i], add) : swap32_combine(va[i], vb[i], mx);
        }
        // U[j] and U[j + 2] -> W[j]: row r holds trial j + 2 r
        float W[2][NV];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < NV; ++i)
                W[j][i] = i < 5 ? row_allsum(swap16_combine(U[j][i], U[j + 2][i], add))
                                : row_allmax(swap16_combine(U[j][i], U[j + 2][i], mx));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float v = kt;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                v = (f >= 1 && fw == w && fk == 0) ? W[j][5 + w] : v;
                v = (f >= 1 && fw == w && fk == 1) ? W[j][0] : v;
                v = (f >= 1 && fw == w && fk == 2) ? W[j][1 + w] : v;
            }
            const int trial = b0 + j + 2 * row;
            if (f < 13 && slot0 + trial < cnt)
                reinterpret_cast<float *>(a.partials)[((size_t)(first + slot0 + trial) * a.ntt + tt) * kPartStride + f] = v;
        }
    }
}

// float64 counterparts of the permlane combines (two swaps per value, one per dword)
__device__ __forceinline__ double vmax_f64(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));  // IEEE mode: skips a NaN operand
    return r;
}
__device__ __forceinline__ double f64_of(unsigned lo, unsigned hi)
{
    return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}
template <class Op>
__device__ __forceinline__ double swap32_combine_f64(double a, double b, Op op)
{
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    return op(f64_of((unsigned)lo[0], (unsigned)hi[0]), f64_of((unsigned)lo[1], (unsigned)hi[1]));
}
template <class Op>
__device__ __forceinline__ double swap16_combine_f64(double a, double b, Op op)
{
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    return op(f64_of((unsigned)lo[0], (unsigned)hi[0]), f64_of((unsigned)lo[1], (unsigned)hi[1]));
}

// Search-mode outputs of a channel-mode wave with float64 accumulators (the reference-
// precision search, acc='f64') for a FULL time tile: the partial record of write_outputs
// (kt | max, sum, sum of squares of the 1/2/4/8-sample rebinned series), computed as
// stats_full_pairs does for float32 - per-lane statistics without bounds tests, widths 2/4/8
// by DPP row shifts accumulated on every lane and the misaligned lanes dropped once, and the
// wave reductions of the 8 trials together on the permlane32/16 swaps, lane 16 r + f
// storing field f of row r's trial.  Round 3 reduced every statistic of every trial with
// its own 6-step DPP chain (about 480 instructions per trial: the larger part of the C1
// kernel).  All sums in float64 (<= 11 roundings per term: gamma = 2^-44 holds).
// E = 1: lane l owns samples t0 + l + 64 k; E = 2: pairs t0 + 2 l + 128 j + {0, 1}.
template <int E, int K, int D = kD>
__device__ __forceinline__ void stats_full_f64(const double (&acc)[D][K], const DedispArgs &a, int first, int slot0,
                                               int cnt, int tt, int lane)
{
    constexpr int NV = 9;  // sum y, sum of squares w = 1, 2, 4, 8, max w = 1, 2, 4, 8
    static_assert(D == 8 || D == 4, "8 or 4 trials per wave");
    double kt;  // the tile mean of the wave's first trial (the shift of every record)
    {
        double s0 = acc[0][0];
#pragma unroll
        for (int k = 1; k < K; ++k) s0 += acc[0][k];
        const uint64_t b = __builtin_bit_cast(uint64_t, wave_sum_to63(s0));
        kt = f64_of((unsigned)__builtin_amdgcn_readlane((int)(uint32_t)b, 63),
                    (unsigned)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63)) *
             (1.0 / (64.0 * K));
    }
    const double k2 = 2.0 * kt, k4 = 4.0 * kt, k8 = 8.0 * kt;
    const bool m2ok = E == 2 || (lane & 1) == 0;                 // aligned width-2 windows
    const bool m4ok = E == 2 ? (lane & 1) == 0 : (lane & 3) == 0;
    const bool m8ok = E == 2 ? (lane & 3) == 0 : (lane & 7) == 0;
    auto lane_stats = [&](int d, double (&v)[NV]) {
        double s1 = 0.0, q1 = 0.0, q2 = 0.0, q4 = 0.0, q8 = 0.0;
        double m1 = -INFINITY, m2 = -INFINITY, m4 = -INFINITY, m8 = -INFINITY;
        auto w1 = [&](double x) {
            const double y = x - kt;
            s1 += y;
            q1 = __builtin_fma(y, y, q1);
            m1 = vmax_f64(m1, x);
        };
        auto wn = [&](double r, double k, double &q, double &m) {
            const double y = r - k;
            q = __builtin_fma(y, y, q);
            m = vmax_f64(m, r);
        };
        if constexpr (E == 1) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const double x = acc[d][k];
                w1(x);
                const double r2 = x + dpp_undef<0x101>(x);  // row_shl:1, zero past the row
                wn(r2, k2, q2, m2);
                const double r4 = r2 + dpp_undef<0x102>(r2);
                wn(r4, k4, q4, m4);
                const double r8 = r4 + dpp_undef<0x104>(r4);
                wn(r8, k8, q8, m8);
            }
        } else {
#pragma unroll
            for (int j = 0; j < K / 2; ++j) {
                const double x0 = acc[d][2 * j], x1 = acc[d][2 * j + 1];
                w1(x0);
                w1(x1);
                const double r2 = x0 + x1;
                wn(r2, k2, q2, m2);
                const double r4 = r2 + dpp_undef<0x101>(r2);
                wn(r4, k4, q4, m4);
                const double r8 = r4 + dpp_undef<0x102>(r4);
                wn(r8, k8, q8, m8);
            }
        }
        v[0] = s1;
        v[1] = q1;
        v[2] = m2ok ? q2 : 0.0;
        v[3] = m4ok ? q4 : 0.0;
        v[4] = m8ok ? q8 : 0.0;
        v[5] = m1;
        v[6] = m2ok ? m2 : -INFINITY;
        v[7] = m4ok ? m4 : -INFINITY;
        v[8] = m8ok ? m8 : -INFINITY;
    };
    auto add = [](double x, double y) { return x + y; };
    auto mx = [](double x, double y) { return vmax_f64(x, y); };
    auto row_all = [&](double v, bool is_max) {
        if (is_max) {
            v = vmax_f64(v, dpp_undef<0xB1>(v));
            v = vmax_f64(v, dpp_undef<0x4E>(v));
            v = vmax_f64(v, dpp_undef<0x124>(v));
            return vmax_f64(v, dpp_undef<0x128>(v));
        }
        v += dpp_undef<0xB1>(v);
        v += dpp_undef<0x4E>(v);
        v += dpp_undef<0x124>(v);
        return v + dpp_undef<0x128>(v);
    };
    // Trials in pairs (k, k + 4): swap32 -> every value holds trial k in lanes 0-31 and
    // k + 4 in lanes 32-63; then swap16 pairs two VALUES of the pair ((s1, q1), (q2, q4),
    // (q8, q8), (m1, m2), (m4, m8)): rows 0 / 1 hold the first / second value for trial k,
    // rows 2 / 3 for trial k + 4, and 4 fused row steps give every lane its row's total.
    // Lane 16 r + f stores field f of its row's trial when that row holds the field's value
    // (one store instruction per pair).  One pair at a time (scheduling barriers between
    // them), so the accumulators die as the partials are made: <= 128 VGPRs, 4 waves per
    // SIMD (8 trials at once, as stats_full_pairs does for float32, took 158-178).
    const int li = lane & 15, row = lane >> 4, rp = row & 1;
    const bool st_lane = rp == 0 ? (li <= 2 || li == 5 || li == 6 || li == 7 || li == 8 || li == 11 || li == 12)
                                 : (li == 3 || li == 4 || li == 9 || li == 10);
#pragma unroll
    for (int k = 0; k < D / 2; ++k) {
        double va[NV], vb[NV];
        lane_stats(k, va);
        __builtin_amdgcn_sched_barrier(0);
        lane_stats(k + D / 2, vb);
        double U[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i)
            U[i] = i < 5 ? swap32_combine_f64(va[i], vb[i], add) : swap32_combine_f64(va[i], vb[i], mx);
        const double P0 = row_all(swap16_combine_f64(U[0], U[1], add), false);  // s1 | q1
        const double P1 = row_all(swap16_combine_f64(U[2], U[3], add), false);  // q2 | q4
        const double P2 = row_all(swap16_combine_f64(U[4], U[4], add), false);  // q8 | q8
        const double P3 = row_all(swap16_combine_f64(U[5], U[6], mx), true);    // m1 | m2
        const double P4 = row_all(swap16_combine_f64(U[7], U[8], mx), true);    // m4 | m8
        // field li: 0 kt, 1 + 3 w + {0 max, 1 sum, 2 sum of squares} for width index w
        double v = kt;
        v = (li == 1 || li == 4) ? P3 : v;
        v = (li == 2 || li == 3 || li == 5 || li == 8 || li == 11) ? P0 : v;
        v = (li == 6 || li == 9) ? P1 : v;
        v = (li == 7 || li == 10) ? P4 : v;
        v = li == 12 ? P2 : v;
        const int trial = row < 2 ? k : k + D / 2;
        if (st_lane && slot0 + trial < cnt)
            reinterpret_cast<double *>(a.partials)[((size_t)(first + slot0 + trial) * a.ntt + tt) * kPartStride + li] = v;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Outputs of one wave: the dedispersed plane rows of its D trials, or their per-tile
// partial statistics (1/2/4/8-sample rebinned sums: max, shifted sum, shifted sum of
// squares; lane-local in the accumulation type, then float64 wave reductions).
template <typename Tl, typename Ta, int K, int D, bool PLANE, bool STATS>
__device__ __forceinline__ void write_outputs(const Ta (&acc)[D][K], const DedispArgs &a, int first, int slot0,
                                              int cnt, int t0, int tt, int lane)
{
    constexpr int E = 8 / (int)sizeof(Tl);
    constexpr int J = K / E;
    const int n = a.n;
    // sample index of acc[.][k] for this lane
    auto sample = [&](int k) { return t0 + E * lane + 64 * E * (k / E) + (k % E); };

    if constexpr (PLANE) {
        Ta *plane = reinterpret_cast<Ta *>(a.plane);
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (slot0 + d < cnt) {
                Ta *orow = plane + (size_t)(first + slot0 + d) * (size_t)a.ld_plane;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int t = sample(k);
                    if (t < n) orow[t] = acc[d][k];
                }
            }
        }
    }
    if constexpr (STATS) {
        // Per trial: lane-local stats of the 1/2/4/8-sample rebinned sums in the
        // accumulation type (few terms), then float64 wave reductions.
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (slot0 + d >= cnt) continue;
            Ta kt;  // lane 0's first sample: the shift that keeps the sums well conditioned
            if constexpr (sizeof(Ta) == 4) {
                kt = __builtin_bit_cast(Ta, __builtin_amdgcn_readlane(__builtin_bit_cast(int, acc[d][0]), 0));
            } else {
                const uint64_t b = __builtin_bit_cast(uint64_t, acc[d][0]);
                kt = __builtin_bit_cast(Ta, (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 0) |
                                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 0) << 32));
            }
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
                    mx[w] = max_nn(mx[w], r);
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
                    r += row_down<1>(r);                  // width 4
                    account(2, r, t, (lane & 1) == 0);
                    r += row_down<2>(r);                  // width 8
                    account(3, r, t, (lane & 3) == 0);
                } else {
                    Ta r = acc[d][j];
                    const int t = sample(j);
                    account(0, r, t, true);
                    r += row_down<1>(r);
                    account(1, r, t, (lane & 1) == 0);
                    r += row_down<2>(r);
                    account(2, r, t, (lane & 3) == 0);
                    r += row_down<4>(r);
                    account(3, r, t, (lane & 7) == 0);
                }
            }
            Ta *p = reinterpret_cast<Ta *>(a.partials) + ((size_t)(first + slot0 + d) * a.ntt + tt) * kPartStride;
            const bool full = t0 + J * 64 * E <= n;  // uniform
            double x1_0 = 0.0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const Ta m = wave_max_to63(mx[w]);
                // In a full tile every width covers all TT samples, so the shifted sums
                // of the four rebinned series are the same sum (sum_t x - TT kt): one
                // reduction serves all widths.
                const double x1 = (w > 0 && full) ? x1_0 : wave_sum_to63_acc<Ta>(s1[w]);
                if (w == 0) x1_0 = x1;
                const double x2 = wave_sum_to63_acc<Ta>(s2[w]);
                if (lane == 63) {
                    p[1 + 3 * w] = m;
                    p[2 + 3 * w] = static_cast<Ta>(x1);
                    p[3 + 3 * w] = static_cast<Ta>(x2);
                }
            }
            if (lane == 63) p[0] = kt;
        }
    }
}

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// LDS-DMA of one channel-row window [start, start + cover) mod n (float32) into dst:
// 1 KiB pieces (16 B/lane) while contiguous, per-lane modular dwords if it wraps.
// Called by one wave; lands by the wave's next vmcnt(0) (the next barrier).
__device__ __forceinline__ void dma_row_f32(unsigned char *dst, const float *row, int start, int cover_bytes, int n,
                                            bool small_n, int lane)
{
    if (!small_n && start + cover_bytes / 4 <= n) {
        const char *src = reinterpret_cast<const char *>(row + start);
        int off = 0;
        for (; off + 1024 <= cover_bytes; off += 1024)
            __builtin_amdgcn_global_load_lds((const void *)(src + off + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(dst + off), 16, 0, 0);
        // the 256..768-byte tail in 256-B pieces (one partial 16-B/lane piece instead
        // measured 0.15 ms slower at C2)
        for (; off < cover_bytes; off += 256)
            __builtin_amdgcn_global_load_lds((const void *)(src + off + 4 * lane),
                                             (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
    } else {
        for (int off = 0; off < cover_bytes; off += 256) {
            int idx = start + (off >> 2) + lane;
            if (small_n) {
                idx %= n;
            } else {
                idx = idx >= n ? idx - n : idx;
            }
            __builtin_amdgcn_global_load_lds((const void *)(row + idx),
                                             (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
        }
    }
}

}  // namespace
