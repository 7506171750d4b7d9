// Float64 accumulation in channel order (acc='f64'): dedisp_f64_kernel and its launcher.
// A translation unit of its own so that it can be compiled with
// -mllvm -structurizecfg-skip-uniform-regions=true: the kernel's per-trial state machine
// is an unstructured graph of UNIFORM branches, which the AMDGPU structurizer would
// otherwise rewrite into flag-guarded flow blocks with register copies at every join
// (the first draft spilled 450 bytes per lane).  dedisperse.hip keeps its own options.
//
// Replaces the reference hot loop of dedisperse / _dedisperse / roll_and_sum
// (pulsarutils/dedispersion.py:60-98) with float64 accumulators: bit-identical series.
#include <hip/hip_runtime.h>

#include "dedisp_common.h"

// the state machine's entry labels (T0_0) are reached by falling through
#pragma clang diagnostic ignored "-Wunused-label"

namespace {

// ---------------------------------------------------------------------------------
// Float64 accumulation in channel order with prefetched windows (round 5) - the
// reference-precision path (acc='f64': dedisperse, show=True, search_by_chunks).
//
// Work decomposition: one DM tile of 64 consecutive trials x one 256-sample time tile per
// workgroup of W waves x D trials (round 5 default W = 16, D = 4: 8 waves per SIMD), lane l
// owning samples t0 + l + 64 k, k < 4.  Against round 4's dedisp_kernel (8 waves x 8 trials):
//   * rows are float64 in LDS: float32 inputs are LDS-DMA'd raw and converted once per
//     element and tile by the wave that DMA'd them (no conversion per window reload:
//     the adds read the window registers directly); float64 inputs are DMA'd as they are.
//     Ring of two float64 buffers (+ one raw float32 buffer): one barrier per chunk.
//   * the window of a trial whose shift differs from the previous trial's is not read at
//     that trial (a read + an immediate wait: the wave stalled on LDS latency at every
//     reload, round 4) but PREFETCHED at the previous distinct window's turn: two window
//     buffers w0 / w1, a state machine over the D trials (state S: wS current, the other
//     buffer in flight) whose code for each (trial, state) is written out, so a reload is
//     wait + swap of roles with no register moves.  The last distinct window of a channel
//     prefetches the next channel's first.
// Record per (DM tile, channel, wave): D u32 words, word d: bit 31 trial d's window
// differs from trial d - 1's (set for d = 0), bits 17-29 trial d's window sample offset
// in its row (read for d = 0 at a chunk start), bits 0-16 the byte offset, from the
// chunk's row base, of the window to prefetch when trial d's becomes current (0: none
// left in the chunk - the prefetch then re-reads the row base, harmlessly).  Channel
// order and the float64 adds are the reference's (dedispersion.py:86-98): the series is
// bit-identical.

// LDS-DMA of one float64 channel-row window [start, start + cover) mod n into dst
__device__ __forceinline__ void dma_row_f64(unsigned char *dst, const double *row, int start, int cover_bytes, int n,
                                            bool small_n, int lane)
{
    if (!small_n && start + cover_bytes / 8 <= n) {
        const char *src = reinterpret_cast<const char *>(row + start);
        int off = 0;
        for (; off + 1024 <= cover_bytes; off += 1024)
            __builtin_amdgcn_global_load_lds((const void *)(src + off + 16 * lane),
                                             (__attribute__((address_space(3))) void *)(dst + off), 16, 0, 0);
        for (; off < cover_bytes; off += 256)
            __builtin_amdgcn_global_load_lds((const void *)(src + off + 4 * lane),
                                             (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
    } else {
        for (int off = 0; off < cover_bytes; off += 256) {
            const int byte = off + 4 * lane;
            int idx = start + (byte >> 3);
            if (small_n) {
                idx %= n;
            } else {
                idx = idx >= n ? idx - n : idx;
            }
            __builtin_amdgcn_global_load_lds((const void *)(reinterpret_cast<const char *>(row + idx) + (byte & 7)),
                                             (__attribute__((address_space(3))) void *)(dst + off), 4, 0, 0);
        }
    }
}

// Record of one (DM tile, channel, wave): D u32 words
template <int D>
struct F64Rec {
    typedef uint32_t type __attribute__((ext_vector_type(D)));
};

// W waves x D trials per wave (W D = 64 trials per DM tile, kTPT).  W = 16, D = 4 (round 5
// default): 1024-thread workgroups, two per CU, 8 waves per SIMD at <= 64 VGPRs - twice the
// waves of W = 8, D = 8 to cover the window reads' latency.
template <typename Tin, int W, int D, bool PLANE, bool STATS>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(W == 16 ? 8 : 4)))
dedisp_f64_kernel(DedispArgs a, const int32_t *__restrict__ tile_first, const int32_t *__restrict__ tile_count,
                  const int32_t *__restrict__ tile_rowlen, const int32_t *__restrict__ base_tab,
                  const uint32_t *__restrict__ rec_tab)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool kConv = std::is_same<Tin, float>::value;  // raw float32 rows converted in LDS
    static_assert(kConv || std::is_same<Tin, double>::value, "dedisp_f64_kernel: float32 or float64 input");
    static_assert(W * D == kTPT && (D == 4 || D == 8), "dedisp_f64_kernel: W x D = 64 trials");
    constexpr int K = 4, TT = 64 * K;
    typedef typename F64Rec<D>::type rec_t;

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
    const bool small_n = a.small_n != 0;
    const int chan_bytes = a.row_stride * 8;    // float64 row (no alignment copies)
    const int buf_bytes = a.ncc * chan_bytes;
    const int cover64 = (rowlen * 8 + 255) & ~255;  // bytes of a float64 row moved by DMA
    const int cover32 = (rowlen * 4 + 255) & ~255;  // bytes of a raw float32 row (its stride too)
    unsigned char *raw = smem + 2 * buf_bytes;
    const uint32_t smem_addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;

    double acc[D][K];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] = 0.0;

    const int32_t *base = base_tab + (size_t)dt * a.nchan;
    const rec_t *recs = reinterpret_cast<const rec_t *>(rec_tab) + (size_t)dt * a.nchan * W + wave;
    const Tin *data = reinterpret_cast<const Tin *>(a.data);
    const int nchunks = (a.nchan + a.ncc - 1) / a.ncc;

    // this wave's rows of chunk k: ci = wave + W m (it DMAs them and, for float32 inputs,
    // converts them, so neither step needs a barrier of its own)
    auto issue_dma = [&](int k, int b) {
        const int c0 = k * a.ncc;
        const int nc = min(a.ncc, a.nchan - c0);
        for (int ci = wave; ci < nc; ci += W) {
            const int c = c0 + ci;
            int start = ld_uniform(base + c) + t0;
            if (start >= n) start -= n;
            if (start >= n) start -= n;
            const Tin *row = data + (size_t)c * (size_t)a.ld;
            if constexpr (kConv)
                dma_row_f32(raw + ci * cover32, row, start, cover32, n, small_n, lane);
            else
                dma_row_f64(smem + b * buf_bytes + ci * chan_bytes, row, start, cover64, n, small_n, lane);
        }
    };
    auto convert = [&](int k, int b) {
        const int nc = min(a.ncc, a.nchan - k * a.ncc);
        for (int ci = wave; ci < nc; ci += W) {
            const float *src = reinterpret_cast<const float *>(raw + ci * cover32);
            double *dst = reinterpret_cast<double *>(smem + b * buf_bytes + ci * chan_bytes);
            for (int j = 2 * lane; j < rowlen; j += 128) {
                const float2 v = *reinterpret_cast<const float2 *>(src + j);
                *reinterpret_cast<double2 *>(dst + j) = double2{(double)v.x, (double)v.y};
            }
        }
    };

    issue_dma(0, 0);
    for (int k = 0; k < nchunks; ++k) {
        const int c0 = k * a.ncc;
        const int nc = min(a.ncc, a.nchan - c0);
        const int b = k & 1;
        // this wave's DMA landed (explicit: a workgroup barrier does not wait for vmcnt)
        asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
        if constexpr (kConv) {
            // buffer b was last read in chunk k - 2's sum, before every wave's barrier of
            // chunk k - 1
            convert(k, b);
            __syncthreads();  // buffer b complete
            if (k + 1 < nchunks) issue_dma(k + 1, 0);  // this wave's raw rows are converted
        } else {
            __syncthreads();  // buffer b landed; every wave left buffer b ^ 1
            if (k + 1 < nchunks) issue_dma(k + 1, b ^ 1);
        }
        if (!active) continue;
        const uint32_t rows = smem_addr + (uint32_t)(b * buf_bytes) + 8u * lane;
        const rec_t *rc = recs + (size_t)c0 * W;
        rec_t ra = ld_uniform(rc);
        double w0[4], w1[4];
        // chunk start: channel c0's first window into w1, state 0 (trial 0's reload makes
        // w1 current and prefetches the next window into w0)
        prefetch_window<4>(w1, rows + 8u * ((ra[0] >> 17) & 0x1fffu));
        // trial d in state S (P: label prefix, R: the channel's record): a reload waits for
        // the other buffer, prefetches the next window into this one (a harmless re-read of
        // the row base when no window is left in the chunk) and continues in the other
        // state.  Every (trial, state) has its own code: no register moves.
#define PU_F64_ADD(D_, W_)                                                                      \
    {                                                                                          \
        acc[D_][0] += W_[0];                                                                   \
        acc[D_][1] += W_[1];                                                                   \
        acc[D_][2] += W_[2];                                                                   \
        acc[D_][3] += W_[3];                                                                   \
        pin_accumulators(acc[D_]);                                                             \
    }
#define PU_F64_TRIAL(P, R, D_, S_, WS, WO)                                                     \
    P##T##D_##_##S_:                                                                           \
    if (R[D_] & 0x80000000u) {                                                                 \
        wait_window<4>(WO);                                                                    \
        prefetch_window<4>(WS, rows + (R[D_] & 0x1ffffu));                                     \
        PU_F64_ADD(D_, WO)                                                                     \
        goto P##T##D_##_flip_##S_;                                                             \
    }                                                                                          \
    PU_F64_ADD(D_, WS)                                                                         \
    goto P##T##D_##_keep_##S_;
        // every label's successor: (d + 1, same state) or (d + 1, other state)
#define PU_F64_EDGES(P, D_, N_)                                                                \
    P##T##D_##_keep_0:                                                                         \
    goto P##T##N_##_0;                                                                         \
    P##T##D_##_flip_0:                                                                         \
    goto P##T##N_##_1;                                                                         \
    P##T##D_##_keep_1:                                                                         \
    goto P##T##N_##_1;                                                                         \
    P##T##D_##_flip_1:                                                                         \
    goto P##T##N_##_0;
#define PU_F64_PAIR(P, R, D_, N_)                                                              \
    PU_F64_TRIAL(P, R, D_, 0, w0, w1) PU_F64_TRIAL(P, R, D_, 1, w1, w0) PU_F64_EDGES(P, D_, N_)
#define PU_F64_END(P, N_)                                                                      \
    P##T##N_##_0:                                                                              \
    state = 0;                                                                                 \
    goto P##done;                                                                              \
    P##T##N_##_1:                                                                              \
    state = 1;                                                                                 \
    P##done:;
#define PU_F64_CHANNEL4(P, R)                                                                  \
    if (state) goto P##T0_1;                                                                   \
    PU_F64_PAIR(P, R, 0, 1) PU_F64_PAIR(P, R, 1, 2) PU_F64_PAIR(P, R, 2, 3) PU_F64_PAIR(P, R, 3, 4) \
    PU_F64_END(P, 4)
#define PU_F64_CHANNEL8(P, R)                                                                  \
    if (state) goto P##T0_1;                                                                   \
    PU_F64_PAIR(P, R, 0, 1) PU_F64_PAIR(P, R, 1, 2) PU_F64_PAIR(P, R, 2, 3) PU_F64_PAIR(P, R, 3, 4) \
    PU_F64_PAIR(P, R, 4, 5) PU_F64_PAIR(P, R, 5, 6) PU_F64_PAIR(P, R, 6, 7) PU_F64_PAIR(P, R, 7, 8) \
    PU_F64_END(P, 8)
        // two channels per iteration with ping-pong records: a record is loaded a channel
        // ahead and consumed only after the channel before it (rotating one record through
        // a copy made the compiler wait for the just-issued scalar load at every channel
        // start); a real loop, not unrolled (LLVM unrolled round 5's first goto cycle ~20
        // times and spilled); the state carries over in a scalar
        int state = 0;
#pragma nounroll
        for (int ci = 0; ci < nc; ci += 2) {
            rec_t rb = ld_uniform(rc + (size_t)min(ci + 1, nc - 1) * W);
            if constexpr (D == 4) {
                PU_F64_CHANNEL4(A4, ra)
            } else {
                PU_F64_CHANNEL8(A8, ra)
            }
            asm volatile("" : "+s"(rb));
            if (ci + 1 >= nc) break;
            ra = ld_uniform(rc + (size_t)min(ci + 2, nc - 1) * W);
            if constexpr (D == 4) {
                PU_F64_CHANNEL4(B4, rb)
            } else {
                PU_F64_CHANNEL8(B8, rb)
            }
            asm volatile("" : "+s"(ra));
        }
#undef PU_F64_ADD
#undef PU_F64_TRIAL
#undef PU_F64_EDGES
#undef PU_F64_PAIR
#undef PU_F64_END
#undef PU_F64_CHANNEL4
#undef PU_F64_CHANNEL8
    }
    if (!active) return;

    if constexpr (STATS && !PLANE) {
        if (t0 + TT <= n) {
            stats_full_f64<1, K, D>(acc, a, first, slot0, cnt, tt, lane);
            return;
        }
    }
    write_outputs<double, double, K, D, PLANE, STATS>(acc, a, first, slot0, cnt, t0, tt, lane);
}

// the production shape: 16 waves x 4 trials (kF64Waves in dedisperse.hip's planner)
constexpr int kF64W = 16, kF64D = 4;

template <typename Tin>
int launch(bool plane, const DedispArgs &a, size_t lds_bytes, const int32_t *first, const int32_t *count,
           const int32_t *rowlen, const int32_t *base, const uint32_t *rec, hipStream_t s)
{
    const dim3 grid((unsigned)((int64_t)a.ndt * a.ntt_run)), block(64 * kF64W);
    auto go = [&](auto kern) {
        if (lds_bytes > 64 * 1024) {
            int rc = pu::hip_check(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes),
                                   "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
            if (rc) return rc;
        }
        hipLaunchKernelGGL(kern, grid, block, lds_bytes, s, a, first, count, rowlen, base, rec);
        return pu::launch_check("dedisp_f64_kernel");
    };
    return plane ? go(dedisp_f64_kernel<Tin, kF64W, kF64D, true, false>)
                 : go(dedisp_f64_kernel<Tin, kF64W, kF64D, false, true>);
}

}  // namespace

// Called by dedisperse.hip's dispatch (plain types across the translation units).
int pu_dd_launch_f64(bool tin_f32, bool plane, const void *args, size_t args_bytes, size_t lds_bytes,
                     const int32_t *first, const int32_t *count, const int32_t *rowlen, const int32_t *base,
                     const void *rec8, void *stream, int waves)
{
    PU_REQUIRE(waves == kF64W, "pu_dd_launch_f64: planned for %d waves, kernel built for %d", waves, kF64W);
    PU_REQUIRE(args_bytes == sizeof(DedispArgs), "pu_dd_launch_f64: argument block size mismatch");
    const DedispArgs &a = *reinterpret_cast<const DedispArgs *>(args);
    const uint32_t *r = reinterpret_cast<const uint32_t *>(rec8);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return tin_f32 ? launch<float>(plane, a, lds_bytes, first, count, rowlen, base, r, s)
                   : launch<double>(plane, a, lds_bytes, first, count, rowlen, base, r, s);
}
