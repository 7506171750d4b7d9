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
//   * no scalar memory traffic in the channel loop: the window records travel with the
//     rows (one 256-byte LDS-DMA per channel and chunk, all waves' records), each channel's
//     record is read from LDS one channel ahead and moved into scalars after the wait that
//     trial 0 needs anyway; every channel pair's reload count is even (planner), so pairs
//     start and end in state 0 and no state variable crosses them.  Per channel: two
//     v_readfirstlane, D - 1 scalar tests and the loop's two (round 5's first form,
//     scalar-loaded records two channels per iteration with a state carried over: ~22
//     scalar instructions per channel, more than its vector ones - SQ_INSTS_SALU 1.26x
//     SQ_INSTS_VALU at C2, profiles/r05/counters/).
// Record per (DM tile, channel, wave): D u16 words, word d = 0 when trial d reads trial
// d - 1's window, else 1 + the offset in float64 elements, from the chunk's row base, of
// the window to prefetch when trial d's becomes current (planner: dedisperse.hip, pu_plan create).  A
// table after the records holds each channel's first window offset (read at chunk starts).
// Channel order and the float64 adds are the reference's (dedispersion.py:86-98): the
// series is bit-identical.

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

// One channel's record (D = 4 u16, uniform across the wave) read from LDS into VGPRs,
// issued without a wait (ds_read_b64: 2 LDS cycles, a 16-byte record's ds_read_b128 takes
// 4); wait_window_record() waits for it together with a window.
__device__ __forceinline__ void prefetch_record(u32x2 &r, uint32_t addr)
{
    asm volatile("ds_read_b64 %0, %1" : "=&v"(r) : "v"(addr) : "memory");
}
__device__ __forceinline__ void wait_window_record(double (&w)[4], u32x2 &r)
{
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(r) : : "memory");
}
__device__ __forceinline__ u32x2 readfirstlane2(const u32x2 &v)
{
    u32x2 s;
    s[0] = __builtin_amdgcn_readfirstlane(v[0]);
    s[1] = __builtin_amdgcn_readfirstlane(v[1]);
    return s;
}
// word d of a record in scalars (d0 | d1 << 16, d2 | d3 << 16)
#define PU_F64_WORD(R, D_) (((D_) & 1) ? (R[(D_) >> 1] >> 16) : (R[(D_) >> 1] & 0xffffu))

// W waves x D trials per wave (W D = 64 trials per DM tile, kTPT): W = 16, D = 4 -
// 1024-thread workgroups, two per CU, 8 waves per SIMD at <= 64 VGPRs to cover the window
// reads' latency (round 5: against W = 8, D = 8 at 4 waves per SIMD, 72.2 -> 66.4 ms at C2).
template <typename Tin, int W, int D, bool PLANE, bool STATS>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(8)))
dedisp_f64_kernel(DedispArgs a, const int32_t *__restrict__ tile_first, const int32_t *__restrict__ tile_count,
                  const int32_t *__restrict__ tile_rowlen, const int32_t *__restrict__ base_tab,
                  const uint32_t *__restrict__ rec_tab, const uint32_t *__restrict__ first_tab)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool kConv = std::is_same<Tin, float>::value;  // raw float32 rows converted in LDS
    static_assert(kConv || std::is_same<Tin, double>::value, "dedisp_f64_kernel: float32 or float64 input");
    static_assert(W * D == kTPT && D == 4 && W == 16, "dedisp_f64_kernel: 16 waves x 4 trials");
    constexpr int K = 4, TT = 64 * K;
    constexpr int kRecBytes = 2 * D * W;  // one channel's records, all waves (u16 words)

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
    const int raw_bytes = kConv ? a.ncc * ((a.row_stride * 4 + 255) & ~255) : 0;
    const int rec_slot = (a.ncc + 2) * kRecBytes;   // + 2 channels: read-ahead, 256-byte DMA pieces
    unsigned char *raw = smem + 2 * buf_bytes;
    unsigned char *recs_lds = smem + 2 * buf_bytes + raw_bytes;
    const uint32_t smem_addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char *)smem;

    double acc[D][K];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] = 0.0;

    const int32_t *base = base_tab + (size_t)dt * a.nchan;
    const unsigned char *rec_g = reinterpret_cast<const unsigned char *>(rec_tab) + (size_t)dt * a.nchan * kRecBytes;
    const uint32_t *first_g = first_tab + (size_t)dt * a.nchan * W + wave;
    const Tin *data = reinterpret_cast<const Tin *>(a.data);
    const int nchunks = (a.nchan + a.ncc - 1) / a.ncc;

    // this wave's rows of chunk k, ci = wave + W m (it DMAs them and, for float32 inputs,
    // converts them, so neither step needs a barrier of its own), rows into float64 buffer
    // b (float64 input) or the raw buffer (float32); the chunk's records in 256-byte pieces
    // (two channels each; the last piece may read past the records, into the first-window
    // table that follows them)
    auto issue_dma = [&](int k, int b) {
        const int c0 = k * a.ncc;
        const int nc = min(a.ncc, a.nchan - c0);
        for (int q = wave; 2 * q < nc; q += W) {
            // the lane's byte offset made opaque here: hoisted out of the chunk loop, the
            // per-lane 64-bit address (rec_g + lane) stayed live across the sum and spilled
            uint32_t lane4 = 4u * (uint32_t)lane;
            asm volatile("" : "+v"(lane4));
            __builtin_amdgcn_global_load_lds((const void *)(rec_g + (size_t)(c0 + 2 * q) * kRecBytes + lane4),
                                             (__attribute__((address_space(3))) void *)(recs_lds + (k & 1) * rec_slot +
                                                                                         q * 2 * kRecBytes),
                                             4, 0, 0);
        }
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
            __syncthreads();  // buffer b and record slot b complete
            if (k + 1 < nchunks) issue_dma(k + 1, 0);  // this wave's raw rows are converted
        } else {
            __syncthreads();  // buffer b landed; every wave left buffer b ^ 1
            if (k + 1 < nchunks) issue_dma(k + 1, b ^ 1);
        }
        if (!active) continue;
        const uint32_t rows = smem_addr + (uint32_t)(b * buf_bytes) + 8u * lane;
        const uint32_t rows_m8 = rows - 8u;  // reload words are 1 + the offset in float64 elements
        // this wave's records of the chunk in LDS: channel ci at rec_v + ci * kRecBytes
        uint32_t rec_v = smem_addr + (uint32_t)(2 * buf_bytes + raw_bytes + b * rec_slot + wave * 2 * D);
        double w0[4], w1[4];
        u32x2 vr;
        // chunk start: channel c0's first window into w1 (state 0: trial 0 makes w1
        // current) and its record in flight
        prefetch_window<4>(w1, rows + ld_uniform(first_g + (size_t)c0 * W));
        prefetch_record(vr, rec_v);
        // Channel code: trial 0 always reloads; trials 1..D-1 run a two-state machine
        // (state S: wS current, the other buffer in flight) whose code for each (trial,
        // state) is written out, so a reload is a wait + a swap of roles with no register
        // moves.  Channels are walked in pairs: the planner makes every pair's reload count
        // even (a trial re-reading its predecessor's window where needed; a lone last
        // channel's count on its own), so a pair starts and ends in state 0 with the next
        // channel's first window in flight in w1 - one entry, one exit, no state variable;
        // the pair's second channel has an entry for each state.  Trial 0's wait also covers
        // the channel's record (read during the previous channel's trial 0), which it moves
        // into scalars before starting the next channel's read.
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
    if (PU_F64_WORD(R, D_) != 0u) {                                                            \
        wait_window<4>(WO);                                                                    \
        prefetch_window<4>(WS, rows_m8 + (PU_F64_WORD(R, D_) << 3));                           \
        PU_F64_ADD(D_, WO)                                                                     \
        goto P##T##D_##_flip_##S_;                                                             \
    }                                                                                          \
    PU_F64_ADD(D_, WS)                                                                         \
    goto P##T##D_##_keep_##S_;
#define PU_F64_EDGES(P, D_, N_)                                                                \
    P##T##D_##_keep_0:                                                                         \
    goto P##T##N_##_0;                                                                         \
    P##T##D_##_flip_0:                                                                         \
    goto P##T##N_##_1;                                                                         \
    P##T##D_##_keep_1:                                                                         \
    goto P##T##N_##_1;                                                                         \
    P##T##D_##_flip_1:                                                                         \
    goto P##T##N_##_0;
        // trial 0 entered in state S (WS: the previous channel's last window, WO: this
        // channel's first, in flight); continues at trial 1 in the other state
#define PU_F64_ENTRY(P, R, RO, S_, WS, WO, N_)                                                 \
    wait_window_record(WO, vr);                                                                \
    R = readfirstlane2(vr);                                                                    \
    prefetch_record(vr, RO);                                                                   \
    prefetch_window<4>(WS, rows_m8 + (PU_F64_WORD(R, 0) << 3));                                \
    PU_F64_ADD(0, WO)                                                                          \
    goto P##T1_##N_;
#define PU_F64_TRIALS(P, R)                                                                    \
    PU_F64_TRIAL(P, R, 1, 0, w0, w1) PU_F64_TRIAL(P, R, 1, 1, w1, w0) PU_F64_EDGES(P, 1, 2)    \
    PU_F64_TRIAL(P, R, 2, 0, w0, w1) PU_F64_TRIAL(P, R, 2, 1, w1, w0) PU_F64_EDGES(P, 2, 3)    \
    PU_F64_TRIAL(P, R, 3, 0, w0, w1) PU_F64_TRIAL(P, R, 3, 1, w1, w0) PU_F64_EDGES(P, 3, 4)
        u32x2 ra, rb;
        // a real loop, not unrolled (LLVM unrolled round 5's first goto cycle ~20 times and
        // spilled)
#pragma nounroll
        for (int ci = 0; ci < nc; ci += 2) {
            PU_F64_ENTRY(A, ra, rec_v + (ci + 1) * kRecBytes, 0, w0, w1, 1)
            PU_F64_TRIALS(A, ra)
        AT4_0:
            if (ci + 1 >= nc) goto chunk_done;
            goto BE0;
        AT4_1:  // (a lone last channel always ends in state 0)
            if (ci + 1 >= nc) goto chunk_done;
            goto BE1;
        BE0:
            PU_F64_ENTRY(B, rb, rec_v + (ci + 2) * kRecBytes, 0, w0, w1, 1)
        BE1:
            PU_F64_ENTRY(B, rb, rec_v + (ci + 2) * kRecBytes, 1, w1, w0, 0)
            PU_F64_TRIALS(B, rb)
        BT4_1:  // never reached (even pair reload counts): joins state 0 without an exit of its own
            goto BT4_0;
        BT4_0:;
        }
    chunk_done:
        // the last prefetches (a re-read of the row base, or a record past the chunk's)
        // land before the next chunk's DMA can overwrite anything
        wait_window_record(w1, vr);
#undef PU_F64_ADD
#undef PU_F64_TRIAL
#undef PU_F64_EDGES
#undef PU_F64_ENTRY
#undef PU_F64_TRIALS
    }
#undef PU_F64_WORD
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
           const int32_t *rowlen, const int32_t *base, const uint32_t *rec, const uint32_t *first_off, hipStream_t s)
{
    const dim3 grid((unsigned)((int64_t)a.ndt * a.ntt_run)), block(64 * kF64W);
    auto go = [&](auto kern) {
        if (lds_bytes > 64 * 1024) {
            int rc = pu::hip_check(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes),
                                   "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
            if (rc) return rc;
        }
        hipLaunchKernelGGL(kern, grid, block, lds_bytes, s, a, first, count, rowlen, base, rec, first_off);
        return pu::launch_check("dedisp_f64_kernel");
    };
    return plane ? go(dedisp_f64_kernel<Tin, kF64W, kF64D, true, false>)
                 : go(dedisp_f64_kernel<Tin, kF64W, kF64D, false, true>);
}

}  // namespace

// Called by dedisperse.hip's dispatch (plain types across the translation units).
int pu_dd_launch_f64(bool tin_f32, bool plane, const void *args, size_t args_bytes, size_t lds_bytes,
                     const int32_t *first, const int32_t *count, const int32_t *rowlen, const int32_t *base,
                     const void *rec8, const void *first_off, void *stream, int waves)
{
    PU_REQUIRE(waves == kF64W, "pu_dd_launch_f64: planned for %d waves, kernel built for %d", waves, kF64W);
    PU_REQUIRE(args_bytes == sizeof(DedispArgs), "pu_dd_launch_f64: argument block size mismatch");
    const DedispArgs &a = *reinterpret_cast<const DedispArgs *>(args);
    const uint32_t *r = reinterpret_cast<const uint32_t *>(rec8);
    const uint32_t *f = reinterpret_cast<const uint32_t *>(first_off);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    return tin_f32 ? launch<float>(plane, a, lds_bytes, first, count, rowlen, base, r, f, s)
                   : launch<double>(plane, a, lds_bytes, first, count, rowlen, base, r, f, s);
}
