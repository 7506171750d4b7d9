// Incoherent (brute-force) shift-and-sum dedispersion for gfx950 (MI355X).
//
// Replaces the reference hot loop (pulsarutils/dedispersion.py):
//   _dedispersion_search :174-202  (prange over trials -> workgroups over DM tiles)
//   dedisperse/_dedisperse/roll_and_sum :60-98 (circular shift-and-sum, channel order)
//
// out_d[t] = sum_c x[c][(t + s[d][c]) mod N]   (s = dedispersion_shifts, any sign)
//
// Mapping:
//   * one workgroup = 4 waves = one DM tile (4*D trials) x one time tile (64*K samples);
//     each wave owns D trials, lane l owns samples t0 + l + 64k, k < K  -> D*K
//     accumulators in VGPRs.
//   * channel rows are staged in LDS, ncc channels per step, each row covering
//     [t0 + smin_c, t0 + 64K + smax_c) mod N: the modular halo of the tile.
//   * per (channel, trial) the shift relative to smin_c is wave-uniform (SGPR); the
//     K-sample window is re-read from LDS only when it changes from the previous
//     trial (adjacent plan trials differ by <= 1 sample per channel), so most adds
//     reuse registers: LDS traffic ~ (1 + (D-1)|slope_c|)/D dwords per add.
//   * accumulation in channel order 0..nchan-1, like the reference; with a float64
//     accumulator the series is bit-identical to the reference's.
//   * epilogue: either the dedispersed plane (coalesced stores), or per-tile partial
//     statistics of the 1/2/4/8-sample rebinned series (max, shifted sum, shifted
//     sum of squares) reduced by pu_finalize_kernel in a fixed order.
//   * blockIdx is remapped XCD-aware so all DM tiles of a time tile run on one XCD
//     and share the staged input through its L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "pu_common.h"

namespace {

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kPartStride = 16;  // doubles per (trial, time tile) partial record
constexpr size_t kLdsBudget = 32 * 1024;
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

// Read one K-sample window of a staged row into registers: J = 4 ds_read_b64 at
// 512-byte strides (lane l gets 8 contiguous bytes of each 512-byte slice).  Written
// as one asm block that overwrites the window in place, so the register allocator
// never keeps two windows alive (the reuse branch would otherwise make phi copies),
// and that waits for its own LDS reads.
__device__ __forceinline__ void read_window(double (&w)[4], uint32_t addr)
{
    asm volatile(
        "ds_read_b64 %0, %4\n\t"
        "ds_read_b64 %1, %4 offset:512\n\t"
        "ds_read_b64 %2, %4 offset:1024\n\t"
        "ds_read_b64 %3, %4 offset:1536\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(w[0]), "=v"(w[1]), "=v"(w[2]), "=v"(w[3])
        : "v"(addr)
        : "memory");
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

// Kernel geometry per lane: E = 8 / sizeof(Tl) consecutive samples per 8-byte LDS
// read, J = 4 reads per window, K = E*J samples per lane:
//   sample(l, j, e) = t0 + E*l + 64*E*j + e.
// float rows are staged twice (copy q holds row[start + q + i]) so every 8-byte read
// is aligned whatever the parity of the shift.
template <typename Tin, typename Tl, typename Ta, int D, bool PLANE, bool STATS>
__global__ void __launch_bounds__(kThreads)
dedisp_kernel(DedispArgs a, const int32_t *__restrict__ tile_first,
              const int32_t *__restrict__ tile_count, const int32_t *__restrict__ tile_rowlen,
              const int32_t *__restrict__ base_tab, const uint16_t *__restrict__ rel_tab)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int E = 8 / (int)sizeof(Tl);
    constexpr int J = 4;
    constexpr int K = E * J;
    constexpr int TT = 64 * K;
    constexpr int TPT = kWaves * D;  // trials per tile

    const int wg = pu::xcd_remap(blockIdx.x, gridDim.x);
    const int dt = wg % a.ndt;
    const int tt = wg / a.ndt;
    const int t0 = tt * TT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int first = tile_first[dt];
    const int cnt = tile_count[dt];
    const int rowlen = tile_rowlen[dt];
    const int slot0 = wave * D;
    const bool active = slot0 < cnt;
    const int n = a.n;
    const int stride = a.row_stride;            // elements per copy (even)
    const int chan_bytes = E * stride * (int)sizeof(Tl);
    // LDS: [rel: ncc x TPT u16][rows: ncc x E copies x stride]
    uint16_t *lds_rel = reinterpret_cast<uint16_t *>(smem);
    const int rel_bytes = (a.ncc * TPT * 2 + 15) & ~15;
    Tl *lds_rows = reinterpret_cast<Tl *>(smem + rel_bytes);
    const uint32_t rows_addr = (uint32_t)(uintptr_t)lds_rows;
    const uint32_t lane_addr = rows_addr + 8u * lane;

    Ta acc[D][K];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[d][k] = Ta(0);

    const int32_t *base = base_tab + (size_t)dt * a.nchan;
    const uint16_t *rel = rel_tab + (size_t)dt * a.nchan * TPT;
    const Tin *data = reinterpret_cast<const Tin *>(a.data);

    for (int c0 = 0; c0 < a.nchan; c0 += a.ncc) {
        const int nc = min(a.ncc, a.nchan - c0);
        __syncthreads();
        // ---- stage: relative shifts of the chunk, then E copies of each row window
        for (int e = tid; e < nc * TPT; e += kThreads) lds_rel[e] = rel[(size_t)c0 * TPT + e];
        for (int ci = 0; ci < nc; ++ci) {
            const int c = c0 + ci;
            const Tin *row = data + (size_t)c * (size_t)a.ld;
            int start = base[c] + t0;
            if (start >= n) start -= n;
            Tl *dst = lds_rows + (size_t)ci * E * stride;
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
        __syncthreads();
        if (!active) continue;
        // ---- accumulate: per channel, D trials x K samples, window reused while the
        // (wave-uniform) shift does not change from one trial to the next
        for (int ci = 0; ci < nc; ++ci) {
            const uint32_t *rr32 = reinterpret_cast<const uint32_t *>(lds_rel + ci * TPT + slot0);
            uint32_t rw[D / 2];
#pragma unroll
            for (int q = 0; q < D / 2; ++q) rw[q] = __builtin_amdgcn_readfirstlane(rr32[q]);
            const uint32_t cbase = lane_addr + (uint32_t)(ci * chan_bytes);
            double w[4];
            int prev = -1;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int s = (int)((rw[d >> 1] >> (16 * (d & 1))) & 0xffffu);
                if (d == 0 || s != prev) {
                    uint32_t off;
                    if constexpr (E == 2)
                        off = (uint32_t)((s & 1) * stride * 4 + (s & ~1) * 4);
                    else
                        off = (uint32_t)(s * 8);
                    read_window(w, cbase + off);
                    prev = s;
                }
#pragma unroll
                for (int k = 0; k < K; ++k) acc[d][k] += static_cast<Ta>(window_elem<Tl>(w, k));
                pin_accumulators(acc[d]);
            }
        }
    }
    if (!active) return;

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
#pragma unroll
        for (int d = 0; d < D; ++d) {
            if (slot0 + d >= cnt) break;
            const double kt = static_cast<double>(__shfl(acc[d][0], 0, 64));
            double mx[4], s1[4], s2[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                mx[w] = -INFINITY;
                s1[w] = 0.0;
                s2[w] = 0.0;
            }
            auto account = [&](int w, Ta r, int t, bool lane_ok) {
                const int width = 1 << w;
                if (lane_ok && t + width <= n) {
                    const double rv = static_cast<double>(r);
                    const double y = rv - width * kt;
                    mx[w] = fmax(mx[w], rv);
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
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    mx[w] = fmax(mx[w], shfl_xor(mx[w], off));
                    s1[w] += shfl_xor(s1[w], off);
                    s2[w] += shfl_xor(s2[w], off);
                }
            }
            if (lane == 0) {
                double *p = a.partials + ((size_t)(first + slot0 + d) * a.ntt + tt) * kPartStride;
                p[0] = kt;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    p[1 + 3 * w] = mx[w];
                    p[2 + 3 * w] = s1[w];
                    p[3 + 3 * w] = s2[w];
                }
            }
        }
    }
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
    int D, K, lds_elem, acc_f64;
};

// D trials per wave; K samples per lane = (8 / LDS element size) * 4 reads
constexpr VariantInfo kVariants[V_COUNT] = {
    {8, 8, 4, 0},  // u8 in, f32 LDS, f32 acc (exact: sums < 2^24)
    {8, 8, 4, 0},  // f32
    {8, 4, 8, 1},  // f64 in, f64 LDS, f64 acc (bit-exact vs reference)
    {8, 8, 4, 1},  // u8 in, f32 LDS, f64 acc
    {8, 8, 4, 1},  // f32 in, f32 LDS, f64 acc (bit-exact vs reference)
    {8, 8, 4, 0},  // f64 in, f32 LDS, f32 acc
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

template <typename Tin, typename Tl, typename Ta, int D>
int launch_variant(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s);

}  // namespace

struct pu_plan {
    int dtype = 0, acc = 0, variant = 0;
    int64_t nchan = 0, n = 0, ndm = 0;
    int D = 0, K = 0, TT = 0, tpt = 0;  // trials per tile
    int ndt = 0, ntt = 0, ncc = 0, row_stride = 0, small_n = 0, max_spread = 0;
    size_t lds_bytes = 0;
    int32_t *d_first = nullptr, *d_count = nullptr, *d_rowlen = nullptr, *d_base = nullptr;
    uint16_t *d_rel = nullptr;
    // optional kernel timing: event pairs recorded around each dedispersion launch
    std::vector<hipEvent_t> ev_start, ev_stop;
    int64_t launches = 0;
};

namespace {

template <typename Tin, typename Tl, typename Ta, int D>
int launch_variant(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    const dim3 grid((unsigned)((int64_t)p->ndt * p->ntt)), block(kThreads);
    if (plane)
        hipLaunchKernelGGL((dedisp_kernel<Tin, Tl, Ta, D, true, false>), grid, block, p->lds_bytes, s,
                           a, p->d_first, p->d_count, p->d_rowlen, p->d_base, p->d_rel);
    else
        hipLaunchKernelGGL((dedisp_kernel<Tin, Tl, Ta, D, false, true>), grid, block, p->lds_bytes, s,
                           a, p->d_first, p->d_count, p->d_rowlen, p->d_base, p->d_rel);
    return pu::launch_check("dedisp_kernel");
}

int dispatch_variant(const pu_plan *p, const DedispArgs &a, bool plane, hipStream_t s)
{
    switch (p->variant) {
    case V_U8_F32: return launch_variant<uint8_t, float, float, 8>(p, a, plane, s);
    case V_F32_F32: return launch_variant<float, float, float, 8>(p, a, plane, s);
    case V_F64_F64: return launch_variant<double, double, double, 8>(p, a, plane, s);
    case V_U8_F64: return launch_variant<uint8_t, float, double, 8>(p, a, plane, s);
    case V_F32_F64: return launch_variant<float, float, double, 8>(p, a, plane, s);
    case V_F64_F32: return launch_variant<double, float, float, 8>(p, a, plane, s);
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
    (void)hipFree(p->d_rel);
    delete p;
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
    p->D = kVariants[v].D;
    p->K = kVariants[v].K;
    p->TT = 64 * p->K;
    p->tpt = kWaves * p->D;
    const int esz = kVariants[v].lds_elem;

    // ---- greedy DM tiles: up to tpt consecutive trials whose per-channel shift
    // spread (max - min) stays <= kMaxSpread
    std::vector<int32_t> first, count, rowlen, base;
    std::vector<uint16_t> rel;
    std::vector<int64_t> mn((size_t)nchan), mx((size_t)nchan);
    int64_t i = 0;
    int max_rowlen = 0;
    while (i < ndm) {
        const int64_t *s0 = shifts + i * nchan;
        for (int64_t c = 0; c < nchan; ++c) mn[c] = mx[c] = s0[c];
        int64_t j = i + 1;
        while (j < ndm && j - i < p->tpt) {
            const int64_t *sj = shifts + j * nchan;
            bool ok = true;
            for (int64_t c = 0; c < nchan; ++c) {
                const int64_t lo = std::min(mn[c], sj[c]), hi = std::max(mx[c], sj[c]);
                if (hi - lo > kMaxSpread) {
                    ok = false;
                    break;
                }
            }
            if (!ok) break;
            for (int64_t c = 0; c < nchan; ++c) {
                mn[c] = std::min(mn[c], sj[c]);
                mx[c] = std::max(mx[c], sj[c]);
            }
            ++j;
        }
        const int cntt = (int)(j - i);
        first.push_back((int32_t)i);
        count.push_back(cntt);
        int spread = 0;
        const size_t rbase = rel.size();
        rel.resize(rbase + (size_t)nchan * p->tpt, 0);
        for (int64_t c = 0; c < nchan; ++c) {
            int64_t b = mn[c] % n;
            if (b < 0) b += n;
            base.push_back((int32_t)b);
            for (int s = 0; s < cntt; ++s) {
                int64_t r = (shifts[(i + s) * nchan + c] - mn[c]) % n;  // >= 0
                rel[rbase + (size_t)c * p->tpt + s] = (uint16_t)r;
                spread = std::max(spread, (int)r);
            }
        }
        p->max_spread = std::max(p->max_spread, spread);
        const int rl = p->TT + spread;
        rowlen.push_back(rl);
        max_rowlen = std::max(max_rowlen, rl);
        i = j;
    }
    p->ndt = (int)first.size();
    p->ntt = (int)((n + p->TT - 1) / p->TT);
    const int ecopies = 8 / esz;  // float rows are staged twice (8-byte aligned pair reads)
    p->row_stride = (max_rowlen + 3) & ~3;
    // one wrap per staged index needs rowlen + 1 <= n
    p->small_n = (int64_t)max_rowlen + 1 > n ? 1 : 0;
    const size_t per_chan = (size_t)ecopies * p->row_stride * esz + (size_t)p->tpt * 2;
    p->ncc = (int)std::max<int64_t>(1, std::min<int64_t>(nchan, (int64_t)(kLdsBudget / per_chan)));
    p->lds_bytes = (((size_t)p->ncc * p->tpt * 2 + 15) & ~(size_t)15) + (size_t)p->ncc * ecopies * p->row_stride * esz;
    if ((int64_t)p->ndt * p->ntt >= (int64_t(1) << 31)) {
        free_plan(p);
        pu::set_error("pu_plan_create: grid too large");
        return PU_EINVAL;
    }
    if (p->lds_bytes > 64 * 1024) {
        free_plan(p);
        pu::set_error("pu_plan_create: LDS row of %d elements does not fit", p->row_stride);
        return PU_EUNSUPPORTED;
    }

    auto upload = [](auto **dst, const auto &vec) -> int {
        const size_t bytes = vec.size() * sizeof(vec[0]);
        int rc = pu::hip_check(hipMalloc((void **)dst, std::max<size_t>(bytes, 16)), "hipMalloc(plan)");
        if (rc) return rc;
        return pu::hip_check(hipMemcpy(*dst, vec.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy(plan)");
    };
    int rc = PU_OK;
    if (!rc) rc = upload(&p->d_first, first);
    if (!rc) rc = upload(&p->d_count, count);
    if (!rc) rc = upload(&p->d_rowlen, rowlen);
    if (!rc) rc = upload(&p->d_base, base);
    if (!rc) rc = upload(&p->d_rel, rel);
    if (rc) {
        free_plan(p);
        return rc;
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
    const int64_t v[] = {p->ndm, p->ndt, p->ntt, p->tpt, p->TT, p->ncc,
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
    a.plane = plane;
    a.ld_plane = ld_plane;
    return dispatch(p, a, true, pu::as_stream(stream));
}

}  // extern "C"
