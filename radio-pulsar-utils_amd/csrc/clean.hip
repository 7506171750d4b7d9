// RFI-cleaning reductions and apply passes for gfx950 (MI355X).
//
// Replaces the 2-D array passes of the reference cleaning path
// (pulsarutils/clean.py:58-111, 114-133) with bit-exact HIP kernels.  The masks the
// reference derives are threshold comparisons on these reductions, so every sum is
// reproduced in numpy's exact order (SURVEY.md §8 a-R; oracle/numpy_order.py):
//
//   add.reduce over a contiguous row  = 0 + pw(block_0) + pw(block_1) + ...,
//       blocks of 8192 elements, pw = numpy pairwise_sum (8 strided accumulators
//       over 128-element leaves, halving splits at n/2 - (n/2)%8)
//   mean(0) / zero-DM light curve      = sequential over rows
//
// Everything is compiled with -ffp-contract=off: a fused multiply-add would change
// the rounding of x*f - mu and of the squared deviations.
//
// Kernels
//   rowsum_chunk_kernel  one workgroup per (row, full 8192 block): leaves read straight
//                        into registers, 8-accumulator leaf sums, in-order pairwise
//                        tree by xor-shuffles.
//   rowsum_tail_kernel   one lane per row for the trailing partial block (irregular
//                        pairwise tree; compile-time-bounded recursion).
//   rowsum_combine       sequential 0 + block sums (+ true_divide by the count).
//   colmean_kernel       V adjacent columns per lane, rows in order (clean.py:77).
//   gauss_lds_kernel     scipy correlate1d symmetric order, mode 'reflect' (:79), from
//                        an LDS window (gauss_kernel: direct form for huge radii).
//   apply_kernel         (x*f - mu)/mu, bad rows zeroed, optional column mean (:81-94),
//                        V adjacent columns per lane.
#include <atomic>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "pu_common.h"

namespace {

constexpr int kBlock = 8192;   // numpy ufunc buffer size
constexpr int kLeaf = 128;     // numpy PW_BLOCKSIZE
constexpr int kScaleRows = 16;  // rows per workgroup of the scaled (MODE 2) row sums
                                // (C4 sweep: f32 191 vs 206 us at 4; u8 73 vs 86 us)

template <typename Tin, typename Ta, int MODE>
__device__ __forceinline__ Ta load_val(const Tin *row, int64_t t, Ta center, const double *scale)
{
    if constexpr (MODE == 0) {
        return static_cast<Ta>(row[t]);
    } else if constexpr (MODE == 1) {
        const Ta d = static_cast<Ta>(row[t]) - center;
        return d * d;
    } else if constexpr (MODE == 4) {
        const Ta v = static_cast<Ta>(row[t]);
        return v * v;
    } else {
        return static_cast<Ta>(static_cast<double>(row[t]) * scale[t]);
    }
}

// numpy pairwise_sum over [off, off+n) of a row, one lane.  DEPTH bounds the
// recursion at compile time (n <= 8192 needs < 10 levels).
template <typename Tin, typename Ta, int MODE, int DEPTH>
__device__ Ta pairwise_lane(const Tin *row, int64_t off, int64_t n, Ta center, const double *scale)
{
    if (n < 8) {
        Ta r = Ta(0);
        for (int64_t i = 0; i < n; ++i) r += load_val<Tin, Ta, MODE>(row, off + i, center, scale);
        return r;
    }
    if constexpr (DEPTH > 0) {
        if (n > kLeaf) {
            int64_t n2 = n / 2;
            n2 -= n2 % 8;
            const Ta l = pairwise_lane<Tin, Ta, MODE, DEPTH - 1>(row, off, n2, center, scale);
            const Ta r = pairwise_lane<Tin, Ta, MODE, DEPTH - 1>(row, off + n2, n - n2, center, scale);
            return l + r;
        }
    }
    Ta r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = load_val<Tin, Ta, MODE>(row, off + j, center, scale);
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += load_val<Tin, Ta, MODE>(row, off + i + j, center, scale);
    Ta res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += load_val<Tin, Ta, MODE>(row, off + i, center, scale);
    return res;
}

// V consecutive elements moved by one global load / store instruction.
template <typename T, int V>
struct alignas(sizeof(T) * V) Vec {
    T v[V];
};

template <typename T, int V>
__device__ __forceinline__ Vec<T, V> load_vec(const T *p)
{
    return *reinterpret_cast<const Vec<T, V> *>(p);
}

// load_val on an element already in registers (s = scale[t] for MODE 2).
template <typename Tin, typename Ta, int MODE>
__device__ __forceinline__ Ta elem_val(Tin x, Ta center, double s)
{
    if constexpr (MODE == 0) {
        return static_cast<Ta>(x);
    } else if constexpr (MODE == 1) {
        const Ta d = static_cast<Ta>(x) - center;
        return d * d;
    } else if constexpr (MODE == 4) {
        const Ta v = static_cast<Ta>(x);
        return v * v;
    } else {
        return static_cast<Ta>(static_cast<double>(x) * s);
    }
}

// Full 8192-element blocks: 64 leaves of 128, read straight into registers.
// Thread (b = tid/4, q = tid%4) owns accumulators r[2q], r[2q+1] of leaf b and loads
// its 16 element pairs (stride 8) with all loads in flight; the leaf total is
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) via two xor-shuffles.  The 64 leaves combine
// as the perfect binary tree pairwise_sum builds for n = 8192: leaf distances 1..8
// are lane distances 4..32 inside a wave (left + right at the even lane), the last
// two levels are (W0+W1)+(W2+W3) over the four waves.  PAIR: element pairs (and
// the scale pairs of MODE 2) are single 2-element vector loads.  A workgroup sums
// the same block of R consecutive rows, so MODE 2 reads its scale pairs once per R
// rows instead of once per row.
//
// MOM (MODE 0, pu_row_moments): the same pass also sums, in float64 and in any order,
// d = x - c and d^2 with c = the row's first element - the shifted moments from which
// measure_channel_variability's std is certified without a second pass (clean.py).
template <typename Tin, typename Ta, int MODE, bool PAIR, int R, bool MOM = false>
__global__ void __launch_bounds__(256)
rowsum_chunk_kernel(const Tin *__restrict__ x, int64_t ld, int64_t nrows, int64_t nfull, int64_t nblk_row,
                    const Ta *__restrict__ centers, const double *__restrict__ scale,
                    Ta *__restrict__ block_sums, double *__restrict__ moments = nullptr)
{
    // mom_tot has one slot per wave, not per row, and only row0's moments are stored
    static_assert(!MOM || R == 1, "rowsum_chunk_kernel: MOM needs R == 1");
    __shared__ Ta wave_tot[R][4];
    __shared__ double mom_tot[2][4];
    const int64_t row0 = (blockIdx.x / nfull) * R;
    const int64_t blk = blockIdx.x % nfull;
    const int tid = threadIdx.x;
    const int b = tid >> 2, q = tid & 3;
    const int64_t e0 = blk * kBlock + b * kLeaf + 2 * q;
    double sa[16], sc[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        if constexpr (MODE == 2 && PAIR) {
            const Vec<double, 2> s = load_vec<double, 2>(scale + e0 + 8 * m);
            sa[m] = s.v[0];
            sc[m] = s.v[1];
        } else if constexpr (MODE == 2) {
            sa[m] = scale[e0 + 8 * m];
            sc[m] = scale[e0 + 8 * m + 1];
        } else {
            sa[m] = sc[m] = 0.0;
        }
    }
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
        const int64_t row = row0 + rr;
        if (row >= nrows) break;
        const Tin *rp = x + row * ld + e0;
        const Ta center = MODE == 1 ? centers[row] : Ta(0);
        Tin a[16], c[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            if constexpr (PAIR) {
                const Vec<Tin, 2> p = load_vec<Tin, 2>(rp + 8 * m);
                a[m] = p.v[0];
                c[m] = p.v[1];
            } else {
                a[m] = rp[8 * m];
                c[m] = rp[8 * m + 1];
            }
        }
        if constexpr (sizeof(Tin) == 1 && MODE == 0) {
            // 8-bit sums (round 5): every partial sum of bytes - and of (x - c) and (x - c)^2 -
            // is an integer far below 2^53, so the float64 sums are exact in ANY order and
            // integer adds give the same values bit for bit, at a fraction of the float64
            // work (the moments pass was bound by it: 3.3 TB/s of its 8-bit reads)
            uint32_t si = 0;
#pragma unroll
            for (int m = 0; m < 16; ++m) si += (uint32_t)a[m] + (uint32_t)c[m];
#pragma unroll
            for (int s = 1; s < 64; s <<= 1) si += __shfl_xor(si, s, 64);  // <= 64 * 32 * 255
            if ((tid & 63) == 0) wave_tot[rr][tid >> 6] = static_cast<Ta>(si);
            if constexpr (MOM) {
                const int cs = (int)x[row * ld];
                int m1 = 0;
                uint32_t m2 = 0;
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    const int da = (int)a[m] - cs, dc = (int)c[m] - cs;
                    m1 += da + dc;
                    m2 += (uint32_t)(da * da) + (uint32_t)(dc * dc);
                }
#pragma unroll
                for (int s = 1; s < 64; s <<= 1) {  // |m1| <= 64 * 32 * 255, m2 <= 64 * 32 * 255^2 < 2^32
                    m1 += __shfl_xor(m1, s, 64);
                    m2 += __shfl_xor(m2, s, 64);
                }
                if ((tid & 63) == 0) {
                    mom_tot[0][tid >> 6] = static_cast<double>(m1);
                    mom_tot[1][tid >> 6] = static_cast<double>(m2);
                }
            }
            continue;
        }
        Ta r0 = elem_val<Tin, Ta, MODE>(a[0], center, sa[0]);
        Ta r1 = elem_val<Tin, Ta, MODE>(c[0], center, sc[0]);
#pragma unroll
        for (int m = 1; m < 16; ++m) {
            r0 += elem_val<Tin, Ta, MODE>(a[m], center, sa[m]);
            r1 += elem_val<Tin, Ta, MODE>(c[m], center, sc[m]);
        }
        Ta t = r0 + r1;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) t += __shfl_xor(t, s, 64);
        if ((tid & 63) == 0) wave_tot[rr][tid >> 6] = t;
        if constexpr (MOM) {
            const double cs = static_cast<double>(x[row * ld]);
            double m1 = 0.0, m2 = 0.0;
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const double da = static_cast<double>(a[m]) - cs, dc = static_cast<double>(c[m]) - cs;
                m1 += da + dc;
                m2 += da * da + dc * dc;
            }
#pragma unroll
            for (int s = 1; s < 64; s <<= 1) {
                m1 += __shfl_xor(m1, s, 64);
                m2 += __shfl_xor(m2, s, 64);
            }
            if ((tid & 63) == 0) {
                mom_tot[0][tid >> 6] = m1;
                mom_tot[1][tid >> 6] = m2;
            }
        }
    }
    __syncthreads();
    if (tid < R && row0 + tid < nrows)
        block_sums[(row0 + tid) * nblk_row + blk] =
            (wave_tot[tid][0] + wave_tot[tid][1]) + (wave_tot[tid][2] + wave_tot[tid][3]);
    if constexpr (MOM) {
        if (tid < 2 && row0 < nrows)
            moments[(row0 * nblk_row + blk) * 2 + tid] =
                (mom_tot[tid][0] + mom_tot[tid][1]) + (mom_tot[tid][2] + mom_tot[tid][3]);
    }
}

template <typename Tin, typename Ta, int MODE, bool MOM = false>
__global__ void __launch_bounds__(64)
rowsum_tail_kernel(const Tin *__restrict__ x, int64_t ld, int64_t nrows, int64_t n, int64_t nfull,
                   int64_t nblk_row, const Ta *__restrict__ centers, const double *__restrict__ scale,
                   Ta *__restrict__ block_sums, double *__restrict__ moments = nullptr)
{
    const int64_t row = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (row >= nrows) return;
    const Ta center = MODE == 1 ? centers[row] : Ta(0);
    const int64_t off = nfull * kBlock;
    block_sums[row * nblk_row + nfull] =
        pairwise_lane<Tin, Ta, MODE, 10>(x + row * ld, off, n - off, center, scale);
    if constexpr (MOM) {
        const double cs = static_cast<double>(x[row * ld]);
        double m1 = 0.0, m2 = 0.0;
        for (int64_t i = off; i < n; ++i) {
            const double d = static_cast<double>(x[row * ld + i]) - cs;
            m1 += d;
            m2 += d * d;
        }
        moments[(row * nblk_row + nfull) * 2] = m1;
        moments[(row * nblk_row + nfull) * 2 + 1] = m2;
    }
}

// pu_row_moments' combine, one launch (round 5: two before): per row the block sums in
// block order into the mean (rowsum_combine's arithmetic) and (c, sum(x - c),
// sum((x - c)^2)), c = the row's first element, from the per-block moment pairs (float64).
template <typename Tin, typename Ta>
__global__ void row_moments_combine(const Ta *__restrict__ block_sums, const double *__restrict__ blk,
                                    const Tin *__restrict__ x, int64_t ld, int64_t nrows, int64_t nblk_row,
                                    double divisor, Ta *__restrict__ means, double *__restrict__ out)
{
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    Ta acc = Ta(0);
    double m1 = 0.0, m2 = 0.0;
    // unrolled: 24 independent loads in flight per step (one at a time, the dependent adds
    // put every load's latency in series: 13 us for C4's 1024 rows x 32 blocks)
#pragma unroll 8
    for (int64_t k = 0; k < nblk_row; ++k) {
        acc += block_sums[row * nblk_row + k];
        m1 += blk[(row * nblk_row + k) * 2];
        m2 += blk[(row * nblk_row + k) * 2 + 1];
    }
    means[row] = static_cast<Ta>(static_cast<double>(acc) / divisor);
    out[row * 3] = static_cast<double>(x[row * ld]);
    out[row * 3 + 1] = m1;
    out[row * 3 + 2] = m2;
}

template <typename Ta>
__global__ void rowsum_combine(const Ta *__restrict__ block_sums, int64_t nrows, int64_t nblk_row,
                               double divisor, Ta *__restrict__ out)
{
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= nrows) return;
    Ta acc = Ta(0);
#pragma unroll 8
    for (int64_t k = 0; k < nblk_row; ++k) acc += block_sums[row * nblk_row + k];
    if (divisor > 0) acc = static_cast<Ta>(static_cast<double>(acc) / divisor);
    out[row] = acc;
}

// Column passes: a lane owns V adjacent columns and walks the rows in order (the
// numpy order of mean(0) and of the row loop of clean.py:81-94).  Per-row scalars
// (skip flag, channel mean) are staged in LDS per chunk of kRowChunk rows.
constexpr int kRowChunk = 4096;
constexpr int kBatchBytes = 128;  // per lane and register buffer: U = kBatchBytes / (V * elem)
constexpr int kMaxBatchRows = 32;

// Rows [0, rn) of a column strip, in order: batches of U rows alternate between two
// register buffers, the next batch's loads issued before the current batch is
// consumed (no register copies, so a wait never covers the batch in flight).
template <typename Tin, int V, typename Body, int BB = kBatchBytes>
__device__ __forceinline__ void walk_rows(const Tin *p, int64_t ld, int rn, Body &&body)
{
    constexpr int U = std::max(1, std::min(kMaxBatchRows, BB / (V * (int)sizeof(Tin))));
    Vec<Tin, V> a[U], b[U];
    auto load = [&](Vec<Tin, V>(&dst)[U], int i0) {
        if (i0 + U <= rn) {
#pragma unroll
            for (int k = 0; k < U; ++k) dst[k] = load_vec<Tin, V>(p + (int64_t)(i0 + k) * ld);
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k)
                if (i0 + k < rn) dst[k] = load_vec<Tin, V>(p + (int64_t)(i0 + k) * ld);
        }
    };
    auto run = [&](Vec<Tin, V>(&src)[U], int i0) {
        if (i0 + U <= rn) {
#pragma unroll
            for (int k = 0; k < U; ++k) body(i0 + k, src[k]);
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k)
                if (i0 + k < rn) body(i0 + k, src[k]);
        }
    };
    load(a, 0);
    for (int i0 = 0; i0 < rn; i0 += 2 * U) {
        if (i0 + U < rn) load(b, i0 + U);
        run(a, i0);
        if (i0 + 2 * U < rn) load(a, i0 + 2 * U);
        if (i0 + U < rn) run(b, i0 + U);
    }
}

// Skipped rows add +0.0 (a select, not a branch): acc starts at +0.0 and never
// becomes -0.0 under round-to-nearest, so acc + 0.0 == acc bit for bit, and NaN or
// Inf in a skipped row never reaches the sum.
template <typename Tin, int V, int BB>
__global__ void __launch_bounds__(256)
colmean_kernel(const Tin *__restrict__ x, int64_t nrows, int64_t col0, int64_t ncols, int64_t ld,
               const uint8_t *__restrict__ skip, double *__restrict__ out)
{
    __shared__ uint8_t sk[kRowChunk];
    const int64_t c = col0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
    const bool active = c < col0 + ncols;
    double acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.0;
    int64_t ngood = 0;
    auto body_fn = [&](int i, const Vec<Tin, V> &v) {
        const bool s = sk[i] != 0;
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += s ? 0.0 : static_cast<double>(v.v[j]);
    };
    for (int64_t r0 = 0; r0 < nrows; r0 += kRowChunk) {
        const int rn = (int)(nrows - r0 < kRowChunk ? nrows - r0 : kRowChunk);
        __syncthreads();
        for (int i = threadIdx.x; i < rn; i += 256) sk[i] = skip ? skip[r0 + i] : 0;
        __syncthreads();
        for (int i = 0; i < rn; ++i) ngood += sk[i] ? 0 : 1;
        if (!active) continue;
        walk_rows<Tin, V, decltype(body_fn) &, BB>(x + r0 * ld + c, ld, rn, body_fn);
    }
    if (!active) return;
#pragma unroll
    for (int j = 0; j < V; ++j) out[c + j] = acc[j] / static_cast<double>(ngood);
}

// 8-bit column sums by row segments.  Every partial sum of 8-bit values is an integer
// (< 2^53), so float64 accumulation is exact in any order: the sequential chain of
// colmean_kernel and a sum of per-segment integer sums give the same bits.  Segments of
// kColSegRows rows fit u16 (256 x 255 = 65280), two columns per dword lane half
// (bytes 0/2 and 1/3 masked with 0x00ff00ff: the halves never carry into each other), so a
// row of 8 columns costs one 8-byte load and four adds.  The (up to 4) u16 segment sums of
// column c are written into out[c]'s 8 bytes; colsum_u8_finish_kernel adds them and divides
// in place.  4 x the lanes of the row-sequential kernel for the same bytes.
constexpr int kColSegRows = 256;
constexpr int kColSegMax = 4;

__global__ void __launch_bounds__(256)
colsum_u8_seg_kernel(const uint8_t *__restrict__ x, int64_t nrows, int64_t ncols, int64_t ld,
                     const uint8_t *__restrict__ skip, uint16_t *__restrict__ part)
{
    __shared__ uint8_t sk[kColSegRows];
    const int seg = blockIdx.y;
    const int64_t r0 = (int64_t)seg * kColSegRows;
    const int rn = (int)(nrows - r0 < kColSegRows ? nrows - r0 : kColSegRows);
    if ((int)threadIdx.x < rn) sk[threadIdx.x] = skip ? skip[r0 + threadIdx.x] : 0;
    __syncthreads();
    const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (c >= ncols) return;
    const uint8_t *p = x + r0 * ld + c;
    uint32_t a02 = 0, a13 = 0, a46 = 0, a57 = 0;  // u16 pairs: columns (0,2), (1,3), (4,6), (5,7)
    constexpr int B = 16;                          // rows in flight per lane
    for (int i0 = 0; i0 < rn; i0 += B) {
        uint2 v[B];
#pragma unroll
        for (int k = 0; k < B; ++k)
            if (i0 + k < rn) v[k] = *reinterpret_cast<const uint2 *>(p + (int64_t)(i0 + k) * ld);
#pragma unroll
        for (int k = 0; k < B; ++k) {
            if (i0 + k < rn && !sk[i0 + k]) {
                a02 += v[k].x & 0x00ff00ffu;
                a13 += (v[k].x >> 8) & 0x00ff00ffu;
                a46 += v[k].y & 0x00ff00ffu;
                a57 += (v[k].y >> 8) & 0x00ff00ffu;
            }
        }
    }
    uint16_t *q = part + c * kColSegMax + seg;  // out[c] viewed as 4 x u16
    const uint32_t s[8] = {a02 & 0xffffu, a13 & 0xffffu, a02 >> 16, a13 >> 16,
                           a46 & 0xffffu, a57 & 0xffffu, a46 >> 16, a57 >> 16};
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j * kColSegMax] = (uint16_t)s[j];
}

__global__ void __launch_bounds__(256)
colsum_u8_finish_kernel(double *__restrict__ out, int64_t ncols, int nseg, int64_t nrows,
                        const uint8_t *__restrict__ skip)
{
    __shared__ int cnt[256];
    int good = 0;
    for (int64_t r = threadIdx.x; r < nrows; r += 256) good += (skip && skip[r]) ? 0 : 1;
    cnt[threadIdx.x] = good;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) cnt[threadIdx.x] += cnt[threadIdx.x + off];
        __syncthreads();
    }
    const double ngood = (double)cnt[0];
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= ncols) return;
    const uint64_t w = reinterpret_cast<const uint64_t *>(out)[c];
    uint32_t tot = 0;
    for (int k = 0; k < nseg; ++k) tot += (uint32_t)((w >> (16 * k)) & 0xffffu);
    out[c] = (double)tot / ngood;
}

__device__ __forceinline__ int64_t reflect_index(int64_t i, int64_t n)
{
    // scipy 'reflect' (d c b a | a b c d | d c b a): period 2n, half-sample symmetric
    const int64_t p = 2 * n;
    int64_t m = i % p;
    if (m < 0) m += p;
    return m >= n ? p - 1 - m : m;
}

// Direct form (radius too large for the LDS window).
__global__ void gauss_kernel(const double *__restrict__ x, int64_t n, const double *__restrict__ w,
                             int64_t r, double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double acc = x[i] * w[r];
    for (int64_t jj = -r; jj < 0; ++jj)
        acc += (x[reflect_index(i + jj, n)] + x[reflect_index(i - jj, n)]) * w[r + jj];
    out[i] = acc;
}

// LDS form: a workgroup stages its 256 outputs' window x[i0-r, i0+256+r) (reflected
// once, at staging) and the r+1 weights, then every tap is two LDS reads and one
// broadcast read, in scipy's symmetric order.
constexpr int kGaussMaxR = 2048;

__global__ void __launch_bounds__(256)
gauss_lds_kernel(const double *__restrict__ x, int64_t n, const double *__restrict__ w, int r,
                 double *__restrict__ out)
{
    extern __shared__ double gsm[];
    double *ws = gsm;              // r + 1 weights
    double *xs = gsm + (r + 1);    // 256 + 2r window
    const int64_t i0 = (int64_t)blockIdx.x * 256;
    for (int k = threadIdx.x; k <= r; k += 256) ws[k] = w[k];
    for (int k = threadIdx.x; k < 256 + 2 * r; k += 256) {
        const int64_t g = i0 - r + k;
        xs[k] = x[(g >= 0 && g < n) ? g : reflect_index(g, n)];
    }
    __syncthreads();
    const int64_t i = i0 + threadIdx.x;
    if (i >= n) return;
    const double *xc = xs + r + threadIdx.x;
    double acc = xc[0] * ws[r];
    for (int jj = -r; jj < 0; ++jj) acc += (xc[jj] + xc[-jj]) * ws[r + jj];
    out[i] = acc;
}

// Pair form (r <= kGaussMaxR): each thread computes TWO adjacent outputs i, i+1 and steps
// two taps at a time through 16-B LDS reads (x pairs and weight pairs): per 2 taps one
// new left pair, one new right pair and one weight pair serve 4 output-taps, 3 LDS reads
// where the one-output form needs 6.  Same per-output order as scipy (and as
// gauss_lds_kernel): acc = x[i] w[r], then acc += (x[i+j] + x[i-j]) w[r+j], j = -r..-1.
constexpr int kGaussPad = 2;
typedef double f64x2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256)
gauss_pair_kernel(const double *__restrict__ x, int64_t n, const double *__restrict__ w, int r,
                  double *__restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) double gsm2[];
    const int wn = (r + 2) & ~1;  // weights padded to an even count: the window stays 16-B aligned
    double *ws = gsm2;
    double *xs = gsm2 + wn;       // x[i0 - r - pad, i0 + 512 + r + pad), reflected at staging
    const int64_t i0 = (int64_t)blockIdx.x * 512;
    const int span = 512 + 2 * r + 2 * kGaussPad;
    for (int k = threadIdx.x; k < wn; k += 256) ws[k] = k <= r ? w[k] : 0.0;
    for (int k = threadIdx.x; k < span; k += 256) {
        const int64_t g = i0 - r - kGaussPad + k;
        xs[k] = x[(g >= 0 && g < n) ? g : reflect_index(g, n)];
    }
    __syncthreads();
    const int t2 = 2 * (int)threadIdx.x;
    const int64_t i = i0 + t2;
    const double *xc = xs + t2 + r + kGaussPad;  // xc[q] = x[i + q]; xc + j is 16-B aligned for j = -r + 2m
    double a0 = xc[0] * ws[r], a1 = xc[1] * ws[r];
    int j = -r;
    f64x2 L01 = *reinterpret_cast<const f64x2 *>(xc + j);  // x[i+j], x[i+j+1]
    f64x2 R23 = *reinterpret_cast<const f64x2 *>(xc - j);  // x[i-j], x[i-j+1]
    for (; j + 1 < 0; j += 2) {
        const f64x2 L23 = *reinterpret_cast<const f64x2 *>(xc + j + 2);      // x[i+j+2], x[i+j+3]
        const f64x2 R01 = *reinterpret_cast<const f64x2 *>(xc - j - 2);      // x[i-j-2], x[i-j-1]
        const f64x2 wp = *reinterpret_cast<const f64x2 *>(ws + r + j);       // w[r+j], w[r+j+1]
        a0 += (L01.x + R23.x) * wp.x;  // tap j
        a1 += (L01.y + R23.y) * wp.x;
        a0 += (L01.y + R01.y) * wp.y;  // tap j + 1
        a1 += (L23.x + R23.x) * wp.y;
        L01 = L23;
        R23 = R01;
    }
    if (j < 0) {  // odd r: the last tap, j = -1
        a0 += (L01.x + R23.x) * ws[r - 1];
        a1 += (L01.y + R23.y) * ws[r - 1];
    }
    if (i < n) out[i] = a0;
    if (i + 1 < n) out[i + 1] = a1;
}

// Quad form (round 4, the default for r <= kGaussMaxR): each thread computes FOUR adjacent
// outputs i..i+3 from two sliding register windows, left x[i+j .. i+j+3] and right
// x[i-j .. i-j+3]; per two taps one new 16-B pair enters each window, so the LDS traffic
// per output-tap is 4 B (pair form: 12 B) plus a broadcast weight pair.  The next two
// taps' pairs are read one iteration ahead.  1024 outputs per workgroup (one workgroup per CU
// at n = 2^18, one wave per SIMD: the f64 adds, not LDS, set the pace).  Per output the
// order is scipy's: acc = x[i] w[r], then acc += (x[i+j] + x[i-j]) w[r+j], j = -r..-1.
constexpr int kGaussQuadThreads = 256;

// One workgroup's 4 T outputs [i0, i0 + 4 T) into a[4] (thread t: outputs i0 + 4 t + q).
// gsm4: LDS of ((r + 2) & ~1) + 4 T + 2 r + 2 kGaussPad doubles.  Returns after the last
// LDS read of the workgroup's staging only once every thread has passed the staging barrier
// (callers that restage must __syncthreads() first).
template <int T>
__device__ __forceinline__ void gauss_quad_segment(const double *__restrict__ x, int64_t n, const double *__restrict__ w,
                                                   int r, int64_t i0, double *gsm4, double (&a)[4])
{
    const int wn = (r + 2) & ~1;  // weights padded to an even count: the window stays 16-B aligned
    double *ws = gsm4;
    double *xs = gsm4 + wn;       // x[i0 - r - pad, i0 + 1024 + r + pad), reflected at staging
    const int span = (4 * T) + 2 * r + 2 * kGaussPad;
    for (int k = threadIdx.x; k < wn; k += T) ws[k] = k <= r ? w[k] : 0.0;
    const int64_t g0 = i0 - r - kGaussPad;
    if (g0 >= 0 && g0 + span <= n) {  // interior workgroup (uniform): no reflection
        for (int k = threadIdx.x; k < span; k += T) xs[k] = x[g0 + k];
    } else {
        for (int k = threadIdx.x; k < span; k += T) {
            const int64_t g = g0 + k;
            xs[k] = x[(g >= 0 && g < n) ? g : reflect_index(g, n)];
        }
    }
    __syncthreads();
    const int t4 = 4 * (int)threadIdx.x;
    // xc[q] = x[i + q]; xc + m is 16-B aligned whenever m + r is even (pad even, t4 even)
    const double *xc = xs + t4 + r + kGaussPad;
    auto pair = [&](int m) { return *reinterpret_cast<const f64x2 *>(xc + m); };
    auto wpair = [&](int m) { return *reinterpret_cast<const f64x2 *>(ws + r + m); };  // w[r+m], w[r+m+1]
    const double wr = ws[r];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = xc[q] * wr;
    int j = -r;
    f64x2 l01 = pair(j), l23 = pair(j + 2);    // left  window xc[j .. j+3]
    f64x2 r01 = pair(-j), r23 = pair(-j + 2);  // right window xc[-j .. -j+3]
    // the next two taps' window and weight pairs are read one iteration ahead (one wave per
    // SIMD: nothing else covers the LDS latency)
    f64x2 p = {0.0, 0.0}, s = {0.0, 0.0}, wp = {0.0, 0.0};
    if (r >= 2) {
        p = pair(j + 4);   // xc[j+4], xc[j+5]
        s = pair(-j - 2);  // xc[-j-2], xc[-j-1]
        wp = wpair(j);
    }
#pragma unroll 2
    for (; j + 1 < 0; j += 2) {
        const int jn = j + 3 < 0 ? j + 2 : j;  // the last iteration reloads its own (in bounds)
        const f64x2 pn = pair(jn + 4), sn = pair(-jn - 2), wpn = wpair(jn);
        const double w0 = wp.x, w1 = wp.y;
        // tap j: left xc[j+q], right xc[q-j]
        a[0] += (l01.x + r01.x) * w0;
        a[1] += (l01.y + r01.y) * w0;
        a[2] += (l23.x + r23.x) * w0;
        a[3] += (l23.y + r23.y) * w0;
        // tap j+1: left xc[j+1+q], right xc[q-j-1]
        a[0] += (l01.y + s.y) * w1;
        a[1] += (l23.x + r01.x) * w1;
        a[2] += (l23.y + r01.y) * w1;
        a[3] += (p.x + r23.x) * w1;
        l01 = l23;
        l23 = p;
        r23 = r01;
        r01 = s;
        p = pn;
        s = sn;
        wp = wpn;
    }
    if (j < 0) {  // odd r: the last tap, j = -1
        const double w0 = ws[r - 1];
        a[0] += (l01.x + r01.x) * w0;
        a[1] += (l01.y + r01.y) * w0;
        a[2] += (l23.x + r23.x) * w0;
        a[3] += (l23.y + r23.y) * w0;
    }
}

template <int T>
__global__ void __launch_bounds__(T)
gauss_quad_kernel(const double *__restrict__ x, int64_t n, const double *__restrict__ w, int r,
                  double *__restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) double gsm4[];
    const int64_t i0 = (int64_t)blockIdx.x * (4 * T);
    double a[4];
    gauss_quad_segment<T>(x, n, w, r, i0, gsm4, a);
    const int64_t i = i0 + 4 * (int)threadIdx.x;
    if (i + 3 < n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
        *reinterpret_cast<f64x2 *>(out + i) = f64x2{a[0], a[1]};
        *reinterpret_cast<f64x2 *>(out + i + 2) = f64x2{a[2], a[3]};
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (i + q < n) out[i + q] = a[q];
    }
}

__global__ void ratio_kernel(double num, const double *__restrict__ x, int64_t n, double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = num / x[i];
}

// (x*f - mu)/mu per element, bad channels written as 0.0, column mean of the result
// accumulated over channels in order.  Same column layout as colmean_kernel; the
// channel means and bad flags are staged in LDS per row chunk.
//
// ZDM (opt-in zero-DM subtraction, no reference counterpart: clean.py:77-82 only
// divides by the smoothed zero-DM series): the strip is walked twice.  The first walk
// sums the normalised values over channels in order (bad channels add +0.0, so the sum
// is the good channels' sum bit for bit); the second writes e - S[t]/ngood for good
// channels and 0.0 for bad ones.  col_means (the cut_outliers series) is S[t]/nchan of
// the normalised data BEFORE the subtraction, as without ZDM.
template <typename Tin, int V, bool NT, bool ZDM, int BB = kBatchBytes>
__global__ void __launch_bounds__(256)
apply_kernel(const Tin *__restrict__ x, int64_t nchan, int64_t col0, int64_t ncols, int64_t ld,
             const double *__restrict__ factor, const double *__restrict__ spec,
             const uint8_t *__restrict__ bad, double *__restrict__ out, int64_t ld_out,
             double *__restrict__ col_means, int64_t ngood)
{
    __shared__ double mus[kRowChunk];
    __shared__ uint8_t bads[kRowChunk];
    const int64_t c = col0 + ((int64_t)blockIdx.x * 256 + threadIdx.x) * V;
    const bool active = c < col0 + ncols;
    double f[V], acc[V], zsub[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        f[j] = active ? factor[c + j] : 0.0;
        acc[j] = 0.0;
        zsub[j] = 0.0;
    }
    auto stage = [&](int64_t r0, int rn) {
        __syncthreads();
        for (int i = threadIdx.x; i < rn; i += 256) {
            mus[i] = spec[r0 + i];
            bads[i] = bad ? bad[r0 + i] : 0;
        }
        __syncthreads();
    };
    if constexpr (ZDM) {
        for (int64_t r0 = 0; r0 < nchan; r0 += kRowChunk) {
            const int rn = (int)(nchan - r0 < kRowChunk ? nchan - r0 : kRowChunk);
            stage(r0, rn);
            if (!active) continue;
            auto sum_fn = [&](int i, const Vec<Tin, V> &v) {
                const double mu = mus[i];
                const bool b = bads[i] != 0;
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    double e = static_cast<double>(v.v[j]) * f[j];
                    e = (e - mu) / mu;
                    acc[j] += b ? 0.0 : e;
                }
            };
            walk_rows<Tin, V, decltype(sum_fn) &, BB>(x + r0 * ld + c, ld, rn, sum_fn);
        }
#pragma unroll
        for (int j = 0; j < V; ++j) zsub[j] = ngood > 0 ? acc[j] / static_cast<double>(ngood) : 0.0;
    }
    for (int64_t r0 = 0; r0 < nchan; r0 += kRowChunk) {
        const int rn = (int)(nchan - r0 < kRowChunk ? nchan - r0 : kRowChunk);
        stage(r0, rn);
        if (!active) continue;
        double *o = out + r0 * ld_out + c;
        auto apply_fn = [&](int i, const Vec<Tin, V> &v) {
            const double mu = mus[i];
            const bool b = bads[i] != 0;
            Vec<double, V> res;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                double e = static_cast<double>(v.v[j]) * f[j];
                e = (e - mu) / mu;
                if constexpr (ZDM) {
                    res.v[j] = b ? 0.0 : e - zsub[j];
                } else {
                    res.v[j] = b ? 0.0 : e;
                    acc[j] += res.v[j];
                }
            }
            if constexpr (NT && V % 2 == 0) {
                // 16-byte non-temporal stores (round 3: one 8-byte store per column)
                typedef double f64x2 __attribute__((ext_vector_type(2)));
#pragma unroll
                for (int j = 0; j < V; j += 2)
                    __builtin_nontemporal_store(f64x2{res.v[j], res.v[j + 1]},
                                                reinterpret_cast<f64x2 *>(o + (int64_t)i * ld_out + j));
            } else if constexpr (NT) {
#pragma unroll
                for (int j = 0; j < V; ++j) __builtin_nontemporal_store(res.v[j], o + (int64_t)i * ld_out + j);
            } else {
                *reinterpret_cast<Vec<double, V> *>(o + (int64_t)i * ld_out) = res;
            }
        };
        walk_rows<Tin, V, decltype(apply_fn) &, BB>(x + r0 * ld + c, ld, rn, apply_fn);
    }
    if (!active || !col_means) return;
#pragma unroll
    for (int j = 0; j < V; ++j) col_means[c + j] = acc[j] / static_cast<double>(nchan);
}

// ---------------------------------------------------------------- cut_outliers
// clean.py:93-105 on the device.  Only the last window (16) of the reference loop
// survives: lc_rebin = uniform_filter1d(lc, 16) (mode reflect: window [i-8, i+7]),
// sd = np.std(lc_rebin[::16]), bad = lc_rebin > 5 sd | lc_rebin < -3 sd.
//
// scipy evaluates lc_rebin as a sequential running sum (tmp += (x[i+7] - x[i-9]) / 16),
// a chain no parallel order reproduces bit for bit.  The kernels instead compute each
// window sum directly (u[i]) and CERTIFY every decision: with L = max |lc|, both the
// chain value v[i] and u[i] lie within (2n + 64) 2^-53 L of the exact windowed mean
// (per-step rounding of the chain <= 1.5 2^-53 L, of the 16-term sum <= 16 2^-53 L),
// and |std(u) - std(v)| <= max |u - v| plus rounding.  A comparison is decided only
// when u is farther than that bound from the threshold; otherwise (or on NaN) the
// state's flag is raised and outlier_exact_kernel, on the same stream, recomputes the
// mask with scipy's running sum and numpy's std order (ws[0:4] then only reports that
// the exact path ran).  So the mask equals the reference's bit for bit either way.
struct OutlierState {
    uint32_t flag;             // 1: a decision was ambiguous or a value NaN (ABI: bytes 0-3)
    uint32_t nbad;             // bad time bins (ABI: bytes 4-7)
    unsigned long long lbits;  // max |lc| as ordered bits (non-negative doubles)
    double sd;
    double up, down;           // 5 sd, -3 sd
    double margin_up, margin_down;
};

__device__ __forceinline__ int64_t reflect_small(int64_t i, int64_t n)
{
    // scipy 'reflect' for |offset| <= n (windows of 16 at the ends)
    if (i < 0) i = -i - 1;
    if (i >= n) i = 2 * n - 1 - i;
    return i < 0 ? 0 : (i >= n ? n - 1 : i);
}

__global__ void __launch_bounds__(256)
outlier_window_kernel(const double *__restrict__ lc, int64_t n, double *__restrict__ u, double *__restrict__ u16,
                      OutlierState *st)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    double s = 0.0, a = 0.0;
    bool nan = false;
    if (i < n) {
        for (int j = -8; j < 8; ++j) s += lc[(i + j >= 0 && i + j < n) ? i + j : reflect_small(i + j, n)];
        u[i] = s / 16.0;
        if ((i & 15) == 0) u16[i >> 4] = s / 16.0;  // u[::16], compact for the std pass
        const double x = lc[i];
        nan = x != x;
        a = fabs(x);
    }
    // block max of |lc| (non-negative doubles order like their bit patterns)
    unsigned long long b = nan ? ~0ull : (unsigned long long)__double_as_longlong(a);
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(b, off, 64);
        b = o > b ? o : b;
    }
    __shared__ unsigned long long wm[4];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = wm[0];
        for (int w = 1; w < 4; ++w) m = wm[w] > m ? wm[w] : m;
        if (m == ~0ull) atomicOr(&st->flag, 1u);
        else atomicMax(&st->lbits, m);
    }
}

// Block-wide sum (1024 threads): wave sums by xor shuffles, then the 16 wave totals.
__device__ __forceinline__ double block_sum_1024(double v, double *red)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int t = threadIdx.x;
    __syncthreads();  // red is reused between calls
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) tot += red[w];
    return tot;
}

// One workgroup: sd = std(u[::16]) (two passes over the compact copy), thresholds and
// certification margins.  (Any summation order: the margins bound the difference.)
__global__ void __launch_bounds__(1024) outlier_std_kernel(const double *__restrict__ u16, int64_t n, OutlierState *st)
{
    __shared__ double red[16];
    const int t = threadIdx.x;
    const int64_t m = (n + 15) / 16;
    double s = 0.0;
    for (int64_t k = t; k < m; k += 1024) s += u16[k];
    const double mean = block_sum_1024(s, red) / (double)m;
    s = 0.0;
    for (int64_t k = t; k < m; k += 1024) {
        const double d = u16[k] - mean;
        s += d * d;
    }
    const double ss = block_sum_1024(s, red);
    if (t == 0) {
        const double sd = sqrt(ss / (double)m);
        const double L = __longlong_as_double((long long)st->lbits);
        const double E = ((double)(2 * n + 64) * 0x1p-53) * L + 1e-300;  // |u - v| bound
        const double Es = E + 1e-12 * sd;                                  // |std(u) - std(v)| bound
        st->sd = sd;
        st->up = 5.0 * sd;
        st->down = -3.0 * sd;
        st->margin_up = E + 5.0 * Es + 1e-15 * (L + 5.0 * sd);
        st->margin_down = E + 3.0 * Es + 1e-15 * (L + 3.0 * sd);
        if (sd != sd) st->flag |= 1u;
    }
}

// Certified decisions, one lane per time bin: the mask, the flag (an ambiguous
// comparison raises it; outlier_exact_kernel then redoes the mask) and the list of the
// bad bins (st->nbad entries; one atomic per wave that has any, lanes in column order).
__global__ void __launch_bounds__(256)
outlier_mask_kernel(const double *__restrict__ u, int64_t n, OutlierState *st, uint8_t *__restrict__ mask,
                    int32_t *__restrict__ list)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint8_t b = 0;
    if (i < n) {
        const double v = u[i];
        const double du = v - st->up, dd = v - st->down;
        const bool amb = !(fabs(du) > st->margin_up) || !(fabs(dd) > st->margin_down);
        if (amb) atomicOr(&st->flag, 1u);
        b = (du > 0.0 || dd < 0.0) ? 1 : 0;
        mask[i] = b;
    }
    const uint64_t bal = __ballot(b != 0);
    if (!bal) return;
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == __ffsll((unsigned long long)bal) - 1) base = atomicAdd(&st->nbad, (uint32_t)__popcll(bal));
    base = __shfl(base, __ffsll((unsigned long long)bal) - 1, 64);
    if (b) list[base + __popcll(bal & ((uint64_t(1) << lane) - 1))] = (int32_t)i;
}

// numpy add.reduce of a contiguous double vector (0 + pairwise sums of 8192-element
// blocks) by one lane; each block is staged in LDS by the whole workgroup first.
__device__ double reduce_sum_staged(const double *__restrict__ a, int64_t m, double *stage)
{
    double acc = 0.0;
    for (int64_t b = 0; b < m; b += kBlock) {
        const int len = (int)(m - b < kBlock ? m - b : kBlock);
        __syncthreads();
        for (int k = threadIdx.x; k < len; k += blockDim.x) stage[k] = a[b + k];
        __syncthreads();
        if (threadIdx.x == 0) acc += pairwise_lane<double, double, 0, 10>(stage, 0, len, 0.0, nullptr);
    }
    return acc;  // valid in lane 0
}

// The reference's own arithmetic for the rare case (the flag is set: a certified decision
// was ambiguous, or the light curve holds NaN / inf), on the device so that the common
// path needs no host round trip (round 4; the host used to rerun scipy).  One
// workgroup:
//  * scipy.ndimage.uniform_filter1d(lc, 16) (mode 'reflect', origin 0): the running sum
//    tmp = (sum of the first window) / 16, then tmp += (x[i + 7] - x[i - 9]) / 16 - the
//    differences of a chunk by all lanes into LDS (each is scipy's single rounding),
//    the chain by lane 0 (its order is the whole point);
//  * np.std(lc_rebin[::16]): numpy's add.reduce order for the mean and for the squared
//    deviations (a compact copy in tmp);
//  * bad = lc_rebin > 5 sd | lc_rebin < -3 sd (NaN compares false, as in numpy).
// Restatement checked bit for bit against scipy / numpy on CPU
// (tests/test_oracle.py::test_cut_outliers_exact_restatement).
__device__ void outlier_exact_body(const double *__restrict__ lc, int64_t n, OutlierState *st, double *__restrict__ v,
                                   double *__restrict__ tmp, uint8_t *__restrict__ mask, int32_t *__restrict__ list)
{
    __shared__ double stage[kBlock];
    __shared__ double thr[2];
    constexpr int kSize = 16, kOrig = kSize / 2;  // window [i - 8, i + 7]
    const int t = threadIdx.x;
    auto ext = [&](int64_t k) { return lc[reflect_small(k - kOrig, n)]; };  // scipy's extended line
    double s = 0.0;
    if (t == 0) {
        for (int j = 0; j < kSize; ++j) s += ext(j);
        s /= (double)kSize;
        v[0] = s;
    }
    for (int64_t c0 = 1; c0 < n; c0 += kBlock) {
        const int len = (int)(n - c0 < kBlock ? n - c0 : kBlock);
        __syncthreads();
        for (int k = t; k < len; k += 256) stage[k] = (ext(c0 + k + kSize - 1) - ext(c0 + k - 1)) / (double)kSize;
        __syncthreads();
        if (t == 0)
            for (int k = 0; k < len; ++k) {
                s += stage[k];
                v[c0 + k] = s;
            }
    }
    __syncthreads();
    __threadfence_block();
    const int64_t m = (n + 15) / 16;
    for (int64_t k = t; k < m; k += 256) tmp[k] = v[16 * k];
    __threadfence_block();
    const double mean = reduce_sum_staged(tmp, m, stage) / (double)m;  // lane 0
    __syncthreads();
    if (t == 0) thr[0] = mean;
    __syncthreads();
    for (int64_t k = t; k < m; k += 256) {
        const double d = tmp[k] - thr[0];
        tmp[k] = d * d;
    }
    __threadfence_block();
    const double ss = reduce_sum_staged(tmp, m, stage);
    __syncthreads();
    if (t == 0) {
        const double sd = sqrt(ss / (double)m);
        thr[0] = 5.0 * sd;
        thr[1] = -3.0 * sd;
        st->sd = sd;
        st->up = thr[0];
        st->down = thr[1];
        st->nbad = 0;
        st->flag = 1;
    }
    __syncthreads();
    __threadfence_block();
    for (int64_t i = t; i < n; i += 256) {
        const double x = v[i];
        const uint8_t b = (x > thr[0] || x < thr[1]) ? 1 : 0;
        mask[i] = b;
        if (b) list[atomicAdd(&st->nbad, 1u)] = (int32_t)i;  // any order: the zeroing is idempotent
    }
}

__global__ void __launch_bounds__(256)
outlier_exact_kernel(const double *__restrict__ lc, int64_t n, OutlierState *st, double *__restrict__ v,
                     double *__restrict__ tmp, uint8_t *__restrict__ mask, int32_t *__restrict__ list, int force)
{
    if (!force && st->flag == 0) return;
    outlier_exact_body(lc, n, st, v, tmp, mask, list);
}

// Zero the plane's bad columns (the final list): one workgroup per row, the list's
// entries over the lanes (entries of a wave are consecutive columns of a burst, so the
// stores coalesce).  Row-major: each row's 2 MiB page is touched by one workgroup instead
// of once per 64-column block of bad bins (15 us -> a few at C4).
__global__ void __launch_bounds__(256)
outlier_zero_kernel(const int32_t *__restrict__ list, const OutlierState *st, double *__restrict__ out,
                    int64_t nrows, int64_t ld)
{
    const uint32_t nbad = st->nbad;
    double *row = out + (int64_t)blockIdx.x * ld;
    for (uint32_t k = threadIdx.x; k < nbad; k += 256) row[list[k]] = 0.0;
}

__global__ void zero_cols_kernel(double *out, int64_t nrows, int64_t ld, const int64_t *__restrict__ cols,
                                 int64_t ncols)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = blockIdx.y;
    for (int64_t rr = r; rr < nrows; rr += gridDim.y)
        if (k < ncols) out[rr * ld + cols[k]] = 0.0;
}

// ---------------------------------------------------------------- median
// np.median of a float64 series on the device (clean.py:80), so the factor pass
// does not wait on a host round trip.  Radix select over order-preserving 64-bit
// keys: six digit passes (11,11,11,11,11,9 bits, high to low) narrow the key
// prefixes of the two order statistics numpy averages (k = n/2-1 and n/2 for even
// n, n/2 twice for odd n).  Each pass is ONE histogram kernel (LDS bins, one global
// atomic add per non-empty bin and workgroup): its workgroups first select the
// previous pass's bin from that pass's global histogram themselves (every workgroup
// computes the same prefix; workgroup 0 records it), and clear the buffer the next
// pass will fill (three rotating buffers).  A one-workgroup final kernel selects the
// last digit.  The result is numpy's mean of the two values, add.reduce order:
// (0 + ((0 + a) + b)) / 2; any NaN gives NaN.  8 launches (was 14).
constexpr int kMedBitsMax = 11;
constexpr int kMedBins = 1 << kMedBitsMax;
constexpr int kMedPasses = 6;
constexpr int kMedBufs = 3;

struct MedState {
    uint64_t prefix[kMedPasses + 1][2];  // key prefix of each target before pass p
    int64_t k[kMedPasses + 1][2];        // its rank among the keys with that prefix
    uint32_t nan;
    uint32_t pad;
};

__host__ __device__ constexpr int med_shift(int p) { return 64 - kMedBitsMax * (p + 1) > 0 ? 64 - kMedBitsMax * (p + 1) : 0; }
__host__ __device__ constexpr int med_bits(int p) { return 64 - kMedBitsMax * p - med_shift(p); }

__device__ __forceinline__ uint64_t order_key(double d)
{
    const uint64_t u = static_cast<uint64_t>(__double_as_longlong(d));
    return (u >> 63) ? ~u : (u | (uint64_t(1) << 63));
}

__device__ __forceinline__ double key_value(uint64_t k)
{
    const uint64_t u = (k >> 63) ? (k & ~(uint64_t(1) << 63)) : ~k;
    return __longlong_as_double(static_cast<long long>(u));
}

__global__ void median_init_kernel(MedState *st, uint32_t *hist, int64_t n)
{
    const int t = threadIdx.x;
    if (t == 0) {
        st->prefix[0][0] = st->prefix[0][1] = 0;
        st->k[0][0] = (n % 2 == 0) ? n / 2 - 1 : n / 2;
        st->k[0][1] = n / 2;
        st->nan = 0;
    }
    for (int i = t; i < kMedBufs * 2 * kMedBins; i += blockDim.x) hist[i] = 0;
}

// Block-wide selection (256 threads): the bin of ``hj`` holding rank k; thread t owns
// bins [8t, 8t+8).  Returns (bin, rank inside the bin) to every thread.
__device__ void med_select_block(const uint32_t *hj, int64_t k, uint32_t *scan, int64_t *res, int &bin,
                                 int64_t &rem)
{
    const int t = threadIdx.x;
    uint32_t c[8], sum = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        c[b] = hj[8 * t + b];
        sum += c[b];
    }
    scan[t] = sum;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        const uint32_t v = t >= off ? scan[t - off] : 0;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
    }
    const int64_t before = (int64_t)scan[t] - sum;
    if (k >= before && k < before + (int64_t)sum) {
        int64_t r = k - before;
        int b = 0;
        while (r >= (int64_t)c[b]) r -= c[b++];
        res[0] = 8 * t + b;
        res[1] = r;
    }
    __syncthreads();
    bin = (int)res[0];
    rem = res[1];
    __syncthreads();
}

// Prefix and rank of both targets before pass ``pass`` (pass >= 1), from the previous
// pass's histogram.
__device__ void med_prefix(const MedState *st, const uint32_t *hist, int pass, uint32_t *scan, int64_t *res,
                           uint64_t (&pfx)[2], int64_t (&kk)[2])
{
    const uint32_t *hp = hist + (size_t)((pass - 1) % kMedBufs) * 2 * kMedBins;
    for (int j = 0; j < 2; ++j) {
        int bin;
        int64_t rem;
        med_select_block(hp + j * kMedBins, st->k[pass - 1][j], scan, res, bin, rem);
        pfx[j] = st->prefix[pass - 1][j] | ((uint64_t)bin << med_shift(pass - 1));
        kk[j] = rem;
    }
}

__global__ void __launch_bounds__(256)
median_hist_kernel(const double *__restrict__ x, int64_t n, MedState *st, uint32_t *hist, int pass)
{
    __shared__ uint32_t h[2][kMedBins];
    __shared__ uint32_t scan[256];
    __shared__ int64_t res[2];
    uint64_t pfx[2] = {0, 0};
    int64_t kk[2] = {st->k[0][0], st->k[0][1]};
    if (pass > 0) {
        med_prefix(st, hist, pass, scan, res, pfx, kk);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->prefix[pass][0] = pfx[0];
            st->prefix[pass][1] = pfx[1];
            st->k[pass][0] = kk[0];
            st->k[pass][1] = kk[1];
        }
    }
    // clear the buffer the NEXT pass accumulates into (nobody reads it during this pass)
    uint32_t *nxt = hist + (size_t)((pass + 1) % kMedBufs) * 2 * kMedBins;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < 2 * kMedBins; i += gridDim.x * 256) nxt[i] = 0;
    for (int i = threadIdx.x; i < 2 * kMedBins; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    const int shift = med_shift(pass), bits = med_bits(pass);
    const uint64_t dmask = (uint64_t(1) << bits) - 1;
    const int hs = shift + bits;  // bits above the digit must match the prefix
    uint32_t nans = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double d = x[i];
        if (d != d) {
            ++nans;
            continue;
        }
        const uint64_t k = order_key(d);
        const uint32_t dig = (uint32_t)((k >> shift) & dmask);
        if (hs >= 64 || (k >> hs) == (pfx[0] >> hs)) atomicAdd(&h[0][dig], 1u);
        if (hs >= 64 || (k >> hs) == (pfx[1] >> hs)) atomicAdd(&h[1][dig], 1u);
    }
    if (pass == 0 && nans) atomicAdd(&st->nan, nans);
    __syncthreads();
    uint32_t *cur = hist + (size_t)(pass % kMedBufs) * 2 * kMedBins;
    for (int i = threadIdx.x; i < 2 * kMedBins; i += 256) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(&cur[i], c);
    }
}

// One workgroup: the last digit, then numpy's mean of the two order statistics.
__global__ void __launch_bounds__(256) median_final_kernel(MedState *st, const uint32_t *hist, int64_t n,
                                                           double *out)
{
    __shared__ uint32_t scan[256];
    __shared__ int64_t res[2];
    uint64_t pfx[2];
    int64_t kk[2];
    med_prefix(st, hist, kMedPasses, scan, res, pfx, kk);
    if (threadIdx.x != 0) return;
    if (st->nan) {
        out[0] = __longlong_as_double(0x7ff8000000000000ll);
        return;
    }
    const double a = key_value(pfx[0]);
    if (n % 2 == 0) {
        const double b = key_value(pfx[1]);
        out[0] = (0.0 + ((0.0 + a) + b)) / 2.0;
    } else {
        out[0] = (0.0 + (0.0 + a)) / 1.0;
    }
}

// ---------------------------------------------------------------- grid barrier
// A monotonic arrival counter for the one-launch cut_outliers (every wave's vmcnt(0), the
// workgroup barrier, lane 0's agent release, the arrival, a relaxed poll with s_sleep, the
// agent acquire - MI355X_MICROARCH.md, inter-workgroup visibility).  Round 5 also tried it
// for renormalize_data's light-curve chain (Gaussian + six radix-select passes + ratio in one
// launch, smoothed values kept in LDS): 103 us with this barrier, 123 us with the fenced form
// of every pass, against 79 us for the ten launches (scripts/bench_lc.py, n = 2^18, sigma
// 101): at 256 workgroups a barrier costs ~7 us, a kernel boundary ~1.5 us, so the chain
// stays launch-by-launch (pu_lc_factor).
struct LcState {
    unsigned arrive;  // grid-barrier arrivals within a launch (outlier_fused_kernel)
    unsigned leave;   // workgroups past the last barrier
    unsigned nan;     // NaNs among the smoothed values
    unsigned pad[61];
};
static_assert(sizeof(LcState) == 256, "LcState");

__device__ __forceinline__ void lc_grid_barrier(LcState *st, unsigned target)
{
    asm volatile("s_waitcnt vmcnt(0)" : : : "memory");  // this wave's histogram atomics done
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
        __hip_atomic_fetch_add(&st->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(&st->arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
            __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" : : : "memory");
    }
    __syncthreads();
}

// ---------------------------------------------------------------- cut_outliers, one launch
// pu_cut_outliers' window means, std, certified decisions, exact fallback and column zeroing
// (clean.py:93-105) in ONE launch (round 5; until round 4: a state fill + five kernels).
// Phases separated by grid barriers (lc_grid_barrier; the counters sit in the workspace
// head cleared by the call's one 128-byte fill):
//   1. each workgroup: u = the 16-window means of its segments (kept in LDS and stored for
//      the exact path), the partial sum of u[::16], max |lc| and the NaN flag;
//   2. mean of u[::16] -> the partial sum of squared deviations;
//   3. sd, thresholds and certification margins (every workgroup computes the same values
//      from the same totals) -> the mask, the ambiguity flag, the bad-bin list;
//   4. only when the flag is set: workgroup 0 redoes the mask with the reference's own
//      arithmetic (outlier_exact_body), the others wait;
//   5. the bad columns of the plane zeroed, rows dealt over the workgroups.
// The sums in phases 1-2 are float64 atomics (any order: the certification margins bound
// the difference from scipy's chain, as in outlier_std_kernel).
struct OutlierBar {
    unsigned arrive, leave;
    double sum_u16, sum_sq;
};

__global__ void __launch_bounds__(256)
outlier_fused_kernel(const double *__restrict__ lc, int64_t n, OutlierState *st, OutlierBar *ob,
                     double *__restrict__ u, double *__restrict__ u16, uint8_t *__restrict__ mask,
                     int32_t *__restrict__ list, double *__restrict__ out, int64_t nrows, int64_t ld_out, int segs)
{
    extern __shared__ __attribute__((aligned(16))) double usm[];  // [segs][1024] window means
    __shared__ double red[4];
    __shared__ unsigned long long wm[4];
    const int t = threadIdx.x;
    const unsigned G = gridDim.x;
    LcState *bar = reinterpret_cast<LcState *>(ob);  // arrive at offset 0 (lc_grid_barrier's counter)
    auto block_sum = [&](double v) {
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        __syncthreads();
        if ((t & 63) == 0) red[t >> 6] = v;
        __syncthreads();
        return (red[0] + red[1]) + (red[2] + red[3]);
    };
    // 1. window means, sum of u[::16], max |lc|, NaN
    double s16 = 0.0;
    unsigned long long lb = 0;
    bool nan = false;
    for (int sg = 0; sg < segs; ++sg) {
        const int64_t i0 = ((int64_t)blockIdx.x + (int64_t)G * sg) * 1024;
        if (i0 >= n) break;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = i0 + q * 256 + t;
            double w = 0.0;
            if (i < n) {
                double sw = 0.0;
                for (int j = -8; j < 8; ++j) sw += lc[(i + j >= 0 && i + j < n) ? i + j : reflect_small(i + j, n)];
                w = sw / 16.0;
                u[i] = w;
                if ((i & 15) == 0) {
                    u16[i >> 4] = w;
                    s16 += w;
                }
                const double x = lc[i];
                nan = nan || x != x;
                const unsigned long long ab = (unsigned long long)__double_as_longlong(fabs(x));
                lb = ab > lb ? ab : lb;
            }
            usm[sg * 1024 + q * 256 + t] = w;
        }
    }
    {
        const double tot = block_sum(s16);
        unsigned long long b = nan ? ~0ull : lb;
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(b, off, 64);
            b = o > b ? o : b;
        }
        if ((t & 63) == 0) wm[t >> 6] = b;
        __syncthreads();
        if (t == 0) {
            unsigned long long m = wm[0];
            for (int w = 1; w < 4; ++w) m = wm[w] > m ? wm[w] : m;
            if (m == ~0ull) atomicOr(&st->flag, 1u);
            else atomicMax(&st->lbits, m);
            atomicAdd(&ob->sum_u16, tot);
        }
    }
    lc_grid_barrier(bar, G);
    // 2. squared deviations of u[::16] from their mean
    const int64_t m = (n + 15) / 16;
    const double mean = __hip_atomic_load(&ob->sum_u16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / (double)m;
    double ssq = 0.0;
    for (int sg = 0; sg < segs; ++sg) {
        const int64_t i0 = ((int64_t)blockIdx.x + (int64_t)G * sg) * 1024;
        if (i0 >= n) break;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = i0 + q * 256 + t;
            if (i < n && (i & 15) == 0) {
                const double d = usm[sg * 1024 + q * 256 + t] - mean;
                ssq += d * d;
            }
        }
    }
    {
        const double tot = block_sum(ssq);
        if (t == 0) atomicAdd(&ob->sum_sq, tot);
    }
    lc_grid_barrier(bar, 2 * G);
    // 3. thresholds, margins (outlier_std_kernel's), decisions, the bad-bin list
    const double ss = __hip_atomic_load(&ob->sum_sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double sd = sqrt(ss / (double)m);
    const double L = __longlong_as_double(
        (long long)__hip_atomic_load(&st->lbits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const double E = ((double)(2 * n + 64) * 0x1p-53) * L + 1e-300;
    const double Es = E + 1e-12 * sd;
    const double up = 5.0 * sd, down = -3.0 * sd;
    const double margin_up = E + 5.0 * Es + 1e-15 * (L + 5.0 * sd);
    const double margin_down = E + 3.0 * Es + 1e-15 * (L + 3.0 * sd);
    if (blockIdx.x == 0 && t == 0) {
        st->sd = sd;
        st->up = up;
        st->down = down;
        st->margin_up = margin_up;
        st->margin_down = margin_down;
        if (sd != sd) atomicOr(&st->flag, 1u);
    }
    const int lane = t & 63;
    for (int sg = 0; sg < segs; ++sg) {
        const int64_t i0 = ((int64_t)blockIdx.x + (int64_t)G * sg) * 1024;
        if (i0 >= n) break;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t i = i0 + q * 256 + t;
            uint8_t b = 0;
            if (i < n) {
                const double v = usm[sg * 1024 + q * 256 + t];
                const double du = v - up, dd = v - down;
                const bool amb = !(fabs(du) > margin_up) || !(fabs(dd) > margin_down);
                if (amb) atomicOr(&st->flag, 1u);
                b = (du > 0.0 || dd < 0.0) ? 1 : 0;
                mask[i] = b;
            }
            const uint64_t bal = __ballot(b != 0);
            if (bal) {
                uint32_t base = 0;
                if (lane == __ffsll((unsigned long long)bal) - 1) base = atomicAdd(&st->nbad, (uint32_t)__popcll(bal));
                base = __shfl(base, __ffsll((unsigned long long)bal) - 1, 64);
                if (b) list[base + __popcll(bal & ((uint64_t(1) << lane) - 1))] = (int32_t)i;
            }
        }
    }
    lc_grid_barrier(bar, 3 * G);
    // 4. the rare exact path (uniform: every workgroup reads the same flag)
    if (__hip_atomic_load(&st->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        if (blockIdx.x == 0) outlier_exact_body(lc, n, st, u, u16, mask, list);
        lc_grid_barrier(bar, 4 * G);
    }
    // 5. zero the bad columns, rows over the workgroups
    const uint32_t nbad = __hip_atomic_load(&st->nbad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int64_t r = blockIdx.x; r < nrows; r += G) {
        double *row = out + r * ld_out;
        for (uint32_t k = t; k < nbad; k += 256) row[list[k]] = 0.0;
    }
}

// ---------------------------------------------------------------- noisy channels
// get_noisier_channels' decision on the device (clean.py:58-67, stats.py:11-32): one
// workgroup, spec of n <= kNoisyMax channel means in T (float32 for float32 input, else
// float64: numpy's mean dtype).  The host path it replaces did medfilt + ref_mad in numpy
// after a read-back of spec; every step here keeps numpy's dtypes (NEP 50) and order:
//   smooth = medfilt(spec, 7)           rank 3 of the zero-padded 7-window (T, exact)
//   d = diff(spec)                      T, then float64: statsmodels 0.12.2's mad starts with
//                                       array_like(a, dtype=np.double) (robust/scale.py:49)
//   m = median(d)                       float64: the middle element, or (a + b) / 2
//   e = |d - m| / c                     float64
//   rm = median(e) / sqrt(2)            float64
//   mask = spec > smooth + 5 rm         float64
// A non-finite spec (NaN / inf: medfilt's and median's handling of them is left to
// numpy / scipy) sets *flag and leaves mask unwritten: the caller then takes the host path.
constexpr int kNoisyMax = 4096;

template <typename T>
__device__ void bitonic_sort_lds(T *v, int m)  // m: power of two, 1024 threads
{
    for (int k = 2; k <= m; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < m; i += 1024) {
                const int l = i ^ j;
                if (l > i) {
                    const T a = v[i], b = v[l];
                    const bool up = (i & k) == 0;
                    if (up ? (b < a) : (a < b)) {
                        v[i] = b;
                        v[l] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// x of lane (lane ^ J) within the wave, on the VALU (no LDS round trip): DPP quad
// permutes for J = 1, 2, row rotations for 4, 8 (J = 4: rotations by 4 and 12, the one
// whose source is lane ^ 4 picked per lane - sel4, computed once by the caller from the
// same rotation of the lane ids), the gfx950 permlane swaps for 16, 32 (the pair returns
// rows / halves exchanged: lanes in the upper row / half take the first result).
template <int J>
__device__ __forceinline__ double lane_xor(double x, int lane, bool sel4)
{
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    uint32_t w[2] = {(uint32_t)u, (uint32_t)(u >> 32)};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int v = (int)w[h];
        if constexpr (J == 1) {
            w[h] = (uint32_t)__builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
        } else if constexpr (J == 2) {
            w[h] = (uint32_t)__builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
        } else if constexpr (J == 4) {
            const int a = __builtin_amdgcn_mov_dpp(v, 0x124, 0xf, 0xf, false);  // row_ror:4
            const int b = __builtin_amdgcn_mov_dpp(v, 0x12C, 0xf, 0xf, false);  // row_ror:12
            w[h] = (uint32_t)(sel4 ? a : b);
        } else if constexpr (J == 8) {
            w[h] = (uint32_t)__builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false);  // row_ror:8
        } else if constexpr (J == 16) {
            const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
            w[h] = (lane & 16) ? (uint32_t)r[0] : (uint32_t)r[1];
        } else {
            static_assert(J == 32, "lane_xor: J = 1 .. 32");
            const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
            w[h] = (lane & 32) ? (uint32_t)r[0] : (uint32_t)r[1];
        }
    }
    return __builtin_bit_cast(double, (uint64_t)w[0] | ((uint64_t)w[1] << 32));
}

// min / max of two doubles that are never NaN (the sorts' callers check: __syncthreads_or) in
// one instruction each (a compare + two selects per 32-bit half otherwise)
__device__ __forceinline__ double min_nn(double a, double b)
{
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double max_nn(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// the bitonic compare-exchange of x with its partner y: the smaller value stays when
// keep_min (exact: min / max of non-NaN values)
__device__ __forceinline__ double bitonic_keep(double x, double y, bool keep_min)
{
    const double lo = min_nn(x, y), hi = max_nn(x, y);
    return keep_min ? lo : hi;
}

// the in-wave bitonic steps j = J, J/2, .., 1 of merge size k (lane_xor exchanges)
template <int J>
__device__ __forceinline__ void bitonic_wave_steps(double &x, int i, int k, int lane, bool sel4)
{
    const double y = lane_xor<J>(x, lane, sel4);
    x = bitonic_keep(x, y, ((i & J) == 0) == ((i & k) == 0));
    if constexpr (J > 1) bitonic_wave_steps<J / 2>(x, i, k, lane, sel4);
}

// NV independent ascending sorts over the 1024 threads of the workgroup, one value of each
// per thread in x[q] (thread i ends with the i-th smallest of sort q), the sorts sharing
// every barrier.  Bitonic: the 45 of the 55 steps whose partner is in the same wave
// exchange on the VALU (lane_xor: DPP and permlane swaps, no barrier; round 5 first:
// __shfl_xor, an LDS permute per step), the 10 with a partner in another wave through ex
// (NV x 2048 doubles of LDS, two alternating halves per sort: one barrier per step).  ex
// must be free on entry; the caller synchronises before reusing it.  No value is NaN (each
// caller tests that first and hands the decision to the host), so min / max are exact.
template <int NV>
__device__ void sort_regs_1024(double (&x)[NV], double *ex)
{
    const int i = threadIdx.x;
    const int lane = i & 63;
    // the lane whose value row_ror:4 brings (whatever the rotation's direction)
    const bool sel4 = __builtin_amdgcn_mov_dpp(lane, 0x124, 0xf, 0xf, false) == (lane ^ 4);
    // merge sizes 2 .. 64 inside each wave
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        bitonic_wave_steps<1>(x[q], i, 2, lane, sel4);
        bitonic_wave_steps<2>(x[q], i, 4, lane, sel4);
        bitonic_wave_steps<4>(x[q], i, 8, lane, sel4);
        bitonic_wave_steps<8>(x[q], i, 16, lane, sel4);
        bitonic_wave_steps<16>(x[q], i, 32, lane, sel4);
        bitonic_wave_steps<32>(x[q], i, 64, lane, sel4);
    }
    int half = 0;
    for (int k = 128; k <= 1024; k <<= 1) {
        for (int j = k >> 1; j >= 64; j >>= 1) {
            double *e = ex + 1024 * half;
#pragma unroll
            for (int q = 0; q < NV; ++q) e[2048 * q + i] = x[q];
            __syncthreads();
            half ^= 1;  // the next exchange writes the other half: no second barrier
            const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
#pragma unroll
            for (int q = 0; q < NV; ++q) x[q] = bitonic_keep(x[q], e[2048 * q + (i ^ j)], keep_min);
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) bitonic_wave_steps<32>(x[q], i, k, lane, sel4);
    }
}

// Ascending sort of v[0, m) (m a power of two) by 1024 threads.  m <= 1024: one element per
// thread, +inf padding to 1024, sort_regs_1024 with v itself as the exchange (v must hold
// 2048 elements).  Larger m: bitonic_sort_lds.
__device__ void sort_1024(double *v, int m)
{
    if (m > 1024) {
        bitonic_sort_lds(v, m);
        return;
    }
    const int i = threadIdx.x;
    double x[1] = {i < m ? v[i] : INFINITY};
    __syncthreads();  // every thread has its element before v is reused as the exchange
    sort_regs_1024<1>(x, v);
    __syncthreads();  // every exchange read is done
    if (i < m) v[i] = x[0];
    __syncthreads();
}

template <typename T>
__device__ T median_sorted(const T *v, int cnt)  // numpy: middle element / mean of the two
{
    if (cnt & 1) return v[cnt / 2];
    const T s = v[cnt / 2 - 1] + v[cnt / 2];
    return s / T(2);
}

template <typename T>
__global__ void __launch_bounds__(1024)
noisy_channels_kernel(const T *__restrict__ spec, int n, double c, uint8_t *__restrict__ mask,
                      int32_t *__restrict__ flag)
{
    __shared__ T sp[kNoisyMax];
    __shared__ double ev[kNoisyMax];  // the sorted differences, then the sorted e (float64)
    const int tid = threadIdx.x;
    int nonfinite = 0;
    for (int i = tid; i < n; i += 1024) {
        const T v = spec[i];
        sp[i] = v;
        nonfinite |= !isfinite((double)v);
    }
    if (__syncthreads_or(nonfinite)) {
        if (tid == 0) flag[0] = 1;
        return;
    }
    int m = 1;
    while (m < n - 1) m <<= 1;
    // the differences in T (np.diff of the T spectrum), then exactly widened to float64
    for (int i = tid; i < m; i += 1024) ev[i] = i < n - 1 ? (double)T(sp[i + 1] - sp[i]) : INFINITY;
    __syncthreads();
    sort_1024(ev, m);
    const double med = median_sorted(ev, n - 1);
    __syncthreads();  // every thread has read the median before ev is overwritten
    int nan_e = 0;
    for (int i = tid; i < m; i += 1024) {
        ev[i] = i < n - 1 ? fabs((double)T(sp[i + 1] - sp[i]) - med) / c : INFINITY;
        nan_e |= isnan(ev[i]);
    }
    // a NaN (inf - inf after a float32 difference overflowed) would be dropped by the
    // register sort's min / max: the host decides
    if (__syncthreads_or(nan_e)) {
        if (tid == 0) flag[0] = 1;
        return;
    }
    sort_1024(ev, m);
    const double rm = median_sorted(ev, n - 1) / 1.4142135623730951;  // np.sqrt(2)
    const double thr = 5.0 * rm;
    for (int i = tid; i < n; i += 1024) {
        T w[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const int k = i + j - 3;
            w[j] = (k >= 0 && k < n) ? sp[k] : T(0);
        }
        // rank 3 of 7 (a full insertion sort of the window: exact selection)
#pragma unroll
        for (int a = 1; a < 7; ++a)
#pragma unroll
            for (int b = a; b > 0; --b)
                if (w[b] < w[b - 1]) {
                    const T t = w[b];
                    w[b] = w[b - 1];
                    w[b - 1] = t;
                }
        mask[i] = (double)sp[i] > (double)w[3] + thr ? 1 : 0;
    }
    if (tid == 0) flag[0] = 0;
}

// ---------------------------------------------------------------- variability mask
// measure_channel_variability's certified decision (clean.py:114-133) on the device: the
// host restatement clean._certified_variability, step for step in float64 (same operation
// order), from the means pass's numpy means (T) and shifted moments (c, s1, s2) per row:
//   V = s2 - 2 dm s1 + n dm^2, dm = m - c;  eV = (s2 + 2 |dm| sqrt(n s2) + n dm^2) mef
//   s_lo / s_hi = numpy's std bounds;  q1..q3 intervals = the k-th smallest s_lo / s_hi of
//   the good channels (k = nrows/4, nrows/2, 3 nrows/4: the reference's indices);
//   the limit intervals; a channel is decided when it is clear of both.
// One workgroup, nrows <= kNoisyMax: bad channels' bounds are +inf in the two bitonic
// sorts, so the k-th smallest of all is the k-th smallest good one.  *flag = 1 (mask not
// written) for non-finite statistics, too few good channels, or any undecided channel:
// the caller then runs the exact second pass.
__device__ __forceinline__ void variability_bounds(double m, const double *mom, double nd, double mef, double gam,
                                                   double u, double &lo, double &hi)
{
    const double c = mom[0], s1 = mom[1], s2 = mom[2];
    const double dm = m - c;
    const double V = (s2 - (2.0 * dm) * s1) + (nd * dm) * dm;
    const double eV = ((s2 + (2.0 * fabs(dm)) * sqrt(nd * s2)) + (nd * dm) * dm) * mef + 1e-300;
    lo = sqrt(fmax(V - eV, 0.0) * (1.0 - gam) / nd * (1.0 - u)) * (1.0 - u);
    hi = sqrt((V + eV) * (1.0 + gam) / nd * (1.0 + u)) * (1.0 + u);
}

template <typename T>
__global__ void __launch_bounds__(1024)
variability_cert_kernel(const T *__restrict__ means, const double *__restrict__ mom, int nrows, double nd,
                        double mef, double gam, double u, const uint8_t *__restrict__ bad,
                        uint8_t *__restrict__ mask, int32_t *__restrict__ flag)
{
    __shared__ double lo[kNoisyMax], hi[kNoisyMax];
    __shared__ int gsum;
    const int tid = threadIdx.x;
    if (tid == 0) gsum = 0;
    __syncthreads();
    int nonfinite = 0, good = 0;
    for (int i = tid; i < nrows; i += 1024) {
        const double m = (double)means[i];
        nonfinite |= !isfinite(m) || !isfinite(mom[3 * i]) || !isfinite(mom[3 * i + 1]) || !isfinite(mom[3 * i + 2]);
        good += bad[i] == 0;
    }
    if (good) atomicAdd(&gsum, good);
    const int any_nf = __syncthreads_or(nonfinite);  // (also orders the LDS adds before the read)
    const int ngood = gsum;
    if (any_nf || nrows / 4 * 3 >= ngood) {
        if (tid == 0) flag[0] = 1;
        return;
    }
    int m2 = 1;
    while (m2 < nrows) m2 <<= 1;
    for (int i = tid; i < m2; i += 1024) {
        double a = INFINITY, b = INFINITY;
        if (i < nrows && bad[i] == 0) variability_bounds((double)means[i], mom + 3 * i, nd, mef, gam, u, a, b);
        lo[i] = a;
        hi[i] = b;
    }
    __syncthreads();
    sort_1024(lo, m2);
    sort_1024(hi, m2);
    const double a1 = lo[nrows / 4], b1 = hi[nrows / 4];
    const double a2 = lo[nrows / 2], b2 = hi[nrows / 2];
    const double a3 = lo[nrows / 4 * 3], b3 = hi[nrows / 4 * 3];
    const double r = 4.0 * u * (b2 + 2.0 * (b3 - a1)) + 1e-300;
    const double low_lo = (2.0 * a1 - b2) - r, low_hi = (2.0 * b1 - a2) + r;
    const double hi_lo = (2.0 * a3 - b2) - r, hi_hi = (2.0 * b3 - a2) + r;
    int unsure = 0;
    for (int i = tid; i < nrows; i += 1024) {
        double sl, sh;
        variability_bounds((double)means[i], mom + 3 * i, nd, mef, gam, u, sl, sh);
        const bool below = sh < low_lo, above = sl > hi_hi;
        const bool sure = (below || sl >= low_hi) && (above || sh <= hi_lo);
        const bool b = bad[i] != 0;
        unsure |= !b && !sure;
        mask[i] = (below || above || b) ? 1 : 0;
    }
    const int any_unsure = __syncthreads_or(unsure);
    if (tid == 0) flag[0] = any_unsure ? 1 : 0;
}

// get_noisier_channels' decision and then measure_channel_variability's for that mask, in
// ONE workgroup and one launch (n <= 1024; round 5: the two kernels above back to back).
// Thread i owns channel i: the noisy-channel steps of noisy_channels_kernel (the two sorts
// of the differences, the 7-window rank), the mask kept in a register as the variability
// certification's bad mask (variability_cert_kernel's steps, the channel's std bounds
// computed once, the lower- and upper-bound sorts sharing their barriers).  spec = the
// row means (numpy's mean dtype T), mom their shifted moments (pu_row_moments).
constexpr int kMasksMax = 1024;

template <typename T>
__global__ void __launch_bounds__(1024)
channel_masks_kernel(const T *__restrict__ spec, const double *__restrict__ mom, int n, double c, double nd,
                     double mef, double gam, double u, uint8_t *__restrict__ nmask, int32_t *__restrict__ nflag,
                     uint8_t *__restrict__ vmask, int32_t *__restrict__ vflag)
{
    __shared__ double ex[2 * 2048];
    __shared__ T sp[kMasksMax];
    __shared__ double ord[8];  // order statistics handed between threads
    const int tid = threadIdx.x;
    const bool in = tid < n;
    const T sv = in ? spec[tid] : T(0);
    if (in) sp[tid] = sv;
    if (__syncthreads_or(in && !isfinite((double)sv))) {
        if (tid == 0) {
            nflag[0] = 1;  // the host decides both masks
            vflag[0] = 1;
        }
        return;
    }
    // ---- noisy channels (clean.py:58-67; noisy_channels_kernel)
    const int nd1 = n - 1;
    const double d = tid < nd1 ? (double)T(sp[tid + 1] - sp[tid]) : INFINITY;
    auto median_of_sorted = [&](double v) {  // numpy's median of the nd1 sorted values
        if (nd1 & 1) {
            if (tid == nd1 / 2) ord[0] = v;
        } else {
            if (tid == nd1 / 2 - 1) ord[0] = v;
            if (tid == nd1 / 2) ord[1] = v;
        }
        __syncthreads();
        const double r = (nd1 & 1) ? ord[0] : (ord[0] + ord[1]) / 2.0;
        __syncthreads();  // ord read by every thread before its next use
        return r;
    };
    double x1[1] = {d};
    sort_regs_1024<1>(x1, ex);
    const double med = median_of_sorted(x1[0]);  // (its barriers also free ex)
    x1[0] = tid < nd1 ? fabs(d - med) / c : INFINITY;
    // the register sorts' v_min_f64 / v_max_f64 drop a NaN operand: a NaN here (a float32
    // difference that overflowed to inf, then inf - inf) hands both decisions to the host
    if (__syncthreads_or(isnan(x1[0]))) {
        if (tid == 0) {
            nflag[0] = 1;
            vflag[0] = 1;
        }
        return;
    }
    sort_regs_1024<1>(x1, ex);
    const double rm = median_of_sorted(x1[0]) / 1.4142135623730951;  // np.sqrt(2)
    const double thr = 5.0 * rm;
    bool bad = false;
    if (in) {
        T w[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const int k = tid + j - 3;
            w[j] = (k >= 0 && k < n) ? sp[k] : T(0);
        }
#pragma unroll
        for (int a = 1; a < 7; ++a)
#pragma unroll
            for (int b = a; b > 0; --b)
                if (w[b] < w[b - 1]) {
                    const T t = w[b];
                    w[b] = w[b - 1];
                    w[b - 1] = t;
                }
        bad = (double)sv > (double)w[3] + thr;
        nmask[tid] = bad ? 1 : 0;
    }
    if (tid == 0) nflag[0] = 0;
    // ---- variability (clean.py:114-133; variability_cert_kernel) with bad = the noisy mask
    const double *mr = mom + 3 * (in ? tid : 0);
    const bool nf = in && (!isfinite(mr[0]) || !isfinite(mr[1]) || !isfinite(mr[2]));
    const int any_nf = __syncthreads_or(nf);
    const int ngood = __syncthreads_count(in && !bad);
    if (any_nf || n / 4 * 3 >= ngood) {
        if (tid == 0) vflag[0] = 1;
        return;
    }
    double sl = INFINITY, sh = INFINITY;
    if (in) variability_bounds((double)sv, mr, nd, mef, gam, u, sl, sh);
    double x2[2] = {in && !bad ? sl : INFINITY, in && !bad ? sh : INFINITY};
    if (__syncthreads_or(isnan(x2[0]) || isnan(x2[1]))) {  // (NaN bounds: the host decides)
        if (tid == 0) vflag[0] = 1;
        return;
    }
    sort_regs_1024<2>(x2, ex);
    const int k1 = n / 4, k2 = n / 2, k3 = n / 4 * 3;
    if (tid == k1) { ord[2] = x2[0]; ord[3] = x2[1]; }
    if (tid == k2) { ord[4] = x2[0]; ord[5] = x2[1]; }
    if (tid == k3) { ord[6] = x2[0]; ord[7] = x2[1]; }
    __syncthreads();
    const double a1 = ord[2], b1 = ord[3], a2 = ord[4], b2 = ord[5], a3 = ord[6], b3 = ord[7];
    const double r = 4.0 * u * (b2 + 2.0 * (b3 - a1)) + 1e-300;
    const double low_lo = (2.0 * a1 - b2) - r, low_hi = (2.0 * b1 - a2) + r;
    const double hi_lo = (2.0 * a3 - b2) - r, hi_hi = (2.0 * b3 - a2) + r;
    int unsure = 0;
    if (in) {
        const bool below = sh < low_lo, above = sl > hi_hi;
        const bool sure = (below || sl >= low_hi) && (above || sh <= hi_lo);
        unsure = !bad && !sure;
        vmask[tid] = (below || above || bad) ? 1 : 0;
    }
    const int any_unsure = __syncthreads_or(unsure);
    if (tid == 0) vflag[0] = any_unsure ? 1 : 0;
}

__global__ void ratio_dev_kernel(const double *__restrict__ num, const double *__restrict__ x, int64_t n,
                                 double *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = num[0] / x[i];
}

template <typename Tin, typename Ta, int MODE>
int row_sums_t(const void *x, int64_t nrows, int64_t n, int64_t ld, const void *center, const double *scale,
               double divisor, void *out, void *ws, hipStream_t s)
{
    const int64_t nfull = n / kBlock;
    const int64_t tail = n % kBlock;
    const int64_t nblk_row = nfull + (tail ? 1 : 0);
    Ta *bs = reinterpret_cast<Ta *>(ws);
    const Tin *xp = reinterpret_cast<const Tin *>(x);
    const Ta *cp = reinterpret_cast<const Ta *>(center);
    if (nfull > 0) {
        // pair loads need 2-element alignment of every row (and of the scale vector)
        const bool pair = reinterpret_cast<uintptr_t>(x) % (2 * sizeof(Tin)) == 0 && ld % 2 == 0 &&
                          (MODE != 2 || reinterpret_cast<uintptr_t>(scale) % 16 == 0);
        // MODE 2: R rows per workgroup share the scale pairs (PU_CLEAN_SCALE_ROWS: 4, 8, 16)
        int rsel = kScaleRows;
        rsel = pu::knob("PU_CLEAN_SCALE_ROWS", rsel);
        auto go = [&](auto rc_) {
            constexpr int R = MODE == 2 ? decltype(rc_)::value : 1;
            const int64_t ngroups = (nrows + R - 1) / R;
            PU_REQUIRE(ngroups * nfull < (int64_t(1) << 31), "pu_row_sums: too many blocks");
            if (pair)
                hipLaunchKernelGGL((rowsum_chunk_kernel<Tin, Ta, MODE, true, R>), dim3((unsigned)(ngroups * nfull)),
                                   dim3(256), 0, s, xp, ld, nrows, nfull, nblk_row, cp, scale, bs);
            else
                hipLaunchKernelGGL((rowsum_chunk_kernel<Tin, Ta, MODE, false, R>),
                                   dim3((unsigned)(ngroups * nfull)), dim3(256), 0, s, xp, ld, nrows, nfull,
                                   nblk_row, cp, scale, bs);
            return pu::launch_check("rowsum_chunk_kernel");
        };
        int rc;
        if constexpr (MODE == 2) {
            rc = rsel >= 16 ? go(std::integral_constant<int, 16>{})
                            : rsel >= 8 ? go(std::integral_constant<int, 8>{}) : go(std::integral_constant<int, 4>{});
        } else {
            rc = go(std::integral_constant<int, 1>{});
        }
        if (rc) return rc;
    }
    if (tail) {
        hipLaunchKernelGGL((rowsum_tail_kernel<Tin, Ta, MODE>), dim3((unsigned)((nrows + 63) / 64)), dim3(64), 0, s,
                           xp, ld, nrows, n, nfull, nblk_row, cp, scale, bs);
        int rc = pu::launch_check("rowsum_tail_kernel");
        if (rc) return rc;
    }
    hipLaunchKernelGGL((rowsum_combine<Ta>), dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, s, bs, nrows,
                       nblk_row, divisor, reinterpret_cast<Ta *>(out));
    return pu::launch_check("rowsum_combine");
}

// numpy's row means (MODE 0 order, divided by n) and, in the same pass, the shifted
// moments of every row (pu_row_moments).  ws: the block sums, then 2 doubles per block.
template <typename Tin, typename Ta>
int row_moments_t(const void *x, int64_t nrows, int64_t n, int64_t ld, void *means, double *moments, void *ws,
                  hipStream_t s)
{
    const int64_t nfull = n / kBlock;
    const int64_t tail = n % kBlock;
    const int64_t nblk_row = nfull + (tail ? 1 : 0);
    Ta *bs = reinterpret_cast<Ta *>(ws);
    double *mb = reinterpret_cast<double *>(reinterpret_cast<char *>(ws) +
                                            (((size_t)nrows * nblk_row * sizeof(double) + 255) & ~size_t(255)));
    const Tin *xp = reinterpret_cast<const Tin *>(x);
    if (nfull > 0) {
        PU_REQUIRE(nrows * nfull < (int64_t(1) << 31), "pu_row_moments: too many blocks");
        const bool pair = reinterpret_cast<uintptr_t>(x) % (2 * sizeof(Tin)) == 0 && ld % 2 == 0;
        if (pair)
            hipLaunchKernelGGL((rowsum_chunk_kernel<Tin, Ta, 0, true, 1, true>), dim3((unsigned)(nrows * nfull)),
                               dim3(256), 0, s, xp, ld, nrows, nfull, nblk_row, nullptr, nullptr, bs, mb);
        else
            hipLaunchKernelGGL((rowsum_chunk_kernel<Tin, Ta, 0, false, 1, true>), dim3((unsigned)(nrows * nfull)),
                               dim3(256), 0, s, xp, ld, nrows, nfull, nblk_row, nullptr, nullptr, bs, mb);
        int rc = pu::launch_check("rowsum_chunk_kernel");
        if (rc) return rc;
    }
    if (tail) {
        hipLaunchKernelGGL((rowsum_tail_kernel<Tin, Ta, 0, true>), dim3((unsigned)((nrows + 63) / 64)), dim3(64), 0,
                           s, xp, ld, nrows, n, nfull, nblk_row, nullptr, nullptr, bs, mb);
        int rc = pu::launch_check("rowsum_tail_kernel");
        if (rc) return rc;
    }
    hipLaunchKernelGGL((row_moments_combine<Tin, Ta>), dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, s, bs, mb,
                       xp, ld, nrows, nblk_row, (double)n, reinterpret_cast<Ta *>(means), moments);
    return pu::launch_check("row_moments_combine");
}

template <typename Tin>
int row_sums_in(int mode, bool f32acc, const void *x, int64_t nrows, int64_t n, int64_t ld, const void *center,
                const double *scale, double divisor, void *out, void *ws, hipStream_t s)
{
    if (mode == 2) return row_sums_t<Tin, double, 2>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    if (mode == 3) return row_sums_t<Tin, double, 0>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    if (mode == 4) return row_sums_t<Tin, double, 4>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    if (f32acc) {
        if (mode == 0) return row_sums_t<Tin, float, 0>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
        return row_sums_t<Tin, float, 1>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    }
    if (mode == 0) return row_sums_t<Tin, double, 0>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
    return row_sums_t<Tin, double, 1>(x, nrows, n, ld, center, scale, divisor, out, ws, s);
}

unsigned blocks_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

// Widest V in {vmax, .., 2} with every row start of p (stride ld elements) aligned
// to V elements; 1 otherwise.
template <typename T>
int pick_vec(const void *p, int64_t ld, int vmax)
{
    for (int v = vmax; v > 1; v >>= 1)
        if (reinterpret_cast<uintptr_t>(p) % (v * sizeof(T)) == 0 && ld % v == 0) return v;
    return 1;
}

// Column lanes: V adjacent columns per lane (16-byte loads at most).  Measured on C4
// (1024 x 2^18): the read-only mean pass is fastest with wide lanes (V=4), the
// apply pass (float64 stores, a division per element) with the most waves (V=1).
// PU_CLEAN_VMAX overrides both (1, 2 or 4).
int vec_max(size_t elem, int dflt)
{
    const int env = pu::knob("PU_CLEAN_VMAX", 0);
    const int v = env > 0 ? env : dflt;
    const int w = v >= 4 ? 4 : v >= 2 ? 2 : 1;
    return elem >= 8 && w > 2 ? 2 : w;
}

// Columns [0, n - n%V) with V-wide lanes, the rest with scalar lanes.
template <typename Tin, typename Launch>
int column_launches(int v, int64_t n, Launch &&launch)
{
    const int64_t nv = n - n % v;
    if (nv > 0) {
        if constexpr (sizeof(Tin) < 8)
            if (v == 4) launch(std::integral_constant<int, 4>{}, 0, nv);
        if (v == 2) launch(std::integral_constant<int, 2>{}, 0, nv);
        if (v == 1) launch(std::integral_constant<int, 1>{}, 0, nv);
    }
    if (n > nv) launch(std::integral_constant<int, 1>{}, nv, n - nv);
    return PU_OK;
}

template <typename Tin>
int col_means_t(const void *x, int64_t nrows, int64_t n, int64_t ld, const uint8_t *skip, double *out, hipStream_t s)
{
    if constexpr (sizeof(Tin) == 1) {
        // 8-bit input: exact integer sums by row segments (PU_COLSEG=0: the sequential kernel)
        static const bool seg = pu::knob("PU_COLSEG", 1) != 0;
        const int nseg = (int)((nrows + kColSegRows - 1) / kColSegRows);
        if (seg && nseg <= kColSegMax && n % 8 == 0 && ld % 8 == 0 && reinterpret_cast<uintptr_t>(x) % 8 == 0) {
            hipLaunchKernelGGL(colsum_u8_seg_kernel, dim3(blocks_for(n / 8, 256), nseg), dim3(256), 0, s,
                               reinterpret_cast<const uint8_t *>(x), nrows, n, ld, skip,
                               reinterpret_cast<uint16_t *>(out));
            hipLaunchKernelGGL(colsum_u8_finish_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, out, n, nseg,
                               nrows, skip);
            return PU_OK;
        }
    }
    const int v = pick_vec<Tin>(x, ld, vec_max(sizeof(Tin), 4));
    // bytes of rows in flight per lane and register buffer (PU_CLEAN_BATCH: 128, 256 or 512)
    int bb = 256;  // C4 sweep (profiles/r02_clean/): f32 V=4 190 us vs 212 us at 128 B
    bb = pu::knob("PU_CLEAN_BATCH", bb);
    return column_launches<Tin>(v, n, [&](auto vc, int64_t col0, int64_t ncols) {
        constexpr int V = decltype(vc)::value;
        if (bb >= 512)
            hipLaunchKernelGGL((colmean_kernel<Tin, V, 512>), dim3(blocks_for(ncols / V, 256)), dim3(256), 0, s,
                               reinterpret_cast<const Tin *>(x), nrows, col0, ncols, ld, skip, out);
        else if (bb >= 256)
            hipLaunchKernelGGL((colmean_kernel<Tin, V, 256>), dim3(blocks_for(ncols / V, 256)), dim3(256), 0, s,
                               reinterpret_cast<const Tin *>(x), nrows, col0, ncols, ld, skip, out);
        else
            hipLaunchKernelGGL((colmean_kernel<Tin, V, kBatchBytes>), dim3(blocks_for(ncols / V, 256)), dim3(256),
                               0, s, reinterpret_cast<const Tin *>(x), nrows, col0, ncols, ld, skip, out);
    });
}

// Output plane written with non-temporal stores: on for 8-bit input (C4 u8 apply
// 542 -> 481 us), off for float input (606 vs 623 us); PU_CLEAN_NT=0/1 overrides.
bool nt_stores(size_t elem)
{
    const int env = pu::knob("PU_CLEAN_NT", -1);
    return env >= 0 ? env != 0 : elem == 1;
}

template <typename Tin>
int renorm_apply_t(const void *x, int64_t nchan, int64_t n, int64_t ld, const double *factor, const double *spec,
                   const uint8_t *bad, double *out, int64_t ld_out, double *col_means, int64_t ngood_zdm,
                   hipStream_t s)
{
    // C4 sweep (profiles/r02_clean/): f32 V=4 615 us (V=1 640), u8 V=2 + nt stores 480 us
    const int vm = vec_max(sizeof(Tin), sizeof(Tin) == 4 ? 4 : sizeof(Tin) == 1 ? 2 : 1);
    const int v = std::min(pick_vec<Tin>(x, ld, vm), pick_vec<double>(out, ld_out, vm));
    const bool zdm = ngood_zdm >= 0;
    return column_launches<Tin>(v, n, [&](auto vc, int64_t col0, int64_t ncols) {
        constexpr int V = decltype(vc)::value;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks_for(ncols / V, 256)), dim3(256), 0, s,
                               reinterpret_cast<const Tin *>(x), nchan, col0, ncols, ld, factor, spec, bad, out,
                               ld_out, col_means, ngood_zdm);
        };
        const bool nt = nt_stores(sizeof(Tin));
        // bytes of rows in flight per lane and register buffer (PU_APPLY_BATCH)
        int bb = kBatchBytes;
        bb = pu::knob("PU_APPLY_BATCH", bb);
        auto pick = [&](auto ntc, auto zc) {
            constexpr bool NT = decltype(ntc)::value, Z = decltype(zc)::value;
            if (bb >= 512) go(apply_kernel<Tin, V, NT, Z, 512>);
            else if (bb >= 256) go(apply_kernel<Tin, V, NT, Z, 256>);
            else go(apply_kernel<Tin, V, NT, Z, kBatchBytes>);
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        if (zdm)
            nt ? pick(T_{}, T_{}) : pick(F_{}, T_{});
        else
            nt ? pick(T_{}, F_{}) : pick(F_{}, F_{});
    });
}

}  // namespace

extern "C" {

size_t pu_row_sums_workspace_bytes(int64_t nrows, int64_t n)
{
    const int64_t nblk = (n + kBlock - 1) / kBlock;
    return (size_t)(nrows > 0 ? nrows : 0) * (size_t)(nblk > 0 ? nblk : 1) * sizeof(double);
}

int pu_row_sums(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, int mode, const void *center,
                const double *scale, double divisor, void *out, void *ws, size_t ws_bytes, void *stream)
{
    PU_REQUIRE(x && out, "pu_row_sums: NULL pointer");
    PU_REQUIRE(nrows > 0 && n > 0 && ld >= n, "pu_row_sums: bad shape");
    PU_REQUIRE(mode >= 0 && mode <= 4, "pu_row_sums: bad mode %d", mode);
    PU_REQUIRE(mode != 1 || center, "pu_row_sums: mode 1 needs center");
    PU_REQUIRE(mode != 2 || scale, "pu_row_sums: mode 2 needs scale");
    PU_REQUIRE(ws && ws_bytes >= pu_row_sums_workspace_bytes(nrows, n), "pu_row_sums: workspace too small");
    hipStream_t s = pu::as_stream(stream);
    switch (dtype) {
    case PU_U8: return row_sums_in<uint8_t>(mode, false, x, nrows, n, ld, center, scale, divisor, out, ws, s);
    case PU_F32: return row_sums_in<float>(mode, true, x, nrows, n, ld, center, scale, divisor, out, ws, s);
    case PU_F64: return row_sums_in<double>(mode, false, x, nrows, n, ld, center, scale, divisor, out, ws, s);
    }
    pu::set_error("pu_row_sums: unsupported dtype %d", dtype);
    return PU_EUNSUPPORTED;
}

size_t pu_row_moments_workspace_bytes(int64_t nrows, int64_t n)
{
    const int64_t nblk = (n + kBlock - 1) / kBlock;
    const size_t nb = (size_t)(nrows > 0 ? nrows : 0) * (size_t)(nblk > 0 ? nblk : 1);
    return ((nb * sizeof(double) + 255) & ~size_t(255)) + nb * 2 * sizeof(double);
}

int pu_row_moments(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, void *means, double *moments,
                   void *ws, size_t ws_bytes, void *stream)
{
    PU_REQUIRE(x && means && moments, "pu_row_moments: NULL pointer");
    PU_REQUIRE(nrows > 0 && n > 0 && ld >= n, "pu_row_moments: bad shape");
    PU_REQUIRE(ws && ws_bytes >= pu_row_moments_workspace_bytes(nrows, n) && reinterpret_cast<uintptr_t>(ws) % 8 == 0,
               "pu_row_moments: workspace too small or not 8-byte aligned");
    hipStream_t s = pu::as_stream(stream);
    switch (dtype) {
    case PU_U8: return row_moments_t<uint8_t, double>(x, nrows, n, ld, means, moments, ws, s);
    case PU_F32: return row_moments_t<float, float>(x, nrows, n, ld, means, moments, ws, s);
    case PU_F64: return row_moments_t<double, double>(x, nrows, n, ld, means, moments, ws, s);
    }
    pu::set_error("pu_row_moments: unsupported dtype %d", dtype);
    return PU_EUNSUPPORTED;
}

int pu_col_means(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, const uint8_t *skip, double *out,
                 void *stream)
{
    PU_REQUIRE(x && out, "pu_col_means: NULL pointer");
    PU_REQUIRE(nrows > 0 && n > 0 && ld >= n, "pu_col_means: bad shape");
    hipStream_t s = pu::as_stream(stream);
    switch (dtype) {
    case PU_U8: col_means_t<uint8_t>(x, nrows, n, ld, skip, out, s); break;
    case PU_F32: col_means_t<float>(x, nrows, n, ld, skip, out, s); break;
    case PU_F64: col_means_t<double>(x, nrows, n, ld, skip, out, s); break;
    default: pu::set_error("pu_col_means: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("colmean_kernel");
}

int pu_gaussian_filter1d(const double *x, int64_t n, const double *w, int64_t r, double *out, void *stream)
{
    PU_REQUIRE(x && w && out && n > 0 && r >= 0, "pu_gaussian_filter1d: bad arguments");
    if (r <= kGaussMaxR) {
        static const bool single = pu::knob("PU_GAUSS_SINGLE", 0) != 0;  // the one-output form, for A/B
        if (single) {
            const size_t lds = (size_t)(r + 1 + 256 + 2 * r) * sizeof(double);
            hipLaunchKernelGGL(gauss_lds_kernel, dim3(blocks_for(n, 256)), dim3(256), lds, pu::as_stream(stream), x,
                               n, w, (int)r, out);
            return pu::launch_check("gauss_lds_kernel");
        }
        static const bool pair = pu::knob("PU_GAUSS_PAIR", 0) != 0;  // the round-3 two-output form, for A/B
        if (pair) {
            const size_t lds = (size_t)(((r + 2) & ~int64_t(1)) + 512 + 2 * r + 2 * kGaussPad) * sizeof(double);
            hipLaunchKernelGGL(gauss_pair_kernel, dim3(blocks_for(n, 512)), dim3(256), lds, pu::as_stream(stream), x,
                               n, w, (int)r, out);
            return pu::launch_check("gauss_pair_kernel");
        }
        // threads per workgroup (4 outputs each): PU_GAUSS_THREADS 64 / 128 / 256 (A/B)
        const int gt = pu::knob("PU_GAUSS_THREADS", kGaussQuadThreads);
        auto quad = [&](auto tc) {
            constexpr int T = decltype(tc)::value;
            const size_t lds = (size_t)(((r + 2) & ~int64_t(1)) + 4 * T + 2 * r + 2 * kGaussPad) * sizeof(double);
            hipLaunchKernelGGL(gauss_quad_kernel<T>, dim3(blocks_for(n, 4 * T)), dim3(T), lds, pu::as_stream(stream),
                               x, n, w, (int)r, out);
        };
        if (gt <= 64) quad(std::integral_constant<int, 64>{});
        else if (gt <= 128) quad(std::integral_constant<int, 128>{});
        else quad(std::integral_constant<int, 256>{});
        return pu::launch_check("gauss_quad_kernel");
    }
    hipLaunchKernelGGL(gauss_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, pu::as_stream(stream), x, n, w, r, out);
    return pu::launch_check("gauss_kernel");
}

int pu_ratio(double num, const double *x, int64_t n, double *out, void *stream)
{
    PU_REQUIRE(x && out && n > 0, "pu_ratio: bad arguments");
    hipLaunchKernelGGL(ratio_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, pu::as_stream(stream), num, x, n, out);
    return pu::launch_check("ratio_kernel");
}

static int renorm_apply_any(const void *x, int dtype, int64_t nchan, int64_t n, int64_t ld, const double *factor,
                            const double *spec, const uint8_t *bad, double *out, int64_t ld_out, double *col_means,
                            int64_t ngood_zdm, void *stream)
{
    PU_REQUIRE(x && factor && spec && out, "pu_renorm_apply: NULL pointer");
    PU_REQUIRE(nchan > 0 && n > 0 && ld >= n && ld_out >= n, "pu_renorm_apply: bad shape");
    hipStream_t s = pu::as_stream(stream);
    const int64_t g = ngood_zdm;
    switch (dtype) {
    case PU_U8: renorm_apply_t<uint8_t>(x, nchan, n, ld, factor, spec, bad, out, ld_out, col_means, g, s); break;
    case PU_F32: renorm_apply_t<float>(x, nchan, n, ld, factor, spec, bad, out, ld_out, col_means, g, s); break;
    case PU_F64: renorm_apply_t<double>(x, nchan, n, ld, factor, spec, bad, out, ld_out, col_means, g, s); break;
    default: pu::set_error("pu_renorm_apply: unsupported dtype %d", dtype); return PU_EUNSUPPORTED;
    }
    return pu::launch_check("apply_kernel");
}

int pu_renorm_apply(const void *x, int dtype, int64_t nchan, int64_t n, int64_t ld, const double *factor,
                    const double *spec, const uint8_t *bad, double *out, int64_t ld_out, double *col_means,
                    void *stream)
{
    return renorm_apply_any(x, dtype, nchan, n, ld, factor, spec, bad, out, ld_out, col_means, -1, stream);
}

int pu_renorm_apply_zero_dm(const void *x, int dtype, int64_t nchan, int64_t n, int64_t ld, const double *factor,
                            const double *spec, const uint8_t *bad, int64_t ngood, double *out, int64_t ld_out,
                            double *col_means, void *stream)
{
    PU_REQUIRE(ngood >= 0 && ngood <= nchan, "pu_renorm_apply_zero_dm: ngood %lld outside [0, nchan]",
               (long long)ngood);
    return renorm_apply_any(x, dtype, nchan, n, ld, factor, spec, bad, out, ld_out, col_means, ngood, stream);
}

size_t pu_cut_outliers_workspace_bytes(int64_t n)
{
    const size_t m = (size_t)(n > 0 ? n : 0);
    return 256 + (m + (m + 15) / 16) * sizeof(double) + m * sizeof(int32_t);  // state | window means | every 16th | bad list
}

namespace {
// CUs a launch on stream s may use: the current device's, or the stream's CU mask's when it
// has one (pu_stream_create_cu_masked); 0 if they cannot be counted.
int usable_cus(hipStream_t s)
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    static std::atomic<int> ncu[64];
    cus = dev < 64 ? ncu[dev].load() : 0;
    if (cus <= 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        if (dev < 64) ncu[dev].store(cus);
    }
    if (s) {
        uint32_t m[32] = {};
        if (hipExtStreamGetCUMask(s, 32, m) == hipSuccess) {
            int c = 0;
            for (uint32_t w : m) c += __builtin_popcount(w);
            if (c > 0 && c < cus) cus = c;
        } else {
            (void)hipGetLastError();
        }
    }
    return cus;
}

int cut_outliers(const double *lc, int64_t n, double *out, int64_t nrows, int64_t ld_out, uint8_t *mask, void *ws,
                 size_t ws_bytes, void *stream, bool exact_only)
{
    PU_REQUIRE(lc && out && mask && n >= 64 && nrows > 0 && ld_out >= n, "pu_cut_outliers: bad arguments");
    PU_REQUIRE(ws && ws_bytes >= pu_cut_outliers_workspace_bytes(n) && reinterpret_cast<uintptr_t>(ws) % 8 == 0,
               "pu_cut_outliers: workspace too small or not 8-byte aligned");
    hipStream_t s = pu::as_stream(stream);
    OutlierState *st = reinterpret_cast<OutlierState *>(ws);
    double *u = reinterpret_cast<double *>(reinterpret_cast<char *>(ws) + 256);
    double *u16 = u + n;
    int32_t *list = reinterpret_cast<int32_t *>(u16 + (n + 15) / 16);
    PU_REQUIRE(nrows < (int64_t(1) << 31), "pu_cut_outliers: too many rows");
    // one 16-byte-multiple fill (the runtime splits a 56-byte memset into two kernels)
    static_assert(sizeof(OutlierState) <= 64, "OutlierState fits the cleared 64 bytes");
    static_assert(sizeof(OutlierBar) <= 64, "OutlierBar fits the cleared 64 bytes after the state");
    bool resident = false;
    if (!exact_only) {
        // one launch with grid barriers (outlier_fused_kernel): at most one workgroup per two
        // CUs the stream may use, each with <= 64 KB of window means in LDS, and never more
        // than the occupancy calculator says can be resident on them together - so every
        // workgroup of the grid is resident and the spinning barrier cannot wait on one that
        // never starts.  Counted per call on the current device and the stream's CU mask (a
        // CU-masked stream, pu_stream_create_cu_masked, sees only its CUs); a grid that would
        // not be resident takes the launch-by-launch path below.
        const int64_t nseg = (n + 1023) / 1024;
        const int cus = usable_cus(s);
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(nseg, std::max(1, cus / 2)));
        const int segs = (int)((nseg + grid - 1) / grid);
        if (cus > 0 && segs <= 8 && nrows < (int64_t(1) << 31)) {
            int dev = 0;
            PU_TRY_HIP(hipGetDevice(&dev));
            static std::atomic<uint64_t> attr_set{0};  // per device: 64 KB static (the exact
                                                      // path's staging) + the window means
            if (dev < 64 && !(attr_set.load() >> dev & 1)) {
                PU_TRY_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(outlier_fused_kernel),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 1024 * (int)sizeof(double)));
                attr_set.fetch_or(uint64_t(1) << dev);
            }
            // resident workgroups per CU at this LDS size (cached per device and size)
            static std::atomic<int> occ[64][9];
            int per_cu = dev < 64 ? occ[dev][segs].load() : 0;
            if (per_cu <= 0) {
                PU_TRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &per_cu, reinterpret_cast<const void *>(outlier_fused_kernel), 256, (size_t)segs * 1024 * sizeof(double)));
                if (dev < 64) occ[dev][segs].store(per_cu);
            }
            resident = (int64_t)per_cu * cus >= grid;
        }
        if (resident) {
            PU_TRY_HIP(hipMemsetAsync(st, 0, 128, s));
            OutlierBar *ob = reinterpret_cast<OutlierBar *>(reinterpret_cast<char *>(ws) + 64);
            hipLaunchKernelGGL(outlier_fused_kernel, dim3(grid), dim3(256), (size_t)segs * 1024 * sizeof(double), s, lc,
                               n, st, ob, u, u16, mask, list, out, nrows, ld_out, segs);
            return pu::launch_check("outlier_fused_kernel");
        }
    }
    PU_TRY_HIP(hipMemsetAsync(st, 0, 64, s));
    if (!exact_only) {
        hipLaunchKernelGGL(outlier_window_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, lc, n, u, u16, st);
        hipLaunchKernelGGL(outlier_std_kernel, dim3(1), dim3(1024), 0, s, u16, n, st);
        hipLaunchKernelGGL(outlier_mask_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, u, n, st, mask, list);
    }
    // returns at once unless the flag is set (or exact_only)
    hipLaunchKernelGGL(outlier_exact_kernel, dim3(1), dim3(256), 0, s, lc, n, st, u, u16, mask, list,
                       exact_only ? 1 : 0);
    hipLaunchKernelGGL(outlier_zero_kernel, dim3((unsigned)nrows), dim3(256), 0, s, list, st, out, nrows, ld_out);
    return pu::launch_check("outlier kernels");
}
}  // namespace

int pu_cut_outliers(const double *lc, int64_t n, double *out, int64_t nrows, int64_t ld_out, uint8_t *mask,
                    void *ws, size_t ws_bytes, void *stream)
{
    return cut_outliers(lc, n, out, nrows, ld_out, mask, ws, ws_bytes, stream, false);
}

int pu_cut_outliers_exact(const double *lc, int64_t n, double *out, int64_t nrows, int64_t ld_out, uint8_t *mask,
                          void *ws, size_t ws_bytes, void *stream)
{
    return cut_outliers(lc, n, out, nrows, ld_out, mask, ws, ws_bytes, stream, true);
}

size_t pu_median_workspace_bytes(void) { return sizeof(MedState) + kMedBufs * 2 * kMedBins * sizeof(uint32_t); }

int pu_median(const double *x, int64_t n, double *out, void *ws, size_t ws_bytes, void *stream)
{
    PU_REQUIRE(x && out && n > 0, "pu_median: bad arguments");
    PU_REQUIRE(ws && ws_bytes >= pu_median_workspace_bytes(), "pu_median: workspace too small");
    PU_REQUIRE(reinterpret_cast<uintptr_t>(ws) % 8 == 0, "pu_median: workspace not 8-byte aligned");
    hipStream_t s = pu::as_stream(stream);
    MedState *st = reinterpret_cast<MedState *>(ws);
    uint32_t *hist = reinterpret_cast<uint32_t *>(st + 1);
    hipLaunchKernelGGL(median_init_kernel, dim3(1), dim3(256), 0, s, st, hist, n);
    // a few elements per thread: fewer workgroups to flush LDS bins to the global histogram
    // (PU_MEDIAN_GRID: most workgroups per pass, tuning)
    int64_t gmax = 256;
    gmax = std::max(1, pu::knob("PU_MEDIAN_GRID", (int)gmax));
    const unsigned grid = std::min<int64_t>(gmax, std::max<int64_t>(1, (n + 1023) / 1024));
    for (int p = 0; p < kMedPasses; ++p)
        hipLaunchKernelGGL(median_hist_kernel, dim3(grid), dim3(256), 0, s, x, n, st, hist, p);
    hipLaunchKernelGGL(median_final_kernel, dim3(1), dim3(256), 0, s, st, hist, n, out);
    return pu::launch_check("median_kernels");
}

int pu_variability_cert(const void *means, int dtype, const double *moments, int64_t nrows, int64_t n, double mef,
                        double gam, double u, const uint8_t *bad, uint8_t *mask, int32_t *flag, void *stream)
{
    PU_REQUIRE(means && moments && bad && mask && flag, "pu_variability_cert: NULL pointer");
    PU_REQUIRE(nrows >= 1 && nrows <= kNoisyMax, "pu_variability_cert: nrows = %lld outside [1, %d]",
               (long long)nrows, kNoisyMax);
    PU_REQUIRE(n >= 1, "pu_variability_cert: n must be positive");
    PU_REQUIRE(dtype == PU_F32 || dtype == PU_F64, "pu_variability_cert: means must be float32 or float64");
    if (dtype == PU_F32)
        hipLaunchKernelGGL(variability_cert_kernel<float>, dim3(1), dim3(1024), 0, pu::as_stream(stream),
                           reinterpret_cast<const float *>(means), moments, (int)nrows, (double)n, mef, gam, u, bad,
                           mask, flag);
    else
        hipLaunchKernelGGL(variability_cert_kernel<double>, dim3(1), dim3(1024), 0, pu::as_stream(stream),
                           reinterpret_cast<const double *>(means), moments, (int)nrows, (double)n, mef, gam, u, bad,
                           mask, flag);
    return pu::launch_check("variability_cert_kernel");
}

int pu_noisy_channels(const void *spec, int dtype, int64_t n, double mad_c, uint8_t *mask, int32_t *flag,
                      void *stream)
{
    PU_REQUIRE(spec && mask && flag, "pu_noisy_channels: NULL pointer");
    PU_REQUIRE(n >= 2 && n <= kNoisyMax, "pu_noisy_channels: n = %lld outside [2, %d]", (long long)n, kNoisyMax);
    PU_REQUIRE(dtype == PU_F32 || dtype == PU_F64, "pu_noisy_channels: spec must be float32 or float64");
    if (dtype == PU_F32)
        hipLaunchKernelGGL(noisy_channels_kernel<float>, dim3(1), dim3(1024), 0, pu::as_stream(stream),
                           reinterpret_cast<const float *>(spec), (int)n, mad_c, mask, flag);
    else
        hipLaunchKernelGGL(noisy_channels_kernel<double>, dim3(1), dim3(1024), 0, pu::as_stream(stream),
                           reinterpret_cast<const double *>(spec), (int)n, mad_c, mask, flag);
    return pu::launch_check("noisy_channels_kernel");
}

int pu_channel_masks(const void *means, int dtype, const double *moments, int64_t nrows, int64_t n, double mad_c,
                     double mef, double gam, double u, uint8_t *noisy, int32_t *noisy_flag, uint8_t *var,
                     int32_t *var_flag, void *stream)
{
    PU_REQUIRE(means && moments && noisy && noisy_flag && var && var_flag, "pu_channel_masks: NULL pointer");
    PU_REQUIRE(nrows >= 2 && nrows <= kMasksMax, "pu_channel_masks: nrows = %lld outside [2, %d]", (long long)nrows,
               kMasksMax);
    PU_REQUIRE(n >= 1, "pu_channel_masks: n must be positive");
    PU_REQUIRE(dtype == PU_F32 || dtype == PU_F64, "pu_channel_masks: means must be float32 or float64");
    if (dtype == PU_F32)
        hipLaunchKernelGGL(channel_masks_kernel<float>, dim3(1), dim3(1024), 0, pu::as_stream(stream),
                           reinterpret_cast<const float *>(means), moments, (int)nrows, mad_c, (double)n, mef, gam, u,
                           noisy, noisy_flag, var, var_flag);
    else
        hipLaunchKernelGGL(channel_masks_kernel<double>, dim3(1), dim3(1024), 0, pu::as_stream(stream),
                           reinterpret_cast<const double *>(means), moments, (int)nrows, mad_c, (double)n, mef, gam,
                           u, noisy, noisy_flag, var, var_flag);
    return pu::launch_check("channel_masks_kernel");
}

int pu_ratio_dev(const double *numerator, const double *x, int64_t n, double *out, void *stream)
{
    PU_REQUIRE(numerator && x && out && n > 0, "pu_ratio_dev: bad arguments");
    hipLaunchKernelGGL(ratio_dev_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, pu::as_stream(stream), numerator, x,
                       n, out);
    return pu::launch_check("ratio_dev_kernel");
}

size_t pu_lc_factor_workspace_bytes(int64_t n)
{
    // the smoothed series, pu_median's workspace and the median
    return (((size_t)std::max<int64_t>(n, 0) * 8 + 255) & ~size_t(255)) + pu_median_workspace_bytes() + 64;
}

int pu_lc_factor(const double *lc, int64_t n, const double *w, int64_t r, double *factor, double *median_out, void *ws,
                 size_t ws_bytes, void *stream)
{
    PU_REQUIRE(lc && w && factor && n > 0 && r >= 0, "pu_lc_factor: bad arguments");
    PU_REQUIRE(ws && ws_bytes >= pu_lc_factor_workspace_bytes(n) && reinterpret_cast<uintptr_t>(ws) % 256 == 0,
               "pu_lc_factor: workspace too small or not 256-byte aligned");
    char *wsb = reinterpret_cast<char *>(ws);
    // Gaussian, median, ratio, launch by launch (a one-launch form with grid barriers measured
    // slower: see the grid-barrier note above)
    double *smooth = reinterpret_cast<double *>(wsb);
    char *mws = wsb + (((size_t)n * 8 + 255) & ~size_t(255));
    double *med = reinterpret_cast<double *>(mws + pu_median_workspace_bytes());
    int rc = pu_gaussian_filter1d(lc, n, w, r, smooth, stream);
    if (!rc) rc = pu_median(smooth, n, median_out ? median_out : med, mws, pu_median_workspace_bytes(), stream);
    if (!rc) rc = pu_ratio_dev(median_out ? median_out : med, smooth, n, factor, stream);
    return rc;
}

int pu_zero_columns(double *out, int64_t nrows, int64_t ld, const int64_t *cols, int64_t ncols, void *stream)
{
    PU_REQUIRE(out && nrows > 0 && ld > 0, "pu_zero_columns: bad arguments");
    if (ncols <= 0) return PU_OK;
    PU_REQUIRE(cols != nullptr, "pu_zero_columns: cols is NULL");
    const unsigned gy = (unsigned)(nrows < 1024 ? nrows : 1024);
    hipLaunchKernelGGL(zero_cols_kernel, dim3(blocks_for(ncols, 256), gy), dim3(256), 0, pu::as_stream(stream), out,
                       nrows, ld, cols, ncols);
    return pu::launch_check("zero_cols_kernel");
}

}  // extern "C"
