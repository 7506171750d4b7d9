/*
 * ORACLE - TEST INFRASTRUCTURE ONLY.  Never linked into or called by the product.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * Plain-C float64 restatement of the reference's dedispersion hot path
 * (matteobachetti/radio-pulsar-utils, pulsarutils/dedispersion.py), with the
 * reference's interpreted-numpy arithmetic order so that results are bit-exact
 * against the golden vectors produced by running the reference itself
 * (tests/golden/make_golden.py):
 *
 *   or_shifts        <- dedispersion_shifts  dedispersion.py:125-139
 *   or_dedisperse    <- dedisperse/_dedisperse/roll_and_sum  :60-98
 *   or_search        <- _dedispersion_search :174-202 (prange -> OpenMP over trials)
 *
 * numpy semantics restated (SURVEY.md §8 a-R, verified by tests/test_oracle.py):
 *   - np.mean / np.sum of a contiguous float64 vector: sequential over 8192-element
 *     blocks, each block pairwise-summed (numpy pairwise_sum, PW_BLOCKSIZE 128).
 *   - np.std: mean -> x - mean -> x*x -> pairwise sum -> / n -> sqrt.
 *   - x // y on doubles: fmod-based divmod with the snapped quotient.
 *   - x ** -2 on scalars: libm pow.
 * Build: oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off, no fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { OR_U8 = 0, OR_F32 = 1, OR_F64 = 2 };

static volatile double kMinusTwo = -2.0; /* keep pow(x,-2) a libm call */

static double py_floordiv(double a, double b)
{
    double mod = fmod(a, b);
    if (b == 0.0) return a / b;
    double div = (a - mod) / b;
    if (mod != 0.0) {
        if ((b < 0) != (mod < 0)) div -= 1.0;
    }
    double fl;
    if (div != 0.0) {
        fl = floor(div);
        if (div - fl > 0.5) fl += 1.0;
    } else {
        fl = copysign(0.0, a / b);
    }
    return fl;
}

int or_shifts(int64_t nchan, double dm, double start_freq, double bandwidth,
              double sample_time, int64_t *out)
{
    double dfreq = bandwidth / (double)nchan;
    double stop = start_freq + bandwidth;
    double center = (stop + start_freq) / 2.0;
    double k = 4149.0 * dm;
    double ref = k * pow(center, kMinusTwo);
    for (int64_t i = 0; i < nchan; ++i) {
        double f = start_freq + (double)i * dfreq;
        double delay = k * pow(f, kMinusTwo) - ref;
        double q = py_floordiv(delay, sample_time);
        out[i] = (int64_t)nearbyint(q);
    }
    return 0;
}

static inline double load_elem(const void *x, int dtype, int64_t i)
{
    switch (dtype) {
    case OR_U8: return (double)((const uint8_t *)x)[i];
    case OR_F32: return (double)((const float *)x)[i];
    default: return ((const double *)x)[i];
    }
}

/* sum[t] += row[(t + shift) mod n] for t in [0,n): roll_and_sum with
 * N = normalize_shifts(-shift) (dedispersion.py:97), channel by channel. */
void or_dedisperse(const void *data, int dtype, int64_t nchan, int64_t n, int64_t ld,
                   const int64_t *shifts, double *sum)
{
    memset(sum, 0, sizeof(double) * (size_t)n);
    size_t esz = dtype == OR_U8 ? 1 : dtype == OR_F32 ? 4 : 8;
    for (int64_t c = 0; c < nchan; ++c) {
        const char *row = (const char *)data + (size_t)c * (size_t)ld * esz;
        int64_t sh = (-shifts[c]) % n;
        if (sh < 0) sh += n; /* roll amount in [0, n) */
        int64_t from_end = n - sh;
        for (int64_t i = 0; i < sh; ++i) sum[i] += load_elem(row, dtype, from_end + i);
        for (int64_t i = 0; i < from_end; ++i) sum[sh + i] += load_elem(row, dtype, i);
    }
}

/* numpy pairwise_sum for doubles (loops_utils.h.src), PW_BLOCKSIZE = 128 */
static double pairwise(const double *a, int64_t n)
{
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise(a, n2) + pairwise(a + n2, n - n2);
    }
}

/* np.add.reduce over a contiguous float64 vector: 8192-element buffered blocks */
double or_np_sum(const double *a, int64_t n)
{
    double res = 0.0;
    for (int64_t s = 0; s < n; s += 8192) {
        int64_t m = n - s < 8192 ? n - s : 8192;
        res += pairwise(a + s, m);
    }
    return res;
}

static double np_max(const double *a, int64_t n)
{
    double m = a[0];
    for (int64_t i = 1; i < n; ++i) {
        if (isnan(a[i]) || isnan(m)) { m = NAN; break; }
        if (a[i] > m) m = a[i];
    }
    return m;
}

/* np.std(a) (ddof 0); scratch holds n doubles */
double or_np_std(const double *a, int64_t n, double *scratch)
{
    double mean = or_np_sum(a, n) / (double)n;
    for (int64_t i = 0; i < n; ++i) {
        double d = a[i] - mean;
        scratch[i] = d * d;
    }
    return sqrt(or_np_sum(scratch, n) / (double)n);
}

/* One trial of _dedispersion_search (dedispersion.py:182-201) on a dedispersed
 * series ``dd`` (n doubles).  work: 2n doubles. */
static void trial_stats_w(const double *dd, int64_t n, double *work, double *max_out,
                          double *std_out, double *snr_out, int64_t *win_out, double *snr_w)
{
    double *shifted = work, *reb = work + n;
    double mean = or_np_sum(dd, n) / (double)n;
    for (int64_t i = 0; i < n; ++i) shifted[i] = dd[i] - mean;
    double best_snr = 0.0;
    int64_t best_win = 0;
    for (int wp = 0; wp < 4; ++wp) {
        int64_t w = (int64_t)1 << wp;
        int64_t nb = n / w;
        if (nb == 0) { /* np.max of an empty array raises in the reference */
            continue;
        }
        for (int64_t i = 0; i < nb; ++i) {
            double acc = 0.0;
            for (int64_t j = 0; j < w; ++j) acc += shifted[i * w + j];
            reb[i] = acc;
        }
        double mx = np_max(reb, nb);
        /* np.std(reb) needs a scratch vector distinct from reb: reuse the tail of
         * ``shifted`` is not allowed, so compute in two passes without scratch */
        double m2 = or_np_sum(reb, nb) / (double)nb;
        double *sq = (double *)malloc(sizeof(double) * (size_t)nb);
        for (int64_t i = 0; i < nb; ++i) {
            double d = reb[i] - m2;
            sq[i] = d * d;
        }
        double sd = sqrt(or_np_sum(sq, nb) / (double)nb);
        free(sq);
        double snr = mx / sd;
        if (snr_w) snr_w[wp] = snr;
        if (snr > best_snr) {
            best_snr = snr;
            best_win = w;
        }
    }
    *max_out = np_max(shifted, n);
    {
        double m2 = or_np_sum(shifted, n) / (double)n;
        double *sq = (double *)malloc(sizeof(double) * (size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            double d = shifted[i] - m2;
            sq[i] = d * d;
        }
        *std_out = sqrt(or_np_sum(sq, n) / (double)n);
        free(sq);
    }
    *snr_out = best_snr;
    *win_out = best_win;
}

void or_trial_stats(const double *dd, int64_t n, double *work, double *max_out,
                    double *std_out, double *snr_out, int64_t *win_out)
{
    trial_stats_w(dd, n, work, max_out, std_out, snr_out, win_out, NULL);
}

/* _dedispersion_search: trials in parallel (numba prange -> OpenMP).
 * dedisp_out (nullable): [ndm][n] float64 dedispersed series.
 * snr_w_out (nullable, test-side only): [ndm][4] the S/N of each rebin width 1/2/4/8
 * (entries of widths longer than the series are left as they are). */
int or_search_w(const void *data, int dtype, int64_t nchan, int64_t n, int64_t ld,
                const double *dms, int64_t ndm, double start_freq, double bandwidth,
                double sample_time, double *max_out, double *std_out, double *snr_out,
                int64_t *win_out, double *dedisp_out, double *snr_w_out, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int err = 0;
#pragma omp parallel
    {
        double *dd = (double *)malloc(sizeof(double) * (size_t)n * 3);
        int64_t *sh = (int64_t *)malloc(sizeof(int64_t) * (size_t)nchan);
        if (!dd || !sh) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 1)
            for (int64_t i = 0; i < ndm; ++i) {
                or_shifts(nchan, dms[i], start_freq, bandwidth, sample_time, sh);
                or_dedisperse(data, dtype, nchan, n, ld, sh, dd);
                if (dedisp_out) memcpy(dedisp_out + (size_t)i * (size_t)n, dd, sizeof(double) * (size_t)n);
                trial_stats_w(dd, n, dd + n, &max_out[i], &std_out[i], &snr_out[i], &win_out[i],
                              snr_w_out ? snr_w_out + 4 * i : NULL);
            }
        }
        free(dd);
        free(sh);
    }
    return err ? -1 : 0;
}

int or_search(const void *data, int dtype, int64_t nchan, int64_t n, int64_t ld,
              const double *dms, int64_t ndm, double start_freq, double bandwidth,
              double sample_time, double *max_out, double *std_out, double *snr_out,
              int64_t *win_out, double *dedisp_out, int nthreads)
{
    return or_search_w(data, dtype, nchan, n, ld, dms, ndm, start_freq, bandwidth, sample_time, max_out,
                       std_out, snr_out, win_out, dedisp_out, NULL, nthreads);
}

int or_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
