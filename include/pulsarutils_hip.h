/*
 * pulsarutils_hip.h - C-ABI of the MI355X (gfx950) dedispersion + cleaning library
 * (libpulsarutils_hip.so).  Plain pointers and sizes only; no torch types.
 *
 * The reference (matteobachetti/radio-pulsar-utils, package ``pulsarutils``) is pure
 * Python + numba; it has no FFI of its own.  Each entry point below replaces one
 * reference function (cited file:line, paths relative to the reference root); the
 * Python host layer (radio-pulsar-utils_amd/pulsarutils) binds them with ctypes
 * exactly as INTEGRATION.md shows.
 *
 * Conventions
 *  - Device pointers are owned by the caller (e.g. torch tensors).  Host pointers
 *    are marked "host".  Row-major 2-D arrays carry a leading dimension ``ld``
 *    (elements).
 *  - Calls are asynchronous on ``stream`` (a hipStream_t passed as void*; NULL = the
 *    null stream) and never throw - except pu_plan_search / pu_plan_finalize, which
 *    synchronise ``stream`` once to settle their certification step (see
 *    pu_plan_finalize) and return final outputs.  They return PU_OK (0) or a negative PU_E* code;
 *    pu_last_error() returns a thread-local message for the last failure.
 *  - The caller selects the device (hipSetDevice) before calling.
 */
#ifndef PULSARUTILS_HIP_H
#define PULSARUTILS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types */
#define PU_U8 0
#define PU_F32 1
#define PU_F64 2
#define PU_I64 3 /* rebin/roll helpers only */

/* accumulation type of the dedispersion sum */
#define PU_ACC_NATIVE 0 /* u8 -> f32 (exact), f32 -> f32, f64 -> f64 */
#define PU_ACC_F32 1
#define PU_ACC_F64 2 /* float64 accumulator in channel order: bit-exact vs the reference */

/* status codes */
#define PU_OK 0
#define PU_EINVAL (-1)
#define PU_EHIP (-2)
#define PU_ENOMEM (-3)
#define PU_EUNSUPPORTED (-4)

const char *pu_version(void);
const char *pu_last_error(void);

/* ------------------------------------------------------------------ planner (host) */

/* Replaces dedispersion_shifts (pulsarutils/dedispersion.py:125-139) for ``ndm``
 * trials at once.  float64 with CPython scalar semantics (libm pow, float floor
 * division, rint).  host: dms[ndm], out[ndm][nchan]. */
int pu_shift_table(int64_t nchan, const double *dms, int64_t ndm, double start_freq,
                   double bandwidth, double sample_time, int64_t *out);

/* ------------------------------------------------------------------ dedispersion */

typedef struct pu_plan pu_plan;

/* Build a dedispersion plan for ``ndm`` trials over an (nchan, nsamples) filterbank
 * of element type ``dtype``.  host: shifts[ndm][nchan] = the reference's per-channel
 * integer delays (dedispersion_shifts output, any sign).  Tiles DM trials x time,
 * derives per-tile LDS halos and uploads the metadata to the current device.
 * Replaces the per-trial shift computation + normalize_shifts of
 * _dedispersion_search (dedispersion.py:183-184, 97, 101-122). */
int pu_plan_create(pu_plan **plan, int dtype, int acc, int64_t nchan, int64_t nsamples,
                   const int64_t *shifts, int64_t ndm);
/* Same, choosing the float32-accumulation strategy: ``group`` = channels summed into
 * one exact partial-sum row per distinct relative-shift vector:
 * 0 = default (the cheapest of the wide / tall shapes with G = 4 and 8 by the planner's
 * cost model, falling back to smaller groups / channel mode when the trial grid does not
 * suit them), 1 = channel mode, 2/4/8.  Float64 accumulation always runs channel mode
 * (the reference's channel order).  = pu_plan_create_ex with opts {group, -1, 0, -1, -1}. */
int pu_plan_create_grouped(pu_plan **plan, int dtype, int acc, int64_t nchan, int64_t nsamples,
                           const int64_t *shifts, int64_t ndm, int group);

/* Explicit planner options (the production library reads no environment: every
 * strategy choice is an argument here or a default).  -1 / 0 = automatic. */
typedef struct pu_plan_opts {
    int32_t group;          /* 0 auto, 1 channel mode, 2 / 4 / 8 */
    int32_t shape;          /* subband workgroup shape: -1 auto, 0 wide, 1 pair, 2 tall */
    int32_t lds_budget_kb;  /* 0: default (160 KiB subband, 64 KiB channel mode) */
    int32_t u8_dma;         /* -1 auto (8-bit rows by LDS-DMA when n % 4 == 0), 0 global-memory build */
    int32_t dt_major;       /* -1 auto item order, 0 time-tile major, 1 DM-tile major */
    int32_t slot16;         /* 16-bit integer slots for 8-bit rows by LDS-DMA in 256-sample
                             * time tiles: -1 auto (= 1), 0 never (float32 slots), 1 every
                             * group size (round 6: -1 meant groups of <= 4 channels) */
    int32_t reserved[2];    /* zero */
} pu_plan_opts;
int pu_plan_create_ex(pu_plan **plan, int dtype, int acc, int64_t nchan, int64_t nsamples,
                      const int64_t *shifts, int64_t ndm, const pu_plan_opts *opts);
void pu_plan_destroy(pu_plan *plan);

/* Device scratch bytes pu_plan_search needs (per-tile partial statistics). */
size_t pu_plan_workspace_bytes(const pu_plan *plan);

/* Replaces _dedispersion_search (dedispersion.py:174-202): for every trial the
 * circular shift-and-sum over channels, mean subtraction, and the S/N of the
 * 1/2/4/8-sample rebinned series; outputs max, std, best snr, best rebin (device,
 * [ndm] each).  data: device (nchan rows of ld elements). */
int pu_plan_search(pu_plan *plan, const void *data, int64_t ld, double *max_out,
                   double *std_out, double *snr_out, int32_t *rebin_out, void *workspace,
                   size_t workspace_bytes, void *stream);

/* pu_plan_search split in two, for pipelining (multi-GPU: the search of early time
 * chunks overlaps the broadcast of later ones).  search_tiles runs the
 * shift-and-sum + per-tile statistics of time tiles [tt_begin, tt_end) only (time
 * tile = pu_plan_info "time_tile" samples; a tile reads its window plus the shift
 * halo, modulo nsamples); once every tile has run, finalize combines the per-tile
 * records into the per-trial outputs exactly as pu_plan_search does. */
int pu_plan_search_tiles(pu_plan *plan, const void *data, int64_t ld, int64_t tt_begin,
                         int64_t tt_end, void *workspace, size_t workspace_bytes, void *stream);
int pu_plan_finalize(pu_plan *plan, const void *data, int64_t ld, double *max_out,
                     double *std_out, double *snr_out, int32_t *rebin_out, void *workspace,
                     size_t workspace_bytes, void *stream);

/* pu_plan_finalize of trials [trial_begin, trial_end) only (time-tile sharding across
 * GPUs, DESIGN.md §5: each rank searches a range of time tiles for every trial, the
 * per-tile records of each trial are moved to the rank that owns the trial, and the owner
 * finalizes its trials).  The records are the workspace's first bytes, trial-major:
 * record (trial d, time tile t) = rec_stride elements of rec_elem_bytes (float32 or
 * float64) at element (d ntt + t) rec_stride (pu_plan_info "rec_elem_bytes",
 * "rec_stride"); only the range's records are read.  Outputs are indexed by plan trial
 * (arrays of ndm; only [trial_begin, trial_end) written).  Certification as in
 * pu_plan_finalize (flagged trials recomputed exactly from data, which must then hold the
 * whole filterbank).  The replaced reference code is the same (dedispersion.py:174-202). */
int pu_plan_finalize_range(pu_plan *plan, const void *data, int64_t ld, int64_t trial_begin,
                           int64_t trial_end, double *max_out, double *std_out, double *snr_out,
                           int32_t *rebin_out, void *workspace, size_t workspace_bytes, void *stream);

/* The finalize of trials [trial_begin, trial_end) without the exact recomputation, for
 * time-tile sharding where each rank holds only its time slice of the filterbank
 * (DESIGN.md §5): the fast statistics are written (outputs indexed by plan trial) and the
 * trials certification would recompute are returned instead - counts[0] = how many,
 * counts[1] = of which with a non-finite partial; the first min(count, cap) plan trial
 * indices into flagged (host, ascending).  Synchronises stream.  The caller settles them
 * (pulsarutils.parallel: a non-finite input anywhere -> the NaN rule for every trial;
 * otherwise each rank's slice of pu_plan_exact_series, gathered, + pu_series_stats). */
int pu_plan_finalize_range_flagged(pu_plan *plan, int64_t trial_begin, int64_t trial_end,
                                   double *max_out, double *std_out, double *snr_out, int32_t *rebin_out,
                                   void *workspace, size_t workspace_bytes, int32_t *flagged, int64_t cap,
                                   int64_t *counts, void *stream);

/* The reference's float64 dedispersed series (channel order, dedispersion.py:86-98, bit
 * for bit) of m plan trials (host indices) at samples [t_begin, t_end) into out (device,
 * m x (t_end - t_begin) contiguous).  Sample t reads column (t + shift) mod nsamples of each
 * channel: a time-split rank computes its own samples from the columns it holds.
 * Synchronises. */
int pu_plan_exact_series(pu_plan *plan, const void *data, int64_t ld, const int32_t *trials, int64_t m,
                         int64_t t_begin, int64_t t_end, double *out, void *stream);

/* *flag (device int32) = 1 if any of the nrows x ncols float32 / float64 elements (row
 * stride ld) is NaN or +-inf, else 0 (always 0 for uint8).  Asynchronous on stream. */
int pu_nonfinite_any(const void *data, int dtype, int64_t nrows, int64_t ncols, int64_t ld, int32_t *flag,
                     void *stream);

/* Certification (pu_plan_search and pu_plan_finalize).  The fast
 * path's per-trial statistics are summed in another order than numpy's; a trial whose
 * result that order could change - a zero or rounding-level std (constant input), a
 * non-finite value, or (float64 accumulation, and uint8 input with exact float32 sums)
 * two windows' S/N within the rounding bound of each other - is recomputed exactly:
 * its series by float64 channel-order dedispersion (bit-identical to the reference's
 * dedisperse) and its statistics by pu_series_stats.  An input holding NaN or +-inf
 * gives every trial the reference's result max = std = NaN, snr = 0, rebin = 0.
 * Both calls therefore synchronise ``stream`` once before returning (the outputs are
 * final when they return).  pu_plan_info reports the trials of the last call that
 * were recomputed ("cert_rechecked") and whether the NaN rule applied ("cert_nan"). */

/* The reference's statistics of given float64 dedispersed series, in numpy's exact
 * order (dedispersion.py:186-201, bit-exact): for each row r of series (rows x n,
 * leading dimension ld) max = np.max(s), std = np.std(s) with s = row - np.mean(row),
 * and the best S/N over the 1/2/4/8-sample rebinned s (quick_resample order) with the
 * reference's strict first-best rule from (0, 0).  Outputs go to position index[r]
 * (device int32; NULL = r).  workspace: 256-byte aligned; rows are processed in
 * batches of as many as pu_series_stats_workspace_bytes(batch, n) <= workspace_bytes
 * allows (at least one). */
size_t pu_series_stats_workspace_bytes(int64_t rows, int64_t n);
int pu_series_stats(const double *series, int64_t rows, int64_t n, int64_t ld,
                    const int32_t *index, double *max_out, double *std_out, double *snr_out,
                    int32_t *rebin_out, void *workspace, size_t workspace_bytes, void *stream);

/* Replaces dedisperse (dedispersion.py:93-98) for every trial of the plan: writes
 * the dedispersed plane plane[trial * ld_plane + t] in the accumulation type
 * (float32 or float64), the show=True plane of dedispersion_search (:214-227). */
int pu_plan_dedisperse(pu_plan *plan, const void *data, int64_t ld, void *plane,
                       int64_t ld_plane, void *stream);

/* The plan's DM tiles in launch order (tile t = trials first[t] .. first[t] + count[t] - 1);
 * writes up to ``n`` of each (either pointer may be NULL) and returns the tile count. */
int pu_plan_dm_tiles(const pu_plan *plan, int32_t *first, int32_t *count, int n);
/* pu_plan_dedisperse restricted to one DM tile ``dt`` of the plan: the tile's trials'
 * rows (dedispersion.py:93-98) at plane rows 0 .. count[dt] - 1, computed by the very
 * kernel instantiation, tables and tiling a full launch of the plan uses (parity tests
 * of a production plan's series at full size without its whole plane). */
int pu_plan_dedisperse_dm_tile(pu_plan *plan, const void *data, int64_t ld, int64_t dt,
                               void *plane, int64_t ld_plane, void *stream);

/* Measurement (bench.py): record a HIP event pair on the launch stream around each
 * of the next ``nslots`` dedispersion-kernel launches of this plan (0 disables). */
int pu_plan_enable_timing(pu_plan *plan, int nslots);
/* Synchronises on the recorded events and writes up to ``n`` kernel durations (ms,
 * launch order).  Returns the number written, or a negative PU_E* code. */
int pu_plan_kernel_times(pu_plan *plan, float *ms, int n);

/* Diagnostics: in the PU_STAMPS build (make stamps -> libpulsarutils_hip_stamps.so) the
 * first call arms per-phase shader-clock stamps of the subband kernel and returns 0;
 * later calls synchronise, write up to ``n`` (<= 8) summed wave-cycle totals {stage
 * metadata, barrier A wait, build, barrier B wait, DMA issue, sum, epilogue, -} and
 * reset them.  Returns 0 in the production build. */
int pu_plan_stamps(pu_plan *plan, int64_t *out, int n);

/* Introspection (tests / DESIGN.md): fills up to ``n`` of
 * {ndm, dm_tiles, time_tiles, trials_per_tile, time_tile, chans_per_step,
 *  row_stride, lds_bytes, acc_is_f64, max_spread, group, slots, stages,
 *  slot_bytes, raw_stride, exec_adds, lds_traffic, cert_rechecked, cert_nan, cert_std,
 *  cert_sign, cert_tie, cert_us, kernel, rec_elem_bytes, rec_stride}: exec_adds and lds_traffic are the adds and LDS bytes (reads,
 *  writes, DMA) one launch executes (subband mode; 0 otherwise); the cert_* fields
 *  describe the last search's certification step (see pu_plan_finalize): trials
 *  recomputed, the NaN rule, and how many trials each check flagged (std not above its
 *  rounding bound, S/N sign, S/N tie) and the host microseconds spent settling them;
 *  kernel: 0 dedisp_kernel (channel order), 1 dedisp_f64_kernel, 2 dedisp_sub_kernel
 *  (float32 slots), 3 dedisp_sub_kernel with 16-bit integer slots (8-bit input);
 *  rec_elem_bytes / rec_stride: the per-(trial, time tile) record layout at the start of
 *  the workspace (pu_plan_finalize_range).  Returns the count written. */
int pu_plan_info(const pu_plan *plan, int64_t *info, int n);

/* ------------------------------------------------------------------ streams */

/* A compute stream on the current device whose CU mask leaves ``reserve`` CUs out
 * (spread over the XCDs), for launching the search while an RCCL collective runs on
 * another stream: the collective's workgroups find those CUs free (the search holds one
 * 160 KiB-LDS workgroup per CU).  No reference counterpart (multi-GPU path, DESIGN.md
 * §5; the reference's parallelism is numba prange, dedispersion.py:181).
 * *stream: hipStream_t as void*, released with pu_stream_destroy. */
int pu_stream_create_cu_masked(int reserve, void **stream);
int pu_stream_destroy(void *stream);

/* ------------------------------------------------------------------ cleaning */

/* Per-row sums in numpy's exact add.reduce order (8192-element blocks, each
 * pairwise-summed), the reductions behind ndarray.mean(1) / np.std(axis=1) in
 * get_noisier_channels (clean.py:60), measure_channel_variability (clean.py:119)
 * and renormalize_data (clean.py:84).
 *   mode 0: sum of x                     (acc: f32 for f32 input, else f64)
 *   mode 1: sum of (x - center[r])^2     (center: device [nrows], acc type)
 *   mode 2: sum of f64(x) * scale[t]     (scale: device [n] f64; acc f64)
 *   mode 3: sum of f64(x)                (acc f64 for every input type)
 *   mode 4: sum of f64(x)^2              (acc f64; get_spectral_stats, stats.py:46-47)
 * out: device [nrows] in the acc type; ``divisor`` > 0 divides each sum in float64
 * and rounds to the acc type (numpy true_divide by the count). */
int pu_row_sums(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, int mode,
                const void *center, const double *scale, double divisor, void *out,
                void *workspace, size_t workspace_bytes, void *stream);
size_t pu_row_sums_workspace_bytes(int64_t nrows, int64_t n);

/* One pass for get_noisier_channels + measure_channel_variability (clean.py:60, 119):
 * means[r] = ndarray.mean(1) exactly as pu_row_sums mode 0 with divisor n (f32 for f32
 * input, else f64), and moments[3 r .. 3 r + 2] = (c, sum(x - c), sum((x - c)^2)) in
 * float64, c = x[r, 0], summed in no particular order.  The caller certifies the
 * std-based decisions from the moments (pulsarutils.clean._certified_variability) and
 * runs the exact second pass (pu_row_sums mode 1) only when one is within its rounding
 * bound.  ws: pu_row_moments_workspace_bytes(nrows, n), 8-byte aligned. */
int pu_row_moments(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld, void *means,
                   double *moments, void *workspace, size_t workspace_bytes, void *stream);
size_t pu_row_moments_workspace_bytes(int64_t nrows, int64_t n);

/* Column means over the rows with skip[r] == 0, sequential in row order
 * (renormalize_data's zero-DM light curve, clean.py:77).  out: device [n] f64. */
int pu_col_means(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld,
                 const uint8_t *skip, double *out, void *stream);

/* scipy.ndimage.gaussian_filter of a 1-D float64 series, mode 'reflect', in
 * scipy's symmetric correlate1d order (clean.py:79).  weights: device [2r+1]. */
int pu_gaussian_filter1d(const double *x, int64_t n, const double *weights, int64_t radius,
                         double *out, void *stream);

/* factor[t] = numerator / x[t] (clean.py:80). */
int pu_ratio(double numerator, const double *x, int64_t n, double *out, void *stream);

/* np.median of a float64 device series (clean.py:80 ``np.median(lc_smooth)``) into
 * out[0] on the device, bit-exact: radix select of the two middle order statistics,
 * numpy's mean of them; NaN if any element is NaN.  ws: pu_median_workspace_bytes(),
 * 8-byte aligned. */
/* get_noisier_channels' decision (pulsarutils/clean.py:58-67 with stats.py:11-32 ref_mad):
 * mask[i] = spec[i] > medfilt(spec, 7)[i] + 5 * ref_mad(spec), numpy's dtypes and order
 * (spec float32 for float32 input, float64 otherwise; mad_c = statsmodels' MAD constant
 * norm.ppf(3/4)).  One workgroup, 2 <= n <= 4096.  *flag = 1 (mask not written) when spec
 * holds a NaN / inf: the caller decides those on the host. */
int pu_noisy_channels(const void *spec, int dtype, int64_t n, double mad_c, uint8_t *mask, int32_t *flag,
                      void *stream);

/* measure_channel_variability's decision (pulsarutils/clean.py:114-133) certified from
 * the means pass: means[nrows] (dtype PU_F32 / PU_F64: numpy's mean dtype) and
 * moments[nrows][3] = (c, sum(x - c), sum((x - c)^2)) in float64 (pu_row_moments), n
 * samples per row; mef, gam, u: the error factors of clean._certified_variability (the
 * moments' relative error bound, numpy's std summation bound, the unit roundoff).
 * mask[i] = std outside the quartile limits, or bad[i].  One workgroup, nrows <= 4096.
 * *flag = 1 (mask not written, or not certified) for non-finite statistics, too few good
 * channels for the reference's quartile indices, or a channel within its bound of a
 * limit: the caller then computes numpy's std exactly (pu_row_sums mode 1). */
int pu_variability_cert(const void *means, int dtype, const double *moments, int64_t nrows, int64_t n,
                        double mef, double gam, double u, const uint8_t *bad, uint8_t *mask,
                        int32_t *flag, void *stream);

/* get_noisier_channels and then measure_channel_variability(badchans_mask=<that mask>)
 * (pulsarutils/clean.py:58-67, then :114-133) in ONE launch: pu_noisy_channels' decision on
 * spec = means (noisy[nrows], *noisy_flag), then pu_variability_cert's with the noisy mask
 * as bad (var[nrows], *var_flag), same arguments and flag meanings as those two calls
 * (mad_c: pu_noisy_channels'; mef, gam, u: pu_variability_cert's).  One workgroup,
 * 2 <= nrows <= 1024; a non-finite spec sets both flags. */
int pu_channel_masks(const void *means, int dtype, const double *moments, int64_t nrows, int64_t n,
                     double mad_c, double mef, double gam, double u, uint8_t *noisy,
                     int32_t *noisy_flag, uint8_t *var, int32_t *var_flag, void *stream);

size_t pu_median_workspace_bytes(void);
int pu_median(const double *x, int64_t n, double *out, void *ws, size_t ws_bytes, void *stream);

/* factor[t] = numerator[0] / x[t] with the numerator in device memory (clean.py:80). */
int pu_ratio_dev(const double *numerator, const double *x, int64_t n, double *out, void *stream);

/* renormalize_data's light-curve chain (clean.py:77-82 after the zero-DM column means):
 * lc_smooth = gaussian_filter(lc, sigma) (weights: device [2r+1], as pu_gaussian_filter1d),
 * med = np.median(lc_smooth) (as pu_median), factor[t] = med / lc_smooth[t] (as
 * pu_ratio_dev) - those three calls on one stream, with their scratch in one workspace.
 * median_out: device [1] or NULL.  ws: pu_lc_factor_workspace_bytes(n), 256-byte aligned. */
size_t pu_lc_factor_workspace_bytes(int64_t n);
int pu_lc_factor(const double *lc, int64_t n, const double *weights, int64_t radius, double *factor,
                 double *median_out, void *ws, size_t ws_bytes, void *stream);

/* renormalize_data apply pass (clean.py:81-94): out[c][t] = bad[c] ? 0 :
 * (f64(x[c][t]) * factor[t] - spec[c]) / spec[c]; if col_means != NULL it also
 * writes the sequential column mean of ``out`` (the cut_outliers light curve). */
int pu_renorm_apply(const void *x, int dtype, int64_t nchan, int64_t n, int64_t ld,
                    const double *factor, const double *spec, const uint8_t *bad,
                    double *out, int64_t ld_out, double *col_means, void *stream);

/* Opt-in zero-DM subtraction (BASELINE north_star "zero-DM subtraction"; the reference
 * has no counterpart: clean.py:77-82 only DIVIDES by the smoothed zero-DM series, so
 * renormalize_data keeps this off by default).  As pu_renorm_apply, then for every
 * good channel out[c][t] -= S[t] / ngood, S[t] = the in-order sum over channels of the
 * normalised values (bad channels contribute +0.0); bad channels stay 0.  ngood =
 * the number of channels with bad[c] == 0.  col_means (if not NULL) is S[t] / nchan,
 * i.e. the cut_outliers light curve of the data BEFORE the subtraction. */
int pu_renorm_apply_zero_dm(const void *x, int dtype, int64_t nchan, int64_t n, int64_t ld,
                            const double *factor, const double *spec, const uint8_t *bad,
                            int64_t ngood, double *out, int64_t ld_out, double *col_means,
                            void *stream);

/* cut_outliers of renormalize_data (clean.py:93-105) on the device: from the column
 * means lc[n] of the renormalised plane (pu_renorm_apply's col_means), mask[t] =
 * uniform_filter1d(lc, 16)[t] > 5 sd  or  < -3 sd, sd = np.std(uniform_filter1d(lc,
 * 16)[::16]), and out[:, t] = 0 where mask[t].  scipy's running-sum order is not
 * reproducible in parallel: every decision is first made on directly summed windows and
 * CERTIFIED against a rigorous rounding bound of both orders; when a decision is closer
 * to its threshold than the bound (or a value is NaN) the flag word ws[0:4] (uint32) is
 * set and a one-workgroup kernel on the same stream recomputes the mask with scipy's and
 * numpy's own arithmetic (running sum, add.reduce order).  Either way the mask and the
 * zeroed columns are the reference's, with no host round trip (round 4: the caller used
 * to redo the step with scipy).  ws[4:8] (uint32) = number of bad bins.  n >= 64; ws:
 * pu_cut_outliers_workspace_bytes(n), 8-byte aligned.
 * pu_cut_outliers_exact: the exact path only (testing, or callers that want it). */
size_t pu_cut_outliers_workspace_bytes(int64_t n);
int pu_cut_outliers(const double *lc, int64_t n, double *out, int64_t nrows, int64_t ld_out,
                    uint8_t *mask, void *workspace, size_t workspace_bytes, void *stream);
int pu_cut_outliers_exact(const double *lc, int64_t n, double *out, int64_t nrows, int64_t ld_out,
                          uint8_t *mask, void *workspace, size_t workspace_bytes, void *stream);

/* out[:, cols[k]] = 0 for k < ncols (clean.py:105). cols: device int64. */
int pu_zero_columns(double *out, int64_t nrows, int64_t ld_out, const int64_t *cols,
                    int64_t ncols, void *stream);

/* ------------------------------------------------------------------ rebin / roll */

/* quick_resample (dedispersion.py:38-57): out[r][i] = 0 + sum_{j<w} x[r][i*w+j]
 * in float64, i < n/w. */
int pu_rebin_time(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld,
                  int64_t rebin, double *out, void *stream);

/* quick_chan_rebin (dedispersion.py:15-35): out[g][t] = sum_{j<r} x[g*r+j][t]
 * sequentially; output type: f32->f32, f64->f64, u8->u64, i64->i64. */
int pu_rebin_chan(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld,
                  int64_t rebin, void *out, void *stream);

/* apply_dm_shifts_to_data (dedispersion.py:254-258): out[c][t] =
 * x[c][(t + shift[c]) mod n] (shift = rint of the reference shift; any sign). */
int pu_roll_rows(const void *x, int dtype, int64_t nrows, int64_t n, int64_t ld,
                 const int64_t *shifts, void *out, void *stream);

/* roll_and_sum (dedispersion.py:60-83), in place on a float64 accumulator:
 * sum[t] += f64(x[(t - roll) mod n]). */
int pu_roll_and_sum(const void *x, int dtype, int64_t n, int64_t roll, double *sum,
                    void *stream);

/* (rows, cols) -> (cols, rows) transpose of 1/2/4/8-byte elements: the time-major ->
 * channel-major reordering sigpyproc's FilReader.readBlock performs on SIGPROC data
 * (clean.py:327, stats.py:45).  dst[c * ld_dst + r] = src[r * ld_src + c]. */
int pu_transpose(const void *src, int elem_bytes, int64_t rows, int64_t cols, int64_t ld_src,
                 void *dst, int64_t ld_dst, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PULSARUTILS_HIP_H */
