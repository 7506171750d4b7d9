"""HIP cleaning parity (GPU): channel masks, time-bin masks and renormalised data are
bit-exact against the reference's own outputs (goldens) and the numpy oracle."""
import hashlib
from dataclasses import replace

import numpy as np
import pytest

from oracle import clean_oracle as co
from pulsarutils import clean as C
from pulsarutils import synth
from pulsarutils.configs import CONFIGS

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def check_case(golden, tag, x):
    arrays, meta = golden
    assert sha(x) == meta[f"{tag}_input_sha256"]
    import torch
    from pulsarutils import _hip
    xd = _hip.to_device(x)
    means = C.channel_means_device(xd).cpu().numpy()
    np.testing.assert_array_equal(means, arrays[f"{tag}_spec_mean"])
    std = np.sqrt(C.channel_variances_device(xd).cpu().numpy())
    np.testing.assert_array_equal(std, arrays[f"{tag}_spec_std"])
    bad = C.get_noisier_channels(x)
    np.testing.assert_array_equal(bad, arrays[f"{tag}_noisier"])
    np.testing.assert_array_equal(C.measure_channel_variability(x), arrays[f"{tag}_variability"])
    np.testing.assert_array_equal(C.measure_channel_variability(x, badchans_mask=bad),
                                  arrays[f"{tag}_variability_masked"])
    for cut in (False, True):
        key = f"{tag}_renorm_{'cut' if cut else 'nocut'}"
        out, bins = C.renormalize_device(xd, badchans_mask=bad, cut_outliers=cut)
        ren = out.cpu().numpy()
        if sha(ren) != meta[key + "_sha256"]:
            ref = co.renormalize(x, badchans_mask=bad, cut_outliers=cut)
            diff = np.argwhere(ren != ref)
            pytest.fail(f"{key}: {len(diff)} elements differ, first {diff[:5].tolist()}")
        if cut:
            expect = arrays[key + "_badbins"]
            np.testing.assert_array_equal(np.nonzero(bins.cpu().numpy())[0], expect)
        del out
        torch.cuda.empty_cache()


@pytest.mark.parametrize("dt", ["f32", "u8", "f64"])
def test_clean_ragged(gpu, golden, dt):
    rag = replace(CONFIGS["C4"], nchan=100, nsamples=12345, seed=77)
    check_case(golden, f"rag{dt}", synth.rfi_filterbank_np(rag, dtype=dt))


@pytest.mark.parametrize("dt", ["f32", "u8"])
def test_clean_c4_bitexact(gpu, golden, dt):
    check_case(golden, f"c4{dt}", synth.rfi_filterbank_np(CONFIGS["C4"], dtype=dt))


def test_clean_c1_float64(gpu, golden):
    arrays, meta = golden
    from test_gpu_dedisperse import c1_input
    x = c1_input()
    bad = C.get_noisier_channels(x)
    np.testing.assert_array_equal(bad, arrays["c1_noisier"])
    np.testing.assert_array_equal(C.measure_channel_variability(x), arrays["c1_variability"])
    ren = C.renormalize_data(x, badchans_mask=bad, cut_outliers=True)
    assert sha(ren) == meta["c1_renorm_cut_sha256"]


def test_renormalize_api_matches_oracle_small(gpu):
    rng = np.random.default_rng(9)
    x = (rng.random((20, 700)) * 5 + 1).astype(np.float32)
    bad = np.zeros(20, bool)
    bad[[3, 7]] = True
    np.testing.assert_array_equal(C.renormalize_data(x, badchans_mask=bad, cut_outliers=True),
                                  co.renormalize(x, badchans_mask=bad, cut_outliers=True))
    np.testing.assert_array_equal(C.renormalize_data(x), co.renormalize(x))


def test_renormalize_channel_mask_reuse(gpu):
    """renormalize_device reuses the device copy of an unchanged channel mask (round 5):
    alternating masks A, B, A, an all-false mask (None) and A again, also on a second
    stream, each equal to the numpy restatement - a changed mask is never served stale."""
    import torch
    from pulsarutils import _hip
    rng = np.random.default_rng(21)
    x = (rng.random((24, 900)) * 5 + 1).astype(np.float32)
    xd = _hip.to_device(x)
    a = np.zeros(24, bool)
    a[[1, 5]] = True
    b = np.zeros(24, bool)
    b[[5, 17, 20]] = True
    s2 = torch.cuda.Stream()
    for i, m in enumerate([a, b, a, None, a, b]):
        def run():
            out, _ = C.renormalize_device(xd, badchans_mask=m, cut_outliers=True)
            return out.cpu().numpy()
        if i >= 4:
            s2.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s2):
                got = run()
        else:
            got = run()
        np.testing.assert_array_equal(got, co.renormalize(x, badchans_mask=m, cut_outliers=True))


@pytest.mark.parametrize("dt", ["f32", "u8", "f64"])
@pytest.mark.parametrize("n,pad,off", [(12346, 6, 0), (16388, 4, 2), (8192 * 2 + 8, 0, 1)])
def test_clean_strided_views(gpu, dt, n, pad, off):
    """Row stride / base alignment select the vector width of the column and row
    kernels (4, 2 or 1 elements): padded and offset views match numpy bit for bit."""
    import torch
    from pulsarutils import _hip
    rag = replace(CONFIGS["C4"], nchan=37, nsamples=n, seed=5)
    x = synth.rfi_filterbank_np(rag, dtype=dt)
    big = np.zeros((x.shape[0], off + n + pad), dtype=x.dtype)
    big[:, off:off + n] = x
    xd = _hip.to_device(big)[:, off:off + n]
    assert xd.stride(0) == off + n + pad
    np.testing.assert_array_equal(C.channel_means_device(xd).cpu().numpy(), x.mean(1))
    np.testing.assert_array_equal(np.sqrt(C.channel_variances_device(xd).cpu().numpy()), np.std(x, axis=1))
    bad = np.zeros(x.shape[0], bool)
    bad[[2, 30]] = True
    out, bins = C.renormalize_device(xd, badchans_mask=bad, cut_outliers=True)
    np.testing.assert_array_equal(out.cpu().numpy(), co.renormalize(x, badchans_mask=bad, cut_outliers=True))
    del out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dt", ["f32", "u8"])
def test_zero_dm_subtraction_c4(gpu, golden, dt):
    """Opt-in zero-DM subtraction (north_star; no reference counterpart, so parity is
    unpinned and checked against the numpy restatement in oracle/clean_oracle.py) at C4
    with the bad channels of get_noisier_channels and the outlier cut; the default path
    stays the reference's (golden SHA-256)."""
    import torch
    from pulsarutils import _hip
    arrays, meta = golden
    x = synth.rfi_filterbank_np(CONFIGS["C4"], dtype=dt)
    bad = C.get_noisier_channels(x)
    assert bad.any()
    xd = _hip.to_device(x)
    out, bins = C.renormalize_device(xd, badchans_mask=bad, cut_outliers=True, zero_dm=True)
    got = out.cpu().numpy()
    del out
    ref, ref_bins = co.renormalize(x, badchans_mask=bad, cut_outliers=True, zero_dm=True, return_badbins=True)
    np.testing.assert_array_equal(bins.cpu().numpy(), ref_bins)
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]
    # the subtraction removes the good channels' per-time-bin mean (up to rounding)
    good = ~bad
    assert np.abs(got[good].mean(0)).max() < 1e-12
    assert not got[bad].any()
    # default (zero_dm=False) is unchanged: the reference's own output
    out, _ = C.renormalize_device(xd, badchans_mask=bad, cut_outliers=True)
    assert sha(out.cpu().numpy()) == meta[f"c4{dt}_renorm_cut_sha256"]
    del out
    torch.cuda.empty_cache()


def test_cut_outliers_device_certified(gpu):
    """cut_outliers runs on the device (pu_cut_outliers): the mask and the zeroed plane
    equal the reference restatement (scipy's running-sum uniform_filter1d) on random
    light curves with injected spikes and dips, N from 64 up; a NaN in a good channel
    raises the certification flag and the exact path (on the device since round 4) gives
    the reference result."""
    import torch
    from pulsarutils import _hip
    rng = np.random.default_rng(17)
    for nchan, n in [(5, 64), (9, 100), (31, 4097), (64, 70001)]:
        x = (rng.random((nchan, n)) * 5 + 10).astype(np.float32)
        for t0 in rng.integers(0, n - 4, 3):
            x[:, t0:t0 + 3] += 40.0
        x[:, rng.integers(0, n)] -= 9.0
        bad = np.zeros(nchan, bool)
        bad[0] = True
        out, bins = C.renormalize_device(_hip.to_device(x), badchans_mask=bad, cut_outliers=True)
        ref, ref_bins = co.renormalize(x, badchans_mask=bad, cut_outliers=True, return_badbins=True)
        np.testing.assert_array_equal(bins.cpu().numpy(), ref_bins)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
    x = (rng.random((8, 500)) * 5 + 10)
    x[3, 100] = np.nan
    got = C.renormalize_data(x, cut_outliers=True)
    want = co.renormalize(x, cut_outliers=True)
    assert np.array_equal(got, want, equal_nan=True)
    torch.cuda.synchronize()


def test_cut_outliers_exact_path_on_device(gpu):
    """The exact path of pu_cut_outliers (round 4: scipy's running-sum uniform_filter1d
    and numpy's std order in one workgroup, instead of a host round trip) gives the
    reference's mask bit for bit - forced through pu_cut_outliers_exact on spiky light
    curves whose bins sit within rounding of the thresholds too, and reached through the
    flag by a NaN - and zeroes exactly the bad columns of the plane."""
    import torch
    from scipy.ndimage import uniform_filter1d
    from pulsarutils import _hip
    lib = _hip.lib()
    rng = np.random.default_rng(29)
    for n in (64, 1000, 70001, 262144):
        lc = rng.standard_normal(n) * 0.01
        lc[rng.integers(0, n, 9)] += 0.3
        reb = uniform_filter1d(lc, 16)
        sd = np.std(reb[::16])
        lc[n // 2:n // 2 + 16] += (5 * sd - reb[n // 2 + 8])  # a window mean at the threshold
        reb = uniform_filter1d(lc, 16)
        sd = np.std(reb[::16])
        want = (reb > 5 * sd) | (reb < -3 * sd)
        nrows = 3
        for fn in (lib.pu_cut_outliers_exact, lib.pu_cut_outliers):
            out = torch.ones((nrows, n), dtype=torch.float64, device="cuda")
            col = torch.from_numpy(lc).cuda()
            ws = torch.empty(lib.pu_cut_outliers_workspace_bytes(n), dtype=torch.uint8, device="cuda")
            mask = torch.empty(n, dtype=torch.uint8, device="cuda")
            _hip.check(fn(_hip.ptr(col), n, _hip.ptr(out), nrows, out.stride(0), _hip.ptr(mask), _hip.ptr(ws),
                          ws.numel(), _hip.stream_ptr()), "cut_outliers")
            got = mask.cpu().numpy().astype(bool)
            np.testing.assert_array_equal(got, want, err_msg=f"n {n} {fn.__name__}")
            o = out.cpu().numpy()
            assert not o[:, want].any() and (o[:, ~want] == 1.0).all()
            assert int(ws[4:8].view(torch.int32).item()) == int(want.sum())
    # NaN: the flag routes to the exact path; numpy's comparisons with NaN are False
    lc = rng.standard_normal(5000)
    lc[1234] = np.nan
    out = torch.ones((2, 5000), dtype=torch.float64, device="cuda")
    col = torch.from_numpy(lc).cuda()
    ws = torch.empty(lib.pu_cut_outliers_workspace_bytes(5000), dtype=torch.uint8, device="cuda")
    mask = torch.empty(5000, dtype=torch.uint8, device="cuda")
    _hip.check(lib.pu_cut_outliers(_hip.ptr(col), 5000, _hip.ptr(out), 2, 5000, _hip.ptr(mask), _hip.ptr(ws),
                                   ws.numel(), _hip.stream_ptr()), "pu_cut_outliers")
    reb = uniform_filter1d(lc, 16)
    sd = np.std(reb[::16])
    np.testing.assert_array_equal(mask.cpu().numpy().astype(bool), (reb > 5 * sd) | (reb < -3 * sd))
    assert int(ws[0:4].view(torch.int32).item()) == 1


def test_zero_dm_small_cases(gpu):
    """Ragged sizes, all channels bad, no channel bad."""
    rng = np.random.default_rng(13)
    for nchan, n in [(7, 333), (33, 5000)]:
        x = (rng.random((nchan, n)) * 5 + 1).astype(np.float32)
        for bad in (np.zeros(nchan, bool), np.ones(nchan, bool), rng.random(nchan) < 0.3):
            got = C.renormalize_data(x, badchans_mask=bad, cut_outliers=True, zero_dm=True)
            want = co.renormalize(x, badchans_mask=bad, cut_outliers=True, zero_dm=True)
            np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("n", [1, 2, 3, 8, 1001, 4096, 262144, 262145])
def test_median_device_matches_numpy(gpu, n):
    """np.median (clean.py:80) by device radix select: random, tied, signed-zero,
    infinite and NaN series, odd and even lengths, a smoothed light curve (the
    renormalisation's input), a constant series, two tight clusters and the two middle
    values far apart in key space."""
    from scipy.ndimage import gaussian_filter1d
    from pulsarutils import _hip
    rng = np.random.default_rng(n)
    cases = [rng.standard_normal(n) * 1e3,
             rng.integers(-3, 4, n).astype(np.float64),             # heavy ties
             np.where(rng.random(n) < 0.5, -0.0, 0.0),                # signed zeros only
             np.concatenate([rng.standard_normal(n - 1), [np.inf]]),
             np.abs(rng.standard_normal(n)) + 1.0,
             gaussian_filter1d(rng.standard_normal(n), 101 if n > 1000 else 2) * 1e-3 + 1.0,
             np.full(n, 3.25),
             np.where(rng.random(n) < 0.5, 1.0, np.nextafter(1.0, 2.0))]
    if n >= 4:
        far = rng.standard_normal(n) * 1e-3
        far[:2] = [-1e300, 1e300]
        cases.append(far)
    if n > 2:
        nan = rng.standard_normal(n)
        nan[n // 3] = np.nan
        cases.append(nan)
    for a in cases:
        got = C.median_device(_hip.to_device(a)).cpu().numpy()[0]
        want = np.median(a)
        assert np.array_equal(np.array([got]), np.array([want]), equal_nan=True), (n, got, want)
        assert np.signbit(got) == np.signbit(want)


@pytest.mark.parametrize("n,sigma", [(12345, 101), (262144, 101), (1000, 3), (777, 2.6), (3001, 2.7), (50, 7),
                                     (10, 5), (1, 1), (513, 0.2)])
def test_gaussian_filter1d_vs_scipy(gpu, n, sigma):
    """pu_gaussian_filter1d (the pair kernel; odd radii 11 and 1 exercise its last-tap
    path, n < radius the repeated reflection) equals scipy's gaussian_filter1d bit for bit."""
    import torch
    from scipy.ndimage import gaussian_filter1d
    from pulsarutils import _hip
    rng = np.random.default_rng(n)
    x = rng.normal(size=n) * 10 + 100
    dw, radius = C._gaussian_weights_device(sigma, torch.device("cuda", 0))
    xd = torch.from_numpy(x).cuda()
    out = torch.empty_like(xd)
    lib = _hip.lib()
    _hip.check(lib.pu_gaussian_filter1d(_hip.ptr(xd), n, _hip.ptr(dw), radius, _hip.ptr(out), _hip.stream_ptr()),
               "pu_gaussian_filter1d")
    np.testing.assert_array_equal(out.cpu().numpy(), gaussian_filter1d(x, sigma, mode="reflect"))


@pytest.mark.parametrize("nrows,ncols", [(300, 4096), (1024, 2048), (1, 64), (257, 8 * 1000)])
def test_col_means_u8_segments(gpu, nrows, ncols):
    """pu_col_means on 8-bit input takes the row-segment kernel (exact integer partial sums;
    a partial last segment, skipped rows, a single row) and must equal the float64 mean over
    the unskipped rows bit for bit."""
    import torch
    from pulsarutils import _hip
    rng = np.random.default_rng(nrows * 7 + ncols)
    x = rng.integers(0, 256, size=(nrows, ncols), dtype=np.uint8)
    skip = (rng.random(nrows) < 0.2).astype(np.uint8)
    if nrows > 1:
        skip[0] = 1
    xd, sd = torch.from_numpy(x).cuda(), torch.from_numpy(skip).cuda()
    out = torch.empty(ncols, dtype=torch.float64, device="cuda")
    lib = _hip.lib()
    _hip.check(lib.pu_col_means(_hip.ptr(xd), _hip.dtype_code(xd.dtype), nrows, ncols, ncols, _hip.ptr(sd),
                                _hip.ptr(out), _hip.stream_ptr()), "pu_col_means")
    good = skip == 0
    with np.errstate(invalid="ignore"):
        ref = x[good].astype(np.float64).sum(axis=0) / float(good.sum())
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("nrows", [1, 3, 100, 1024, 1031])
@pytest.mark.parametrize("ncols,ld", [(1, 1), (77, 80), (4099, 4099), (4096, 4096)])
def test_col_means_f32_certified(gpu, nrows, ncols, ld):
    """pu_col_means on float32 input (the zero-DM light curve, clean.py:77: numpy's
    float64 mean(0), a sequential chain over the rows): columns with a tiny value beside
    large ones, huge and tiny values (the chain's roundings), NaN / inf in a used and in a
    skipped row, all-zero columns, ragged widths (V = 1 tails) and a padded row stride:
    equal to numpy bit for bit.  (Round 4 also ran a row-quarters kernel certified exact
    per column against it: 268 vs 236 us at C4, not kept; profiles/r04/experiments/.)"""
    import torch
    from pulsarutils import _hip
    rng = np.random.default_rng(nrows * 31 + ncols)
    x = np.abs(rng.standard_normal((nrows, ld))).astype(np.float32) * 3
    skip = (rng.random(nrows) < 0.2).astype(np.uint8)
    if nrows > 2:
        skip[1] = 1
    k = min(ncols, 12)
    cols = rng.choice(ncols, size=k, replace=False)
    for j, c in enumerate(cols):
        r = int(rng.integers(0, nrows))
        kind = j % 6
        if kind == 0:
            x[r, c] = 1e-30                       # uncertifiable: the chain
        elif kind == 1:
            x[:, c] = rng.random(nrows).astype(np.float32) * np.float32(1e30)
            x[r, c] = 1.0                          # rounds in the chain
        elif kind == 2:
            x[r, c] = np.nan
        elif kind == 3 and nrows > 2:
            x[1, c] = np.inf                       # in a skipped row: no effect
        elif kind == 4:
            x[:, c] = 0.0
        else:
            x[r, c] = -x[r, c]
    xd, sd = torch.from_numpy(x).cuda(), torch.from_numpy(skip).cuda()
    out = torch.empty(ncols, dtype=torch.float64, device="cuda")
    _hip.check(_hip.lib().pu_col_means(_hip.ptr(xd), _hip.PU_F32, nrows, ncols, ld, _hip.ptr(sd), _hip.ptr(out),
                                       _hip.stream_ptr()), "pu_col_means")
    good = skip == 0
    with np.errstate(invalid="ignore"):
        ref = x[good][:, :ncols].astype(np.float64).mean(0) if good.any() else np.full(ncols, np.nan)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def _noisy_host(spec):
    """The reference's decision (clean.py:58-67) on a host spec, numpy / scipy."""
    from scipy.signal import medfilt
    from pulsarutils.stats import ref_mad
    return spec > medfilt(spec, 7) + 5 * ref_mad(spec)


def _noisy_device(spec):
    import torch
    from pulsarutils import _hip
    d = torch.from_numpy(spec).cuda()
    n = spec.size
    off = (n + 3) & ~3
    res = torch.full((off + 4,), 7, dtype=torch.uint8, device=d.device)
    _hip.check(_hip.lib().pu_noisy_channels(_hip.ptr(d), _hip.dtype_code(d.dtype), n, float(C.MAD_C), _hip.ptr(res),
                                            res.data_ptr() + off, _hip.stream_ptr()), "pu_noisy_channels")
    h = res.cpu().numpy()
    return h[:n].astype(bool), int(h[off:off + 4].view(np.int32)[0])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("n", [2, 3, 7, 8, 64, 255, 1000, 1024, 1025, 1026, 4095, 4096])
def test_noisy_channels_device_matches_host(gpu, dt, n):
    """pu_noisy_channels (get_noisier_channels' medfilt + ref_mad + comparison on the
    device) equals the numpy / scipy decision bit for bit: noisy spectra with spikes, a
    constant spectrum (MAD 0), quantised values (ties in the sorts and windows), both
    parities of n - 1 (the two medians' middle-pair means)."""
    rng = np.random.default_rng(n)
    cases = [rng.normal(100, 1, n), np.full(n, 3.5), np.round(rng.normal(10, 2, n)) / 4,
             rng.normal(0, 1e-3, n) + 1e6]
    spike = rng.normal(50, 0.5, n)
    spike[rng.choice(n, max(1, n // 20), replace=False)] += 40
    cases.append(spike)
    for c in cases:
        spec = c.astype(dt)
        mask, flag = _noisy_device(spec)
        assert flag == 0
        np.testing.assert_array_equal(mask, _noisy_host(spec))


def test_noisy_channels_float32_mad_golden(gpu, golden):
    """the float32 spectrum whose mask depends on statsmodels' float64 mad
    (tests/golden: reference run, mad cross-checked against the real statsmodels 0.12.2):
    the device decision, through get_noisier_channels on host and device data, equals it."""
    import torch
    arrays, _ = golden
    spec = arrays["noisy32_spec"]
    mask, flag = _noisy_device(spec)
    assert flag == 0
    np.testing.assert_array_equal(mask, arrays["noisy32_mask"])
    x = np.repeat(spec[:, None], 4, axis=1)
    np.testing.assert_array_equal(C.get_noisier_channels(x), arrays["noisy32_mask"])
    got = C.get_noisier_channels(torch.from_numpy(x).cuda())
    np.testing.assert_array_equal(got.cpu().numpy() if hasattr(got, "cpu") else got, arrays["noisy32_mask"])


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
def test_noisy_channels_nonfinite_flag(gpu, bad):
    """A NaN / inf channel mean sets the flag (mask left alone); get_noisier_channels then
    decides on the host, as the reference does."""
    spec = np.random.default_rng(1).normal(100, 1, 512)
    spec[17] = bad
    mask, flag = _noisy_device(spec)
    assert flag == 1
    assert (mask == (7 != 0)).all()  # untouched (the fill byte)
    x = np.random.default_rng(2).normal(0, 1, (64, 4096)).astype(np.float32)
    x[5, 100] = bad
    np.testing.assert_array_equal(C.get_noisier_channels(x), _noisy_host(x.mean(1)))


@pytest.mark.parametrize("nchan", [16, 600, 1500])
def test_noisy_channels_overflowing_differences(gpu, nchan):
    """a finite float32 spectrum whose np.diff overflows to +-inf (means of
    +-3e38) makes the median of the differences NaN (inf - inf), which the device's register
    sorts (v_min_f64 / v_max_f64 drop NaN) cannot order: both kernels raise the flag and the
    masks come from the host's numpy / scipy arithmetic - the same as the reference's."""
    from pulsarutils import _hip
    spec = np.where(np.arange(nchan) % 2 == 0, 3e38, -3e38).astype(np.float32)
    assert np.isfinite(spec).all() and not np.isfinite(np.diff(spec)).all()
    mask, flag = _noisy_device(spec)
    assert flag == 1
    x = np.repeat(spec[:, None], 1, axis=1)
    np.testing.assert_array_equal(C.get_noisier_channels(x), _noisy_host(spec))
    if nchan <= 1024:
        xd = _hip.to_device(x)
        C.invalidate_channel_means()
        np.testing.assert_array_equal(C.get_noisier_channels(xd), _noisy_host(spec))
        np.testing.assert_array_equal(C.measure_channel_variability(xd),
                                      co.channel_variability(x, badchans_mask=None))


def test_noisy_channels_wide_band_host_path(gpu):
    """More channels than one workgroup decides (4097): the host path, same mask."""
    x = np.random.default_rng(3).normal(0, 1, (4097, 256)).astype(np.float32)
    x[100] += 5
    np.testing.assert_array_equal(C.get_noisier_channels(x), _noisy_host(x.mean(1)))


@pytest.mark.parametrize("n", [1, 15, 16, 100, 8192, 65536, 65537, 200003])
@pytest.mark.parametrize("padded", [False, True])
def test_u8_row_sums_exact(gpu, n, padded):
    """8-bit Σx (mean, modes 0/3) and Σx² (mode 4) equal numpy's float64 results bit for
    bit, for contiguous and padded (ld > n) rows, full 8192-blocks and tails."""
    import torch
    from pulsarutils import _hip
    from pulsarutils.stats import _chunk_row_sums
    rng = np.random.default_rng(n)
    x = rng.integers(0, 256, (37, n), dtype=np.uint8)
    x[3] = 255
    ld = (n + 15) // 16 * 16 + 16 if padded else n
    buf = torch.zeros((37, ld), dtype=torch.uint8, device="cuda")
    buf[:, :n] = torch.from_numpy(x).cuda()
    xd = buf[:, :n]
    np.testing.assert_array_equal(C.channel_means_device(xd).cpu().numpy(), x.mean(1))
    np.testing.assert_array_equal(_chunk_row_sums(xd, 3).cpu().numpy(), x.astype(float).sum(1))
    np.testing.assert_array_equal(_chunk_row_sums(xd, 4).cpu().numpy(), (x.astype(float) ** 2).sum(1))


@pytest.mark.parametrize("dtype", [np.float32, np.uint8, np.float64])
@pytest.mark.parametrize("n", [8192, 20000, 262144])
def test_row_moments_one_pass(gpu, dtype, n):
    """pu_row_moments (round 4): the means are pu_row_sums mode 0's bit for bit (numpy's
    mean(1)), and the shifted moments (c, sum(x - c), sum((x - c)^2)) match float64 numpy
    to rounding - the inputs of measure_channel_variability's certification."""
    from pulsarutils import _hip
    rng = np.random.default_rng(n + 3)
    x = rng.normal(100.0, 5.0, (37, n))
    x = (np.clip(x, 0, 255) if dtype == np.uint8 else x).astype(dtype)
    xd = _hip.to_device(x)
    means, mom = C._row_moments(xd)
    ref_means = C._row_sums(xd, 0, divisor=n)
    np.testing.assert_array_equal(means.cpu().numpy(), ref_means.cpu().numpy())
    np.testing.assert_array_equal(means.cpu().numpy(), x.mean(1))
    xd64 = x.astype(np.float64)
    d = xd64 - xd64[:, :1]
    want = np.stack([xd64[:, 0], d.sum(1), (d * d).sum(1)], axis=1)
    got = mom.cpu().numpy()
    np.testing.assert_array_equal(got[:, 0], want[:, 0])
    np.testing.assert_allclose(got[:, 1], want[:, 1], rtol=1e-9, atol=1e-6 * np.abs(d).sum(1).max())
    np.testing.assert_allclose(got[:, 2], want[:, 2], rtol=1e-12)


def test_variability_one_pass_and_fallback(gpu):
    """measure_channel_variability: certified from the one-pass moments on ordinary data
    (one read pass: the variance pass is not run), and the exact second pass when a
    channel's std is moved onto the upper limit; both equal the reference."""
    from pulsarutils import _hip
    rng = np.random.default_rng(47)
    nchan, n = 64, 65536
    x = rng.normal(10.0, 1.0, (nchan, n)).astype(np.float32) * rng.uniform(0.8, 1.2, nchan)[:, None].astype(np.float32)
    bad = np.zeros(nchan, bool)
    bad[3] = True
    xd = _hip.to_device(x)
    calls = []
    orig = C.channel_variances_device
    C.channel_variances_device = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    try:
        C.invalidate_channel_means()
        np.testing.assert_array_equal(C.measure_channel_variability(xd, badchans_mask=bad),
                                      co.channel_variability(x, badchans_mask=bad))
        assert not calls  # certified: no second pass
        # channel j (the lowest std) onto the upper limit of the others
        spec = np.std(x, axis=1)
        j = int(np.argmin(np.where(bad, np.inf, spec)))
        rest = np.sort(np.delete(spec, [j, 3]))
        q2, q3 = rest[nchan // 2], rest[nchan // 4 * 3]
        hi = q2 + 2 * (q3 - q2)
        x[j] = ((x[j].astype(np.float64) - x[j].mean()) * (float(hi) / float(spec[j])) + 10.0).astype(np.float32)
        want = co.channel_variability(x, badchans_mask=bad)
        C.invalidate_channel_means()
        got = C.measure_channel_variability(_hip.to_device(x), badchans_mask=bad)
        np.testing.assert_array_equal(got, want)
    finally:
        C.channel_variances_device = orig


@pytest.mark.parametrize("dtype", [np.float32, np.uint8, np.float64])
@pytest.mark.parametrize("nchan,n", [(4, 5000), (100, 12345), (1024, 16384), (4096, 2048)])
def test_variability_cert_device_matches_host(gpu, dtype, nchan, n):
    """pu_variability_cert (round 5) = the host restatement _certified_variability: the
    same certified-or-not outcome and, when certified, the same mask (which then equals
    the reference's decision: checked against the oracle too); masks with bad channels,
    too many bad channels (not certifiable), a channel forced onto a limit."""
    from pulsarutils import _hip
    import torch
    rng = np.random.default_rng(nchan + n)
    x = rng.normal(100.0, 5.0, (nchan, n)) * rng.uniform(0.7, 1.4, nchan)[:, None]
    x = (np.clip(x, 0, 255) if dtype == np.uint8 else x).astype(dtype)
    cases = [np.zeros(nchan, bool), rng.random(nchan) < 0.1, rng.random(nchan) < 0.3]
    if nchan >= 8:
        many = np.ones(nchan, bool)
        many[: nchan // 4] = False  # nchan // 4 * 3 >= good: the reference's indices fail
        cases.append(many)
    xd = _hip.to_device(x)
    C.invalidate_channel_means()
    means, mom = C._cached_stats(xd)
    off = (nchan + 3) & ~3
    for bad in cases:
        host = C._certified_variability(means.cpu().numpy().astype(np.float64), mom.cpu().numpy(), n,
                                        means.dtype == torch.float32, bad)
        badd = torch.from_numpy(bad.astype(np.uint8)).to(xd.device)
        res = torch.zeros(off + 4, dtype=torch.uint8, device=xd.device)
        C._launch_variability(xd, badd, res.data_ptr(), res.data_ptr() + off)
        h = res.cpu().numpy()
        flag = int(h[off:off + 4].view(np.int32)[0])
        assert flag == (host is None), (flag, host is None)
        if host is not None:
            np.testing.assert_array_equal(h[:nchan].astype(bool), host)
            if bad.sum() < nchan // 2:
                np.testing.assert_array_equal(host, co.channel_variability(x, badchans_mask=bad))


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.uint8])
@pytest.mark.parametrize("nchan", [2, 3, 5, 8, 63, 64, 65, 500, 1023, 1024])
def test_channel_masks_one_launch_matches_two_kernels(gpu, dtype, nchan):
    """pu_channel_masks (round 5: both decisions in one workgroup) writes the same bytes as
    pu_noisy_channels followed by pu_variability_cert with the noisy mask as bad - masks and
    flags - on spectra with noisy channels, a channel at the variability limit region, and
    a non-finite spectrum (both flags set)."""
    from pulsarutils import _hip
    import torch
    rng = np.random.default_rng(7 * nchan + np.dtype(dtype).itemsize)
    ns = 2048
    for case in range(3):
        x = rng.normal(100.0, 5.0, (nchan, ns)) * rng.uniform(0.7, 1.4, nchan)[:, None]
        if case >= 1:
            x[rng.random(nchan) < 0.1] += 40.0  # noisy channels
        x = (np.clip(x, 0, 255) if dtype == np.uint8 else x).astype(dtype)
        if case == 2 and dtype != np.uint8:
            x[nchan // 2, 3] = np.nan
        xd = _hip.to_device(x)
        C.invalidate_channel_means()
        means, mom = C._cached_stats(xd)
        mef, gam, u = C._variability_args(means, ns)
        off = (nchan + 3) & ~3
        lib = _hip.lib()
        one = torch.full((2 * (off + 4),), 7, dtype=torch.uint8, device=xd.device)
        b = one.data_ptr()
        _hip.check(lib.pu_channel_masks(_hip.ptr(means), _hip.dtype_code(means.dtype), _hip.ptr(mom), nchan, ns,
                                        float(C.MAD_C), mef, gam, u, b, b + off, b + off + 4, b + 2 * off + 4,
                                        _hip.stream_ptr()), "pu_channel_masks")
        two = torch.full((2 * (off + 4),), 7, dtype=torch.uint8, device=xd.device)
        b = two.data_ptr()
        _hip.check(lib.pu_noisy_channels(_hip.ptr(means), _hip.dtype_code(means.dtype), nchan, float(C.MAD_C), b,
                                         b + off, _hip.stream_ptr()), "pu_noisy_channels")
        h1, h2 = one.cpu().numpy(), two.cpu().numpy()
        nflag = int(h2[off:off + 4].view(np.int32)[0])
        assert int(h1[off:off + 4].view(np.int32)[0]) == nflag
        if nflag:
            assert case == 2 and dtype != np.uint8
            assert int(h1[2 * off + 4:2 * off + 8].view(np.int32)[0]) == 1
            continue
        np.testing.assert_array_equal(h1[:nchan], h2[:nchan])
        _hip.check(lib.pu_variability_cert(_hip.ptr(means), _hip.dtype_code(means.dtype), _hip.ptr(mom), nchan, ns,
                                           mef, gam, u, b, b + off + 4, b + 2 * off + 4, _hip.stream_ptr()),
                   "pu_variability_cert")
        h2 = two.cpu().numpy()
        vflag = int(h2[2 * off + 4:2 * off + 8].view(np.int32)[0])
        assert int(h1[2 * off + 4:2 * off + 8].view(np.int32)[0]) == vflag
        if not vflag:
            np.testing.assert_array_equal(h1[off + 4:off + 4 + nchan], h2[off + 4:off + 4 + nchan])


@pytest.mark.parametrize("dt", ["f32", "u8"])
def test_masks_one_readback_on_device_tensor(gpu, golden, dt):
    """get_noisier_channels on a device tensor also decides measure_channel_variability
    for its own mask (one read-back for both); the next call with that mask returns the
    kept result without a GPU call, a different mask or a modified tensor recomputes -
    all equal to the reference's goldens / oracle."""
    from pulsarutils import _hip
    arrays, meta = golden
    x = synth.rfi_filterbank_np(CONFIGS["C4"], dtype=dt)
    xd = _hip.to_device(x)
    C.invalidate_channel_means()
    bad = C.get_noisier_channels(xd)
    np.testing.assert_array_equal(bad, arrays[f"c4{dt}_noisier"])
    lib = _hip.lib()
    calls = []
    orig = C._launch_variability
    C._launch_variability = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    try:
        got = C.measure_channel_variability(xd, badchans_mask=bad)
        assert not calls  # decided with get_noisier_channels' read-back
        np.testing.assert_array_equal(got, arrays[f"c4{dt}_variability_masked"])
        other = bad.copy()
        other[0] = not other[0]
        got2 = C.measure_channel_variability(xd, badchans_mask=other)
        assert calls
        np.testing.assert_array_equal(got2, co.channel_variability(x, badchans_mask=other))
        np.testing.assert_array_equal(C.measure_channel_variability(xd), arrays[f"c4{dt}_variability"])
    finally:
        C._launch_variability = orig
    del lib


@pytest.mark.parametrize("n,sigma", [(262144, 101), (262145, 101), (262143, 55), (1, 1), (7, 2), (1000, 3),
                                     (3 * 262144 + 17, 101), (2 * 262144, 0.2), (12345, 600)])
def test_light_curve_factor(gpu, n, sigma):
    """pu_lc_factor (clean.py:79-80: Gaussian, median, factor) equals scipy's
    gaussian_filter1d + np.median + the division bit for bit, and the three separate device
    calls; long series (n > 2^18), odd and even n, n < radius, a NaN (median NaN), a
    constant light curve, r > 2048 (sigma 600).  Repeated calls give the same bits."""
    import torch
    from scipy.ndimage import gaussian_filter1d
    from pulsarutils import _hip
    rng = np.random.default_rng(n)
    dev = torch.device("cuda", 0)
    dw, radius = C._gaussian_weights_device(sigma, dev)
    cases = [rng.normal(size=n) * 10 + 100, np.full(n, 4.5)]
    if n > 8:
        spiky = rng.normal(size=n) + 50
        spiky[rng.integers(0, n, 5)] = 1e6
        cases.append(spiky)
        nan = rng.normal(size=n) + 3
        nan[n // 2] = np.nan
        cases.append(nan)
    lib = _hip.lib()
    for x in cases:
        smooth = gaussian_filter1d(x, sigma, mode="reflect")
        med = np.median(smooth)
        want = med / smooth
        xd = torch.from_numpy(x).to(dev)
        for rep in range(2):
            medd = torch.empty(1, dtype=torch.float64, device=dev)
            got = C.light_curve_factor(xd, dw, radius, median_out=medd)
            np.testing.assert_array_equal(got.cpu().numpy(), want)
            assert np.array_equal(medd.cpu().numpy(), [med], equal_nan=True)
        # the launch-by-launch device path
        sm = torch.empty_like(xd)
        _hip.check(lib.pu_gaussian_filter1d(_hip.ptr(xd), n, _hip.ptr(dw), radius, _hip.ptr(sm), _hip.stream_ptr()),
                   "pu_gaussian_filter1d")
        f3 = torch.empty_like(xd)
        _hip.check(lib.pu_ratio_dev(_hip.ptr(C.median_device(sm)), _hip.ptr(sm), n, _hip.ptr(f3), _hip.stream_ptr()),
                   "pu_ratio_dev")
        assert torch.equal(f3.isnan(), got.isnan()) and torch.equal(f3.nan_to_num(), got.nan_to_num())


def test_stream_ptr_is_torch_current_stream(gpu):
    """_hip.stream_ptr() (read raw, round 5) is torch's current stream, also inside a
    ``torch.cuda.stream`` block, and an explicit stream's own handle (the null stream: a NULL pointer, c_void_p(0).value is None)."""
    from pulsarutils import _hip
    import torch
    assert (_hip.stream_ptr().value or 0) == torch.cuda.current_stream().cuda_stream
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        assert (_hip.stream_ptr().value or 0) == s.cuda_stream
    assert (_hip.stream_ptr(s).value or 0) == s.cuda_stream
    assert (_hip.stream_ptr().value or 0) == torch.cuda.current_stream().cuda_stream
