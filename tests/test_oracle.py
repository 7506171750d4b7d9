"""The oracle (test infrastructure) pinned against the reference's own outputs.

Golden vectors come from executing the reference source (tests/golden/make_golden.py).
"""
import hashlib

import numpy as np
import pytest

import oracle
from oracle import clean_oracle as co
from oracle import numpy_order as no
from pulsarutils.configs import CONFIGS
from pulsarutils import simulate, synth


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_oracle_shifts_match_reference(golden, name):
    arrays, _ = golden
    c = CONFIGS[name]
    dms = arrays[f"plan_{name}"]
    for row, i in zip(arrays[f"shifts_{name}"], arrays[f"shiftidx_{name}"]):
        got = oracle.shifts(c.nchan, dms[i], c.start_freq, c.bandwidth, c.tsamp)
        np.testing.assert_array_equal(got, row.astype(np.int64))


def _c1_input():
    c = CONFIGS["C1"]
    np.random.seed(c.seed)
    arr, _ = simulate.simulate_test_data(dm=c.pulse_dm, tsamp=c.tsamp, nsamples=c.nsamples, nchan=c.nchan,
                                         start_freq=c.start_freq, bandwidth=c.bandwidth)
    return arr


def test_oracle_dedisperse_bitexact_c1(golden):
    arrays, meta = golden
    c = CONFIGS["C1"]
    arr = _c1_input()
    assert sha(arr) == meta["c1_input_sha256"]
    dms = arrays["plan_C1"]
    for k, i in enumerate(arrays["c1_dedisp_rows_idx"]):
        sh = oracle.shifts(c.nchan, dms[i], c.start_freq, c.bandwidth, c.tsamp)
        dd = oracle.dedisperse(arr, sh)
        assert sha(dd) == meta[f"c1_dedisp_sha256_{i}"]
        np.testing.assert_array_equal(dd[::16], arrays["c1_dedisp_rows"][k])


def test_oracle_search_bitexact_c1(golden):
    arrays, _ = golden
    c = CONFIGS["C1"]
    arr = _c1_input()
    mx, sd, snr, win = oracle.search(arr, arrays["plan_C1"], c.start_freq, c.bandwidth, c.tsamp)
    np.testing.assert_array_equal(mx, arrays["c1_table_max"])
    np.testing.assert_array_equal(sd, arrays["c1_table_std"])
    np.testing.assert_array_equal(snr, arrays["c1_table_snr"])
    np.testing.assert_array_equal(win, arrays["c1_table_rebin"])


def test_oracle_search_bitexact_test_config(golden):
    arrays, meta = golden
    np.random.seed(0)
    arr, h = simulate.simulate_test_data(150)
    assert sha(arr) == meta["test_input_sha256"]
    mx, sd, snr, win = oracle.search(arr, arrays["test_table_DM"], h["fbottom"], h["bandwidth"], h["tsamp"])
    np.testing.assert_array_equal(mx, arrays["test_table_max"])
    np.testing.assert_array_equal(sd, arrays["test_table_std"])
    np.testing.assert_array_equal(snr, arrays["test_table_snr"])
    np.testing.assert_array_equal(win, arrays["test_table_rebin"])
    # the reference test's own assertion (tests/test_dedispersion.py:25)
    assert np.isclose(arrays["test_table_DM"][np.argmax(snr)], 150, atol=1)


def test_oracle_pulseinfo_search_and_plane(golden):
    """clean.dedispersion_search's PulseInfo route (clean.py:136-180): grid, plane
    (dedisperse per trial, float64) and table of the oracle equal the reference's."""
    import hashlib
    from pulsarutils.dedispersion import dedispersion_plan
    arrays, meta = golden
    a = meta["pinfo_args"]
    np.random.seed(a["seed"])
    tsamp_sim = 1 / a["pulse_freq"] / a["nbin"]
    arr, _ = simulate.simulate_test_data(dm=a["dm"], tsamp=tsamp_sim, nsamples=a["nbin"], nchan=a["nchan"],
                                         start_freq=a["start_freq"], bandwidth=a["bandwidth"])
    assert sha(arr) == meta["pinfo_input_sha256"]
    sample_time = 1 / a["pulse_freq"] / a["nbin"]  # clean.py:141
    dms = dedispersion_plan(a["nchan"], a["dmmin"], a["dmmax"], a["start_freq"], a["bandwidth"], sample_time)
    np.testing.assert_array_equal(dms, arrays["pinfo_table_DM"])
    plane = np.array([oracle.dedisperse(arr, oracle.shifts(a["nchan"], dm, a["start_freq"], a["bandwidth"],
                                                           sample_time)) for dm in dms])
    assert hashlib.sha256(plane.tobytes()).hexdigest() == meta["pinfo_plane_sha256"]
    mx, sd, snr, win = oracle.search(arr, dms, a["start_freq"], a["bandwidth"], sample_time)
    for got, col in zip((mx, sd, snr, win), ("max", "std", "snr", "rebin")):
        np.testing.assert_array_equal(got, arrays[f"pinfo_table_{col}"])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("n", [5, 127, 129, 1000, 8192, 8193, 20000, 65536 + 77])
def test_numpy_order_emulation(dt, n):
    rng = np.random.default_rng(n)
    x = (rng.random((3, n)) * 3 - 1).astype(dt)
    np.testing.assert_array_equal(no.row_sums(x), x.sum(1))
    np.testing.assert_array_equal(no.col_sums(x), x.sum(0))


def test_mad_matches_statsmodels(golden):
    arrays, meta = golden
    a = arrays["refmad_in_f64"]
    assert co.ref_mad(a) == arrays["refmad_out_f64"]
    assert co.ref_mad(a.astype(np.float32)) == arrays["refmad_out_f32"]
    if "refmad_f64_real_statsmodels" in meta:
        assert float(co.ref_mad(a)) == meta["refmad_f64_real_statsmodels"]
    # float32 input: statsmodels widens it to float64, cross-checked against the
    # real package in /opt/conda/bin/python3.9 by make_golden.py
    assert float(co.ref_mad(a.astype(np.float32))) == meta["refmad_f32_real_statsmodels"]


def test_noisier_channels_float32_mad_dtype(golden):
    """A float32 spectrum whose mask depends on the mad's dtype (make_golden.py, seed in
    the meta): the reference (statsmodels' float64 mad, cross-checked against the real
    package) keeps channel 100; a float32 median / |d - m| would flag it."""
    from scipy.signal import medfilt
    arrays, meta = golden
    spec = arrays["noisy32_spec"]
    x = np.repeat(spec[:, None], 4, axis=1)
    np.testing.assert_array_equal(co.noisier_channels(x), arrays["noisy32_mask"])
    assert float(co.ref_mad(spec)) == meta["noisy32_refmad_real_statsmodels"]
    d = np.diff(spec)  # the float32-median variant flips the decision
    m32 = np.median(np.abs(d - np.apply_over_axes(np.median, d, 0)) / co.MAD_C) / np.sqrt(2)
    assert (spec > medfilt(spec, 7) + 5 * m32)[100] and not arrays["noisy32_mask"][100]


def _check_clean(arrays, meta, tag, x):
    assert sha(x) == meta[f"{tag}_input_sha256"]
    bad = co.noisier_channels(x)
    np.testing.assert_array_equal(bad, arrays[f"{tag}_noisier"])
    np.testing.assert_array_equal(co.channel_variability(x), arrays[f"{tag}_variability"])
    np.testing.assert_array_equal(co.channel_variability(x, bad), arrays[f"{tag}_variability_masked"])
    for cut in (False, True):
        ren = co.renormalize(x, badchans_mask=bad, cut_outliers=cut)
        assert sha(ren) == meta[f"{tag}_renorm_{'cut' if cut else 'nocut'}_sha256"]


@pytest.mark.parametrize("dt", ["f32", "u8", "f64"])
def test_oracle_clean_ragged(golden, dt):
    from dataclasses import replace
    arrays, meta = golden
    rag = replace(CONFIGS["C4"], nchan=100, nsamples=12345, seed=77)
    _check_clean(arrays, meta, f"rag{dt}", synth.rfi_filterbank_np(rag, dtype=dt))


def test_oracle_clean_c4_f32(golden):
    arrays, meta = golden
    _check_clean(arrays, meta, "c4f32", synth.rfi_filterbank_np(CONFIGS["C4"], dtype="f32"))


def test_oracle_rebin_roll(golden):
    arrays, _ = golden
    x = arrays["rebin_in"]
    for r in (1, 2, 3, 8):
        np.testing.assert_array_equal(co.quick_resample(x, r), arrays[f"resample_{r}"])
        np.testing.assert_array_equal(co.quick_chan_rebin(x, r), arrays[f"chanrebin_{r}"])
    np.testing.assert_array_equal(co.apply_dm_shifts(x, arrays["roll_shifts"]), arrays["roll_out"])


# ------------------------------------------------------------------ degenerate trials
import degenerate_cases as DC  # noqa: E402


def _deg_inputs(golden, case):
    arrays, meta = golden
    k = DC.key(case)
    x = DC.make(case)
    assert sha(x) == meta[k + "_input_sha256"], case
    return x, arrays[k + "_dms"], [arrays[f"{k}_{c}"] for c in ("max", "std", "snr", "rebin")]


@pytest.mark.parametrize("case", [c for c in DC.CASES if not c.startswith("c2:")] + ["c2:block8:f32"])
def test_oracle_degenerate_trials_bitexact(golden, case):
    """The oracle's search reproduces the reference's degenerate-trial semantics bit for
    bit (NaN-propagating max/std, NaN S/N never wins, +-inf S/N from a zero std, exact
    and rounding-broken ties keep the first strictly larger S/N): golden tables from
    executing the reference (make_golden.py, degenerate section)."""
    x, dms, ref = _deg_inputs(golden, case)
    _, f0, bw, ts = DC.band(case)
    got = oracle.search(x, dms, f0, bw, ts, nthreads=8)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)


def test_cut_outliers_exact_restatement():
    """The order outlier_exact_kernel follows (the device's exact cut_outliers path,
    round 4) is scipy's and numpy's bit for bit: uniform_filter1d(lc, 16) as scipy's
    running sum, np.std(lc_rebin[::16]) in add.reduce order - spiky light curves,
    lengths 64 .. 2^18 + 1, a NaN (propagates through the running sum)."""
    from scipy.ndimage import uniform_filter1d
    rng = np.random.default_rng(23)
    for n in (64, 100, 4097, 70001, 262145):
        lc = rng.standard_normal(n) * 3.0 + 0.5
        lc[rng.integers(0, n, 7)] += 40.0
        got = co.uniform_filter1d_running(lc)
        want = uniform_filter1d(lc, 16)
        np.testing.assert_array_equal(got, want)
        assert co.std_numpy_order(want[::16]) == np.std(want[::16])
    lc = rng.standard_normal(500)
    lc[300] = np.nan
    np.testing.assert_array_equal(co.uniform_filter1d_running(lc), uniform_filter1d(lc, 16))
