"""HIP dedispersion parity (GPU): through the C-ABI, against the oracle and the goldens.

Tolerances:
* float64 accumulation (acc='f64', and float64 input by default): bit-exact series.
* uint8 input, float32 accumulation: bit-exact (all partial sums are integers < 2**24).
* float32 input, float32 accumulation: |gpu - ref| <= nchan * 2**-24 * sum_c |x_c| per sample.
* search statistics: max/std/snr within 1e-5 relative (1e-9 for float64 accumulation);
  argmax DM and rebin equal unless the top two S/N are within that tolerance.
"""
import hashlib

import numpy as np
import pytest

import oracle
from pulsarutils import dedispersion as D
from pulsarutils import simulate, _hip
from pulsarutils.configs import CONFIGS

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def c1_input():
    c = CONFIGS["C1"]
    np.random.seed(c.seed)
    arr, _ = simulate.simulate_test_data(dm=c.pulse_dm, tsamp=c.tsamp, nsamples=c.nsamples, nchan=c.nchan,
                                         start_freq=c.start_freq, bandwidth=c.bandwidth)
    return arr


def f32_bound(x, shifts):
    """Per-sample first-order bound nchan * 2^-24 * sum_c |x_c[(t+s_c) mod N]|."""
    ax = np.abs(x)  # exact in the input dtype; the oracle sums it in float64
    return x.shape[0] * 2.0 ** -24 * oracle.dedisperse(ax, shifts) + 1e-30


# ------------------------------------------------------------------ doctests / helpers

def test_doctest_quick_chan_rebin(gpu, golden):
    counts = np.array([np.arange(0, 10), np.arange(2, 12), np.arange(1, 11), np.arange(3, 13),
                       np.arange(1, 11), np.arange(3, 13)])
    reb = D.quick_chan_rebin(counts, 2)
    assert reb.dtype == golden[0]["doctest_chan_rebin"].dtype
    np.testing.assert_array_equal(reb, golden[0]["doctest_chan_rebin"])


def test_doctest_quick_resample(gpu, golden):
    counts = np.array([np.arange(1, 11), np.arange(3, 13)])
    np.testing.assert_array_equal(D.quick_resample(counts, 2), golden[0]["doctest_resample"])


def test_doctest_roll_and_sum_in_place(gpu, golden):
    array = np.arange(10)
    sum_array = np.zeros(10)
    assert np.allclose(D.roll_and_sum(array, sum_array, 3), np.roll(array, 3))
    assert sum_array is D.roll_and_sum(array, sum_array, 3)
    np.testing.assert_array_equal(sum_array, 2 * golden[0]["doctest_roll_and_sum"])


def test_rebin_roll_goldens(gpu, golden):
    arrays, _ = golden
    x = arrays["rebin_in"]
    for r in (1, 2, 3, 8):
        np.testing.assert_array_equal(D.quick_resample(x, r), arrays[f"resample_{r}"])
        np.testing.assert_array_equal(D.quick_chan_rebin(x, r), arrays[f"chanrebin_{r}"])
        np.testing.assert_array_equal(D.quick_chan_rebin(x.astype(np.float32), r),
                                      x.astype(np.float32)[:x.shape[0] // r * r].reshape(-1, r, x.shape[1]).sum(1))
    np.testing.assert_array_equal(D.apply_dm_shifts_to_data(x, arrays["roll_shifts"]), arrays["roll_out"])
    u = (x * 255).astype(np.uint8)
    np.testing.assert_array_equal(D.quick_chan_rebin(u, 3), u[:6].reshape(2, 3, -1).sum(1))
    np.testing.assert_array_equal(D.apply_dm_shifts_to_data(u, arrays["roll_shifts"]),
                                  np.array([np.roll(u[i], -int(np.rint(s))) for i, s in
                                            enumerate(arrays["roll_shifts"])]))


# ------------------------------------------------------------------ dedisperse

def test_dedisperse_bitexact_c1_rows(gpu, golden):
    arrays, meta = golden
    c = CONFIGS["C1"]
    arr = c1_input()
    for k, i in enumerate(arrays["c1_dedisp_rows_idx"]):
        sh = D.dedispersion_shifts(c.nchan, arrays["plan_C1"][i], c.start_freq, c.bandwidth, c.tsamp)
        dd = D.dedisperse(arr, sh)
        assert dd.dtype == np.float64
        assert sha(dd) == meta[f"c1_dedisp_sha256_{i}"]


@pytest.mark.parametrize("dt", ["u8", "f32", "f64"])
@pytest.mark.parametrize("shape", [(1, 7), (3, 100), (17, 1000), (64, 4099), (33, 65536)])
def test_dedisperse_random_shapes_exact_f64(gpu, dt, shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    nchan, n = shape
    x = {"u8": lambda: rng.integers(0, 256, shape).astype(np.uint8),
         "f32": lambda: rng.standard_normal(shape).astype(np.float32),
         "f64": lambda: rng.standard_normal(shape)}[dt]()
    sh = rng.integers(-3 * n, 3 * n, nchan).astype(float)
    np.testing.assert_array_equal(D.dedisperse(x, sh), oracle.dedisperse(x, sh.astype(np.int64)))


def _plane(x, shifts, acc, group=0, info=None, **opts):
    t = _hip.require_gpu()
    xd = _hip.to_device(x)
    plan = _hip.Plan(_hip.dtype_code(xd.dtype), D._acc_code(acc), x.shape[0], x.shape[1], shifts, group=group,
                     **opts)
    if info is not None:
        info.update(plan.info)
    return plan.dedisperse(xd).cpu().numpy()


@pytest.mark.parametrize("group", [1, 2, 4, 8])
@pytest.mark.parametrize("name", ["C1", "C5"])
def test_plane_native_vs_oracle(gpu, golden, name, group):
    """float32 accumulation, channel mode (group 1) and group mode (exact group rows)."""
    arrays, _ = golden
    c = CONFIGS[name]
    rng = np.random.default_rng(11)
    n = min(c.nsamples, 1 << 15)
    x = np.abs(rng.standard_normal((c.nchan, n))).astype(np.float32) * 0.5
    dms = arrays[f"plan_{name}"]
    idx = np.linspace(0, dms.size - 1, 40).astype(int)
    sh = _hip.shift_table(c.nchan, dms[idx], c.start_freq, c.bandwidth, c.tsamp)
    info = {}
    plane = _plane(x, sh, "native", group, info)
    assert plane.dtype == np.float32
    assert info["group"] == group or (group > 1 and info["group"] < group), info
    for k in range(len(idx)):
        ref = oracle.dedisperse(x, sh[k])
        assert np.all(np.abs(plane[k] - ref) <= f32_bound(x, sh[k])), k
    u = (x * 100).astype(np.uint8)
    pu = _plane(u, sh, "native", group)
    for k in range(0, len(idx), 5):
        np.testing.assert_array_equal(pu[k].astype(np.float64), oracle.dedisperse(u, sh[k]))
    p64 = _plane(x, sh, "f64")
    for k in range(0, len(idx), 7):
        np.testing.assert_array_equal(p64[k], oracle.dedisperse(x, sh[k]))


def test_plane_arbitrary_dm_list_large_spread(gpu):
    """Non-plan trial lists (random order, huge shift spreads): tile splitting + halo."""
    rng = np.random.default_rng(5)
    nchan, n = 48, 5000
    x = rng.standard_normal((nchan, n))
    sh = rng.integers(-20000, 20000, (70, nchan))
    plane = _plane(x, sh, "f64")
    for k in range(70):
        np.testing.assert_array_equal(plane[k], oracle.dedisperse(x, sh[k]))
    u = (np.abs(x) * 40).astype(np.uint8)
    for group in (1, 4):
        pu = _plane(u, sh, "native", group)
        for k in range(70):
            np.testing.assert_array_equal(pu[k].astype(np.float64), oracle.dedisperse(u, sh[k]))


@pytest.mark.parametrize("dt", ["u8", "f32", "f64"])
def test_plane_subband_small_lds_budget(gpu, dt):
    """A small LDS budget: one group per stage, short DM tiles, many stages per tile."""
    c = CONFIGS["C5"]
    rng = np.random.default_rng(21)
    n = 1 << 14
    x = rng.random((c.nchan, n)) * 50
    x = {"u8": x.astype(np.uint8), "f32": x.astype(np.float32), "f64": x}[dt]
    dms = np.linspace(c.dmmin, c.dmmax, 90)
    sh = _hip.shift_table(c.nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    info = {}
    plane = _plane(x, sh, "f32" if dt == "f64" else "native", 4, info, lds_budget_kb=96)
    assert info["group"] == 4 and info["stages"] > 2 * info["dm_tiles"], info
    for k in range(0, 90, 7):
        ref = oracle.dedisperse(x, sh[k])
        if dt == "u8":
            np.testing.assert_array_equal(plane[k].astype(np.float64), ref)
        else:
            assert np.all(np.abs(plane[k] - ref) <= f32_bound(x, sh[k])), k


@pytest.mark.parametrize("group", [4, 8])
@pytest.mark.parametrize("shape", ["1", "2"])
@pytest.mark.parametrize("dt", ["u8", "f32"])
def test_plane_subband_pair_shape(gpu, dt, shape, group):
    """The time-tile-256 subband shapes (shape 1 pair: 8 waves x 16 trials, two
    workgroups per CU; 2 tall: 16 waves x 16 trials) against the oracle, ragged N and a
    partial last group (nchan % G != 0 for G = 4 and 8)."""
    c = CONFIGS["C2"]
    rng = np.random.default_rng(33)
    nchan, n = 130, 20000 + 37
    x = rng.random((nchan, n)) * 40
    x = x.astype(np.uint8) if dt == "u8" else x.astype(np.float32)
    dms = np.linspace(0.0, 60.0, 150)
    sh = _hip.shift_table(nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    info = {}
    plane = _plane(x, sh, "native", group, info, shape=int(shape))
    assert info["group"] == group and info["time_tile"] == 256, info
    for k in range(0, 150, 11):
        ref = oracle.dedisperse(x, sh[k])
        if dt == "u8":
            np.testing.assert_array_equal(plane[k].astype(np.float64), ref)
        else:
            assert np.all(np.abs(plane[k] - ref) <= f32_bound(x, sh[k])), k
    g = D._dedispersion_search(x, dms, nchan, c.start_freq, c.bandwidth, c.tsamp)
    o = oracle.search(x, dms, c.start_freq, c.bandwidth, c.tsamp, nthreads=8)
    for a, b in zip(g[:3], o[:3]):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-9)


# ------------------------------------------------------------------ search tables

def test_search_test_config_vs_reference(gpu, golden):
    arrays, meta = golden
    np.random.seed(0)
    arr, h = simulate.simulate_test_data(150)
    assert sha(arr) == meta["test_input_sha256"]
    tab = D.dedispersion_search(arr, 100, 200., h["fbottom"], h["bandwidth"], h["tsamp"])
    np.testing.assert_array_equal(tab["DM"], arrays["test_table_DM"])
    for col in ("max", "std", "snr"):
        np.testing.assert_allclose(tab[col], arrays[f"test_table_{col}"], rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(tab["rebin"], arrays["test_table_rebin"])
    assert tab["rebin"].dtype == np.int32
    # the reference test's assertion (tests/test_dedispersion.py:25)
    assert np.isclose(tab["DM"][np.argmax(tab["snr"])], 150, atol=1)


def test_search_slow_path_plane(gpu, golden):
    arrays, meta = golden
    np.random.seed(0)
    arr, h = simulate.simulate_test_data(150)
    tab, plane = D.dedispersion_search(arr, 100, 200., h["fbottom"], h["bandwidth"], h["tsamp"], show=True)
    assert sha(plane) == meta["test_plane_sha256"]
    assert tab["rebin"].dtype == np.int64
    # the table comes from the float64 plane through pu_series_stats (numpy order):
    # every column bit-identical to the reference's serial path
    for col in ("DM", "max", "std", "snr", "rebin"):
        np.testing.assert_array_equal(tab[col], arrays[f"test_slow_table_{col}"])
    assert np.isclose(tab["DM"][np.argmax(tab["snr"])], 150, atol=1)


def pinfo_case(meta):
    """The PulseInfo input of the clean.dedispersion_search golden (make_golden.py)."""
    from pulsarutils.clean import PulseInfo
    a = meta["pinfo_args"]
    np.random.seed(a["seed"])
    arr, _ = simulate.simulate_test_data(dm=a["dm"], tsamp=1 / a["pulse_freq"] / a["nbin"], nsamples=a["nbin"],
                                         nchan=a["nchan"], start_freq=a["start_freq"], bandwidth=a["bandwidth"])
    assert sha(arr) == meta["pinfo_input_sha256"]
    info = PulseInfo()
    info.allprofs, info.start_freq, info.bandwidth = arr, a["start_freq"], a["bandwidth"]
    info.pulse_freq, info.nbin, info.nchan = a["pulse_freq"], a["nbin"], a["nchan"]
    return info, a


def test_clean_dedispersion_search_pulseinfo(gpu, golden):
    """clean.dedispersion_search(info, dmmin, dmmax) (clean.py:136-180): the PulseInfo
    route (sample_time = 1 / pulse_freq / nbin), float64 plane bit-identical to the
    reference's ``dummy.npy`` memmap, table equal to the reference's (rebin int64)."""
    from pulsarutils import clean as C
    arrays, meta = golden
    info, a = pinfo_case(meta)
    plane, tab = C.dedispersion_search(info, a["dmmin"], a["dmmax"])
    assert plane.dtype == np.float64 and plane.shape == (arrays["pinfo_table_DM"].size, a["nbin"])
    assert sha(plane) == meta["pinfo_plane_sha256"]
    for col in ("DM", "max", "std", "snr", "rebin"):  # bit-identical (pu_series_stats of the plane)
        np.testing.assert_array_equal(tab[col], arrays[f"pinfo_table_{col}"])
    assert tab["rebin"].dtype == np.int64


def test_search_c1_vs_reference(gpu, golden):
    arrays, _ = golden
    c = CONFIGS["C1"]
    arr = c1_input()
    mx, sd, snr, win = D._dedispersion_search(arr, arrays["plan_C1"], c.nchan, c.start_freq, c.bandwidth, c.tsamp)
    np.testing.assert_allclose(mx, arrays["c1_table_max"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(sd, arrays["c1_table_std"], rtol=1e-9)
    np.testing.assert_allclose(snr, arrays["c1_table_snr"], rtol=1e-9)
    np.testing.assert_array_equal(win, arrays["c1_table_rebin"])
    assert win.dtype == np.int32


@pytest.mark.parametrize("acc", ["native", "f32"])
def test_search_c1_float32_accumulation(gpu, golden, acc):
    arrays, _ = golden
    c = CONFIGS["C1"]
    arr = c1_input()
    mx, sd, snr, win = D._dedispersion_search(arr, arrays["plan_C1"], c.nchan, c.start_freq, c.bandwidth, c.tsamp,
                                              acc="f32" if acc == "f32" else None)
    tol = 1e-5 if acc == "f32" else 1e-9
    np.testing.assert_allclose(snr, arrays["c1_table_snr"], rtol=tol)
    np.testing.assert_allclose(sd, arrays["c1_table_std"], rtol=tol)


@pytest.mark.parametrize("group", ["1", "4"])
@pytest.mark.parametrize("dt", ["f32", "u8"])
def test_search_ragged_small(gpu, dt, group):
    """Tiny / ragged inputs: N smaller than a time tile, odd nchan, N % 8 != 0."""
    rng = np.random.default_rng(3)
    for nchan, n in [(3, 37), (5, 200), (31, 1001), (130, 3000)]:
        x = rng.random((nchan, n)) * 10
        x = x.astype(np.float32) if dt == "f32" else x.astype(np.uint8)
        dms = np.linspace(0, 300, 23)
        with D.planner_options(group=int(group)):
            g = D._dedispersion_search(x, dms, nchan, 400., 100., 1e-3)
        o = oracle.search(x, dms, 400., 100., 1e-3)
        for a, b in zip(g[:3], o[:3]):
            np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-9)
        np.testing.assert_array_equal(g[3], o[3])


@pytest.mark.parametrize("name", ["C2", "C5"])
def test_search_full_size_all_trials(gpu, golden, name):
    """Full-size configs on device data; EVERY trial of the grid re-done by the C oracle
    (C2: 1000 trials x 2^20 samples, ~25 s on 16 threads; C5: 500 trials, < 1 s) - the
    whole table against SURVEY §8a's bars, argmax over the whole grid."""
    import torch
    from pulsarutils import synth
    arrays, _ = golden
    c = CONFIGS[name]
    xd = synth.pulsar_filterbank_device(c)
    dms = arrays[f"plan_{name}"]
    (mx, sd, snr, win), plan = D.search_device(xd, dms, c.nchan, c.start_freq, c.bandwidth, c.tsamp)
    torch.cuda.synchronize()
    snr, mx, sd, win = (v.cpu().numpy() for v in (snr, mx, sd, win))
    best = dms[np.argmax(snr)]
    assert abs(best - c.pulse_dm) < 0.5, (best, c.pulse_dm)
    x = xd.cpu().numpy()
    del xd
    torch.cuda.empty_cache()
    omx, osd, osnr, owin, osw = oracle.search(x, dms, c.start_freq, c.bandwidth, c.tsamp, nthreads=16,
                                              return_width_snr=True)
    np.testing.assert_allclose(snr, osnr, rtol=1e-5)
    # max and std from the per-sample float32 bound E_t = nchan 2^-24 sum_c |x_c[t + s_c]|
    # (module docstring): the max of the series moves by <= max_t E_t, the mean by <= its
    # mean, so max - mean by <= 2 max_t E_t; std is 1-Lipschitz in the sup norm (<= max_t
    # E_t).  Plus the statistics' own float64/float32 rounding, 1e-6 relative.  The inputs
    # are non-negative (|N(0, 0.5)| + pulse), so sum_c |x_c[t + s_c]| is the series itself
    # and its maximum is the oracle's max(d) + mean (mean = sum_c mean_c for every trial).
    assert float(x.min()) >= 0.0
    mu = float(x.sum(dtype=np.float64)) / x.shape[1]
    emax = c.nchan * 2.0 ** -24 * (omx + mu) * (1 + 1e-6)
    assert np.all(np.abs(mx - omx) <= 2 * emax + 1e-6 * np.abs(omx))
    assert np.all(np.abs(sd - osd) <= emax + 1e-6 * osd)
    # rebin equal for every trial whose best and second-best window S/N are more than 1e-5
    # apart (the oracle's per-width S/N of each trial decides which trials are ties)
    srt = np.sort(osw, axis=1)
    tie = (srt[:, -1] - srt[:, -2]) <= 1e-5 * np.abs(srt[:, -1])
    assert np.array_equal(win[~tie], owin[~tie]), np.nonzero((win != owin) & ~tie)[0][:10]
    assert tie.sum() <= max(2, dms.size // 100), int(tie.sum())
    # argmax over the whole grid (unless the top two S/N are within the tolerance)
    top2 = np.sort(osnr)[-2:]
    if top2[1] - top2[0] > 1e-5 * top2[1]:
        assert np.argmax(snr) == np.argmax(osnr)


def sampled_trials(snr, n):
    """About ``n`` trials: evenly spaced ones plus the top 5 by S/N (where argmax-DM and
    rebin equality matter)."""
    top = np.argsort(snr)[::-1][:5]
    return np.unique(np.r_[np.linspace(0, snr.size - 1, n - 5).astype(int), top])


@pytest.mark.parametrize("name,group,tile", [("C2", 4, 256), ("C3", 4, 256), ("C5", 4, 256), ("C4", 4, 128)])
def test_default_group_cost_model(gpu, golden, name, group, tile):
    """With no explicit group the planner keeps the cheapest of G = 8 / G = 4 in the wide
    (128-trial DM tiles) and tall (256-trial) shapes by its cost model; at C2/C3/C4/C5 that is the measured winner (profiles/r01_autog/,
    profiles/r03/experiments/ab_*_shape*.log; round 6: C3's 5000 trials tall G = 4 with
    16-bit slots 909.7 ms against tall G = 8 960 ms, profiles/r06/experiments/slot16/).  The default plan's dedispersed rows also
    match the oracle (float32: the summation-order bound; uint8: bit-exact), so the
    numerics do not depend on which plan the model picks."""
    import torch
    from pulsarutils import synth
    c = CONFIGS[name]
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
    sh = _hip.shift_table(c.nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    code = {"u8": _hip.PU_U8, "f32": _hip.PU_F32}[c.dtype]
    plan = _hip.Plan(code, _hip.PU_ACC_NATIVE, c.nchan, c.nsamples, sh)
    assert plan.info["group"] == group and plan.info["trials_per_tile"] == tile, plan.info
    assert plan.info["kernel"] == (3 if name == "C3" else 2), plan.info
    if name == "C3":
        # C3's production plan (5000 trials, tall G = 4, 16-bit slots): test_search_c3_full_size_u8 checks
        # rows of its DM tile that holds the best trial bit-exact, through that plan itself
        # (pu_plan_dedisperse_dm_tile: same instantiation, tables and tiling)
        return
    xd = synth.pulsar_filterbank_device(c)
    plane = plan.dedisperse(xd)
    idx = np.array([0, dms.size // 3, dms.size - 1])
    rows = plane[torch.as_tensor(idx, device=xd.device)].cpu().numpy()
    del plane
    torch.cuda.empty_cache()
    x = xd.cpu().numpy()
    for k, i in enumerate(idx):
        ref = oracle.dedisperse(x, sh[i])
        assert np.all(np.abs(rows[k] - ref) <= f32_bound(x, sh[i])), i


def test_plan_cache_reuse(gpu):
    """Repeated numpy-API calls reuse the cached plan (same results); a different trial
    grid or planner variable builds a new one."""
    c = CONFIGS["C2"]
    rng = np.random.default_rng(7)
    x = rng.random((64, 4096)).astype(np.float32)
    dms = np.linspace(0.0, 30.0, 40)
    args = (64, c.start_freq, c.bandwidth, c.tsamp)
    a = D._dedispersion_search(x, dms, *args)
    _, p1 = D.search_device(x, dms, *args)
    _, p2 = D.search_device(x, dms, *args)
    assert p1 is p2
    b = D._dedispersion_search(x, dms, *args)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)
    _, p3 = D.search_device(x, dms[:-1], *args)
    assert p3 is not p1
    with D.planner_options(shape=1):
        _, p4 = D.search_device(x, dms, *args)
        assert p4 is not p1 and p4.info["time_tile"] == 256
        for u, v in zip(a, D._dedispersion_search(x, dms, *args)):
            np.testing.assert_allclose(u, v, rtol=1e-5)
    _, p5 = D.search_device(x, dms, *args)  # the scope ended: the default plan again
    assert p5 is p1


def test_search_c3_full_size_u8(gpu):
    """Maximum size (C3: 4096 x 2^22 uint8, 5000 trials, 17 GB in HBM): the full search
    finds the injected pulse; the production plan's own rows - the DM tile that holds the
    best trial, dedispersed by that plan (pu_plan_dedisperse_dm_tile: the tall G = 4 16-bit
    slot instantiation, slot/stage/window tables and tiling of the 5000-trial search) - are
    bit-equal to the float64 C oracle for the tile's first, best and last trial (integer
    partial sums < 2^24 are exact in float32), and the statistics match it within SURVEY
    §8a's 1e-5."""
    import torch
    from pulsarutils import synth
    c = CONFIGS["C3"]
    xd = synth.pulsar_filterbank_device(c)
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
    assert dms.size == 5000
    (mx, sd, snr, win), plan = D.search_device(xd, dms, c.nchan, c.start_freq, c.bandwidth, c.tsamp)
    torch.cuda.synchronize()
    assert plan.info["group"] == 4 and plan.info["trials_per_tile"] == 256 and plan.ndm == 5000, plan.info
    assert plan.info["kernel"] == 3, plan.info
    snr = snr.cpu().numpy()
    best = int(np.argmax(snr))
    assert abs(dms[best] - c.pulse_dm) < 0.5, (dms[best], c.pulse_dm)
    first, count = plan.dm_tiles()
    assert int(count.sum()) == dms.size and np.array_equal(np.sort(first), np.cumsum(np.r_[0, count[np.argsort(first)]])[:-1])
    dt = int(np.nonzero((first <= best) & (best < first + count))[0][0])
    rows = plan.dedisperse_dm_tile(xd, dt)
    idx = np.array([int(first[dt]), best, int(first[dt] + count[dt] - 1)])
    plane = rows[torch.as_tensor(idx - int(first[dt]), device=rows.device)].cpu().numpy()
    del rows
    x = xd.cpu().numpy()
    del xd
    torch.cuda.empty_cache()
    omx, osd, osnr, owin, dd = oracle.search(x, dms[idx], c.start_freq, c.bandwidth, c.tsamp,
                                             nthreads=16, return_dedisp=True)
    for k in range(idx.size):
        np.testing.assert_array_equal(plane[k].astype(np.float64), dd[k])
    del dd
    # statistics of ~32 trials (evenly spaced + the top 5 by S/N): argmax DM and rebin pinned
    idx = sampled_trials(snr, 32)
    omx, osd, osnr, owin = oracle.search(x, dms[idx], c.start_freq, c.bandwidth, c.tsamp, nthreads=16)
    np.testing.assert_allclose(snr[idx], osnr, rtol=1e-5)
    np.testing.assert_allclose(sd.cpu().numpy()[idx], osd, rtol=1e-5)
    np.testing.assert_allclose(mx.cpu().numpy()[idx], omx, rtol=1e-5)
    np.testing.assert_array_equal(win.cpu().numpy()[idx], owin)
    assert idx[np.argmax(snr[idx])] == idx[np.argmax(osnr)]


def test_search_u8_bitexact_series_c3_slice(gpu):
    """uint8 C3-like slice: float32 accumulation is exact -> plane equals the float64 oracle."""
    import torch
    from dataclasses import replace
    from pulsarutils import synth
    c = replace(CONFIGS["C3"], nsamples=1 << 16)
    xd = synth.pulsar_filterbank_device(c)
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
    idx = np.linspace(0, dms.size - 1, 5).astype(int)
    sh = _hip.shift_table(c.nchan, dms[idx], c.start_freq, c.bandwidth, c.tsamp)
    plan = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, c.nchan, c.nsamples, sh)
    plane = plan.dedisperse(xd).cpu().numpy()
    x = xd.cpu().numpy()
    for k in range(len(idx)):
        np.testing.assert_array_equal(plane[k].astype(np.float64), oracle.dedisperse(x, sh[k]))
    torch.cuda.synchronize()


@pytest.mark.parametrize("group", [4, 8])
@pytest.mark.parametrize("shape", ["0", "1", "2"])
def test_plane_u8_dma_rows(gpu, shape, group):
    """8-bit rows staged by LDS-DMA (N % 4 == 0): bit-exact against the oracle and the
    global-read build (u8_dma=False), with a partial last group (130 % G != 0), row
    misalignments (base % 4 != 0), a padded row stride and a view whose rows are not
    4-byte aligned."""
    import torch
    c = CONFIGS["C2"]
    rng = np.random.default_rng(44)
    nchan, n = 130, 20000
    x = (rng.random((nchan, n)) * 60).astype(np.uint8)
    dms = np.linspace(0.0, 60.0, 150)
    sh = _hip.shift_table(nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    plan = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, nchan, n, sh, group=group, shape=int(shape))
    assert plan.info["group"] == group, plan.info
    xd = _hip.to_device(x)
    plane = plan.dedisperse(xd).cpu().numpy()
    for k in range(0, 150, 13):
        np.testing.assert_array_equal(plane[k].astype(np.float64), oracle.dedisperse(x, sh[k]))
    ref = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, nchan, n, sh, group=group, shape=int(shape),
                    u8_dma=False).dedisperse(xd).cpu().numpy()
    np.testing.assert_array_equal(plane, ref)
    big = torch.zeros((nchan, n + 8), dtype=torch.uint8, device=xd.device)
    big[:, 4:4 + n] = xd
    np.testing.assert_array_equal(plan.dedisperse(big[:, 4:4 + n]).cpu().numpy(), plane)  # ld = n + 8
    np.testing.assert_array_equal(plan.dedisperse(big[:, 1:1 + n].copy_(xd)).cpu().numpy(), plane)  # copied
    g = plan.search(big[:, 1:1 + n])
    torch.cuda.synchronize()


@pytest.mark.parametrize("group", [4, 8])
def test_plane_u8_global_rows_ragged(gpu, group):
    """8-bit rows read from global memory (N % 4 != 0: no LDS-DMA) with a partial last
    group (nchan % G != 0): bit-exact against the oracle."""
    c = CONFIGS["C2"]
    rng = np.random.default_rng(45)
    nchan, n = 130, 20001
    x = (rng.random((nchan, n)) * 60).astype(np.uint8)
    dms = np.linspace(0.0, 60.0, 150)
    sh = _hip.shift_table(nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    info = {}
    plane = _plane(x, sh, "native", group, info)
    assert info["group"] == group, info
    for k in range(0, 150, 13):
        np.testing.assert_array_equal(plane[k].astype(np.float64), oracle.dedisperse(x, sh[k]))


@pytest.mark.parametrize("dt", ["u8", "f32"])
def test_default_group_ragged_vs_oracle(gpu, dt):
    """No explicit group (automatic G = 4 / 8 choice) at a ragged nchan: the plan the
    planner keeps is reported, and its plane and search match the oracle."""
    c = CONFIGS["C2"]
    rng = np.random.default_rng(46)
    nchan, n = 203, 40000
    x = rng.random((nchan, n)) * 40
    x = x.astype(np.uint8) if dt == "u8" else x.astype(np.float32)
    dms = np.linspace(0.0, 60.0, 300)
    sh = _hip.shift_table(nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    info = {}
    plane = _plane(x, sh, "native", 0, info)
    assert info["group"] in (4, 8), info
    for k in range(0, 300, 23):
        ref = oracle.dedisperse(x, sh[k])
        if dt == "u8":
            np.testing.assert_array_equal(plane[k].astype(np.float64), ref)
        else:
            assert np.all(np.abs(plane[k] - ref) <= f32_bound(x, sh[k])), k
    g = D._dedispersion_search(x, dms, nchan, c.start_freq, c.bandwidth, c.tsamp)
    o = oracle.search(x, dms, c.start_freq, c.bandwidth, c.tsamp, nthreads=16)
    for a, b in zip(g[:3], o[:3]):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-9)
    np.testing.assert_array_equal(g[3], o[3])
    for forced in (4, 8):
        pf = _plane(x, sh, "native", forced)
        if dt == "u8":
            np.testing.assert_array_equal(pf, plane)


@pytest.mark.parametrize("dt,acc,group", [("f32", "native", 0), ("u8", "native", 8), ("f32", "f64", 1),
                                          ("f64", "native", 1), ("f32", "native", 4)])
def test_dedisperse_dm_tile_equals_full_plane(gpu, dt, acc, group):
    """pu_plan_dedisperse_dm_tile: every DM tile's rows equal the full plane's rows of the
    same trials bit for bit (subband and channel mode, sorted tile orders included), and
    the tiles cover the grid exactly once."""
    import torch
    c = CONFIGS["C2"]
    rng = np.random.default_rng(52)
    nchan, n = 96, 12000
    x = rng.random((nchan, n)) * 50
    x = {"f32": x.astype(np.float32), "u8": x.astype(np.uint8), "f64": x}[dt]
    dms = np.linspace(0.0, 300.0, 333)
    sh = _hip.shift_table(nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    code = {"u8": _hip.PU_U8, "f32": _hip.PU_F32, "f64": _hip.PU_F64}[dt]
    accc = {"native": _hip.PU_ACC_NATIVE, "f64": _hip.PU_ACC_F64}[acc]
    plan = _hip.Plan(code, accc, nchan, n, sh, group=group)
    xd = _hip.to_device(x)
    full = plan.dedisperse(xd)
    first, count = plan.dm_tiles()
    assert first.size == plan.info["dm_tiles"] and first.size > 1
    seen = np.zeros(dms.size, int)
    for t in range(first.size):
        rows = plan.dedisperse_dm_tile(xd, t)
        assert rows.shape == (int(count[t]), n)
        assert torch.equal(rows, full[int(first[t]):int(first[t] + count[t])]), t
        seen[first[t]:first[t] + count[t]] += 1
    assert np.all(seen == 1)
    with pytest.raises(ValueError):
        _hip.check(_hip.lib().pu_plan_dedisperse_dm_tile(plan._h, _hip.ptr(xd), xd.stride(0), first.size,
                                                         _hip.ptr(full), full.stride(0), None), "dm_tile")


def _tables_agree(r16, r32):
    """Search tables of the two slot kinds: the series are the same integers, but the plans
    may cut the trials into different DM tiles (the 16-bit slots cap a slot's span), so
    the epilogue's float32 partial sums centre on other tile means - max / std / snr agree
    to float32 summation order (rtol 1e-6, inside SURVEY §8a's 1e-5), rebin exactly."""
    for a, b in zip(r16[:3], r32[:3]):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(r16[3], r32[3])


def _slot16_pair(x, sh, **opts):
    """The same trial grid planned with 16-bit integer slots and with float32 slots:
    (plane16, plane32, search16, search32, info16, info32)."""
    import torch
    xd = _hip.to_device(x)
    out = []
    for s16 in (True, False):
        plan = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, x.shape[0], x.shape[1], sh, slot16=s16, **opts)
        plane = plan.dedisperse(xd).cpu().numpy()
        res = [v.cpu().numpy() for v in plan.search(xd)]
        torch.cuda.synchronize()
        out.append((plane, res, plan.info))
    (p16, r16, i16), (p32, r32, i32) = out
    return p16, p32, r16, r32, i16, i32


@pytest.mark.parametrize("shape", ["tall", "pair"])
@pytest.mark.parametrize("group", [2, 4, 8])
def test_slot16_u8_matches_float_slots_and_oracle(gpu, shape, group):
    """16-bit integer slots (8-bit input, 256-sample tiles): every plane row
    bit-equal to the float64 oracle (integer sums < 2^24 are exact either way) and to the
    float32-slot plan, and the search table (max, std, snr, rebin) equal to the float32-slot
    plan's (_tables_agree) and to the oracle's within 1e-5.  Ragged channel count
    (a partial last group reads the zero row), N not a multiple of the tile, values up to
    255."""
    rng = np.random.default_rng(100 + group)
    nchan, n = 203, 5000
    x = rng.integers(0, 256, (nchan, n)).astype(np.uint8)
    dms = np.linspace(0, 120, 300)
    sh = _hip.shift_table(nchan, dms, 400., 100., 1e-3)
    p16, p32, r16, r32, i16, i32 = _slot16_pair(x, sh, group=group, shape=shape)
    assert i16["kernel"] == 3 and i32["kernel"] == 2, (i16, i32)
    assert i16["group"] == group and i16["time_tile"] == 256
    np.testing.assert_array_equal(p16, p32)
    for k in range(0, sh.shape[0], 13):
        np.testing.assert_array_equal(p16[k].astype(np.float64), oracle.dedisperse(x, sh[k]))
    _tables_agree(r16, r32)
    o = oracle.search(x, dms, 400., 100., 1e-3)
    for a, b in zip(r16[:3], o[:3]):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-9)
    np.testing.assert_array_equal(r16[3], o[3])


def test_slot16_u8_full_scale_sums_and_flushes(gpu):
    """All-255 input on 4096 channels: every window adds 4 x 255 per group, so the packed
    u16 accumulators flush every 64 groups and the 256-unit halves carry the totals up to
    4096 x 255 = 1044480 (< 2^24) - the plane equals the oracle bit for bit; a few rows of
    noise on top make the series differ per trial."""
    rng = np.random.default_rng(7)
    nchan, n = 4096, 2048
    x = np.full((nchan, n), 255, np.uint8)
    x[rng.integers(0, nchan, 50), rng.integers(0, n, 50)] = 0
    dms = np.linspace(0, 30, 40)
    sh = _hip.shift_table(nchan, dms, 1200., 300., 64e-6)
    p16, p32, r16, r32, i16, _ = _slot16_pair(x, sh, group=4, shape="tall")
    assert i16["kernel"] == 3
    np.testing.assert_array_equal(p16, p32)
    for k in (0, 17, 39):
        np.testing.assert_array_equal(p16[k].astype(np.float64), oracle.dedisperse(x, sh[k]))
    _tables_agree(r16, r32)


def test_slot16_u8_long_slots_c3_slice(gpu):
    """C3's own channels and first 625 trials (the 8-GPU shard) at 2^16 samples: slot spans
    up to ~150 samples, so some slots need the fourth 128-element build chunk (len > 384)
    and the O stream's lane-63 hand-over between chunks - plane rows bit-equal to the
    oracle, tables equal to the float32-slot plan's (_tables_agree)."""
    from dataclasses import replace
    from pulsarutils import synth
    c = replace(CONFIGS["C3"], nsamples=1 << 16)
    xd = synth.pulsar_filterbank_device(c)
    x = xd.cpu().numpy()
    del xd
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)[:625]
    sh = _hip.shift_table(c.nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    p16, p32, r16, r32, i16, _ = _slot16_pair(x, sh, group=4, shape="tall")
    assert i16["kernel"] == 3 and i16["group"] == 4, i16
    np.testing.assert_array_equal(p16, p32)
    for k in (0, 300, 624):
        np.testing.assert_array_equal(p16[k].astype(np.float64), oracle.dedisperse(x, sh[k]))
    _tables_agree(r16, r32)


@pytest.mark.parametrize("budget", [0, 64])
def test_slot16_u8_wrapping_windows_and_small_budget(gpu, budget):
    """Short series (windows wrap modulo N: the per-lane modular DMA) with large random
    shifts, and a small LDS budget (one group per stage: the flush counter runs across
    many stages) - planes equal the oracle, tables the float32-slot plan's."""
    rng = np.random.default_rng(9)
    nchan, n = 48, 1024
    x = rng.integers(0, 256, (nchan, n)).astype(np.uint8)
    sh = rng.integers(-20000, 20000, (70, nchan))
    sh = np.sort(sh, axis=0)
    p16, p32, r16, r32, i16, _ = _slot16_pair(x, sh, group=4, shape="tall", lds_budget_kb=budget)
    assert i16["kernel"] == 3, i16
    np.testing.assert_array_equal(p16, p32)
    for k in range(0, 70, 9):
        np.testing.assert_array_equal(p16[k].astype(np.float64), oracle.dedisperse(x, sh[k]))
    _tables_agree(r16, r32)


def test_slot16_default_every_group(gpu):
    """By default the planner uses 16-bit slots for 8-bit rows in 256-sample tiles at every
    group size (G = 8 with the four-per-lane build measured faster than with float32 slots:
    DESIGN.md §4.1b); slot16=True is the same, slot16=False never uses them."""
    x = np.zeros((64, 4096), np.uint8)
    sh = _hip.shift_table(64, np.linspace(0, 50, 40), 400., 100., 1e-3)
    mk = lambda g, s16: _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, 64, 4096, sh, group=g, shape="tall",
                                   slot16=s16).info
    assert mk(8, None)["kernel"] == 3 and mk(4, None)["kernel"] == 3 and mk(2, None)["kernel"] == 3
    assert mk(8, True)["kernel"] == 3 and mk(4, False)["kernel"] == 2 and mk(8, False)["kernel"] == 2


def test_c3_plan_choice_shard_and_full(gpu):
    """The planner's cost model at C3's two measured operating points:
    the 625-trial shard of the 8-GPU split takes tall G = 8 (16-bit slots 113.5 ms, against
    127.2 ms for G = 4), the whole 5000-trial grid tall G = 4 (858 ms, against 936 for G = 8)."""
    c = CONFIGS["C3"]
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
    for ntr, group, kernel in ((625, 8, 3), (5000, 4, 3)):
        sh = _hip.shift_table(c.nchan, dms[:ntr], c.start_freq, c.bandwidth, c.tsamp)
        info = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, c.nchan, c.nsamples, sh).info
        assert (info["group"], info["kernel"], info["trials_per_tile"]) == (group, kernel, 256), (ntr, info)
