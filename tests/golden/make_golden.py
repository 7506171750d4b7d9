"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

Run once in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

The reference modules are executed from /root/reference via ``refload.py`` (numba
stubbed to the identity => interpreted-numpy semantics).  Only data
is written: ``golden.npz`` (arrays, loadable with ``allow_pickle=False``) and
``golden.json`` (scalars, SHA-256 digests).  Inputs are regenerated from seeds by
the tests; their SHA-256 is recorded so a drifting generator is caught.

Cross-check: ``ref_mad`` goldens are recomputed with the real statsmodels 0.12.2
in /opt/conda/bin/python3.9 (numpy 1.26) when that interpreter exists.
"""
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "radio-pulsar-utils_amd"))

from refload import load_reference  # noqa: E402

ref = load_reference()
from pulsarutils.configs import CONFIGS  # noqa: E402  (our package: configs + synth only)
from pulsarutils import synth  # noqa: E402

OUT_NPZ = os.path.join(HERE, "golden.npz")
OUT_JSON = os.path.join(HERE, "golden.json")

arrays = {}
meta = {}
if os.path.exists(OUT_NPZ):
    arrays.update(dict(np.load(OUT_NPZ, allow_pickle=False)))
if os.path.exists(OUT_JSON):
    meta.update(json.load(open(OUT_JSON)))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def have(key):
    return key in arrays or key in meta


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


D = ref.dedispersion

# ---------------------------------------------------------------- doctests
if not have("doctest_normalize"):
    arrays["doctest_normalize"] = D.normalize_shifts(np.array([-1, 0, 2, 4]), 3)
    counts = np.array([np.arange(0, 10), np.arange(2, 12), np.arange(1, 11),
                       np.arange(3, 13), np.arange(1, 11), np.arange(3, 13)])
    arrays["doctest_chan_rebin"] = D.quick_chan_rebin(counts, 2)
    arrays["doctest_resample"] = D.quick_resample(np.array([np.arange(1, 11), np.arange(3, 13)]), 2)
    arrays["doctest_roll_and_sum"] = D.roll_and_sum(np.arange(10), np.zeros(10), 3)
    arrays["doctest_plan"] = D.dedispersion_plan(10, 0, 10, 1400, 128, 0.0005)

# ---------------------------------------------------------------- plans + shift tables
for name, c in CONFIGS.items():
    k = f"plan_{name}"
    if have(k):
        continue
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
    arrays[k] = dms
    nd = dms.size
    idx = np.unique(np.concatenate([[0, nd - 1], np.linspace(0, nd - 1, 10).astype(int)]))
    if name == "C1":
        idx = np.arange(nd)
    arrays[f"shiftidx_{name}"] = idx
    arrays[f"shifts_{name}"] = np.array(
        [D.dedispersion_shifts(c.nchan, dms[i], c.start_freq, c.bandwidth, c.tsamp) for i in idx])
    log("plan", name, nd)

# ---------------------------------------------------------------- test config (seed 0)
if not have("test_table_snr"):
    np.random.seed(0)
    arr, header = ref.simulate.simulate_test_data(150)
    meta["test_input_sha256"] = sha(arr)
    t0 = time.time()
    tab = D.dedispersion_search(arr, 100, 200., header["fbottom"], header["bandwidth"], header["tsamp"])
    log("test fast search", time.time() - t0)
    for col in ("DM", "max", "std", "snr", "rebin"):
        arrays[f"test_table_{col}"] = np.asarray(tab[col])
    tab2, plane = D.dedispersion_search(arr, 100, 200., header["fbottom"], header["bandwidth"],
                                        header["tsamp"], show=True)
    for col in ("DM", "max", "std", "snr", "rebin"):
        arrays[f"test_slow_table_{col}"] = np.asarray(tab2[col])
    plane = np.asarray(plane)
    meta["test_plane_sha256"] = sha(plane)
    arrays["test_plane_rows"] = plane[::16].copy()
    meta["test_best_dm"] = float(tab["DM"][np.argmax(tab["snr"])])

# ---------------------------------------------------------------- C1 (seed 2024)
c1 = CONFIGS["C1"]
if not have("c1_table_snr"):
    np.random.seed(c1.seed)
    arr, header = ref.simulate.simulate_test_data(
        dm=c1.pulse_dm, tsamp=c1.tsamp, nsamples=c1.nsamples, nchan=c1.nchan,
        start_freq=c1.start_freq, bandwidth=c1.bandwidth)
    meta["c1_input_sha256"] = sha(arr)
    dms = arrays["plan_C1"]
    rows = {}
    for i in (0, 30, 60, 99):
        sh = D.dedispersion_shifts(c1.nchan, dms[i], c1.start_freq, c1.bandwidth, c1.tsamp)
        dd = D.dedisperse(arr, sh)
        meta[f"c1_dedisp_sha256_{i}"] = sha(dd)
        rows[i] = dd
    arrays["c1_dedisp_rows_idx"] = np.array(sorted(rows))
    arrays["c1_dedisp_rows"] = np.array([rows[i][::16] for i in sorted(rows)])
    t0 = time.time()
    tab = D.dedispersion_search(arr, c1.dmmin, c1.dmmax, c1.start_freq, c1.bandwidth, c1.tsamp)
    log("C1 search (interpreted reference)", time.time() - t0)
    meta["c1_ref_search_seconds_1thread"] = time.time() - t0
    for col in ("DM", "max", "std", "snr", "rebin"):
        arrays[f"c1_table_{col}"] = np.asarray(tab[col])
    # C1 cleaning leg (float64 input)
    C = ref.clean
    bad = C.get_noisier_channels(arr)
    arrays["c1_noisier"] = bad
    arrays["c1_variability"] = C.measure_channel_variability(arr)
    ren = C.renormalize_data(arr, badchans_mask=bad, cut_outliers=True)
    meta["c1_renorm_cut_sha256"] = sha(ren)
    arrays["c1_renorm_cut_badbins"] = np.nonzero(np.all(ren == 0, axis=0))[0]
    arrays["c1_renorm_cut_sample"] = ren[:, ::256].copy()

# ---------------------------------------------------------------- cleaning goldens
C = ref.clean


def clean_case(tag, x):
    if have(f"{tag}_noisier"):
        return
    meta[f"{tag}_input_sha256"] = sha(x)
    t0 = time.time()
    bad = C.get_noisier_channels(x)
    arrays[f"{tag}_noisier"] = bad
    arrays[f"{tag}_spec_mean"] = x.mean(1)
    arrays[f"{tag}_spec_std"] = np.std(x, axis=1)
    arrays[f"{tag}_variability"] = C.measure_channel_variability(x)
    arrays[f"{tag}_variability_masked"] = C.measure_channel_variability(x, badchans_mask=bad)
    for cut in (False, True):
        ren = C.renormalize_data(x, badchans_mask=bad, cut_outliers=cut)
        key = f"{tag}_renorm_{'cut' if cut else 'nocut'}"
        meta[key + "_sha256"] = sha(ren)
        arrays[key + "_sample"] = ren[:, ::max(1, x.shape[1] // 64)].copy()
        arrays[key + "_rowsum"] = ren.sum(1)
        if cut:
            arrays[key + "_badbins"] = np.nonzero(np.all(ren == 0, axis=0) & ~np.all(bad))[0]
        del ren
    log("clean", tag, x.shape, x.dtype, time.time() - t0)


c4 = CONFIGS["C4"]
for dt in ("f32", "u8"):
    x = synth.rfi_filterbank_np(c4, dtype=dt)
    clean_case(f"c4{dt}", x)
    del x
# ragged shape: N not a multiple of 8192 (pairwise tail chunks), nchan not a power of 2
from dataclasses import replace  # noqa: E402
rag = replace(c4, nchan=100, nsamples=12345, seed=77)
for dt in ("f32", "u8"):
    clean_case(f"rag{dt}", synth.rfi_filterbank_np(rag, dtype=dt))
clean_case("ragf64", synth.rfi_filterbank_np(rag, dtype="f64"))

# ---------------------------------------------------------------- ref_mad
if not have("refmad_in_f64"):
    rng = np.random.default_rng(5)
    a64 = rng.standard_normal(1000) * 3 + 10
    a32 = a64.astype(np.float32)
    arrays["refmad_in_f64"] = a64
    arrays["refmad_out_f64"] = np.array(ref.stats.ref_mad(a64))
    arrays["refmad_out_f32"] = np.array(ref.stats.ref_mad(a32))
    py39 = "/opt/conda/bin/python3.9"
    if os.path.exists(py39):
        code = ("import numpy as np,sys;from statsmodels.robust import mad;"
                "a=np.frombuffer(sys.stdin.buffer.read(),dtype=np.float64);"
                "print(repr(float(mad(np.diff(a))/np.sqrt(2))))")
        r = subprocess.run([py39, "-W", "ignore", "-c", code], input=a64.tobytes(),
                           capture_output=True, check=True)
        meta["refmad_f64_real_statsmodels"] = float(r.stdout.decode().strip())
        log("statsmodels 0.12.2 cross-check", meta["refmad_f64_real_statsmodels"],
            float(arrays["refmad_out_f64"]))


def real_statsmodels_refmad(a):
    """ref_mad of ``a`` (float32 or float64) by the real statsmodels 0.12.2 in py3.9: the
    input's bytes and dtype go through stdin, np.diff runs in that dtype (as in stats.py)."""
    code = ("import numpy as np,sys;from statsmodels.robust import mad;"
            f"a=np.frombuffer(sys.stdin.buffer.read(),dtype=np.{a.dtype.name});"
            "print(repr(float(mad(np.diff(a))/np.sqrt(2))))")
    r = subprocess.run(["/opt/conda/bin/python3.9", "-W", "ignore", "-c", code], input=a.tobytes(),
                       capture_output=True, check=True)
    return float(r.stdout.decode().strip())


# statsmodels' mad converts its input to float64 (array_like dtype=np.double),
# so a float32 spectrum's ref_mad is a float64 median of exactly widened float32
# differences.  Cross-check the float32 input against the real package too, and pin a
# float32 spectrum whose noisier-channel decision depends on it (with a float32 median /
# |d - m| the channel at index 100 flips to "noisy").
if os.path.exists("/opt/conda/bin/python3.9") and not have("refmad_f32_real_statsmodels"):
    a32 = arrays["refmad_in_f64"].astype(np.float32)
    meta["refmad_f32_real_statsmodels"] = real_statsmodels_refmad(a32)
    log("statsmodels 0.12.2 cross-check (float32)", meta["refmad_f32_real_statsmodels"],
        float(arrays["refmad_out_f32"]))
if not have("noisy32_spec"):
    from scipy.signal import medfilt
    from scipy.stats import norm

    def _mad(a, wide):
        a = np.asarray(a, dtype=np.double) if wide else np.asarray(a)
        c = np.median(a) if wide else np.apply_over_axes(np.median, a, 0)
        return np.median(np.abs(a - c) / norm.ppf(3 / 4.))

    for seed in range(2000):  # first seed where a float32 value separates the two thresholds
        rng = np.random.default_rng(seed)
        spec = rng.standard_normal(256).astype(np.float32)
        spec[100] = 50.0  # the two differences at 100 stay extreme: medians independent of it
        thr = [medfilt(spec, 7)[100] + 5 * (_mad(np.diff(spec), w) / np.sqrt(2)) for w in (True, False)]
        lo, hi = min(thr), max(thr)
        v = np.nextafter(np.float32(lo), np.float32(np.inf))
        while v <= lo:
            v = np.nextafter(v, np.float32(np.inf))
        if v < hi:
            spec[100] = v
            break
    x = np.repeat(spec[:, None], 4, axis=1)  # row means (float32 pairwise sums of 4 equal values) = spec
    assert np.array_equal(x.mean(1), spec)
    arrays["noisy32_spec"] = spec
    arrays["noisy32_mask"] = ref.clean.get_noisier_channels(x)
    meta["noisy32_seed"] = seed
    if os.path.exists("/opt/conda/bin/python3.9"):
        meta["noisy32_refmad_real_statsmodels"] = real_statsmodels_refmad(spec)
        assert meta["noisy32_refmad_real_statsmodels"] == float(ref.stats.ref_mad(spec))
    log("noisy32", seed, np.flatnonzero(arrays["noisy32_mask"]))

# ---------------------------------------------------------------- small rebin / roll goldens
if not have("rebin_in"):
    rng = np.random.default_rng(6)
    x = rng.random((6, 1003))
    arrays["rebin_in"] = x
    for r in (1, 2, 3, 8):
        arrays[f"resample_{r}"] = D.quick_resample(x, r)
        arrays[f"chanrebin_{r}"] = D.quick_chan_rebin(x, r)
    sh = rng.integers(-2000, 2000, 6).astype(float)
    arrays["roll_shifts"] = sh
    arrays["roll_out"] = D.apply_dm_shifts_to_data(x, sh)

# ---------------------------------------------------------------- clean.dedispersion_search (clean.py:136-180)
# The PulseInfo route: sample_time = 1 / pulse_freq / nbin (clean.py:141).  The
# reference writes its plane to ``dummy.npy`` in the CWD (clean.py:150-151): it runs
# inside a throw-away directory so nothing lands in the repository.
if not have("pinfo_table_snr"):
    import tempfile

    class _Info:  # the attributes clean.dedispersion_search reads (clean.py:138-141)
        pass

    np.random.seed(31)
    nbin, pulse_freq = 512, 1.7
    arr, _ = ref.simulate.simulate_test_data(dm=60., tsamp=1 / pulse_freq / nbin, nsamples=nbin, nchan=64,
                                             start_freq=1200., bandwidth=200.)
    info = _Info()
    info.allprofs, info.start_freq, info.bandwidth = arr, 1200., 200.
    info.pulse_freq, info.nbin = pulse_freq, nbin
    meta["pinfo_input_sha256"] = sha(arr)
    cwd = os.getcwd()
    tmpd = tempfile.mkdtemp()
    os.chdir(tmpd)
    try:
        plane, tab = ref.clean.dedispersion_search(info, 30., 90.)
        plane = np.array(plane)
    finally:
        os.chdir(cwd)
    meta["pinfo_plane_sha256"] = sha(plane)
    meta["pinfo_args"] = {"seed": 31, "nbin": nbin, "pulse_freq": pulse_freq, "dm": 60., "nchan": 64,
                          "start_freq": 1200., "bandwidth": 200., "dmmin": 30., "dmmax": 90.}
    for col in ("DM", "max", "std", "snr", "rebin"):
        arrays[f"pinfo_table_{col}"] = np.asarray(tab[col])
    log("clean.dedispersion_search (PulseInfo)", plane.shape)

# ---------------------------------------------------------------- file statistics (stats.py:35-90)
# sigpyproc is absent: the reference's get_spectral_stats/get_bad_chans run with their
# ``FilReader`` name bound to our SIGPROC reader (header/readBlock surface).  What this
# pins is the reference's chunked statistics + thresholds; the reader is ours on both sides.
if not have("fil_u8_badchans"):
    import tempfile
    from pulsarutils import sigproc
    tmpd = tempfile.mkdtemp()
    from synth_files import write_stats_file
    for dt in ("u8", "f32"):
        fname, x = write_stats_file(tmpd, dt)
        meta[f"fil_{dt}_sha256"] = sha(x)
        ref.stats.FilReader = sigproc.FilReader
        mean_spec, std_spec = ref.stats.get_spectral_stats(fname)
        arrays[f"fil_{dt}_mean"] = mean_spec
        arrays[f"fil_{dt}_std"] = std_spec
        arrays[f"fil_{dt}_badchans"] = ref.stats.get_bad_chans(fname)
        meta[f"fil_{dt}_badchans_txt"] = open(fname + ".badchans").read()
    log("file statistics goldens")

# ---------------------------------------------------------------- degenerate trials (dedispersion.py:186-201)
# All-zero, constant, NaN/inf-carrying and S/N-tie inputs (tests/degenerate_cases.py).
# The small cases run the reference's ``_dedispersion_search`` as it is.  The C1- and
# C2-shaped cases (too slow for the interpreted roll_and_sum loop: 1e9 Python
# iterations per C2 trial) run it with the module's ``dedisperse`` replaced by a
# vectorised equivalent that adds the same float64 values in the same channel order
# (``s += np.roll(row, normalize_shifts(-shifts, N)[c])``, the reference's own
# normalize_shifts); the replacement is checked bit-for-bit against the reference's
# dedisperse on every small case first.  Everything else (mean, quick_resample,
# np.max / np.std, the strict ``snr > best_snr`` rule) is the reference's code.
import degenerate_cases as DC  # noqa: E402

_orig_dedisperse = D.dedisperse


def _vec_dedisperse(data, shifts):
    N = data.shape[1]
    sh = D.normalize_shifts(-shifts, N)
    s = np.zeros(N)
    for c in range(data.shape[0]):
        s += np.roll(data[c], int(sh[c]))
    return s


def _deg_run(case, patched):
    nchan, f0, bw, ts = DC.band(case)
    x = DC.make(case)
    dms = DC.trial_dms(case.split(":")[0])
    if dms is None:
        dms = D.dedispersion_plan(nchan, DC.SMALL_DM_RANGE[0], DC.SMALL_DM_RANGE[1], f0, bw, ts)
    D.dedisperse = _vec_dedisperse if patched else _orig_dedisperse
    try:
        with np.errstate(all="ignore"):
            out = D._dedispersion_search(x, dms, nchan, f0, bw, ts)
    finally:
        D.dedisperse = _orig_dedisperse
    return x, dms, out


for case in DC.CASES:
    k = DC.key(case)
    if have(k + "_snr"):
        continue
    t0 = time.time()
    small = case.startswith("small:")
    x, dms, out = _deg_run(case, patched=not small)
    if small:
        # the vectorised dedisperse used for the large shapes gives the same bits here
        with np.errstate(all="ignore"):
            sh0 = D.dedispersion_shifts(x.shape[0], dms[-1], *DC.band(case)[1:])
            a, b = _orig_dedisperse(x, sh0), _vec_dedisperse(x, sh0)
        assert a.tobytes() == b.tobytes(), case
        _, _, out2 = _deg_run(case, patched=True)
        for u, v in zip(out, out2):
            assert np.asarray(u).tobytes() == np.asarray(v).tobytes(), case
    meta[k + "_input_sha256"] = sha(x)
    arrays[k + "_dms"] = np.asarray(dms)
    for col, v in zip(("max", "std", "snr", "rebin"), out):
        arrays[f"{k}_{col}"] = np.asarray(v)
    log("degenerate", case, x.shape, f"{time.time() - t0:.1f}s", "rebin", np.asarray(out[3])[:8],
        "snr", np.asarray(out[2])[:4])

np.savez_compressed(OUT_NPZ, **arrays)
json.dump(meta, open(OUT_JSON, "w"), indent=1, sort_keys=True)
log("wrote", OUT_NPZ, os.path.getsize(OUT_NPZ), "bytes;", len(arrays), "arrays,", len(meta), "meta")
