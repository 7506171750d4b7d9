"""File-driven path on the GPU: SIGPROC block transpose, get_spectral_stats /
get_bad_chans (stats.py:35-90) bit-exact vs the reference's own outputs, and the
search_by_chunks driver (clean.py:276-351) vs the oracle composition."""
import os

import numpy as np
import pytest

import oracle
from oracle import clean_oracle as co
from pulsarutils import sigproc, stats
from pulsarutils.dedispersion import dedispersion_plan
from synth_files import write_stats_file

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [np.uint8, np.float32, np.float64, np.uint16])
def test_transpose(gpu, dt):
    import torch
    rng = np.random.default_rng(3)
    x = (rng.random((777, 130)) * 250).astype(dt)
    out = sigproc.transpose_device(torch.from_numpy(x).to(gpu))
    np.testing.assert_array_equal(out.cpu().numpy(), x.T)


@pytest.mark.parametrize("dt", ["u8", "f32"])
def test_spectral_stats_and_bad_chans(gpu, golden, tmp_path, dt):
    arrays, meta = golden
    fname, _ = write_stats_file(str(tmp_path), dt)
    mean_spec, std_spec = stats.get_spectral_stats(fname)
    np.testing.assert_array_equal(mean_spec, arrays[f"fil_{dt}_mean"])
    np.testing.assert_array_equal(std_spec, arrays[f"fil_{dt}_std"])
    bad = stats.get_bad_chans(fname)
    np.testing.assert_array_equal(bad, arrays[f"fil_{dt}_badchans"])
    assert open(fname + ".badchans").read() == meta[f"fil_{dt}_badchans_txt"]
    # second call: served from the cache file, same mask
    np.testing.assert_array_equal(stats.get_bad_chans(fname), bad)


@pytest.mark.parametrize("search_dtype", ["f64", "f32"])
def test_search_by_chunks_finds_pulse(gpu, tmp_path, monkeypatch, search_dtype):
    """A dispersed pulse in a foff<0 u8 file: found in the chunks covering it, and each
    chunk table equals the oracle composition of the reference steps (float64 search:
    1e-9; float32 search of the float32-cast plane: 1e-5)."""
    from pulsarutils import clean, _planner
    nch, ns, tsamp = 64, 20000, 2e-4
    fch1, foff = 1500.0, -300.0 / nch
    rng = np.random.default_rng(21)
    x = np.clip(np.rint(rng.standard_normal((ns, nch)) * 6 + 60), 0, 255)
    # pulse at DM 300 at t = 9000 (channel order in file is descending frequency)
    fbottom = fch1 - 0.5 * foff + foff * nch
    sh = _planner.dedispersion_shifts(nch, 300.0, fbottom, 300.0, tsamp).astype(int)
    for c in range(nch):
        x[(9000 + sh[c]) % ns, nch - 1 - c] += 40
    x = np.clip(x, 0, 255).astype(np.uint8)
    fname = str(tmp_path / "pulse.fil")
    sigproc.write_filterbank(fname, x, fch1=fch1, foff=foff, tsamp=tsamp)
    monkeypatch.chdir(tmp_path)
    prof = []
    cands = clean.search_by_chunks(fname, dmmin=250, dmmax=350, new_sample_time=tsamp, save_candidates=True,
                                   search_dtype=search_dtype, profile=prof)
    assert cands, "pulse not found"
    assert prof and all(k in prof[0] for k in ("h2d", "transpose", "clean", "rebin", "cast", "search"))
    best = max(cands, key=lambda c: c["snr"])
    assert abs(best["dm"] - 300) < 3 and best["istart"] <= 9000 < best["iend"]
    assert os.path.exists(f"pulse_{best['istart']}-{best['iend']}.pkl")
    # oracle composition for that chunk: get_bad_chans -> renormalize -> flip -> search
    mask = np.loadtxt(fname + ".badchans").astype(bool)
    blk = sigproc.FilReader(fname).readBlock(best["istart"], best["iend"] - best["istart"])
    ren = np.ascontiguousarray(co.renormalize(blk, badchans_mask=mask)[::-1])
    if search_dtype == "f32":
        ren = ren.astype(np.float32)
    dms = dedispersion_plan(nch, 250, 350, fbottom, 300.0, tsamp)
    omx, osd, osnr, owin = oracle.search(ren, dms, fbottom, 300.0, tsamp)
    tab = best["table"]
    np.testing.assert_allclose(tab["snr"], osnr, rtol=1e-9 if search_dtype == "f64" else 1e-5)
    np.testing.assert_array_equal(tab["rebin"], owin)
