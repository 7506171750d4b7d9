"""Degenerate search trials (GPU) against golden tables from executing the reference.

The reference's rules (pulsarutils/dedispersion.py:186-201): ``best_snr = 0,
best_win = 0`` replaced only by a strictly greater S/N; ``np.max`` / ``np.std``
propagate NaN; a zero std gives +-inf or NaN S/N.  The HIP search certifies each
trial's fast statistics and recomputes the ones it cannot certify
exactly (float64 channel-order series + numpy-order statistics), so:

* zero / constant / NaN / inf inputs (every trial degenerate): all four columns
  bit-equal to the reference's, whatever the accumulation;
* S/N ties (block-constant integer data at DM 0): with an exact series (uint8 input,
  or float64 accumulation) the tie is recomputed and the rebin column equals the
  reference's; with float32 accumulation of float input the decision is within the
  stated float32 tolerance and only the non-tie trials' rebin is compared;
* every other trial: max/std/snr within 1e-9 (float64 accumulation) or 1e-5 (float32)
  relative, rebin equal.
Goldens: tests/golden/make_golden.py ("degenerate" section); inputs rebuilt by
tests/degenerate_cases.py and pinned by SHA-256.
"""
import hashlib

import numpy as np
import pytest

import degenerate_cases as DC
import oracle
from pulsarutils import _hip
from pulsarutils import dedispersion as D

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _case(golden, case):
    arrays, meta = golden
    k = DC.key(case)
    x = DC.make(case)
    assert sha(x) == meta[k + "_input_sha256"], case
    return x, arrays[k + "_dms"], [arrays[f"{k}_{c}"] for c in ("max", "std", "snr", "rebin")]


def _degenerate(ref):
    """Trials whose reference result is a degenerate one (NaN max, zero or infinite S/N)."""
    mx, sd, snr, _ = ref
    return ~np.isfinite(mx) | ~np.isfinite(snr) | (snr == 0) | (sd == 0)


def _exact_series(x, acc):
    return acc == "f64" or x.dtype == np.float64 or x.dtype == np.uint8


def _check(case, x, got, ref, plan, acc):
    exact = _degenerate(ref)
    exact_series = _exact_series(x, acc)
    rtol = 1e-9 if (acc == "f64" or x.dtype == np.float64) else 1e-5
    tie = case.split(":")[1] == "block8"
    for col, (g, r) in enumerate(zip(got, ref)):
        # degenerate trials: bit for bit (NaN == NaN)
        np.testing.assert_array_equal(g[exact], r[exact], err_msg=f"{case} col {col} degenerate")
        ok = ~exact
        if tie and not exact_series:
            ok &= np.arange(g.size) != 0  # DM 0: the constructed tie, inside the float32 tolerance
        if col < 3:
            np.testing.assert_allclose(g[ok], r[ok], rtol=rtol, atol=1e-300, err_msg=f"{case} col {col}")
        else:
            np.testing.assert_array_equal(g[ok], r[ok], err_msg=f"{case} rebin")
    info = plan.cert_info()
    if case.split(":")[1] in ("nanchan", "nansamp", "posinf", "infs"):
        assert info["nan_rule"], info
    elif exact.all():
        assert info["rechecked"] == exact.size, info
    if tie and exact_series:
        assert info["rechecked"] >= 1, info   # the DM-0 tie was recomputed
        np.testing.assert_array_equal(got[3][0], ref[3][0])


@pytest.mark.parametrize("acc", [None, "f64"])
@pytest.mark.parametrize("case", [c for c in DC.CASES if not c.startswith("c2:")])
def test_degenerate_trials_vs_reference(gpu, golden, case, acc):
    x, dms, ref = _case(golden, case)
    nchan, f0, bw, ts = DC.band(case)
    (mx, sd, snr, win), plan = D.search_device(x, dms, nchan, f0, bw, ts, acc=acc)
    got = [v.cpu().numpy() for v in (mx, sd, snr, win)]
    _check(case, x, got, ref, plan, acc)


@pytest.mark.parametrize("case", [c for c in DC.CASES if c.startswith("c2:")])
def test_degenerate_trials_c2_shape(gpu, golden, case):
    """C2-shaped (1024 x 2^20 float32, the headline config's shape) degenerate inputs
    through the default (float32-accumulation subband) search."""
    import torch
    x, dms, ref = _case(golden, case)
    nchan, f0, bw, ts = DC.band(case)
    xd = torch.from_numpy(x).cuda()
    del x
    (mx, sd, snr, win), plan = D.search_device(xd, dms, nchan, f0, bw, ts)
    got = [v.cpu().numpy() for v in (mx, sd, snr, win)]
    assert plan.info["group"] > 1, plan.info   # the subband (fast) kernel ran
    _check(case, np.empty(0, np.float32), got, ref, plan, None)


def _series_cases():
    rng = np.random.default_rng(8)
    rows = []
    for n in (8, 9, 100, 128, 129, 8192, 8193, 20000, (1 << 16) + 5):
        rows.append(rng.standard_normal(n) * 3 + 7)
        rows.append(np.repeat(rng.integers(0, 9, -(-n // 8)), 8)[:n].astype(np.float64))  # ties
        rows.append(np.full(n, 0.1))
        rows.append(np.zeros(n))
        r = rng.standard_normal(n)
        r[n // 2] = np.nan
        rows.append(r)
        r = rng.standard_normal(n)
        r[0] = np.inf
        rows.append(r)
        rows.append(-np.abs(rng.standard_normal(n)) - 1.0)
    return rows


def test_series_stats_bitexact_vs_oracle(gpu):
    """pu_series_stats (numpy-order mean / quick_resample / max / std, strict first-best
    S/N) equals the oracle's restatement - pinned against the reference's own tables in
    tests/test_oracle.py - bit for bit, on random, tied, constant, zero, NaN, inf and
    all-negative series of ragged lengths (pairwise tails, 8192-element blocks)."""
    import torch
    rows = _series_cases()
    by_n = {}
    for r in rows:
        by_n.setdefault(r.size, []).append(r)
    for n, rs in by_n.items():
        a = np.stack(rs)
        got = [v.cpu().numpy() for v in _hip.series_stats(torch.from_numpy(a).cuda())]
        for i, r in enumerate(rs):
            want = oracle.trial_stats(r)
            np.testing.assert_array_equal(np.array([g[i] for g in got[:3]]), np.array(want[:3]), err_msg=f"n={n} row {i}")
            assert got[3][i] == want[3], (n, i, got[3][i], want[3])


def test_nearconst_f32_c2_shape_vs_oracle(gpu):
    """A near-constant float32 filterbank at C2's shape (1024 x 2^20: 1000 + 1e-3 N(0, 1)),
    through the default float32-accumulation subband search (pinned
    only at 32 x 4096 before).  The float32 series sums (~1e6, ulp 0.06) round by more than
    the series' std (~0.03), so the certification must refuse every trial's
    fast statistics and recompute them exactly: all four columns then equal the C oracle's
    float64 channel-order restatement of the reference (dedispersion.py:86-98, 186-201) bit
    for bit.  Parity against the oracle, not a reference-run golden (the oracle is pinned to
    the reference's own tables elsewhere, tests/test_oracle.py)."""
    import torch
    nchan, n = DC.SHAPES["c2"][:2]
    _, f0, bw, ts = DC.band("c2:zero:f32")
    dms = DC.trial_dms("c2")
    rng = np.random.default_rng(20261018)
    x = rng.standard_normal((nchan, n), dtype=np.float32)
    x *= np.float32(1e-3)
    x += np.float32(1000.0)
    xd = torch.from_numpy(x).cuda()
    (mx, sd, snr, win), plan = D.search_device(xd, dms, nchan, f0, bw, ts)
    got = [v.cpu().numpy() for v in (mx, sd, snr, win)]
    del xd
    assert plan.info["group"] > 1, plan.info   # the subband (fast) kernel ran
    info = plan.cert_info()
    assert info["rechecked"] == dms.size, info
    ref = oracle.search(x, dms, f0, bw, ts, nthreads=16)
    for col, (g, r) in enumerate(zip(got, ref)):
        np.testing.assert_array_equal(g, r, err_msg=f"nearconst c2 col {col}")
