"""measure_channel_variability from one read pass (round 4): the certification of
pulsarutils.clean._certified_variability, on CPU.

The device pass (pu_row_moments) returns numpy's row means and, per row, (c, sum(x - c),
sum((x - c)^2)) in float64 with c = x[r, 0].  Here the same moments are formed with
numpy in float64 (any order: the bound allows it), and whenever the certification answers
it must give the reference's mask (oracle/clean_oracle.channel_variability) bit for bit;
when a channel's std sits within rounding of a limit it must answer None (the caller then
runs the exact second pass).  Float32, float64 and uint8 inputs, masked channels, spiky
and constant channels."""
import numpy as np
import pytest

from oracle import clean_oracle as co
from pulsarutils.clean import _certified_variability


def _moments(x):
    xd = x.astype(np.float64)
    c = xd[:, :1]
    d = xd - c
    return np.stack([c[:, 0], d.sum(1), (d * d).sum(1)], axis=1)


def _means(x):
    return x.mean(1) if x.dtype == np.float32 else x.astype(np.float64).mean(1) if x.dtype == np.uint8 else x.mean(1)


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.uint8])
def test_certified_variability_matches_reference(dtype):
    rng = np.random.default_rng(41)
    answered = 0
    for trial in range(12):
        nchan, n = 64, 20000 + 4099 * trial
        scale = rng.uniform(0.5, 3.0, nchan)
        x = rng.normal(100.0, 1.0, (nchan, n)) * scale[:, None]
        x[rng.integers(0, nchan, 3)] *= 4.0  # loud channels
        if dtype == np.uint8:
            x = np.clip(x, 0, 255)
        x = x.astype(dtype)
        x[5] = x[5, 0]  # a constant channel
        bad = rng.random(nchan) < 0.1
        got = _certified_variability(_means(x), _moments(x), n, dtype == np.float32, bad)
        want = co.channel_variability(x, badchans_mask=bad)
        if got is not None:
            answered += 1
            np.testing.assert_array_equal(got, want)
    assert answered >= 10  # the one-pass answer is the common case


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("which", ["hi", "low"])
def test_certified_variability_declines_at_a_limit(dtype, which):
    """A channel whose moments put its std on a limit (between the limit's bounds)
    cannot be certified: None.  Channel 0's second moment is set so that
    sqrt(V / n) = the reference's limit computed from the other channels' stds."""
    rng = np.random.default_rng(43)
    nchan, n = 33, 30000
    x = rng.normal(10.0, 1.0, (nchan, n)).astype(dtype)
    mom = _moments(x)
    m = _means(x).astype(np.float64)
    spec = np.std(x, axis=1)
    # channel j (the lowest std for "hi", the highest for "low") moves onto the limit:
    # it then sorts last (first), so the quartiles are the others' order statistics at
    # the same (one lower) positions
    j = int(np.argsort(spec)[0 if which == "hi" else -1])
    rest = np.sort(np.delete(spec, j))
    sh = 0 if which == "hi" else -1
    q1, q2, q3 = rest[nchan // 4 + sh], rest[nchan // 2 + sh], rest[nchan // 4 * 3 + sh]
    lim = float(q2 + 2 * (q3 - q2)) if which == "hi" else float(q2 - 2 * (q2 - q1))
    # V_j = n lim^2  ->  s2 = V_j + 2 (m - c) s1 - n (m - c)^2
    dm = m[j] - mom[j, 0]
    mom[j, 2] = n * lim * lim + 2.0 * dm * mom[j, 1] - n * dm * dm
    assert _certified_variability(m, mom, n, dtype == np.float32, np.zeros(nchan, bool)) is None


def test_certified_variability_nonfinite_and_too_few_good():
    x = np.ones((16, 100), np.float32)
    x[3, 7] = np.nan
    assert _certified_variability(np.nanmean(x, 1), _moments(x), 100, True, np.zeros(16, bool)) is None
    y = np.random.default_rng(1).normal(size=(16, 100)).astype(np.float32)
    bad = np.ones(16, bool)
    bad[:4] = False  # 4 good channels: the reference's quartile index 12 raises
    assert _certified_variability(y.mean(1), _moments(y), 100, True, bad) is None


@pytest.mark.parametrize("k", [0, 1, 3, 40])
def test_moment_error_bound_covers_serial_tail(k):
    """pu_row_moments sums a row's trailing partial block (up to 8191 elements)
    serially and then the per-block sums one after another, so the float64 summation depth
    reaches min(n, 8191) + ceil(n / 8192) + the block tree.  At n = 8192 k + 8191 the
    bound's factor must cover that depth, and the rounding error of V formed the device's
    way (blocks as pairwise trees, the tail and the block combine as serial chains) must lie
    inside the bound eV _certified_variability uses."""
    from fractions import Fraction
    from pulsarutils.clean import moment_error_factor
    n = 8192 * k + 8191
    depth = min(n, 8191) + -(-n // 8192)
    assert moment_error_factor(n) >= depth * 2.0 ** -53
    rng = np.random.default_rng(70 + k)
    x = (1000.0 + rng.normal(0.0, 3.0, n)).astype(np.float32).astype(np.float64)
    c = x[0]
    d = x - c
    # the device's order: full blocks by a tree (numpy's pairwise sum here), the tail and the
    # combine as serial float64 chains
    nfull = n // 8192
    blocks1 = [float(np.sum(d[b * 8192:(b + 1) * 8192])) for b in range(nfull)]
    blocks2 = [float(np.sum(d[b * 8192:(b + 1) * 8192] ** 2)) for b in range(nfull)]
    t1 = t2 = 0.0
    for v in d[nfull * 8192:]:
        t1 += float(v)
        t2 += float(v) * float(v)
    s1 = s2 = 0.0
    for a, b in zip(blocks1 + [t1], blocks2 + [t2]):
        s1 += a
        s2 += b
    m = float(np.mean(x))
    dm = m - c
    V = s2 - 2.0 * dm * s1 + n * dm * dm
    exact_d = [Fraction(float(v)) for v in d]
    S1, S2 = sum(exact_d), sum(v * v for v in exact_d)
    Vx = S2 - 2 * Fraction(dm) * S1 + n * Fraction(dm) ** 2
    eV = (s2 + 2.0 * abs(dm) * np.sqrt(n * s2) + n * dm * dm) * moment_error_factor(n)
    assert abs(Fraction(V) - Vx) <= Fraction(eV)


@pytest.mark.parametrize("length", [7, 9, 0])
def test_channel_mask_length_raises_like_numpy(length):
    """A channel mask whose length is not nchan raises numpy's IndexError before anything
    reaches the device (the kernels read exactly nchan mask bytes), as the reference's
    ``spec[~badchans_mask]`` does (clean.py:120)."""
    from pulsarutils import clean
    x = np.ones((8, 64), np.float32)
    if length:  # (numpy lets an empty boolean index through; the reference then fails at
        #          ordered[spec.size // 4] - here the length check raises first)
        with pytest.raises(IndexError):
            np.std(x, axis=1)[~np.zeros(length, bool)]
    with pytest.raises(IndexError, match="boolean index did not match"):
        clean.measure_channel_variability(x, badchans_mask=np.zeros(length, bool))
