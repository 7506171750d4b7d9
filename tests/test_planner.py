"""Host planner (product code) vs the reference's own plan / shift tables."""
import numpy as np
import pytest

from pulsarutils import _planner
from pulsarutils.configs import CONFIGS


def test_doctests(golden):
    arrays, _ = golden
    np.testing.assert_array_equal(_planner.normalize_shifts(np.array([-1, 0, 2, 4]), 3), [2, 0, 2, 1])
    np.testing.assert_array_equal(_planner.normalize_shifts(np.array([-1, 0, 2, 4]), 3),
                                  arrays["doctest_normalize"])
    assert _planner.normalize_shifts(np.array([-1.0]), 3).dtype == np.int32
    tdm = _planner.dedispersion_plan(10, 0, 10, 1400, 128, 0.0005)
    np.testing.assert_array_equal(tdm, arrays["doctest_plan"])
    assert np.isclose(tdm[0], 0) and np.isclose(tdm[-1], 10., atol=1)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_plan_bitexact(golden, name):
    arrays, _ = golden
    c = CONFIGS[name]
    p = _planner.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)
    np.testing.assert_array_equal(p, arrays[f"plan_{name}"])
    assert p.size == c.ntrials


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_python_shifts_bitexact(golden, name):
    arrays, _ = golden
    c = CONFIGS[name]
    dms = arrays[f"plan_{name}"]
    idx = arrays[f"shiftidx_{name}"]
    if name == "C1":
        idx = idx[::7]
    for i in idx:
        got = _planner.dedispersion_shifts(c.nchan, dms[i], c.start_freq, c.bandwidth, c.tsamp)
        k = list(arrays[f"shiftidx_{name}"]).index(i)
        np.testing.assert_array_equal(got, arrays[f"shifts_{name}"][k])


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_cpp_shift_table_bitexact(golden, name):
    """pu_shift_table (C++ in the HIP library; host function, no GPU needed)."""
    from pulsarutils import _hip
    arrays, _ = golden
    c = CONFIGS[name]
    dms = arrays[f"plan_{name}"]
    idx = arrays[f"shiftidx_{name}"]
    got = _hip.shift_table(c.nchan, dms[idx], c.start_freq, c.bandwidth, c.tsamp)
    np.testing.assert_array_equal(got, arrays[f"shifts_{name}"].astype(np.int64))


def test_delta_delay():
    assert _planner.delta_delay(1.0, 1200., 1400.) == 4149. * 1200. ** -2 - 4149. * 1400. ** -2
