"""SIGPROC reader/writer (host side, no GPU): header keys the reference uses
(clean.py:286-294), sigpyproc's derived keys, readBlock shape/order."""
import numpy as np
import pytest

from pulsarutils import sigproc


@pytest.mark.parametrize("dt", [np.uint8, np.float32, np.uint16])
def test_roundtrip(tmp_path, dt):
    rng = np.random.default_rng(1)
    x = (rng.random((1000, 16)) * 200).astype(dt)
    f = str(tmp_path / "a.fil")
    sigproc.write_filterbank(f, x, fch1=1500.0, foff=-3.125, tsamp=1e-4, tstart=59000.5)
    r = sigproc.FilReader(f)
    h = r.header
    assert h["nchans"] == 16 and h["nsamples"] == 1000 and h["tsamp"] == 1e-4
    assert h["tstart"] == 59000.5 and h["foff"] == -3.125
    assert h["bandwidth"] == 50.0
    assert h["ftop"] == 1500.0 + 0.5 * 3.125
    assert h["fbottom"] == h["ftop"] - 50.0
    blk = r.readBlock(100, 300, as_filterbankBlock=False)
    assert blk.shape == (16, 300) and blk.dtype == dt
    np.testing.assert_array_equal(blk, x[100:400].T)
    # short read at the end of the file, like sigpyproc
    assert r.readBlock(900, 500).shape == (16, 100)


def test_bad_header(tmp_path):
    f = tmp_path / "b.fil"
    f.write_bytes(b"\x05\x00\x00\x00hello")
    with pytest.raises(ValueError):
        sigproc.FilReader(str(f))
