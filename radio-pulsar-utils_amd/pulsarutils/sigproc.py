"""SIGPROC filterbank I/O (replaces ``sigpyproc.Readers.FilReader`` for the hot path).

The reference reads files through sigpyproc (``stats.py:36-45``, ``clean.py:284-327``) and
uses these header keys: ``nsamples, tsamp, fbottom, ftop, bandwidth, nchans, foff,
tstart`` (``clean.py:286-294``) and ``readBlock(start, nsamps, as_filterbankBlock=False)``
-> ``(nchans, nsamps)`` (``clean.py:327``, ``stats.py:45``).  sigpyproc is not available in
this image; derived keys follow sigpyproc's Header conventions (parity unpinned by the
reference's tests, which never read a file):

    bandwidth = |foff| * nchans
    ftop      = fch1 - 0.5 * foff
    fbottom   = ftop + foff * nchans        (lower band edge when foff < 0)
    nsamples  = data bytes / (nchans * nifs * nbits / 8)

Samples are memory-mapped (never loaded whole).  The on-disk layout is time-major
(one spectrum per sample); :meth:`FilReader.readBlock` returns channel-major
``(nchans, nsamps)`` like sigpyproc, :meth:`FilReader.read_block_device` transposes on
the GPU (``pu_transpose``) so large blocks never go through a host transpose.
"""
import os
import struct

import numpy as np

_INT_KEYS = {"telescope_id", "machine_id", "data_type", "barycentric", "pulsarcentric", "nbits", "nsamples",
             "nchans", "nifs", "nbeams", "ibeam"}
_DBL_KEYS = {"az_start", "za_start", "src_raj", "src_dej", "tstart", "tsamp", "fch1", "foff", "refdm",
             "period"}
_STR_KEYS = {"source_name", "rawdatafile"}
_DTYPES = {8: np.uint8, 16: np.uint16, 32: np.float32}


def _rd_str(f):
    (n,) = struct.unpack("<i", f.read(4))
    if not 0 < n < 4096:
        raise ValueError("not a SIGPROC header (bad string length)")
    return f.read(n).decode("ascii", errors="replace")


def read_header(fname):
    """Parse a SIGPROC header; returns (dict, header_bytes)."""
    hdr = {}
    with open(fname, "rb") as f:
        if _rd_str(f) != "HEADER_START":
            raise ValueError(f"{fname}: missing HEADER_START")
        while True:
            key = _rd_str(f)
            if key == "HEADER_END":
                break
            if key in _INT_KEYS:
                (hdr[key],) = struct.unpack("<i", f.read(4))
            elif key in _DBL_KEYS:
                (hdr[key],) = struct.unpack("<d", f.read(8))
            elif key in _STR_KEYS:
                hdr[key] = _rd_str(f)
            else:
                raise ValueError(f"{fname}: unknown SIGPROC header key {key!r}")
        hdr_len = f.tell()
    nbits = hdr.get("nbits", 8)
    nchans = hdr["nchans"]
    nifs = hdr.get("nifs", 1)
    data_bytes = os.path.getsize(fname) - hdr_len
    hdr.setdefault("nifs", 1)
    hdr["nsamples"] = data_bytes // (nchans * nifs * nbits // 8)
    foff = hdr["foff"]
    hdr["bandwidth"] = abs(foff) * nchans
    hdr["ftop"] = hdr["fch1"] - 0.5 * foff
    hdr["fbottom"] = hdr["ftop"] + foff * nchans
    hdr["fcenter"] = hdr["ftop"] + 0.5 * foff * nchans
    hdr["hdrlen"] = hdr_len
    return hdr, hdr_len


def write_filterbank(fname, data_tc, fch1, foff, tsamp, tstart=60000.0, source_name="synthetic", nbits=None):
    """Write a time-major (nsamps, nchans) array as a SIGPROC filterbank file."""
    data_tc = np.ascontiguousarray(data_tc)
    nbits = nbits or {np.dtype(np.uint8): 8, np.dtype(np.uint16): 16, np.dtype(np.float32): 32}[data_tc.dtype]

    def s(x):
        b = x.encode()
        return struct.pack("<i", len(b)) + b

    out = [s("HEADER_START"), s("source_name"), s(source_name)]
    for k, v in (("machine_id", 0), ("telescope_id", 0), ("data_type", 1), ("nchans", data_tc.shape[1]),
                 ("nbits", nbits), ("nifs", 1)):
        out += [s(k), struct.pack("<i", v)]
    for k, v in (("fch1", fch1), ("foff", foff), ("tstart", tstart), ("tsamp", tsamp)):
        out += [s(k), struct.pack("<d", v)]
    out.append(s("HEADER_END"))
    with open(fname, "wb") as f:
        f.write(b"".join(out))
        f.write(data_tc.tobytes())


class FilReader:
    """Memory-mapped SIGPROC reader with sigpyproc's ``header`` / ``readBlock`` surface."""

    def __init__(self, fname):
        self.filename = fname
        self.header, self._hdr_len = read_header(fname)
        nbits = self.header.get("nbits", 8)
        if nbits not in _DTYPES:
            raise ValueError(f"{fname}: nbits={nbits} not supported (8, 16, 32)")
        self.dtype = np.dtype(_DTYPES[nbits])
        self._mm = np.memmap(fname, dtype=self.dtype, mode="r", offset=self._hdr_len,
                             shape=(self.header["nsamples"], self.header["nchans"] * self.header["nifs"]))

    def _block_tc(self, start, nsamps):
        start = int(start)
        nsamps = int(min(nsamps, self.header["nsamples"] - start))
        if start < 0 or nsamps < 0:
            raise ValueError("block outside the file")
        return self._mm[start:start + nsamps, :self.header["nchans"]]

    def readBlock(self, start, nsamps, as_filterbankBlock=False):  # noqa: N802 (sigpyproc name)
        """(nchans, nsamps) array in file channel order (host transpose)."""
        return np.ascontiguousarray(self._block_tc(start, nsamps).T)

    def read_block_device(self, start, nsamps, device=None):
        """(nchans, nsamps) device tensor: time-major bytes uploaded, transposed by pu_transpose."""
        from . import _hip
        t = _hip.require_gpu()
        tc = np.ascontiguousarray(self._block_tc(start, nsamps))
        src = t.from_numpy(tc).to(device or t.device("cuda", t.cuda.current_device()))
        return transpose_device(src)


def transpose_device(src):
    """(rows, cols) -> (cols, rows) contiguous, HIP tiled transpose (1/2/4/8-byte elements)."""
    from . import _hip
    t = _hip.require_gpu()
    rows, cols = src.shape
    out = t.empty((cols, rows), dtype=src.dtype, device=src.device)
    _hip.check(_hip.lib().pu_transpose(_hip.ptr(src), src.element_size(), rows, cols, src.stride(0), _hip.ptr(out),
                                       rows, _hip.stream_ptr()), "pu_transpose")
    return out
