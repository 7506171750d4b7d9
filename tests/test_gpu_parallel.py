"""The multi-GPU product path on one GPU: the HIP compute of ``parallel.sharded_search``
under a world-size-1 RCCL (nccl) process group, and the pipelined broadcast + search
(time-tile range launches, pu_plan_search_tiles + pu_plan_finalize) against the one-shot
search.  The multi-rank split / broadcast / gather plumbing is covered on CPU by
tests/test_parallel_gloo.py (gloo, world 2-4)."""
import socket

import numpy as np
import pytest

import oracle
from pulsarutils import _hip, parallel, synth
from pulsarutils import dedispersion as D
from pulsarutils.configs import CONFIGS

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name,chunks", [("C5", 5), ("C2s", 8), ("C3s", 3)])
def test_pipelined_tiles_equal_full_search(gpu, name, chunks):
    """Searching time-tile ranges as chunks land, then finalising, gives the one-shot
    pu_plan_search outputs bit for bit (same kernels, same per-tile records, same
    deterministic finalize order); wrapping tiles wait for the last chunk."""
    import torch
    from dataclasses import replace
    c = {"C5": CONFIGS["C5"], "C2s": replace(CONFIGS["C2"], nchan=256, nsamples=1 << 18),
         "C3s": replace(CONFIGS["C3"], nchan=512, nsamples=1 << 18)}[name]
    xd = synth.pulsar_filterbank_device(c)
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)[:300]
    sh = _hip.shift_table(c.nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    plan = _hip.Plan(_hip.dtype_code(xd.dtype), _hip.PU_ACC_NATIVE, c.nchan, c.nsamples, sh)
    full = [o.cpu().numpy() for o in plan.search(xd)]
    piped = [o.cpu().numpy() for o in parallel.pipelined_broadcast_search(xd, plan, chunks=chunks)]
    torch.cuda.synchronize()
    for a, b in zip(full, piped):
        np.testing.assert_array_equal(a, b)
    # tile-range launches with an empty and a partial range, finalised
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=xd.device)
    ntt = plan.info["time_tiles"]
    plan.search_tiles(xd, 0, 0, ws)
    plan.search_tiles(xd, ntt // 3, ntt, ws)
    plan.search_tiles(xd, 0, ntt // 3, ws)
    for a, b in zip(full, plan.finalize(ws, xd)):
        np.testing.assert_array_equal(a, b.cpu().numpy())
    with pytest.raises(ValueError):
        plan.search_tiles(xd, 0, ntt + 1, ws)


@pytest.mark.parametrize("pipelined", [False, True])
def test_sharded_search_nccl_world1(gpu, pipelined):
    """parallel.sharded_search with the HIP compute (the product path) under a real
    RCCL process group of size 1: equals the single-process search, and the sampled
    trials equal the oracle within SURVEY §8a's 1e-5."""
    import torch
    import torch.distributed as dist
    from dataclasses import replace
    c = replace(CONFIGS["C2"], nchan=256, nsamples=1 << 17)
    xd = synth.pulsar_filterbank_device(c)
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)[:257]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=xd.device)
    try:
        mx, sd, snr, win = parallel.sharded_search(xd, dms, c.nchan, c.start_freq, c.bandwidth, c.tsamp,
                                                   pipelined=pipelined)
    finally:
        dist.destroy_process_group()
    ref = D._dedispersion_search(xd, dms, c.nchan, c.start_freq, c.bandwidth, c.tsamp)
    for a, b in zip((mx, sd, snr, win), ref):
        np.testing.assert_array_equal(a, b)
    assert win.dtype == np.int32
    idx = np.unique(np.r_[np.linspace(0, dms.size - 1, 8).astype(int), np.argmax(snr)])
    o = oracle.search(xd.cpu().numpy(), dms[idx], c.start_freq, c.bandwidth, c.tsamp, nthreads=16)
    np.testing.assert_allclose(snr[idx], o[2], rtol=1e-5)
    np.testing.assert_array_equal(win[idx], o[3])
    torch.cuda.synchronize()


@pytest.mark.parametrize("offset", [0, 5000])
@pytest.mark.parametrize("dt", ["f32", "u8dma", "u8", "f64"])
def test_ready_tiles_read_only_landed_columns(gpu, dt, offset):
    """the halo that gates early tile launches (Plan.tile_window) is checked
    against the kernels' real reads.  Every chunk's not-yet-landed columns are
    overwritten with garbage (NaN / 255) before the tiles ``ready_tiles`` marks are
    searched; the finalised result must equal the one-shot search bit for bit, so no
    ready tile may read past the landed prefix.  Plans: float32 (LDS-DMA rows), 8-bit
    with LDS-DMA rows (N % 4 == 0) and with global-memory rows (N % 4 != 0), float64
    (channel mode); shift tables with a negative (offset 0: the reference's delays
    around the band centre) and a positive smallest shift (offset 5000)."""
    import torch
    c = CONFIGS["C2"]
    nchan = 96
    n = 40962 if dt == "u8" else 40960
    rng = np.random.default_rng(17)
    xh = rng.random((nchan, n)) * 40
    x = torch.from_numpy({"f32": xh.astype(np.float32), "u8dma": xh.astype(np.uint8), "u8": xh.astype(np.uint8),
                          "f64": xh}[dt]).cuda()
    dms = np.linspace(0.0, 80.0, 150)
    sh = _hip.shift_table(nchan, dms, c.start_freq, c.bandwidth, c.tsamp) + offset
    assert (sh.min() < 0) == (offset == 0)
    plan = _hip.Plan(_hip.dtype_code(x.dtype), _hip.PU_ACC_NATIVE, nchan, n, sh)
    full = [o.cpu().numpy() for o in plan.search(x)]
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=x.device)
    done = np.zeros(plan.info["time_tiles"], dtype=bool)
    launched = 0
    for c0, c1 in parallel.column_chunks(n, 6):
        xg = x.clone()
        if c1 < n:
            xg[:, c1:] = 255 if x.dtype == torch.uint8 else float("nan")
        ready = parallel.ready_tiles(plan, c1) & ~done
        idx = np.flatnonzero(ready)
        for run in np.split(idx, np.flatnonzero(np.diff(idx) != 1) + 1) if idx.size else []:
            plan.search_tiles(xg, int(run[0]), int(run[-1]) + 1, ws)
            launched += 1
        done |= ready
        torch.cuda.synchronize()
        del xg
    assert done.all() and launched > 1
    got = [o.cpu().numpy() for o in plan.finalize(ws, x)]
    for a, b in zip(full, got):
        np.testing.assert_array_equal(a, b)


def test_cached_plan_two_threads(gpu):
    """one cached plan searched from two threads at once (ctypes releases the
    GIL), each thread on its own stream; one input is constant, so every one of its trials
    is certified by the exact recheck (resolve_flagged: the pinned CertState read-back and
    the recheck scratch), the other is noise.  Every result equals the single-threaded
    one: the library's per-plan lock keeps the calls' certification state apart."""
    import threading

    import torch
    c = CONFIGS["C5"]
    rng = np.random.default_rng(9)
    n = 1 << 15
    noise = torch.from_numpy((rng.random((c.nchan, n)) * 50).astype(np.uint8)).cuda()
    const = torch.full((c.nchan, n), 7, dtype=torch.uint8, device=noise.device)
    dms = np.linspace(c.dmmin, c.dmmax, 120)
    args = (c.nchan, c.start_freq, c.bandwidth, c.tsamp)
    want = {}
    for name, x in (("noise", noise), ("const", const)):
        (o, plan) = D.search_device(x, dms, *args)
        want[name] = [t.cpu().numpy() for t in o]
        if name == "const":
            assert plan.cert_info()["rechecked"] == dms.size
    _, p1 = D.search_device(noise, dms, *args)
    _, p2 = D.search_device(const, dms, *args)
    assert p1 is p2  # one cached plan serves both inputs
    errors = []

    def worker(name, x):
        try:
            s = torch.cuda.Stream(device=x.device)
            with torch.cuda.stream(s):
                for _ in range(6):
                    o, _ = D.search_device(x, dms, *args)
                    got = [t.cpu().numpy() for t in o]
                    for a, b in zip(want[name], got):
                        np.testing.assert_array_equal(a, b)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(f"{name}: {e!r}")

    th = [threading.Thread(target=worker, args=a) for a in (("noise", noise), ("const", const))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th), "thread hung"
    assert not errors, errors


@pytest.mark.parametrize("name,acc", [("C5", "native"), ("C3s", "native"), ("C5", "f64")])
def test_finalize_range_pieces_equal_full_search(gpu, name, acc):
    """Round 6 (time-tile sharding): the records of a tile-range search, finalized
    in trial ranges (pu_plan_finalize_range), equal the one-shot search bit for bit; the
    deferred form (pu_plan_finalize_range_flagged) writes the same fast statistics and
    returns the trials the one-shot search's certification recomputed, whose exact series
    (pu_plan_exact_series) + pu_series_stats give the one-shot outputs; the records view
    has the documented layout."""
    import torch
    from dataclasses import replace
    c = {"C5": CONFIGS["C5"], "C3s": replace(CONFIGS["C3"], nchan=512, nsamples=1 << 18)}[name]
    xd = synth.pulsar_filterbank_device(c)
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)[:300]
    sh = _hip.shift_table(c.nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    code = {"native": _hip.PU_ACC_NATIVE, "f64": _hip.PU_ACC_F64}[acc]
    plan = _hip.Plan(_hip.dtype_code(xd.dtype), code, c.nchan, c.nsamples, sh)
    full = [o.cpu().numpy() for o in plan.search(xd)]
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=xd.device)
    ntt = plan.info["time_tiles"]
    plan.search_tiles(xd, 0, ntt // 3, ws)
    plan.search_tiles(xd, ntt // 3, ntt, ws)
    rec = plan.records(ws)
    assert rec.shape == (dms.size, ntt, plan.info["rec_stride"])
    assert rec.element_size() == plan.info["rec_elem_bytes"]
    outs = None
    for lo, hi in [(0, 7), (7, 7), (7, 151), (151, dms.size)]:
        outs = plan.finalize_range(ws, xd, lo, hi, out=outs)
    for k in range(4):
        np.testing.assert_array_equal(outs[k].cpu().numpy(), full[k], err_msg=f"output {k}")
    # deferred certification: same fast statistics, flagged trials settled by the caller
    plan.search_tiles(xd, 0, ntt, ws)
    outs2, flagged, nnf = plan.finalize_range_flagged(ws, 0, dms.size)
    assert nnf == 0 and np.all(np.diff(flagged) > 0)
    if flagged.size:
        ser = plan.exact_series(xd, flagged)
        # a sample range is the same samples of the whole series (time-split ranks)
        n3 = c.nsamples // 3 + 5
        assert torch.equal(plan.exact_series(xd, flagged, t_begin=n3, t_end=2 * n3), ser[:, n3:2 * n3])
        st = _hip.series_stats(ser)
        for k in range(4):
            outs2[k][torch.as_tensor(flagged.astype(np.int64), device=xd.device)] = st[k]
    for k in range(4):
        np.testing.assert_array_equal(outs2[k].cpu().numpy(), full[k], err_msg=f"deferred output {k}")


def test_finalize_range_flagged_zero_input_and_nonfinite_scan(gpu):
    """All-zero input: every trial's std is zero, so every trial of the range is flagged and
    its exact series is all zeros; pu_nonfinite_any sees a NaN in a column range only when
    the range holds it."""
    import torch
    from dataclasses import replace
    c = replace(CONFIGS["C3"], nchan=256, nsamples=1 << 16)
    xd = torch.zeros((c.nchan, c.nsamples), dtype=torch.uint8, device="cuda")
    dms = D.dedispersion_plan(c.nchan, c.dmmin, c.dmmax, c.start_freq, c.bandwidth, c.tsamp)[:40]
    sh = _hip.shift_table(c.nchan, dms, c.start_freq, c.bandwidth, c.tsamp)
    plan = _hip.Plan(_hip.dtype_code(xd.dtype), _hip.PU_ACC_NATIVE, c.nchan, c.nsamples, sh)
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=xd.device)
    plan.search_tiles(xd, 0, plan.info["time_tiles"], ws)
    _, flagged, nnf = plan.finalize_range_flagged(ws, 10, 30)
    assert list(flagged) == list(range(10, 30)) and nnf == 0
    assert torch.count_nonzero(plan.exact_series(xd, flagged[:3])) == 0
    assert plan.exact_series(xd, flagged[:3], t_begin=100, t_end=100).shape == (3, 0)
    xf = torch.ones((16, 1000), dtype=torch.float32, device="cuda")
    xf[5, 700] = float("nan")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert int(_hip.nonfinite_any(xf[:, 600:800], flag)[0]) == 1
    assert int(_hip.nonfinite_any(xf[:, :700], flag)[0]) == 0
    assert int(_hip.nonfinite_any(xd[:, :100], flag)[0]) == 0


@pytest.mark.parametrize("dt", ["u8", "f32", "f64"])
def test_exact_series_ranges_equal_oracle_rows(gpu, dt):
    """pu_plan_exact_series (the certification recompute; loads of 8/4/2 channels issued ahead
    of their adds, round 6) equals the oracle's float64 channel-order rows bit for bit, over
    the whole series and over sample ranges that start and end anywhere (ragged n, windows
    wrapping modulo n)."""
    import torch
    n, nchan = 70001, 37
    rng = np.random.default_rng(7)
    x = {"u8": rng.integers(0, 256, (nchan, n)).astype(np.uint8), "f32": rng.random((nchan, n)).astype(np.float32),
         "f64": rng.random((nchan, n))}[dt]
    xd = torch.from_numpy(x).cuda()
    dms = np.linspace(0.0, 400.0, 9)
    sh = _hip.shift_table(nchan, dms, 1200.0, 300.0, 64e-6)
    plan = _hip.Plan(_hip.dtype_code(xd.dtype), _hip.PU_ACC_F64, nchan, n, sh)
    want = np.stack([oracle.dedisperse(x, sh[d]) for d in range(dms.size)])
    tr = np.arange(dms.size, dtype=np.int32)
    np.testing.assert_array_equal(plan.exact_series(xd, tr).cpu().numpy(), want)
    for a, b in [(0, 1), (5, 4100), (n - 700, n), (12345, 12346 + 8 * 513)]:
        np.testing.assert_array_equal(plan.exact_series(xd, tr, t_begin=a, t_end=b).cpu().numpy(), want[:, a:b])
