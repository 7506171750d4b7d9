"""Cost of the receivers' staging -> strided copy in the pipelined multi-GPU step
(parallel.pipelined_broadcast_search, the ``unpack`` phase), measured on one GPU at C3's shape:
8 column chunks of a 4096 x 2^22 uint8 filterbank, each copied from a contiguous staging buffer
into data[:, c0:c1] (the copy a receiving rank does after each chunk's exchange), alone on
the device and beside the rank's search of its 625-trial slice (two streams, as in the step).

    python scripts/unpack_cost.py [chunks]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "radio-pulsar-utils_amd"), REPO]
import torch  # noqa: E402
from pulsarutils import _hip, synth  # noqa: E402
from pulsarutils.configs import CONFIGS  # noqa: E402
from pulsarutils.dedispersion import dedispersion_plan  # noqa: E402
from pulsarutils.parallel import column_chunks, shard_bounds  # noqa: E402

chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cfg = CONFIGS["C3"]
x = synth.pulsar_filterbank_device(cfg)
nchan, n = x.shape
bounds = column_chunks(n, chunks)
width = max(c1 - c0 for c0, c1 in bounds)
staging = torch.empty(nchan * width, dtype=x.dtype, device=x.device)
# the staging buffer holds filterbank bytes (columns [0, width)), so the unpacked data stays a
# noise filterbank: garbage would make every trial degenerate and send it to the exact path
staging.view(nchan, width).copy_(x[:, :width])


def unpack_all(stream):
    with torch.cuda.stream(stream):
        for c0, c1 in bounds:
            buf = staging[:nchan * (c1 - c0)].view(nchan, c1 - c0)
            x[:, c0:c1].copy_(buf)


s = torch.cuda.Stream()
unpack_all(s)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    unpack_all(s)
torch.cuda.synchronize()
alone = (time.perf_counter() - t0) / 3 * 1e3

dms = dedispersion_plan(cfg.nchan, cfg.dmmin, cfg.dmmax, cfg.start_freq, cfg.bandwidth, cfg.tsamp)
lo, hi = shard_bounds(dms.size, 8, 0)
sh = _hip.shift_table(cfg.nchan, dms[lo:hi], cfg.start_freq, cfg.bandwidth, cfg.tsamp)
plan = _hip.Plan(_hip.PU_U8, _hip.PU_ACC_NATIVE, cfg.nchan, cfg.nsamples, sh)
ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=x.device)
plan.search(x, workspace=ws)
torch.cuda.synchronize()
t0 = time.perf_counter()
plan.search(x, workspace=ws)
torch.cuda.synchronize()
search = (time.perf_counter() - t0) * 1e3
comp = torch.cuda.Stream()
torch.cuda.synchronize()
t0 = time.perf_counter()
unpack_all(s)  # enqueued first: pu_plan_search returns after its own stream synchronises
with torch.cuda.stream(comp):
    out = plan.search(x, workspace=ws)
torch.cuda.synchronize()
both = (time.perf_counter() - t0) * 1e3
nbytes = 2 * x.numel()
print(json.dumps({"what": "C3 receivers' unpack copies (staging -> data[:, c0:c1]) per pipelined step, one GPU",
                  "chunks": len(bounds), "bytes_moved": nbytes, "unpack_alone_ms": round(alone, 3),
                  "unpack_GBps": round(nbytes / alone / 1e6, 1), "search_625_ms": round(search, 3),
                  "search_plus_unpack_two_streams_ms": round(both, 3),
                  "unpack_exposed_ms": round(both - search, 3)}))
