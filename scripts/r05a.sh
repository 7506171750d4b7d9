#!/bin/bash
# Round 5, first GPU call: the new parity tests (production C3 tile, tile == full plane,
# mesh collective on 2-3 ranks), a two-rank gloo rehearsal of the N > 1 bench path, and
# the default bench line at HEAD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05a
O=gpurun_out/r05a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dedisperse.py::test_dedisperse_dm_tile_equals_full_plane \
  tests/test_gpu_multirank.py tests/test_gpu_dedisperse.py::test_search_c3_full_size_u8 > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --dist-backend gloo --config C5 --steps 3 --warmup 1 \
  > $O/rehearse_c5_2.json 2> $O/rehearse_c5_2.err || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
exit 0
