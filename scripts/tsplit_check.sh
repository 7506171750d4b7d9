#!/bin/bash
# Round 6: the time-tile sharded N > 1 path on one GPU - the multi-rank GPU tests (dm and
# time decompositions, gloo ranks sharing cuda:0; RCCL world 1), the per-rank times of the
# 8-way time split of C3 next to the DM split's (scripts/shard_times.py), and a 2-rank
# rehearsal of bench.py's N > 1 line (C5, gloo).  Each GPU step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tsplit}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/mr_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/shard_times.py C3 8 time > $OUT/shards_C3_time.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --config C5 --dist-backend gloo --steps 2 --warmup 1 --bcast-chunks 4 \
    > $OUT/mr_bench_c5_time.json 2> $OUT/mr_bench_c5_time.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29534 bench.py --gpus 2 --config C5 --dist-backend gloo --steps 2 --warmup 1 --bcast-chunks 4 \
    --decomposition dm > $OUT/mr_bench_c5_dm.json 2> $OUT/mr_bench_c5_dm.err || exit $?
echo done
