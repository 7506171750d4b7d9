#!/bin/bash
# Closing per-config lines (C1, C5, C3, the C3 625-trial DM shard) at the shipped source, and
# the one-GPU per-rank times of the 8-way C3 split both ways (scripts/shard_times.py: the
# time-tile split, the default N > 1 decomposition, and the DM split).  BENCH=1: also the
# default bench line and its rocprofv3 stats (after the counter files were refreshed, so the
# line reports traffic and lds_cycle_frac).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cfgs}
mkdir -p $OUT
if [ -n "$BENCH" ]; then NB=""; else NB=1; fi
NOTEST=1 NOSMOKE=1 NOBENCH=$NB CFGS=1 TAG=${TAG:-cfgs} bash scripts/refresh.sh || exit $?
timeout -k 10 300 python -u scripts/shard_times.py C3 8 time > $OUT/shards_C3_time.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/shard_times.py C3 8 dm > $OUT/shards_C3_dm.log 2>&1 || exit $?
echo done > $OUT/status2.txt
