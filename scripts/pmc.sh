#!/bin/bash
# PMC passes for the dominant kernel (separate rocprofv3 runs, --pmc only; no sys/runtime
# trace).  Usage: TAG=x bash scripts/pmc.sh [extra bench args]
#   CLEAN=1: profile scripts/bench_clean.py (C4 cleaning kernels) instead of bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
OUT=gpurun_out/${TAG}
mkdir -p $OUT
if [ -n "$CLEAN" ]; then
  CMD="python3 scripts/bench_clean.py --steps 2 --warmup 1 $*"
else
  CMD="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-clean $*"
fi
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
      "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
      "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
[ -n "$HBM_ONLY" ] && SETS=("FETCH_SIZE" "WRITE_SIZE")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?" >> $OUT/status.txt; exit 1; }
done
echo done >> $OUT/status.txt
