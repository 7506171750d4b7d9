#!/bin/bash
# One environment knob over values, C2 and C3 (625 trials), one box.
# Usage: KNOB=PU_DMA_WAVES VALUES="16 8 4" TAG=x bash scripts/knob_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-knob}.log
for rep in 1 2; do
  for v in $VALUES; do
    echo "$KNOB=$v rep=$rep C2" >> $OUT
    env $KNOB=$v PU_SWEEP=4:160:0 PU_ROUNDS=2 timeout -k 10 200 python3 scripts/sweep.py C2 >> $OUT 2>&1 || exit $?
    if [ -z "$NOC3" ]; then
      echo "$KNOB=$v rep=$rep C3-625" >> $OUT
      env $KNOB=$v PU_TRIALS=625 PU_SWEEP=8:160:0 PU_ROUNDS=2 timeout -k 10 200 python3 scripts/sweep.py C3 >> $OUT 2>&1 || exit $?
    fi
  done
done
