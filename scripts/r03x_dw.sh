#!/bin/bash
# DMA-issuing wave count (6/8/10/12 of 16) re-tuned for the tall plans: libraries built
# with each value, interleaved per config (C2, C5, C3 625-trial shard).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03x
mkdir -p $OUT
for cfg in C2 C5 C3; do
  T=0; [ $cfg = C3 ] && T=625
  for r in 1 2; do
    for v in dw6 dw8 dw10 dw12; do
      echo "== $cfg round $r lib $v" >> $OUT/ab_$cfg.log
      PULSARUTILS_HIP_LIB=ab/lib_$v.so PU_AB="AB_LIB=$v" PU_TRIALS=$T timeout -k 10 240 python -u scripts/ab_env.py $cfg 2 >> $OUT/ab_$cfg.log 2>&1 || exit $?
    done
  done
done
echo done > $OUT/status.txt
