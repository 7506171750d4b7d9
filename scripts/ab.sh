#!/bin/bash
# A/B the C2 subband kernel across trees built from earlier commits (ab/<commit>/, built
# in this container) and HEAD, interleaved on one box.  Usage: AB="07a48be 9a9ae53" bash scripts/ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-ab}.log
for rep in 1 2; do
  for c in HEAD $AB; do
    d=.; [ "$c" = HEAD ] || d=ab/$c
    echo "tree=$c rep=$rep" >> $OUT
    (cd $d && PU_SWEEP=${VARIANT:-4:160:0} PU_ROUNDS=2 timeout -k 10 200 python3 scripts/sweep.py ${CFG:-C2}) >> $OUT 2>&1 || exit $?
  done
done
