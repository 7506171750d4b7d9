#!/bin/bash
# Round 4: does the f32 apply pass's write-back slow the NEXT pass?  End-to-end
# renormalize (bench_clean.py, back-to-back calls) with non-temporal stores on / off in
# the apply pass (diagnostic build: PU_CLEAN_NT), interleaved processes, f32 and u8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04g
mkdir -p $OUT
L=radio-pulsar-utils_amd/pulsarutils/_lib/libpulsarutils_hip_stamps.so
for r in 1 2; do
  for dt in f32 u8; do
    for nt in 0 1; do
      echo "== round $r dtype $dt PU_CLEAN_NT=$nt" >> $OUT/nt_ab.log
      PULSARUTILS_HIP_LIB=$L PU_CLEAN_NT=$nt timeout -k 10 200 python -u scripts/bench_clean.py --dtype $dt --steps 20 >> $OUT/nt_ab.log 2>&1 || exit $?
    done
  done
done
echo done > $OUT/status.txt
