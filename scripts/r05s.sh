#!/bin/bash
# Round 5: in-wave bitonic steps on the VALU (DPP / permlane swaps) in the one-workgroup
# sorts of the noisy-channel and variability kernels - cleaning GPU tests, then an
# interleaved A/B of bench_clean (head vs dpp) for f32 and u8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_clean.py > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in ${LIBS:-head dpp}; do
    for d in f32 u8; do
      echo "== round $r lib $v $d" >> $O/ab.log
      PULSARUTILS_HIP_LIB=ab/lib_$v.so timeout -k 10 200 python -u scripts/bench_clean.py --dtype $d --steps 20 --warmup 3 >> $O/ab.log 2>&1 || exit $?
    done
  done
done
exit 0
