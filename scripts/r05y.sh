#!/bin/bash
# Round 5: bitonic steps with v_min_f64 / v_max_f64 - cleaning GPU tests, then an interleaved
# A/B of masks_overhead.py (fused = previous build, minmax = this one), f32 and u8, and
# rocprofv3 kernel stats of the masks path at this build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05y}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_clean.py > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  for v in ${LIBS:-fused minmax}; do
    for d in f32 u8; do
      echo "== round $r lib $v $d" >> $O/ab.log
      PULSARUTILS_HIP_LIB=ab/lib_$v.so timeout -k 10 200 python -u scripts/masks_overhead.py --dtype $d --iters 100 >> $O/ab.log 2>&1 || exit $?
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/masks_overhead.py --iters 30 > $O/prof.log 2>&1 || exit $?
exit 0
