#!/bin/bash
# Round 5: the Gaussian's window reads two iterations ahead - cleaning GPU tests, A/B of
# bench_clean (head vs gpf2), and rocprofv3 kernel stats of bench_clean f32 with each lib.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05an}
mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-r05an} LIBS="head gpf2" bash scripts/r05s.sh || exit $?
for v in head gpf2; do
  PULSARUTILS_HIP_LIB=ab/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 scripts/bench_clean.py --dtype f32 --steps 10 --warmup 2 > $O/prof_$v.log 2>&1 || exit $?
done
exit 0
