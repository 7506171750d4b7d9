#!/bin/bash
# One GPU call: a pytest selection (PYTEST_K, -k expression; PYTEST_FILES), then interleaved
# plan A/B sweeps (SWEEPS="cfg:trials[+first]:variants;..." -> scripts/sweep.py; "625+1875" =
# trials 1875 .. 2499), each step under its
# own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$PYTEST_K$PYTEST_FILES" ]; then
  timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -v -m gpu -x ${PYTEST_K:+-k "$PYTEST_K"} --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || exit $?
fi
IFS=';' read -ra SW <<< "${SWEEPS:-}"
i=0
for sw in "${SW[@]}"; do
  [ -z "$sw" ] && continue
  IFS=':' read -r cfg trials variants <<< "$sw"
  i=$((i+1))
  t0=0
  case "$trials" in *+*) t0=${trials#*+}; trials=${trials%%+*};; esac
  PU_SWEEP="$variants" PU_TRIALS="$trials" PU_TRIAL0="$t0" PU_ROUNDS=${ROUNDS:-3} timeout -k 10 400 python -u scripts/sweep.py $cfg > $OUT/sweep_${i}_${cfg}.log 2>&1 || exit $?
done
echo done > $OUT/status.txt
