#!/bin/bash
# Round 5: dedisperse.hip compiled with other AMDGPU scheduler strategies (same source):
# interleaved A/B of the production build (head) against max-ilp (ilp), max-memory-clause
# (mc) and the AMDGPU register-pressure trackers (trk) at the configs in CFGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05ab}
mkdir -p $O
export TMPDIR=/tmp
for c in ${CFGS:-C2 C5}; do
  case $c in C2) T=1000 ;; C5) T=500 ;; C3) T=625 ;; esac
  LIBS="${LIBS:-head ilp mc trk}" CFG=$c TRIALS=$T ROUNDS=${ROUNDS:-2} bash scripts/ab_lib.sh > $O/ab_$c.log 2>&1 || exit $?
done
exit 0
