#!/bin/bash
# Subband-kernel ablation: time the C2 (CFG) plan with phases skipped (results invalid).
# PU_SUB_SKIP exists only in the diagnostic build (make -C radio-pulsar-utils_amd/csrc stamps).
cd "$GRAFT_REPO_ROOT"
for sk in ${SKIPS:-0 1 2 3 4 7 8 15}; do
  echo "skip=$sk"
  PULSARUTILS_HIP_LIB=radio-pulsar-utils_amd/pulsarutils/_lib/libpulsarutils_hip_stamps.so PU_SUB_SKIP=$sk PU_ROUNDS=1 PU_SWEEP=${PU_SWEEP:-4:160:0} timeout -k 10 120 python3 scripts/sweep.py ${CFG:-C2} 2>&1 | grep SUMMARY || exit 1
done
