#!/bin/bash
# Round 5: DMA-issuing wave count re-swept at the round-5 source (diagnostic build's
# PU_DMA_WAVES knob; stamps build, so absolute times include the stamp reads).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r05ag}
mkdir -p $O
export TMPDIR=/tmp
export PULSARUTILS_HIP_LIB=radio-pulsar-utils_amd/pulsarutils/_lib/libpulsarutils_hip_stamps.so
AB="PU_DMA_WAVES=8;PU_DMA_WAVES=6;PU_DMA_WAVES=10;PU_DMA_WAVES=12;PU_DMA_WAVES=16"
PU_AB="$AB" timeout -k 10 300 python -u scripts/ab_env.py C2 3 > $O/dw_c2.log 2>&1 || exit $?
PU_AB="$AB" timeout -k 10 300 python -u scripts/ab_env.py C5 3 > $O/dw_c5.log 2>&1 || exit $?
PU_TRIALS=625 PU_AB="$AB" timeout -k 10 500 python -u scripts/ab_env.py C3 2 > $O/dw_c3_625.log 2>&1 || exit $?
exit 0
