#!/bin/bash
# C5 / C2 diagnostics at HEAD: phase stamps (diagnostic build) and the C5 workgroup-shape A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03e}; mkdir -p $O
timeout -k 10 200 python -u scripts/stamps.py C2 3 > $O/stamps_c2.jsonl 2> $O/stamps.err || exit $?
timeout -k 10 200 python -u scripts/stamps.py C5 5 > $O/stamps_c5.jsonl 2>> $O/stamps.err || exit $?
PU_AB="PU_SUB_SHAPE=0;PU_SUB_SHAPE=1;PU_SUB_SHAPE=2" timeout -k 10 300 python -u scripts/ab_env.py C5 3 > $O/ab_c5_shape.log 2>&1 || exit $?
