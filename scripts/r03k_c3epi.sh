#!/bin/bash
# C3 epilogue choice: libraries head (247f70e) / new2 (permlane epilogue everywhere) / new3 (round-2 epilogue for G = 8).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r03k}; mkdir -p $O
A=new2 B=new3 CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625_n2n3.log 2>&1 || exit $?
A=head B=new3 CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c3_625_hn3.log 2>&1 || exit $?
A=head B=new3 CFG=C3 TRIALS=0 ROUNDS=1 bash scripts/ab_lib.sh > $O/ab_c3_5000_hn3.log 2>&1 || exit $?
A=new2 B=new3 CFG=C2 TRIALS=0 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2_n2n3.log 2>&1 || exit $?
