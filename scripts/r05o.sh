#!/bin/bash
# Round 5: archived finalize vector-load diff A/B (fin vs c3a) at C5 / C2 / C3 625; SQ
# counters of the C3 625-trial shard and of the float64 C2 kernel at the current source.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o
mkdir -p $O
export TMPDIR=/tmp
LIBS="c3a fin" CFG=C5 TRIALS=500 ROUNDS=3 bash scripts/ab_lib.sh > $O/ab_c5_fin.log 2>&1 || exit $?
LIBS="c3a fin" CFG=C2 TRIALS=1000 ROUNDS=2 bash scripts/ab_lib.sh > $O/ab_c2_fin.log 2>&1 || exit $?
i=0
CMD="python3 bench.py --config C3 --scaling strong --shard 8 --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64"
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc_c3_p$i -o run -- $CMD > $O/pmc_c3_p$i.log 2>&1 || exit $?
done
i=0
CMD="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 --acc f64"
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc_f64_p$i -o run -- $CMD > $O/pmc_f64_p$i.log 2>&1 || exit $?
done
exit 0
