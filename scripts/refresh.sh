#!/bin/bash
# One GPU call that refreshes the judged artefacts at the current tree: the GPU parity
# suite, the default bench line (C2 headline + clean + cpu baseline + C3 strong), the
# rocprofv3 kernel stats of the C2 bench command, and per config the HBM PMC passes
# (FETCH_SIZE, WRITE_SIZE: one rocprofv3 --pmc run each) next to a bench line of the same
# command, summarised by scripts/pmc_json.py.  Each GPU step has its own time limit; the
# script stops at the first step that fails.
#   NOTEST=1: skip the test suite.  NOSMOKE=1: skip __graft_entry__.smoke().  SQ=1: SQ counter
#   passes of the C3 625 shard.  MR=1: a 2-rank rehearsal of the N > 1 bench on this GPU.  PMC="C2 C5 C3 C3_625": the PMC configs.  CFGS=1: also
#   bench lines for C1/C5/C3 (5000) / the C3 625-trial shard.  LDSC="C2 C3_625 C5 C2_f64": one SQ
#   counter pass each (LDS-array cycles, bank conflicts, instruction counts) -> sq_<cfg>.json.
#   UNPACK=1: the multi-GPU receivers' unpack-copy cost at C3's shape (scripts/unpack_cost.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-refresh}
OUT=gpurun_out/${TAG}
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
fi
if [ -z "$NOSMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c3-strong > $OUT/prof.log 2>&1 || exit $?
  python3 scripts/warm_stats.py $OUT/prof --skip 1 > $OUT/rocprof_warm_stats.csv || exit $?
fi
args_of() {
  case $1 in
    C2) echo "--config C2" ;;
    C5) echo "--config C5" ;;
    C3) echo "--config C3" ;;
    C3_625) echo "--config C3 --scaling strong --shard 8" ;;
    C2_f64) echo "--config C2 --acc f64" ;;
    C1) echo "--config C1" ;;
  esac
}
for cfg in ${PMC:-}; do
  A=$(args_of $cfg)
  D=$OUT/pmc_$cfg
  mkdir -p $D
  timeout -k 10 300 python3 -u bench.py $A --steps 3 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong > $D/bench.json 2> $D/bench.err || exit $?
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/p1 -o run -- python3 bench.py $A --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong > $D/p1.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/p2 -o run -- python3 bench.py $A --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong > $D/p2.log 2>&1 || exit $?
  python3 scripts/pmc_json.py $D $cfg $D/bench.json > $D/pmc_json.log 2>&1 || exit $?
done
for cfg in ${LDSC:-}; do
  A=$(args_of $cfg)
  D=$OUT/sq_$cfg
  mkdir -p $D
  PAT=dedisp_sub_kernel; SRC=csrc/dedisperse.hip
  if [ $cfg = C2_f64 ]; then PAT=dedisp_f64_kernel; SRC=csrc/dedisp_f64.hip; fi
  timeout -k 10 300 python3 -u bench.py $A --steps 3 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $D/bench.json 2> $D/bench.err || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $D/p1 -o run -- python3 bench.py $A --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $D/p1.log 2>&1 || exit $?
  python3 scripts/sq_json.py $D $cfg $D/bench.json $PAT $SRC > $D/sq_json.log 2>&1 || exit $?
done
if [ -n "$SQ" ]; then
  # SQ counter passes of the C3 625-trial shard (scalar vs vector issue) at this source
  A=$(args_of C3_625)
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $OUT/sq_c3_625/p$i -o run -- python3 bench.py $A --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 > $OUT/sq_c3_625_p$i.log 2>&1 || exit $?
  done
fi
if [ -n "$MR" ]; then
  # the N > 1 bench path rehearsed with 2 ranks on this one GPU (gloo: both ranks share the
  # device), small config
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --config C5 --dist-backend gloo --steps 2 --warmup 1 --bcast-chunks 4 \
    > $OUT/mr_bench_c5.json 2> $OUT/mr_bench_c5.err || exit $?
fi
if [ -n "$UNPACK" ]; then
  # the receivers' staging -> strided copy of the N > 1 step at C3's shape
  timeout -k 10 300 python3 -u scripts/unpack_cost.py 8 > $OUT/unpack_cost.json 2> $OUT/unpack_cost.err || exit $?
fi
if [ -n "$CFGS" ]; then
  for cfg in C1 C5 C3 C3_625; do
    A=$(args_of $cfg)
    timeout -k 10 300 python -u bench.py $A --steps 5 --warmup 1 --cpu-trials 16 --no-c3-strong > $OUT/cfg_$cfg.json 2> $OUT/cfg_$cfg.err || exit $?
  done
fi
echo done > $OUT/status.txt
exit 0
