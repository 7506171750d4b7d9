#!/bin/bash
# Round 5: one-launch cut_outliers - cleaning GPU tests; per-kernel trace of the C4 cleaning
# steps (f32, u8); the non-temporal apply tail (diagnostic library, PU_APPLY_NT_TAIL) A/B;
# SQ counters of the 16 x 4 float64 kernel at C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_clean.py > $O/tests_clean.log 2>&1 || exit $?
for dt in f32 u8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clean_$dt -o run -- \
    python3 scripts/bench_clean.py --dtype $dt --steps 10 --warmup 2 > $O/prof_clean_$dt.log 2>&1 || exit $?
done
STAMPLIB=radio-pulsar-utils_amd/pulsarutils/_lib/libpulsarutils_hip_stamps.so
for rep in 1 2; do
  for tail in 0 1 2 4; do
    for dt in f32 u8; do
      echo "== rep $rep tail $tail dtype $dt" >> $O/nt_tail.log
      PULSARUTILS_HIP_LIB=$STAMPLIB PU_APPLY_NT_TAIL=$tail timeout -k 10 200 python3 scripts/bench_clean.py \
        --dtype $dt --steps 10 --warmup 2 >> $O/nt_tail.log 2>&1 || exit $?
    done
  done
done
CMD="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-clean --no-c3-strong --no-acc-f64 --acc f64"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc_f64_p$i -o run -- $CMD > $O/pmc_f64_p$i.log 2>&1 || exit $?
done
exit 0
