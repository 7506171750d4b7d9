#!/bin/bash
# Round 4: select build diagnosis (M0-based vs per-lane slot writes), its parity tests, the
# whole GPU suite, then A/B against the round-3 library at C3 (625 / 5000 trials).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
PULSARUTILS_HIP_LIB=ab/lib_addtid.so timeout -k 10 180 python -u scripts/sel_diag.py > $OUT/sel_diag_addtid.log 2>&1 || exit $?
PULSARUTILS_HIP_LIB=ab/lib_new.so timeout -k 10 180 python -u scripts/sel_diag.py > $OUT/sel_diag_new.log 2>&1 || exit $?
timeout -k 10 120 python -u scripts/hbm_ceiling.py > $OUT/hbm_ceiling.jsonl 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_dedisperse.py -k "select_build or u8_dma or c3_full" -v -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_sel.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
SEL_LIBS=new A=head B=new CFG=C3 TRIALS=625 ROUNDS=2 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_625.log 2>&1 || exit $?
SEL_LIBS=new A=head B=new CFG=C3 TRIALS=0 ROUNDS=1 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c3_5000.log 2>&1 || exit $?
echo done > $OUT/status.txt
A=new B=tail CFG=C2 TRIALS=1000 ROUNDS=1 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c2_tail.log 2>&1 || exit $?
A=new B=tail CFG=C5 TRIALS=0 ROUNDS=1 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c5_tail.log 2>&1 || exit $?
echo done2 > $OUT/status2.txt
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c3-strong > $OUT/bench.json 2> $OUT/bench.err || exit $?
echo done3 > $OUT/status3.txt
