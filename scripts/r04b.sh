#!/bin/bash
# Round 4: channel-mode (float64 accumulation) kernel with one-step-ahead window reads
# and J = 2 for float32 rows into float64 accumulators.  GPU suite, A/B against the
# previous library (ab/lib_head.so) at C1 and C2 acc=f64, the bench line (acc_f64
# sub-object), and the rocprofv3 kernel stats of the C1 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit $?
A=head B=pp CFG=C1 TRIALS=0 ROUNDS=2 timeout -k 10 300 bash scripts/ab_lib.sh > $OUT/ab_c1.log 2>&1 || exit $?
A=head B=pp CFG=C2 TRIALS=1000 ROUNDS=1 ACC=f64 timeout -k 10 400 bash scripts/ab_lib.sh > $OUT/ab_c2_f64.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 python -u bench.py --config C1 --steps 20 --warmup 2 --no-clean --no-c3-strong --cpu-trials 16 --cpu-reps 1 > $OUT/bench_c1.json 2> $OUT/bench_c1.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c1 -o run -- python3 bench.py --config C1 --steps 20 --warmup 5 --no-clean --no-c3-strong --no-cpu-baseline --no-acc-f64 > $OUT/prof_c1.log 2>&1 || exit $?
echo done > $OUT/status.txt
