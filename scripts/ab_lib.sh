#!/bin/bash
# Interleaved A/B of two builds of the library (ab/lib_<A>.so vs ab/lib_<B>.so), each round
# in its own process:  A=head B=new CFG=C3 TRIALS=625 ROUNDS=2 bash scripts/ab_lib.sh
# (LIBS="a b c" instead of A / B: any number of libraries)
set -e
A=${A:-head}; B=${B:-new}; CFG=${CFG:-C3}; TRIALS=${TRIALS:-625}; ROUNDS=${ROUNDS:-2}; export AB_ACC=${ACC:-native}
for r in $(seq 1 "$ROUNDS"); do
  for v in ${LIBS:-$A $B}; do
    echo "== round $r lib $v"
    PULSARUTILS_HIP_LIB=ab/lib_$v.so PU_AB="AB_LIB=$v" PU_TRIALS=$TRIALS \
      timeout -k 10 240 python -u scripts/ab_env.py "$CFG" 2
  done
done
