#!/usr/bin/env bash
# Surrogate training-iteration A/B over library variants (alternating processes) + their surrogate tests.
#   tools/gpu_surr_ab.sh OUT ROUNDS lib1.so lib2.so ...   ("base" = kan-odes_amd/kanode/libkanode.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=$1; rounds=$2; shift 2
for l in "$@"; do
  lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
  KANODE_LIB=$PWD/$lib timeout -k 10 200 python -m pytest tests/test_gpu_surrogate.py tests/test_gpu_chain.py -x -q \
     --timeout 120 --timeout-method thread > gpurun_out/surr_tests_$(basename $l .so).txt 2>&1 \
     || { echo "$l tests failed"; tail -20 gpurun_out/surr_tests_$(basename $l .so).txt; exit 3; }
  echo "$l: $(tail -n 1 gpurun_out/surr_tests_$(basename $l .so).txt)" >> $out
done
for r in $(seq 1 $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    for c in burgers512 schrodinger1024; do
      KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/prof_surrogate_train.py --case $c --reps 3 2>&1 | \
        python3 -c "import sys,re; s=sys.stdin.read(); print('$l $c', *re.findall(r\"'(rhs_us|vjp_us|train_iteration_ms)': ([0-9.]+)\", s))" >> $out || exit 3
    done
  done
done
cat $out
