#!/bin/bash
# Surrogate two-launch pullback: parity tests, interleaved A/B, Burgers training kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3prof
mkdir -p $O
timeout -k 10 120 python -u tools/diag/burgers41_spread.py > $O/burgers41_spread.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py \
    tests/test_gpu_native_solve.py -k "surrogate or pair" -m gpu > $O/pair_tests.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc      # test failures are reported; a crash / timeout ends the run
timeout -k 10 300 python -u tools/surr_pair_ab.py > $O/surr_pair_ab.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/burgers -o run -- python3 $R/tools/prof_surrogate_train.py \
    --case burgers512 --reps 2 > $O/burgers_prof.log 2>&1
