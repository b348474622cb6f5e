#!/bin/bash
# Adjoint step records (KANODE_OPT_RECORD_ADJOINT_STEPS) on every adjoint path and the surrogate test's
# derived adaptive bar, then the round-5 anchors (tools/gpu/r5_anchors.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/rec
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_native_solve.py \
  -k "full_size_surrogate or falls_back or fk_small or lv1_wide" -s > $O/tests.txt 2>&1 || exit 3
bash tools/gpu/r5_anchors.sh
