#!/bin/bash
# GPU tests on the mapped step-control scalars, the surrogate pullback ablation, training-leg A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc -le 1 ] || exit $rc
bash tools/surr_ablate.sh abl1 abl2 abl3 abl4 abl5 abl6 abl7 || exit 3
bash tools/gpu/train_ab.sh $O/train_ab.txt 2 base tools/bin/var/oldsolve.so
