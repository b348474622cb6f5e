#!/bin/bash
# surrogate GPU tests on the final pair pullback, then the second ablation round
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py tests/test_gpu_native_solve.py tests/test_gpu_tp.py tests/test_gpu_train.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -le 1 ] || exit $rc
bash tools/surr_ablate.sh abl1 abl3 abl4 abl5 abl6 abl7 abl8 abl9
