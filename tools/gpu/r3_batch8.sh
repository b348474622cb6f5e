#!/bin/bash
# all GPU tests on the polled step control, then training A/B vs the previous commit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b8; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; tail -15 $O/pytest_gpu.txt; [ $rc -le 1 ] || exit $rc
bash tools/gpu/train_ab.sh $O/train_ab.txt 2 base tools/bin/var/prev.so
