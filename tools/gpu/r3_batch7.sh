#!/bin/bash
# all GPU tests on the adaptive combined reductions + host-summed step error, then training A/B vs HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b7; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; tail -15 $O/pytest_gpu.txt; [ $rc -le 1 ] || exit $rc
bash tools/gpu/train_ab.sh $O/train_ab.txt 2 base tools/bin/var/head.so
