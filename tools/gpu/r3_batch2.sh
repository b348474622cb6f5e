#!/bin/bash
# pair pullback with the basis store and the wave-per-unit wide-out parameters: GPU tests, VJP and training A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; tail -5 $O/pytest_gpu.txt; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 python -u tools/surr_vjp_time.py base >> $O/vjp.txt 2>&1 || exit 3
  KANODE_LIB=$PWD/tools/bin/var/oldsolve.so timeout -k 10 120 python -u tools/surr_vjp_time.py r3head >> $O/vjp.txt 2>&1 || exit 3
done
grep -v amdgpu.ids $O/vjp.txt
bash tools/gpu/train_ab.sh $O/train_ab.txt 2 base tools/bin/var/oldsolve.so
