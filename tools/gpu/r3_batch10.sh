#!/bin/bash
# fused pair stages: all GPU tests, then training A/B vs the previous commit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b10; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; tail -15 $O/pytest_gpu.txt; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for l in base tools/bin/var/prev.so; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/train_time.py $(basename $l .so) --no-epoch >> $O/train.txt 2>&1 || exit 3
  done
done
grep -v amdgpu.ids $O/train.txt | sort -k2,2 -k1,1
