#!/bin/bash
# column-contiguous pair dot-product partials: surrogate tests, VJP and training A/B vs the previous commit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b14; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py tests/test_gpu_native_solve.py tests/test_gpu_tp.py tests/test_gpu_train.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -le 1 ] || exit $rc
bash tools/gpu/vjp_ab.sh $O/vjp.txt 2 base tools/bin/var/prev.so || exit 3
for r in 1 2; do
  for l in base tools/bin/var/prev.so; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/train_time.py $(basename $l .so) --no-epoch >> $O/train.txt 2>&1 || exit 3
  done
done
grep -v amdgpu.ids $O/train.txt | sort -k2,2 -k1,1
