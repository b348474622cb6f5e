#!/bin/bash
# forward step kernel with the next row prefetched: FK tests, then epoch A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b12; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_fk_e2e.py tests/test_gpu_native_solve.py tests/test_gpu_adjoint.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  for l in base tools/bin/var/nopf.so tools/bin/var/prev.so; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/train_time.py $(basename $l .so) --no-surrogates >> $O/train.txt 2>&1 || exit 3
  done
done
grep -v amdgpu.ids $O/train.txt | sort -k2,2 -k1,1
