#!/bin/bash
# interleaved A/B: chain kernels staging constants with all loads in flight (working build) vs HEAD's kan_col
# (tools/bin/var/colhead.so) on the LV4096 and LV1 training legs; the chain tests on the working build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_k; mkdir -p $O
for r in 1 2 3; do
  KANODE_LIB=$PWD/tools/bin/var/colhead.so timeout -k 10 120 python3 -u tools/legs.py lv4096_train lv1_train 2>/dev/null | sed "s/^/head $r /" | tee -a $O/ab.txt || exit 3
  timeout -k 10 120 python3 -u tools/legs.py lv4096_train lv1_train 2>/dev/null | sed "s/^/new $r /" | tee -a $O/ab.txt || exit 3
done
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_native_solve.py tests/test_gpu_chain.py tests/test_gpu_train.py > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
exit $rc
