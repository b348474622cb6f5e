#!/bin/bash
# Trainer's pinned loss copy: the training tests, the table tests on the final staging, the small-problem legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_o; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_pp.py tests/test_gpu_fsens.py tests/test_gpu_fk_e2e.py > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 120 python3 -u tools/legs.py lv1_train fk26_train lv4096_train 2>/dev/null | sed "s/^/r$r /" | tee -a $O/legs.txt || exit 3
done
