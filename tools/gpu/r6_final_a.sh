#!/bin/bash
# round-6 closing run, part A: the whole GPU suite and smoke() on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/${R6_FINAL:-r6_final}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?
tail -3 $O/pytest_gpu.txt
grep -E "^FAILED|^ERROR" $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 3; }
tail -1 $O/smoke.txt
