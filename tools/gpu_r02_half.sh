#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/half; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/lib_ab.sh $O/epoch_ab.txt 3 4096 base tools/bin/var/nohalf.so || exit 4
bash tools/lib_ab.sh $O/epoch_ab2048.txt 2 2048 base tools/bin/var/nohalf.so || exit 5
