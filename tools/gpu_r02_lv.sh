#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/lv; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for l in kan-odes_amd/kanode/libkanode.so tools/bin/var/prev.so; do
    KANODE_LIB=$PWD/$l timeout -k 10 200 python -u tools/lv_ab.py 2>&1 | grep lv4096 | sed "s|^|$l |" | tee -a $O/ab.txt || exit 3
  done
done
