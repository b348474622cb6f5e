#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/b6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_rhs.py --op vjp --rounds 5 kan-odes_amd/kanode/libkanode.so tools/bin/var/prev.so > $O/vjp_ab.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/vjp_ab.txt
bash tools/lib_ab.sh $O/epoch_ab.txt 3 4096 base tools/bin/var/prev.so || exit 4
