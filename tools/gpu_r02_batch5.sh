#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/b5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_rhs.py --op vjp --rounds 5 kan-odes_amd/kanode/libkanode.so tools/bin/var/prev.so tools/bin/var/vunroll.so > $O/vjp_ab.txt 2>&1 || exit 3
cat $O/vjp_ab.txt | grep -v amdgpu.ids
bash tools/lib_ab.sh $O/epoch_ab.txt 3 4096 base tools/bin/var/prev.so tools/bin/var/fwpe4.so || exit 4
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err || exit 5
cat $O/bench.json
