#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/wide; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for l in base tools/bin/var/prev.so; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    for c in burgers512 schrodinger1024; do
      KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/prof_surrogate_train.py --case $c --reps 3 2>&1 | grep train_iteration | python3 -c "import sys,ast; s=sys.stdin.read(); d=ast.literal_eval(s[:s.rindex('}')+1]); v=list(d.values())[0]; print('$l', '$c', 'iter_ms %.2f rhs %.2f vjp %.2f' % (v['train_iteration_ms'], v['rhs_us'], v['vjp_us']))" | tee -a $O/ab.txt || exit 3
    done
  done
done
