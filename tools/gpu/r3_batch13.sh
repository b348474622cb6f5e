#!/bin/bash
# table build with one load round: FK tests, then interleaved bench RHS A/B at 1M and 128k trajectories
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b13; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_pp.py tests/test_gpu_fk.py tests/test_gpu_fk_e2e.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do
  for l in base tools/bin/var/prev.so; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    for bt in 1048576 131072; do
      KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-vjp --no-epoch --batch-total $bt > $O/b.json 2>/dev/null || exit 3
      python3 -c "import json;d=json.load(open('$O/b.json'));print('$(basename $l .so)', $bt, round(d['ms_per_step']*1e3,1), 'us/step', round(d['roofline']['frac'],4))" >> $O/ab.txt
    done
  done
done
sort -k2,2n -k1,1 $O/ab.txt
