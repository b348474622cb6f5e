#!/bin/bash
# interleaved A/B: table staging by direct-to-LDS loads (working build) vs HEAD (tools/bin/var/pphead.so):
# the headline RHS + VJP legs and the adaptive epoch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_n; mkdir -p $O
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$PWD/tools/bin/var/pphead.so; else L=""; fi
    KANODE_LIB=$L timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-epoch --no-shard-ceiling --steps 50 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -5 $O/b_${v}_$r.err; exit 3; }
    python3 -c "import json,sys; d=json.loads(open('$O/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, 'rhs_ms %.4f' % d['ms_per_step'], 'vjp_ms %.4f' % d['vjp']['ms_per_step'])" | tee -a $O/ab.txt
    KANODE_LIB=$L timeout -k 10 120 python3 -u tools/epoch_adaptive_ab.py --variants "fk_device_loop=1" --rounds 1 --reps 2 2>&1 | grep round | sed "s/^/$v $r /" | tee -a $O/ab.txt || exit 3
  done
done
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pp.py tests/test_gpu_fk_e2e.py tests/test_gpu_native_solve.py -k "pp or fk or device_loop or fused_finish or e2e" > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
exit $rc
