#!/bin/bash
# the table acceptance fix: FK tests, the epoch drift under training, the VJP drift probe, the RHS/VJP/epoch legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_y; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pp.py tests/test_gpu_fk.py tests/test_gpu_fk_e2e.py tests/test_gpu_fsens.py tests/test_gpu_adjoint.py tests/test_gpu_native_solve.py -k "not lotka" > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/epoch_drift.py 0.01 2>/dev/null | tee $O/drift.txt || exit 3
timeout -k 10 200 python3 -u tools/vjp_drift.py 2>/dev/null > $O/vjp_drift.json || exit 3
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-shard-ceiling --no-dist-surrogates > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('rhs', d['ms_per_step'], 'vjp', d['vjp']['ms_per_step'], 'epoch_adaptive', d['epoch_adaptive']['gpu'], 'fk26', d['fk26_train']['gpu'])"
