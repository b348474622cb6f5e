#!/bin/bash
# per-block table stamps: the table tests, then the headline leg under the kernel trace (fk_pp_build_kernel average)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_m; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pp.py tests/test_gpu_fk.py tests/test_gpu_fk_e2e.py tests/test_gpu_fsens.py > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o head -- python3 -u bench.py --no-cpu-baseline --no-epoch --no-shard-ceiling --no-vjp > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -4 "$f" | cut -c1-220
timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-epoch --no-shard-ceiling > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'vjp', d['vjp']['ms_per_step'])"
