#!/usr/bin/env bash
# adjoint-step rows kernel: parity tests, epoch A/B, kernel trace of the epoch
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/rows; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_solve.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in 4096 1024 8192; do
  timeout -k 10 200 python -u tools/epoch_ab.py --batch $b --rounds 3 --variants "adj_step_rows=1;adj_step_rows=0" > $OUT/epoch_ab_$b.txt 2>&1 || exit 3
  tail -2 $OUT/epoch_ab_$b.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/prof_epoch.py --batch 4096 --reps 3 > $OUT/trace.log 2>&1 || exit 4
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/rows/trace/run_kernel_stats.csv')))
for r in rows[:8]: print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
