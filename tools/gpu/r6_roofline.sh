#!/bin/bash
# Round 6: GPU tests, then the headline roofline reproducible from one file, then the shader clock under the
# FK kernels whose issue floors DESIGN states.
#   head/    rocprofv3 --kernel-trace --stats of bench.py with ONLY the 1M-trajectory RHS leg (no shard_ceiling,
#            VJP, epochs): every fk_rhs_pp_wave_kernel / fk_pp_build_kernel dispatch is a bench step
#   full/    the default bench under the profiler, its trace split by grid size (tools/kstats_by_grid.py)
#   clock_*/ --pmc GRBM_GUI_ACTIVE passes (kernel trace only) -> tools/clock.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_roof; mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
  rc=$?
  tail -1 $O/pytest_gpu.txt
  # a test assertion (rc 1) does not stop the profiles; anything else (timeout, crash) does
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/pytest_gpu.txt; exit 3; fi
  grep -E "^FAILED" $O/pytest_gpu.txt || true
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/head -o run --output-format csv -- \
  python3 bench.py --no-vjp --no-epoch --no-shard-ceiling --no-cpu-baseline --steps 50 --warmup 5 > $O/head.json 2> $O/head.err || { tail -5 $O/head.err; exit 3; }
cat $O/head.json
python3 tools/kstats_by_grid.py $O/head/run_kernel_trace.csv --csv $O/head_by_grid.csv > $O/head_by_grid.txt
cp $O/head/run_kernel_stats.csv $O/head_kernel_stats.csv
head -4 $O/head_by_grid.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/full -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline > $O/full.json 2> $O/full.err || { tail -5 $O/full.err; exit 3; }
python3 tools/kstats_by_grid.py $O/full/run_kernel_trace.csv --csv $O/full_by_grid.csv > $O/full_by_grid.txt
cp $O/full/run_kernel_stats.csv $O/full_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lv4096 -o run --output-format csv -- \
  python3 tools/prof_lv4096.py --reps 5 > $O/lv4096.json 2> $O/lv4096.err || { tail -5 $O/lv4096.err; exit 3; }
cat $O/lv4096.json
python3 tools/kstats_by_grid.py $O/lv4096/run_kernel_trace.csv > $O/lv4096_by_grid.txt
cp $O/lv4096/run_kernel_stats.csv $O/lv4096_kernel_stats.csv
head -12 $O/lv4096_by_grid.txt
for w in epoch_adaptive fk_vjp fk_rhs; do
  if [ $w = epoch_adaptive ]; then cmd="python3 tools/prof_epoch_adaptive.py"; else cmd="python3 tools/prof_kernel.py --what $w --reps 20 --batch 1048576"; fi
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-trace -d $O/clock_$w -o run --output-format csv -- $cmd > $O/clock_$w.log 2>&1 || { echo "clock $w failed"; tail -5 $O/clock_$w.log; exit 3; }
  python3 tools/clock.py $O/clock_$w > $O/clock_$w.txt
  cat $O/clock_$w.txt | head -8
done
# keep the summaries only (the per-dispatch CSVs are large)
rm -rf $O/full $O/lv4096 $O/clock_*/ 2>/dev/null
find $O/head -name "*.csv" ! -name "run_kernel_trace.csv" ! -name "run_kernel_stats.csv" -delete
