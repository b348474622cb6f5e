#!/usr/bin/env bash
# Round evidence on the GPU box -> gpurun_out/profile_$TAG/ (copied into profiles/$TAG by the caller):
#   0. pytest -m gpu (whole suite) and __graft_entry__.smoke()
#   1. bench.py (the driver's command, with cpu_baseline)  -> bench.json
#   2. rocprofv3 --kernel-trace --stats of the same bench    -> kernel_stats.csv
#   3. separate --pmc passes (no trace domains with PMC): FETCH_SIZE, WRITE_SIZE, VALU counters
#   4. tools/traffic.py -> traffic.json (gfx950: FETCH_SIZE x2 for 16-B/lane streaming reads)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/profile_$TAG; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 3; }
  tail -2 $OUT/pytest_gpu.log
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
  tail -2 $OUT/smoke.log
fi
echo "== bench"
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 3; }
cat $OUT/bench.json
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 3; }
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
for w in fk_rhs fk_rhs_rec fk_vjp; do
  for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS"; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $OUT/pmc_${w}_$n -o run --output-format csv -- \
      python3 tools/prof_kernel.py --what $w --reps 5 --batch ${BATCH:-1048576} > $OUT/pmc_${w}_$n.log 2>&1 || { echo "pmc $w $n failed"; tail -5 $OUT/pmc_${w}_$n.log; exit 3; }
  done
done
echo "== epoch kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/epoch -o run --output-format csv -- \
  python3 tools/prof_epoch.py --batch 4096 --reps 3 > $OUT/epoch.log 2>&1 || { tail -5 $OUT/epoch.log; exit 3; }
cp $OUT/epoch/run_kernel_stats.csv $OUT/epoch_kernel_stats.csv
echo "== adaptive epoch and surrogate training kernel traces"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/epoch_adaptive -o run --output-format csv -- \
  python3 tools/prof_epoch_adaptive.py > $OUT/epoch_adaptive.log 2>&1 || { tail -5 $OUT/epoch_adaptive.log; exit 3; }
cp $OUT/epoch_adaptive/run_kernel_stats.csv $OUT/epoch_adaptive_kernel_stats.csv
for c in burgers512 schrodinger1024; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/train_$c -o run --output-format csv -- \
    python3 tools/prof_surrogate_train.py --case $c --reps 2 > $OUT/train_$c.log 2>&1 || { tail -5 $OUT/train_$c.log; exit 3; }
  cp $OUT/train_$c/run_kernel_stats.csv $OUT/train_${c}_kernel_stats.csv
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt
BATCH=${BATCH:-1048576} python3 tools/traffic.py $OUT > $OUT/traffic.json
cat $OUT/pmc_summary.txt $OUT/traffic.json
# the per-dispatch CSVs are tens of MB (gpurun returns at most 64 MiB): keep the summaries only
find $OUT -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
