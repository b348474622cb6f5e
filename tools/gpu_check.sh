#!/usr/bin/env bash
# GPU-box validation step: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r01}
stop_if_bad() {  # $1 = rc, $2 = step; 0 ok, 1 = test failures (keep going), else stop
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP after $2 (rc=$1)"; exit "$1"; fi
}
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -3 $OUT/smoke.log; echo "smoke rc=$rc"; stop_if_bad $rc smoke
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -15 $OUT/pytest_gpu.log; echo "pytest rc=$rc"; stop_if_bad $rc pytest
echo "== bench"; timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
cat $OUT/bench_$TAG.json; tail -3 $OUT/bench_$TAG.err; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"; export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1; rc=$?
  tail -3 $OUT/prof_$TAG.log; echo "rocprof rc=$rc"
  find $OUT/prof_$TAG -name "*stats*" | head
fi
