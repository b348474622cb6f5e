#!/bin/bash
# Round 5: the whole -m gpu suite, then the reference-size training iterations (LV1, FK26) on the default
# library and on the round-4 library (kernel traces + wall time), then one bench.py run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/${1:-small}
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for v in base r4; do
  if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
  timeout -k 10 200 python -u tools/prof_small.py --reps 20 > $O/small_$v.json 2> $O/small_$v.err || exit 3
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_small_$v -o run -- \
      python3 tools/prof_small.py --reps 10 > $O/kt_small_$v.log 2>&1 || exit 3
  rm -f $O/kt_small_$v/*kernel_trace.csv $O/kt_small_$v/*agent_info.csv
done
unset KANODE_LIB
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo ok
