#!/bin/bash
# Round 5 closing evidence after the small-problem work: the whole -m gpu suite, smoke, the default bench line
# (with its CPU baselines) and the reference-size iterations' kernel trace -> gpurun_out/profile_r05b/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && export TMPDIR=/tmp
O=gpurun_out/profile_r05b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 3; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 3; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
cat $O/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/small -o run -- \
  python3 tools/prof_small.py --reps 20 > $O/small.log 2>&1 || exit 3
cp $O/small/run_kernel_stats.csv $O/small_kernel_stats.csv
rm -rf $O/small
echo ok
