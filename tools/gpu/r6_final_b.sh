#!/bin/bash
# round-6 closing run, part B: the default bench line, then the same command under the kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/${R6_FINAL:-r6_final}; mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
tail -c 400 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 -u bench.py > $O/bench_profiled.json 2> $O/bench_profiled.err || { tail -20 $O/bench_profiled.err; exit 3; }
find $O/prof -name "*kernel_stats.csv" | head -2
