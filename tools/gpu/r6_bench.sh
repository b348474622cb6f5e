#!/bin/bash
# the default bench line on the working tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_bench}; mkdir -p $O
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
cat $O/bench.json
