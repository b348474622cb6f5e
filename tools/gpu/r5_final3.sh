#!/bin/bash
# Round 5 closing bench line after the Trainer's native MSE step: smoke and bench.py -> gpurun_out/profile_r05c/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && export TMPDIR=/tmp
O=gpurun_out/profile_r05c
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 3; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
cat $O/bench.json
echo ok
