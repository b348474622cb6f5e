#!/bin/bash
# Round 4: GPU idle gaps of the adaptive reference-problem epoch (kernel trace, gaps by kernel pair).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/gaps
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $O/kt.log 2>&1 &&
python3 tools/trace_gaps.py $O/kt --split 5 > $O/gaps.txt 2>&1
rc=$?
rm -rf $O/kt
exit $rc
