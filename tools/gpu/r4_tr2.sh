#!/bin/bash
# Round 4: the fixed-step combined adjoint step's rows parameter-major too: the whole -m gpu suite, then
# kernel traces of the fixed and adaptive epochs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/tr2
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1
[ $? -le 1 ] || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ep -o run -- \
    python3 tools/prof_epoch.py --batch 4096 --reps 3 > $O/ep.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ea -o run -- \
    python3 tools/prof_epoch_adaptive.py > $O/ea.log 2>&1 || exit 3
rm -f $O/ep/*kernel_trace.csv $O/ep/*agent_info.csv $O/ea/*kernel_trace.csv $O/ea/*agent_info.csv
