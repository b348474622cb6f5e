#!/bin/bash
# Round 4: the reduction / finish kernels with four rows' loads in flight per thread: the whole -m gpu suite,
# kernel traces of the fixed and adaptive epochs, and the adaptive epoch's wall time (bench leg).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/red
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1
[ $? -le 1 ] || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ep -o run -- \
    python3 tools/prof_epoch.py --batch 4096 --reps 3 > $O/ep.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ea -o run -- \
    python3 tools/prof_epoch_adaptive.py > $O/ea.log 2>&1 || exit 3
rm -f $O/ep/*kernel_trace.csv $O/ep/*agent_info.csv $O/ea/*kernel_trace.csv $O/ea/*agent_info.csv
timeout -k 10 300 python -u tools/epoch_adaptive_ab.py --variants "adj_fused_finish=0" --rounds 3 > $O/epoch_adaptive.txt 2>&1
