#!/bin/bash
# Round 4: the combined adaptive step's slab rows parameter-major (coalesced finish loads): the whole -m gpu
# suite, then the adaptive epoch's kernel trace and wall time (twice).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/tr
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1
[ $? -le 1 ] || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_epoch_adaptive.py > $O/kt.log 2>&1 || exit 3
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
timeout -k 10 300 python -u tools/epoch_adaptive_ab.py --variants "adj_fused_finish=0;adj_fused_finish=1" --rounds 2 > $O/wall.txt 2>&1
