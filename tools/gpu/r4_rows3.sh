#!/bin/bash
# Round 4: adjoint rows step with first-point moment initialisation and the host-precomputed 2nd-order
# correction weight: the FK GPU tests, then a kernel trace of the adaptive epoch and the epoch itself.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/rows3
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu \
    > $O/pytest.txt 2>&1; [ $? -le 1 ] || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $O/kt.log 2>&1 || exit 3
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
timeout -k 10 200 python -u tools/epoch_adaptive_ab.py --rounds 3 --reps 2 --variants "adj_step_rows=1" > $O/epoch.txt 2>&1
