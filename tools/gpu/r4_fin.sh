#!/bin/bash
# Round 4: the adaptive adjoint step's finish fused into the rows kernel (KANODE_OPT_ADJ_FUSED_FINISH):
# the targeted tests, the whole -m gpu suite, the epoch A/B (option off / on, interleaved) and a kernel
# trace of the adaptive epoch with the option on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/fin
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_native_solve.py \
    -k "fused_finish or dense_saveat or rows_kernel or options_round_trip" > $O/targeted.txt 2>&1 || exit 3
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1
[ $? -le 1 ] || exit 3
timeout -k 10 400 python -u tools/epoch_adaptive_ab.py --variants "adj_fused_finish=0;adj_fused_finish=1" \
    --rounds 3 > $O/epoch_ab.txt 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_epoch_adaptive.py > $O/kt.log 2>&1
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
