#!/bin/bash
# Round 4: the FK pullback point with its φ′ and swish Horner chains interleaved (rows_hs0, more ILP for
# the latency-bound adjoint rows step): standalone VJP at 1M trajectories (one process, interleaved) and a
# kernel trace of the adaptive epoch; then the short anchor test with its learned source printed.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/rows2
mkdir -p $O
cd $R && export TMPDIR=/tmp
B=kan-odes_amd/kanode/libkanode.so
timeout -k 10 300 python -u tools/ab_rhs.py --op vjp --batch 1048576 --rounds 5 --reps 10 \
    $B tools/bin/var/rows_hs0.so > $O/ab_vjp.txt 2>&1 || exit 3
KANODE_LIB=$R/tools/bin/var/rows_hs0.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/kt_hs0 -o run -- python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $O/kt_hs0.log 2>&1 || exit 3
rm -f $O/kt_hs0/*kernel_trace.csv $O/kt_hs0/*agent_info.csv
timeout -k 10 200 python -u -m pytest -x -v --timeout 180 --timeout-method thread -s tests/test_gpu_anchors.py \
    > $O/pytest_anchors.txt 2>&1
exit 0
