#!/bin/bash
# Round 5: where the adjoint rows step's time goes. Kernel traces of the fixed-step epoch (4,096 FK256
# trajectories) with the default library and with the skeleton variant (tools/bin/var/skel.so: the rows
# step's loads, stage sums, stores and reductions without the per-point pullback), interleaved twice; and
# the adaptive epoch's kernel trace on the default library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/skel
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_native_solve.py -k "rows_kernel and not batch_cap" > $O/tests_base.txt 2>&1 || exit 3
for r in 0 1; do
  for v in base skel; do
    if [ $v = skel ]; then export KANODE_LIB=$R/tools/bin/var/skel.so; else unset KANODE_LIB; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fx_${v}_$r -o run -- \
        python3 tools/prof_epoch.py --batch 4096 --reps 3 > $O/fx_${v}_$r.log 2>&1 || exit 3
    rm -f $O/fx_${v}_$r/*kernel_trace.csv $O/fx_${v}_$r/*agent_info.csv
  done
done
unset KANODE_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ad_base -o run -- \
    python3 tools/prof_epoch_adaptive.py > $O/ad_base.log 2>&1 || exit 3
rm -f $O/ad_base/*kernel_trace.csv $O/ad_base/*agent_info.csv
echo ok
