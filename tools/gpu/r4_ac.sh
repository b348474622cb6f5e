#!/bin/bash
# Round 4: the persistent pair adjoint's phase profile (final kernel), the short anchor test, then the Allen-Cahn source anchor (N_iter = 5e4 at ~17 ms per iteration,
# two initialisations side by side, each stopping at its time budget if the call's limit comes first).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/anchors_ac
mkdir -p $O/s0 $O/s1 $R/gpurun_out/r4/persist
mkdir -p $R/gpurun_out/r4/rows
KANODE_LIB=$R/tools/bin/var/rows_r2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/r4/rows/kt_r2 -o run -- python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 \
    > $R/gpurun_out/r4/rows/kt_r2.log 2>&1 || exit 3
rm -f $R/gpurun_out/r4/rows/kt_r2/*kernel_trace.csv $R/gpurun_out/r4/rows/kt_r2/*agent_info.csv
KANODE_LIB=$R/tools/bin/var/paprof.so timeout -k 10 120 python -u tools/pair_persist_prof.py 0 \
    > $R/gpurun_out/r4/persist/prof_s8_final.txt 2>&1 || exit 3
timeout -k 10 200 python -u -m pytest -x -v --timeout 180 --timeout-method thread -s tests/test_gpu_anchors.py \
    > $O/pytest_anchors.txt 2>&1
rc=$?
timeout -k 10 960 python -u tools/anchors.py ac --seed 0 --max-seconds 840 --out $O/s0 > $O/ac_s0.log 2>&1 &
P1=$!
timeout -k 10 960 python -u tools/anchors.py ac --seed 1 --max-seconds 840 --out $O/s1 > $O/ac_s1.log 2>&1 &
P2=$!
for p in $P1 $P2; do wait $p || rc=$?; done
exit $rc
