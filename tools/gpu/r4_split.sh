#!/bin/bash
# Round 4: the adaptive-epoch A/B over the rows modes of the adjoint step (1 one wave per row; 2 split,
# 768-thread blocks; 3 split, no deferred combinations; 4 split, 256-thread blocks), then the 1024-thread
# finish kernel (variant library) against the base in alternating processes, then a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/split
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/epoch_adaptive_ab.py --rounds 3 --reps 2 \
    --variants "adj_step_rows=1;adj_step_rows=2;adj_step_rows=3;adj_step_rows=4" > $O/ab_adaptive.txt 2>&1 || exit 3
for r in 1 2 3; do
  for l in base fin1024; do
    lib=kan-odes_amd/kanode/libkanode.so; [ $l = fin1024 ] && lib=tools/bin/var/fin1024.so
    KANODE_LIB=$R/$lib timeout -k 10 120 python -u tools/epoch_adaptive_ab.py --rounds 1 --reps 3 \
        --variants "adj_step_rows=2" 2>&1 | grep median_ms | sed "s|^|$l |" >> $O/ab_fin1024.txt || exit 3
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $O/kt.log 2>&1 &&
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
