#!/bin/bash
# Kernel trace of the adaptive FK256 reference-problem epoch and of a Burgers training iteration.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/epoch_adaptive -o run -- python3 $R/tools/prof_epoch_adaptive.py \
    > $O/epoch_adaptive_prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/burgers -o run -- python3 $R/tools/prof_surrogate_train.py \
    --case burgers512 --reps 2 > $O/burgers_prof.log 2>&1
