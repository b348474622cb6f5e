#!/bin/bash
# Adaptive epoch kernel traces at smaller batches (dense-output footprint experiment).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for B in 1024 2048; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/epoch_adaptive_$B -o run -- python3 $R/tools/prof_epoch_adaptive.py \
      --batch $B > $O/epoch_adaptive_$B.log 2>&1 || exit 1
done
