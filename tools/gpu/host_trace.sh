#!/bin/bash
# HIP API + kernel trace of one Burgers training iteration: host time per adjoint stage vs GPU time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=$PWD/gpurun_out/host_trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/burgers -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_surrogate_train.py --case burgers512 --reps 1 > $O/burgers.log 2>&1
