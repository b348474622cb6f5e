#!/bin/bash
# kernel trace (csv) of the adaptive FK256 reference-problem epoch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=$PWD/gpurun_out/trace_ea; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/run -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_epoch_adaptive.py > $O/log.txt 2>&1
