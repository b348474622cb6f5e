#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=$PWD/gpurun_out/trace_bu; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/run -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_surrogate_train.py --case burgers512 --reps 2 > $O/log.txt 2>&1
