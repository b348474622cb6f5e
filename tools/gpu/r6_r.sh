#!/bin/bash
# kernel trace of consecutive adaptive reference epochs under Adam(1e-2): which kernels slow down as p moves
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_r; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o drift -- python3 -u tools/epoch_drift.py 0.01 > $O/drift.txt 2>&1 || { tail -5 $O/drift.txt; exit 3; }
grep eta $O/drift.txt
