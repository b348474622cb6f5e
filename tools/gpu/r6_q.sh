#!/bin/bash
# consecutive adaptive reference epochs with and without parameter updates
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_q; mkdir -p $O
timeout -k 10 300 python3 -u tools/epoch_drift.py 2>/dev/null | tee $O/drift.txt
