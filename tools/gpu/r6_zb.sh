#!/bin/bash
# table path vs the direct per-point kernels over negative and positive states
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_zb; mkdir -p $O
timeout -k 10 200 python3 -u tools/table_vs_direct.py 2>&1 | tail -3 | tee $O/table_vs_direct.txt
