#!/bin/bash
# the all-negative adaptive case: adjoint step sizes on the table path and the direct kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_zd; mkdir -p $O
timeout -k 10 200 python3 -u tools/negvar_steps.py 2>&1 | tail -2 | tee $O/steps.json
