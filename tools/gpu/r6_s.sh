#!/bin/bash
# the VJP's dependence on p and on the states (epoch slowdown under training)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_s; mkdir -p $O
timeout -k 10 300 python3 -u tools/vjp_drift.py 2>/dev/null | tee $O/vjp_drift.json
