#!/bin/bash
# the VJP drift probe on the diagnostic build: how many points take the direct formula
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_w; mkdir -p $O
KANODE_LIB=$PWD/tools/bin/var/clock.so timeout -k 10 300 python3 -u tools/vjp_drift.py --count 2>&1 | tail -3 | tee $O/vjp_drift_count.json
