#!/bin/bash
# (diagnostic build) the table intervals whose points the VJP sends to the direct formula
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_x; mkdir -p $O
KANODE_LIB=$PWD/tools/bin/var/clock.so timeout -k 10 300 python3 -u tools/pp_direct_scan.py 2>&1 | tail -2 | tee $O/scan3.json
