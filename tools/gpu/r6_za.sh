#!/bin/bash
# the negative-state adaptive case under path options (device loop, tables, fused step)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_za; mkdir -p $O
timeout -k 10 300 python3 -u tools/negvar_probe.py 2>&1 | tee $O/variants.txt
