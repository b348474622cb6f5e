#!/bin/bash
# the negative-state adaptive case on the pre-fix table build (tools/bin/var/prefix.so) and on the working build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_zc; mkdir -p $O
KANODE_LIB=$PWD/tools/bin/var/prefix.so timeout -k 10 200 python3 -u tools/negvar_probe.py 2>&1 | grep -E "OK|FAIL" | sed "s/^/prefix /" | tee $O/variants.txt
timeout -k 10 200 python3 -u tools/negvar_probe.py 2>&1 | grep -E "OK|FAIL" | sed "s/^/fixed /" | tee -a $O/variants.txt
