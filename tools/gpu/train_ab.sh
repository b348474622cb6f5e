#!/bin/bash
# Interleaved separate-process A/B of library variants on the training legs (tools/train_time.py):
#   tools/gpu/train_ab.sh OUT ROUNDS base tools/bin/var/x.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=$1; rounds=$2; shift 2
mkdir -p $(dirname $out)
for r in $(seq 1 $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/train_time.py $(basename $l .so) >> $out 2>&1 || exit 3
  done
done
grep -v amdgpu.ids $out
