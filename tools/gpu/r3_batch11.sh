#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b11; mkdir -p $O
bash tools/gpu/vjp_ab.sh $O/vjp.txt 2 base tools/bin/var/mv16.so tools/bin/var/mv24.so || exit 3
for l in base tools/bin/var/mv16.so tools/bin/var/mv24.so; do
  lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
  KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/train_time.py $(basename $l .so) --no-epoch >> $O/train.txt 2>&1 || exit 3
done
grep -v amdgpu.ids $O/train.txt
