#!/bin/bash
# forward step kernel at 4 waves/SIMD (one dispatch round at 4096 rows): epoch A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r3b9; mkdir -p $O
for r in 1 2 3; do
  for l in base tools/bin/var/fwpe4.so; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    KANODE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/train_time.py $(basename $l .so) --no-surrogates >> $O/train.txt 2>&1 || exit 3
  done
done
grep -v amdgpu.ids $O/train.txt | sort -k2,2 -k1,1
