#!/usr/bin/env bash
# Rows adjoint-step variants: epoch A/B in alternating processes + cross-library gradient check.
#   tools/gpu_rows_ab.sh OUT ROUNDS BATCH lib1.so lib2.so ...   ("base" = kan-odes_amd/kanode/libkanode.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=$1; rounds=$2; batch=$3; shift 3
mkdir -p gpurun_out/grad
for r in $(seq 1 $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    n=$(basename $l .so)
    KANODE_LIB=$PWD/$lib timeout -k 10 120 python -u tools/epoch_ab.py --batch $batch --rounds 1 --reps 4 \
      --variants "adj_step_rows=1" --dump-grad gpurun_out/grad/$n.npy 2>&1 | grep median | sed "s|^|$l |" >> $out || exit 3
  done
done
python3 - "$@" <<'P' >> $out
import sys, os, numpy as np
names = [os.path.basename(l).replace(".so", "") for l in sys.argv[1:]]
ref = np.load(f"gpurun_out/grad/{names[0]}.npy")
for n in names:
    g = np.load(f"gpurun_out/grad/{n}.npy")
    print(f"{n}: gradient bitwise equal to {names[0]}: {bool(np.array_equal(g, ref))}, max rel diff "
          f"{np.max(np.abs(g - ref)) / np.max(np.abs(ref)):.2e}")
P
cat $out
