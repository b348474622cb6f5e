#!/usr/bin/env bash
# Interleaved A/B (separate processes, same box) of a cache-policy variant of the step kernels:
# libkanode.so vs libkanode$VAR.so (built with the experiment's -D flag), on the epoch leg.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out; mkdir -p $OUT
VAR=${VAR:-_keep}
for r in 1 2 3; do
  for v in "" $VAR; do
    echo "== round $r lib$v"
    KANODE_LIB=kan-odes_amd/kanode/libkanode$v.so timeout -k 10 120 python3 -u tools/vstep_grid_ab.py --grids 0 --rounds 3 || exit $?
  done
done
