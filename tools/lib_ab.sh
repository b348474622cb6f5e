#!/usr/bin/env bash
# Interleaved separate-process A/B of library variants on the epoch leg:
#   tools/lib_ab.sh OUT ROUNDS BATCH lib1.so lib2.so ...   ("base" = kan-odes_amd/kanode/libkanode.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=$1; rounds=$2; batch=$3; shift 3
for r in $(seq 1 $rounds); do
  for l in "$@"; do
    lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
    KANODE_LIB=$PWD/$lib timeout -k 10 120 python -u tools/epoch_ab.py --batch $batch --rounds 1 --reps 4 --variants "adj_step_rows=1" 2>&1 | grep median | sed "s|^|$l |" >> $out || exit 3
  done
done
cat $out
