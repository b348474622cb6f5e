#!/usr/bin/env bash
# Ablation timing of the surrogate pair pullback: tools/bin/var/abl{1..7}.so (built here by
# tools/build_var.sh NAME "-DKAN_ABL=n" kan_wide.hip) against the product library; results of the
# variants are wrong by construction, only their times are read.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ablate; mkdir -p $O
timeout -k 10 120 python -u tools/surr_vjp_time.py base > $O/times.txt 2>&1 || exit 3
for v in "$@"; do
  KANODE_LIB=$PWD/tools/bin/var/$v.so timeout -k 10 120 python -u tools/surr_vjp_time.py $v >> $O/times.txt 2>&1 || exit 3
done
timeout -k 10 120 python -u tools/surr_vjp_time.py base >> $O/times.txt 2>&1 || exit 3
grep -v amdgpu.ids $O/times.txt
