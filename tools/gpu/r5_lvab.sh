#!/bin/bash
# Round 5: interleaved A/B of the stage-parallel LV adjoint's register variants (per-attempt probe):
# base (opaque lane + LDS tableau), opq (opaque lane only), prev (neither).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/lvab
mkdir -p $O
cd $R && export TMPDIR=/tmp
for r in 1 2 3; do
  for v in base opq prev; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 120 python -u tools/lv_adj_probe.py --reps 50 > $O/probe_${v}_$r.json 2> $O/probe_${v}_$r.err || exit 3
  done
done
unset KANODE_LIB
echo ok
