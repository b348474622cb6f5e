#!/bin/bash
# Round 5: where the stage-parallel Lotka-Volterra adjoint's time goes (per-attempt time of the default, the
# one-wave kernel, and the timing-only variants: no in-loop stage evaluations / fp32 controller powers), and
# the LV1 iteration's host phases.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/lvp
mkdir -p $O
cd $R && export TMPDIR=/tmp
for v in base old noph1 fastpow; do
  if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
  timeout -k 10 120 python -u tools/lv_adj_probe.py --reps 30 > $O/probe_$v.json 2> $O/probe_$v.err || exit 3
done
unset KANODE_LIB
timeout -k 10 200 python -u tools/lv1_host_profile.py --reps 50 > $O/host_profile.txt 2>&1 || exit 3
echo ok
