#!/bin/bash
# Round 5 closing anchors on the final code (the one-workgroup drivers' exp2/log2 controller powers change the
# training trajectories at rounding level): Fisher-KPP source learning, three initialisations at the driver's 2e4
# iterations; Lotka-Volterra seed 1 at the driver's 1e5 iterations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/anchors_final
mkdir -p $O
cd $R
for s in 0 1 2; do
  timeout -k 10 300 python -u tools/anchors.py fk --seed $s --log-every 250 --out $O > $O/fk_seed$s.log 2>&1 || exit 3
done
for s in 1; do
  timeout -k 10 420 python -u tools/anchors.py lv --seed $s --log-every 500 --out $O > $O/lv_seed$s.log 2>&1 || exit 3
done
echo ok
