#!/bin/bash
# Round 5 anchors on the one-workgroup reference-size paths: Fisher-KPP source learning, three
# initialisations at the driver's 2e4 iterations with the learned source's deviation from the recorded fit
# logged every 250 iterations; Lotka-Volterra seeds 1 and 2 at the driver's 1e5 iterations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/anchors
mkdir -p $O
cd $R
for s in 0 1 2; do
  timeout -k 10 300 python -u tools/anchors.py fk --seed $s --log-every 250 --out $O > $O/fk_seed$s.log 2>&1 || exit 3
done
for s in 1 2; do
  timeout -k 10 420 python -u tools/anchors.py lv --seed $s --log-every 500 --out $O > $O/lv_seed$s.log 2>&1 || exit 3
done
echo ok
