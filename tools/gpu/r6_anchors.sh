#!/bin/bash
# Round 6 anchors: the reference's recorded training outcomes through the product path, three initialisations
# each.  Fisher-KPP source (2e4 iterations, the reference's ForwardDiffSensitivity gradient),
# Lotka-Volterra (1e5 iterations, InterpolatingAdjoint), Allen-Cahn source (5e4).  JSONs -> gpurun_out/anchors_r6/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/anchors_r6; mkdir -p $O
for s in 0 1 2; do
  timeout -k 10 240 python3 -u tools/anchors.py fk --seed $s --log-every 250 --out $O || exit 3
done
for s in 0 1 2; do
  timeout -k 10 300 python3 -u tools/anchors.py lv --seed $s --log-every 500 --out $O || exit 3
done
for s in 0 1; do
  timeout -k 10 300 python3 -u tools/anchors.py ac --seed $s --log-every 500 --out $O --max-seconds 240 || exit 3
done
