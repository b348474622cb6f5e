#!/bin/bash
# The reference's recorded training runs through the product path (tools/anchors.py), the Fisher-KPP
# source at its N_iter = 2e4 for three initialisations and Lotka-Volterra at N_iter = 1e5, as concurrent
# processes on the one GPU (each is a chain of small launches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/anchors_full
mkdir -p $O/s0 $O/s1 $O/s2 $O/lv
timeout -k 10 900 python -u tools/anchors.py fk --seed 0 --out $O/s0 > $O/fk_s0.log 2>&1 &
P1=$!
timeout -k 10 900 python -u tools/anchors.py fk --seed 1 --out $O/s1 > $O/fk_s1.log 2>&1 &
P2=$!
timeout -k 10 900 python -u tools/anchors.py fk --seed 2 --out $O/s2 > $O/fk_s2.log 2>&1 &
P3=$!
timeout -k 10 900 python -u tools/anchors.py lv --seed 0 --out $O/lv > $O/lv.log 2>&1 &
P4=$!
rc=0
for p in $P1 $P2 $P3 $P4; do wait $p || rc=$?; done
exit $rc
