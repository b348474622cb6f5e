#!/bin/bash
# Round 4: the short anchor test, then the Allen-Cahn source anchor (N_iter = 5e4 at ~14 ms per iteration),
# two initialisations side by side, each stopping at its time budget if the call's limit comes first.
# Results: profiles/r04/anchors/ac_seed*.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/anchors_ac
mkdir -p $O/s0 $O/s1
timeout -k 10 200 python -u -m pytest -x -v --timeout 180 --timeout-method thread -s tests/test_gpu_anchors.py \
    > $O/pytest_anchors.txt 2>&1
rc=$?
timeout -k 10 960 python -u tools/anchors.py ac --seed 0 --max-seconds 840 --out $O/s0 > $O/ac_s0.log 2>&1 &
P1=$!
timeout -k 10 960 python -u tools/anchors.py ac --seed 1 --max-seconds 840 --out $O/s1 > $O/ac_s1.log 2>&1 &
P2=$!
for p in $P1 $P2; do wait $p || rc=$?; done
exit $rc
