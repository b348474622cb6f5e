#!/bin/bash
# Round 4: grid of the one-launch forward Tsit5 step (KANODE_OPT_GRID_RHS) on the adaptive epoch:
# 0 = occupancy cap (768 blocks = 3,072 waves: 1.33 rows per wave at 4,096 rows), 512 (2 rows per wave),
# 1024 (one row per wave, 1.33 dispatch rounds), 342 (3 rows per wave).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/fgrid
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 500 python -u tools/epoch_adaptive_ab.py --rounds 3 --reps 2 \
    --variants "grid_rhs=0;grid_rhs=512;grid_rhs=1024;grid_rhs=342" > $O/ab.txt 2>&1
