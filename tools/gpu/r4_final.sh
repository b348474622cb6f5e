#!/bin/bash
# Round 4 evidence: the whole -m gpu suite, smoke, bench + rocprof kernel trace + PMC traffic
# (tools/profile_round.sh, TAG r04), then the self-spawned 2-rank gloo rehearsal of the multi-GPU legs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=r04 bash tools/profile_round.sh || exit 3
mkdir -p gpurun_out/r4/dist
timeout -k 10 500 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --batch-total 131072 \
    --no-epoch-adaptive > gpurun_out/r4/dist/bench_gpus2_gloo_final.json 2> gpurun_out/r4/dist/bench_gpus2_final.err
