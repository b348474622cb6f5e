#!/bin/bash
# Two ranks on one GPU over gloo: the multi-rank bench path (FK256 RHS, epoch with the gradient
# all-reduce, BU512 grid-sharded training, SC1024 data-parallel training) end to end.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3prof/dist
mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --batch-total 131072 \
    --no-epoch-adaptive > $O/bench_2ranks_gloo_one_gpu.json 2> $O/bench_2ranks.err
