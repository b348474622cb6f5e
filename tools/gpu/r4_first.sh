#!/bin/bash
# Round 4, first GPU call: the persistent pair adjoint (tests, then A/B), anchor-training probes, the
# self-spawned 2-rank bench (gloo, one GPU) and the GPU tests touched this round.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4
mkdir -p $O/anchors $O/dist
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    "tests/test_gpu_native_solve.py::test_persistent_pair_adjoint_matches_launch_path" > $O/pytest_persist.txt 2>&1 &&
timeout -k 10 200 python -u tools/pair_persist_ab.py burgers512 0 3 > $O/persist_ab.txt 2>&1 &&
timeout -k 10 240 python -u tools/anchors.py fk --iters 2000 --out $O/anchors > $O/anchors/fk_probe.log 2>&1 &&
timeout -k 10 200 python -u tools/anchors.py lv --iters 2000 --out $O/anchors > $O/anchors/lv_probe.log 2>&1 &&
timeout -k 10 200 python -u tools/anchors.py ac --iters 300 --out $O/anchors > $O/anchors/ac_probe.log 2>&1 &&
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tp.py \
    tests/test_gpu_train.py "tests/test_gpu_native_solve.py::test_failed_adjoint_leaves_no_pending_stage" \
    "tests/test_gpu_native_solve.py::test_full_size_surrogate_adjoint_matches_cpu_oracle" -s \
    > $O/pytest_touched.txt 2>&1 &&
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --batch-total 131072 \
    --no-epoch-adaptive > $O/dist/bench_gpus2_gloo_selfspawn.json 2> $O/dist/bench_gpus2.err
