#!/bin/bash
# Round 5 evidence, second part (the first is `TAG=r05 bash tools/profile_round.sh`: tests, smoke, bench, traces,
# PMC): the reference-size iterations' kernel trace (LV1 / FK26), the self-spawned 2-rank gloo rehearsal of the
# multi-GPU legs, and the adaptive epoch's device-vs-host step control A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && export TMPDIR=/tmp
mkdir -p gpurun_out/profile_r05
O=gpurun_out/profile_r05
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/small -o run -- \
  python3 tools/prof_small.py --reps 10 > $O/small.log 2>&1 || exit 3
cp $O/small/run_kernel_stats.csv $O/small_kernel_stats.csv
rm -rf $O/small
mkdir -p $O/dist
timeout -k 10 500 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --batch-total 131072 \
    --no-epoch-adaptive > $O/dist/bench_gpus2_gloo.json 2> $O/dist/bench_gpus2.err || exit 3
timeout -k 10 600 python -u tools/epoch_adaptive_ab.py --variants "fk_device_loop=1;fk_device_loop=0" --rounds 3 \
  --reps 2 > $O/epoch_adaptive_device_loop_ab.txt 2>&1 || exit 3
echo ok
