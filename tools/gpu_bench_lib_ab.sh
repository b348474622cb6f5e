#!/usr/bin/env bash
# bench.py's RHS leg (table rebuilt every step) over library variants, alternating processes:
#   tools/gpu_bench_lib_ab.sh OUT ROUNDS "BATCHES" lib1.so lib2.so ...  ("base" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=$1; rounds=$2; batches=$3; shift 3
for r in $(seq 1 $rounds); do for b in $batches; do for l in "$@"; do
  lib=$l; [ "$l" = base ] && lib=kan-odes_amd/kanode/libkanode.so
  KANODE_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-vjp --no-epoch --steps 100 \
    --batch-total $b > gpurun_out/ab_bench.json 2>/dev/null || exit 3
  python3 -c "import json; d=json.load(open('gpurun_out/ab_bench.json')); print('$l', $b, round(d['ms_per_step']*1e3,1), 'us/step', round(d['roofline']['kernel_ms']*1e3,1), 'us event', '%.3e' % d['value'])" >> $out
done; done; done
cat $out
