#!/bin/bash
# Skipped unchanged uploads + counters in mapped memory: the GPU suite, then LV1 A/B against the previous library
set -e
O=gpurun_out/r6_zg
mkdir -p $O
[ -n "$SKIP_PYTEST" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for r in 1 2 3; do
  KANODE_LIB=$PWD/tools/bin/var/libkanode_base.so timeout -k 10 120 python3 -u tools/lv1_probe.py --reps 100 --rounds 3 > $O/base_$r.json 2>&1
  timeout -k 10 120 python3 -u tools/lv1_probe.py --reps 100 --rounds 3 > $O/new_$r.json 2>&1
done
timeout -k 10 240 python3 -u tools/lv1_iter_cprofile.py --reps 300 > $O/cprofile_new.txt 2>&1
[ -z "$WITH_BENCH" ] || timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
