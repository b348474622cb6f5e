#!/usr/bin/env bash
# Instruction-cache counters over the FK256 epoch (rows adjoint step, forward step, VJP).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/pmc_icache; mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*" $OUT/counters_list.txt | sort -u > $OUT/icache_counters.txt || true
cat $OUT/icache_counters.txt
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --kernel-trace -d $OUT/p1 -o run --output-format csv -- \
  python3 tools/prof_epoch.py --batch 4096 --reps 1 > $OUT/p1.log 2>&1 || { echo "pass failed rc=$?"; tail -5 $OUT/p1.log; exit 3; }
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
