#!/usr/bin/env bash
# Copy the judged artefacts of one profile_round.sh run (gpurun_out/profile_TAG) into profiles/DEST.
set -eu
cd "$(dirname "$0")/.."
src=gpurun_out/profile_$1; dst=profiles/$2
mkdir -p $dst/pmc
for f in bench.json kernel_stats.csv epoch_kernel_stats.csv epoch_adaptive_kernel_stats.csv train_burgers512_kernel_stats.csv train_schrodinger1024_kernel_stats.csv pmc_summary.txt traffic.json pytest_gpu.log smoke.log; do
  [ -f $src/$f ] && cp $src/$f $dst/$f.tmp && mv $dst/$f.tmp $dst/$f
done
[ -f $dst/pytest_gpu.log ] && mv $dst/pytest_gpu.log $dst/pytest_gpu.txt
[ -f $dst/smoke.log ] && mv $dst/smoke.log $dst/smoke.txt
for d in $src/pmc_*/; do
  n=$(basename $d)
  c=$(ls $d/run_counter_collection.csv 2>/dev/null || true)
  [ -n "$c" ] && cp $c $dst/pmc/$n.csv
done
cp $src/traffic.json profiles/traffic.json
echo collected into $dst
