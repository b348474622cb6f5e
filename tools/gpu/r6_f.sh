#!/bin/bash
# phases of the device-controlled loops' finish and forward kernels (clock-probe build); kernel trace of the LV1
# iteration probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_f; mkdir -p $O
KANODE_LIB=$PWD/tools/bin/var/clock.so timeout -k 10 300 python3 -u tools/clock_probe.py > $O/clock_phases.json 2> $O/clock_phases.err || { tail -5 $O/clock_phases.err; exit 3; }
cat $O/clock_phases.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lv1prof -o lv1 -- python3 -u tools/lv1_probe.py --reps 20 --rounds 2 > $O/lv1prof.log 2>&1 || { tail -20 $O/lv1prof.log; exit 3; }
tail -2 $O/lv1prof.log
find $O/lv1prof -name "*kernel_stats.csv" | head -3
