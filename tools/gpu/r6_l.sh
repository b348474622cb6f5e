#!/bin/bash
# phases of the table build (clock-probe build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_l; mkdir -p $O
KANODE_LIB=$PWD/tools/bin/var/clock.so timeout -k 10 300 python3 -u tools/clock_probe.py > $O/clock_phases.json 2> $O/clock_phases.err || { tail -5 $O/clock_phases.err; exit 3; }
cat $O/clock_phases.json
