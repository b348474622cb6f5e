#!/bin/bash
# in-kernel clock probe (diagnostic build), FK seed 0 run longer, then the whole GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_d; mkdir -p $O
KANODE_LIB=$PWD/tools/bin/var/clock.so timeout -k 10 300 python3 -u tools/clock_probe.py > $O/clock_probe.json 2> $O/clock_probe.err || { tail -5 $O/clock_probe.err; exit 3; }
cat $O/clock_probe.json
timeout -k 10 240 python3 -u tools/anchors.py fk --seed 0 --iters 40000 --log-every 1000 --out $O || exit 3
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?
tail -2 $O/pytest_gpu.txt
grep -E "^FAILED|^ERROR" $O/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/pytest_gpu.txt; exit 3; fi
grep -E "deviations|loss_train at 2e4" $O/pytest_gpu.txt || true
