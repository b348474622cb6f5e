#!/bin/bash
# The whole -m gpu suite, the default bench line, the surrogate A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3prof
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u tools/surr_pair_ab.py > $O/surr_pair_ab.txt 2>&1
