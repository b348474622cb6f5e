#!/bin/bash
# the driver's round-end commands on the committed tree: GPU tests, smoke, default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/final; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1 || { tail -20 $O/pytest_gpu.txt; exit 3; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 3; }
tail -1 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['roofline']['frac'], d['epoch_adaptive']['gpu'], d['surrogates']['burgers512']['train_iteration_ms'])"
