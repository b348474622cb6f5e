#!/bin/bash
# Round 4: the saveat values of a Tsit5 step in one launch: the whole -m gpu suite, then the surrogate
# training iterations (bench legs) and the Burgers persistent-adjoint A/B line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/saveat
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1
[ $? -le 1 ] || exit 3
timeout -k 10 200 python -u tools/pair_persist_ab.py burgers512 0 3 > $O/burgers_ab.txt 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_surrogate_train.py --case burgers512 --reps 2 > $O/kt.log 2>&1
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
