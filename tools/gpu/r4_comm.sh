#!/bin/bash
# Round 4: the C-ABI communicator (kanode_comm_*): its GPU tests, then two ranks on this box's GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/comm
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_comm.py > $O/pytest.txt 2>&1 || exit 3
timeout -k 10 300 python -u tools/comm_two_ranks.py > $O/two_ranks.txt 2>&1
echo "two ranks rc $?" >> $O/two_ranks.txt
