#!/bin/bash
# Round 5: the one-wave LV adjoint and the device-controlled FK loops: native-solve GPU tests, the small-problem
# kernel trace (LV1 / FK26 epochs), the FK256 adaptive epoch A/B and its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/lv
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_native_solve.py tests/test_gpu_fk_e2e.py tests/test_gpu_anchors.py > $O/tests.txt 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_small -o run -- \
  python3 tools/prof_small.py --reps 10 > $O/kt_small.log 2>&1 || exit 3
rm -f $O/kt_small/*kernel_trace.csv $O/kt_small/*agent_info.csv
timeout -k 10 400 python -u tools/epoch_adaptive_ab.py --variants "fk_device_loop=1;fk_device_loop=0" --rounds 2 \
  --reps 2 > $O/ab.txt 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 tools/prof_epoch_adaptive.py --reps 2 > $O/kt.log 2>&1 || exit 3
python3 tools/trace_gaps.py $O/kt > $O/gaps.txt 2>&1 || true
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
echo ok
