#!/bin/bash
# Round 6: targeted GPU tests (PYTEST_ARGS, default the new ones) + the lv4096 training trace + a plain bench leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_quick; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-tests/test_gpu_fsens.py tests/test_gpu_train.py tests/test_gpu_native_solve.py -k "fused_chain_adjoint_step or lv4096 or fsens or forward or eval_loss or trainer"} > $O/pytest.txt 2>&1
rc=$?
tail -3 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then tail -30 $O/pytest.txt; exit 3; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/lv4096 -o run --output-format csv -- \
  python3 tools/prof_lv4096.py --reps 5 > $O/lv4096.json 2> $O/lv4096.err || { tail -5 $O/lv4096.err; exit 3; }
cat $O/lv4096.json
python3 tools/kstats_by_grid.py $O/lv4096/run_kernel_trace.csv > $O/lv4096_by_grid.txt
head -8 $O/lv4096_by_grid.txt | cut -c1-170
timeout -k 10 120 python3 tools/prof_lv4096.py --reps 10 > $O/lv4096_plain.json && cat $O/lv4096_plain.json
rm -rf $O/lv4096
