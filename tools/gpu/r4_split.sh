#!/bin/bash
# Round 4: the split-row adjoint step (two waves per 256-point row) — tests, then the adaptive epoch A/B
# over the rows modes (1 one wave per row; 2 split, 768-thread blocks; 3 split, no deferred combinations;
# 4 split, 256-thread blocks) and a kernel-trace of mode 2 vs 1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/split
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "tests/test_gpu_native_solve.py::test_adjoint_step_split_rows_matches_one_wave_rows" \
    "tests/test_gpu_native_solve.py::test_adjoint_step_rows_kernel_matches_persistent_grid" \
    tests/test_gpu_fk_e2e.py > $O/pytest_split.txt 2>&1 &&
timeout -k 10 400 python -u tools/epoch_adaptive_ab.py --rounds 3 --reps 2 \
    --variants "adj_step_rows=1;adj_step_rows=2;adj_step_rows=3;adj_step_rows=4" > $O/ab_adaptive.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $O/kt.log 2>&1 &&
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
