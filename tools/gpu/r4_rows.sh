#!/bin/bash
# Round 4: the one-wave rows adjoint step with the table size compiled in (NI) and λs formed before the
# reloaded dense output is used (LAMFIRST): tests, then alternating-process A/B on the adaptive epoch
# (base = both, rows_ni = NI only, rows_orig = neither, rows_r2 = base + two knot power chains), then a kernel trace of the base.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/rows
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "tests/test_gpu_native_solve.py::test_adjoint_step_rows_kernel_matches_persistent_grid" \
    tests/test_gpu_fk_e2e.py > $O/pytest_rows.txt 2>&1 || exit 3
for r in 1 2 3; do
  for l in base rows_ni rows_orig rows_r2; do
    lib=kan-odes_amd/kanode/libkanode.so; [ $l != base ] && lib=tools/bin/var/$l.so
    KANODE_LIB=$R/$lib timeout -k 10 120 python -u tools/epoch_adaptive_ab.py --rounds 1 --reps 3 \
        --variants "adj_step_rows=1" 2>&1 | grep median_ms | sed "s|^|$l |" >> $O/ab_rows.txt || exit 3
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $O/kt.log 2>&1 &&
rm -f $O/kt/*kernel_trace.csv $O/kt/*agent_info.csv
