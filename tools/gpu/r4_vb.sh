#!/bin/bash
# Round 4: 512-thread blocks for the VJP / adjoint step kernels (variant lib tools/bin/var/vb512.so, one
# block of 8 rows per CU, tables staged once per CU) against the default 256: targeted tests on the
# variant, then the adaptive epoch kernel traces and wall times of both libs, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/vb
mkdir -p $O
cd $R && export TMPDIR=/tmp
V=$R/tools/bin/var/vb512.so
KANODE_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_native_solve.py tests/test_gpu_fk_e2e.py -k "(rows_kernel and not batch_cap) or fused_finish or fk256 or e2e" > $O/tests_var.txt 2>&1 || exit 3
for r in 0 1; do
  for v in def var; do
    if [ $v = var ]; then export KANODE_LIB=$V; else unset KANODE_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${v}_$r -o run -- \
        python3 tools/prof_epoch_adaptive.py > $O/kt_${v}_$r.log 2>&1 || exit 3
    rm -f $O/kt_${v}_$r/*kernel_trace.csv $O/kt_${v}_$r/*agent_info.csv
    timeout -k 10 300 python -u tools/epoch_adaptive_ab.py --variants "adj_fused_finish=0" --rounds 1 > $O/wall_${v}_$r.txt 2>&1 || exit 3
  done
done
unset KANODE_LIB
