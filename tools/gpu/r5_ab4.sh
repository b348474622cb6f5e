#!/bin/bash
# Round 5: the rows kernel's LDS-column combination sums (ldsred.so; pfred.so = with the next-round prefetch):
# targeted tests on the variant, then the adaptive epoch A/B; and the one-workgroup adjoints with the model's
# pullback removed (novjp.so: the drivers alone) against the default, kernel-traced.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/ab4
mkdir -p $O
cd $R && export TMPDIR=/tmp
KANODE_LIB=$R/tools/bin/var/ldsred.so timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
    tests/test_gpu_native_solve.py tests/test_gpu_fk_e2e.py -k "rows_kernel or fused_finish or fk256 or e2e or fk_" \
    > $O/tests_ldsred.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in base ldsred pfred; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ad_${v}_$r -o run -- \
        python3 tools/prof_epoch_adaptive.py > $O/ad_${v}_$r.log 2>&1 || exit 3
    rm -f $O/ad_${v}_$r/*kernel_trace.csv $O/ad_${v}_$r/*agent_info.csv
  done
done
for v in base novjp; do
  if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_small_$v -o run -- \
      python3 tools/prof_small.py --reps 10 > $O/kt_small_$v.log 2>&1 || exit 3
  rm -f $O/kt_small_$v/*kernel_trace.csv $O/kt_small_$v/*agent_info.csv
done
unset KANODE_LIB
echo ok
