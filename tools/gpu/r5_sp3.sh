#!/bin/bash
# Round 5: the stage-parallel Lotka-Volterra adjoint with the coefficients read from LDS (no register copy)
# against the one-wave kernel (tools/bin/var/old.so): native-solve tests, LV1 timing and kernel traces.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/sp3
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_native_solve.py \
    -m gpu > $O/pytest.txt 2>&1 || exit 3
for r in 1 2 3; do
  for v in base old; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 200 python -u tools/prof_small.py --reps 100 --which lv1 > $O/small_${v}_$r.json 2> $O/small_${v}_$r.err || exit 3
  done
done
for v in base old; do
  if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- \
      python3 tools/prof_small.py --reps 10 --which lv1 > $O/kt_$v.log 2>&1 || exit 3
  rm -f $O/kt_$v/*kernel_trace.csv $O/kt_$v/*agent_info.csv
done
unset KANODE_LIB
echo ok
