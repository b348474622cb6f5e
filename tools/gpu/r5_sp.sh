#!/bin/bash
# Round 5: the stage-parallel one-trajectory adjoints (fk_small_adjoint_sp_kernel, kd_chain_adjoint_lvsp_kernel)
# against the previous kernels (tools/bin/var/old.so: KAN_SMALL_SP=0, KAN_LV_SP=0): tests, FK26 / LV1 timing,
# kernel traces, and the Fisher-KPP / Lotka-Volterra anchors at the drivers' iteration counts.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/sp2
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_native_solve.py \
    -m gpu > $O/pytest.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in base old; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 200 python -u tools/prof_small.py --reps 50 > $O/small_${v}_$r.json 2> $O/small_${v}_$r.err || exit 3
  done
done
for v in base old; do
  if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- \
      python3 tools/prof_small.py --reps 10 > $O/kt_$v.log 2>&1 || exit 3
  rm -f $O/kt_$v/*kernel_trace.csv $O/kt_$v/*agent_info.csv
done
unset KANODE_LIB
for s in 1 2; do
  timeout -k 10 300 python -u tools/anchors.py fk --seed $s --log-every 250 --out $O/anchors > $O/fk_seed$s.log 2>&1 || exit 3
done
timeout -k 10 420 python -u tools/anchors.py lv --seed 1 --log-every 500 --out $O/anchors > $O/lv_seed1.log 2>&1 || exit 3
echo ok
