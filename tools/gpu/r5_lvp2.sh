#!/bin/bash
# Round 5: the stage-parallel LV adjoint with qold^β2 on a seventh wave, the fused mse_loss and the cached
# solve arguments: native-solve tests, probe and LV1 / FK26 timing against the one-wave kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/${1:-lvp2}
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_native_solve.py \
    tests/test_gpu_train.py -m gpu > $O/pytest.txt 2>&1 || exit 3
for v in base; do
  if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
  timeout -k 10 120 python -u tools/lv_adj_probe.py --reps 30 > $O/probe_$v.json 2> $O/probe_$v.err || exit 3
done
unset KANODE_LIB
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/prof_small.py --reps 100 > $O/small_$r.json 2> $O/small_$r.err || exit 3
done
timeout -k 10 200 python -u tools/lv1_host_profile.py --reps 50 > $O/host_profile.txt 2>&1 || exit 3
echo ok
