#!/bin/bash
# Round 5: the forward step at 4 waves/SIMD (fwpe4.so: KAN_FSTEP_WPE=4, <= 128 VGPRs, so 4,096 rows are ONE
# dispatch round instead of 1.33) against the default, adaptive epoch kernel traces and epoch times, both
# step controls.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/fwpe
mkdir -p $O
cd $R && export TMPDIR=/tmp
for r in 1 2; do
  for v in base fwpe4; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${v}_$r -o run -- \
        python3 tools/prof_epoch_adaptive.py > $O/kt_${v}_$r.log 2>&1 || exit 3
    rm -f $O/kt_${v}_$r/*kernel_trace.csv $O/kt_${v}_$r/*agent_info.csv
    timeout -k 10 300 python -u tools/epoch_adaptive_ab.py --variants "fk_device_loop=1;fk_device_loop=0" \
        --rounds 1 --reps 2 > $O/ab_${v}_$r.txt 2>&1 || exit 3
  done
done
unset KANODE_LIB
echo ok
