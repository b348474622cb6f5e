#!/bin/bash
# Round 5: the one-workgroup drivers' controller powers as exp2(y·log2 x) (tools/bin/var/owpow.so) against pow:
# kernel traces of the reference-size iterations (FK26, LV1), interleaved twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/powab
mkdir -p $O
cd $R && export TMPDIR=/tmp
for r in 1 2; do
  for v in base owpow; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${v}_$r -o run -- \
        python3 tools/prof_small.py --reps 20 > $O/kt_${v}_$r.log 2>&1 || exit 3
    rm -f $O/kt_${v}_$r/*kernel_trace.csv $O/kt_${v}_$r/*agent_info.csv
  done
done
unset KANODE_LIB
echo ok
