#!/bin/bash
# Round 4: the adjoint finish kernel at 1024 threads per block (one load per slab per thread) vs 256:
# kernel traces of the adaptive epoch with each library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/fin
mkdir -p $O
cd $R && export TMPDIR=/tmp
for l in base fin1024; do
  lib=kan-odes_amd/kanode/libkanode.so; [ $l != base ] && lib=tools/bin/var/$l.so
  KANODE_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$l -o run -- \
      python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $O/kt_$l.log 2>&1 || exit 3
  rm -f $O/kt_$l/*kernel_trace.csv $O/kt_$l/*agent_info.csv
done
