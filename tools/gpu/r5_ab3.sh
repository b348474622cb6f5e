#!/bin/bash
# Round 5: the whole -m gpu suite on the default library (one-workgroup Fisher-KPP path, refactored small-chain
# drivers), the small-chain solve + adjoint bitwise against the round-4 library, then the rows-kernel A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/ab3
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/onewg_dump.py $O/onewg_base.npz > $O/onewg_base.log 2>&1 || exit 3
KANODE_LIB=$R/tools/bin/var/r4.so timeout -k 10 120 python -u tools/onewg_dump.py $O/onewg_r4.npz > $O/onewg_r4.log 2>&1 || exit 3
python -c "
import numpy as np; a=np.load('$O/onewg_base.npz'); b=np.load('$O/onewg_r4.npz')
print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})" > $O/onewg_bitwise.txt 2>&1
for r in 1 2; do
  for v in base l2load nosb; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ad_${v}_$r -o run -- \
        python3 tools/prof_epoch_adaptive.py > $O/ad_${v}_$r.log 2>&1 || exit 3
    rm -f $O/ad_${v}_$r/*kernel_trace.csv $O/ad_${v}_$r/*agent_info.csv
  done
done
unset KANODE_LIB
echo ok
