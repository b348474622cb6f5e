#!/bin/bash
# Round 5 A/B driver: the whole -m gpu suite on the default library, then kernel traces of the adaptive
# reference-problem epoch (and the fixed-step epoch) for each library given, interleaved ROUNDS times.
#   tools/gpu/r5_ab.sh OUTNAME ROUNDS lib1 lib2 ...   ("base" = kan-odes_amd/kanode/libkanode.so,
#                                                       NAME = tools/bin/var/NAME.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/$1
rounds=$2
shift 2
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ad_${v}_$r -o run -- \
        python3 tools/prof_epoch_adaptive.py > $O/ad_${v}_$r.log 2>&1 || exit 3
    rm -f $O/ad_${v}_$r/*kernel_trace.csv $O/ad_${v}_$r/*agent_info.csv
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fx_${v}_$r -o run -- \
        python3 tools/prof_epoch.py --batch 4096 --reps 3 > $O/fx_${v}_$r.log 2>&1 || exit 3
    rm -f $O/fx_${v}_$r/*kernel_trace.csv $O/fx_${v}_$r/*agent_info.csv
  done
done
unset KANODE_LIB
echo ok
