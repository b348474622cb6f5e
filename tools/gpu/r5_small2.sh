#!/bin/bash
# Round 5: -m gpu suite; reference-size iterations (LV1, FK26) timed, kernel-traced and API-traced; the rows
# kernel's next-round L2 prefetch (tools/bin/var/pf.so) against the default on the adaptive epoch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5/${1:-small2}
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/prof_small.py --reps 30 > $O/small_base.json 2> $O/small_base.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_small -o run -- \
    python3 tools/prof_small.py --reps 10 > $O/kt_small.log 2>&1 || exit 3
rm -f $O/kt_small/*kernel_trace.csv $O/kt_small/*agent_info.csv
timeout -k 10 200 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $O/api_fk26 -o run -- \
    python3 tools/prof_small.py --reps 10 --which fk26 > $O/api_fk26.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $O/api_lv1 -o run -- \
    python3 tools/prof_small.py --reps 10 --which lv1 > $O/api_lv1.log 2>&1 || exit 3
for r in 1 2; do
  for v in base pf; do
    if [ $v = base ]; then unset KANODE_LIB; else export KANODE_LIB=$R/tools/bin/var/$v.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ad_${v}_$r -o run -- \
        python3 tools/prof_epoch_adaptive.py > $O/ad_${v}_$r.log 2>&1 || exit 3
    rm -f $O/ad_${v}_$r/*kernel_trace.csv $O/ad_${v}_$r/*agent_info.csv
  done
done
unset KANODE_LIB
echo ok
