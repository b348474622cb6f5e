#!/bin/bash
# LV1 iteration breakdown + concurrent loss_test variant; LV4096 training leg with the folded stops; the fsens,
# anchor and fused-chain tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_e; mkdir -p $O
timeout -k 10 180 python3 -u tools/lv1_probe.py --reps 50 --rounds 5 > $O/lv1_probe.json 2> $O/lv1_probe.err || { tail -5 $O/lv1_probe.err; exit 3; }
cat $O/lv1_probe.json
timeout -k 10 180 python3 -u tools/prof_lv4096.py --reps 10 > $O/lv4096.json 2> $O/lv4096.err || { tail -5 $O/lv4096.err; exit 3; }
cat $O/lv4096.json
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_fsens.py tests/test_gpu_anchors.py tests/test_gpu_native_solve.py -k "fsens or forward_sens or anchors or fisher_kpp_source or lotka or fused_chain or lv4096" > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
grep -E "deviations|loss_train at 2e4" $O/pytest.txt || true
exit $rc
