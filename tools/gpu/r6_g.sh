#!/bin/bash
# interleaved A/B of the adaptive epoch: HEAD's device-loop kernels (tools/bin/var/old.so) vs the controller inputs
# formed off the critical path (the working build); the device-loop tests on the working build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/r6_g; mkdir -p $O
for r in 1 2 3; do
  KANODE_LIB=$PWD/tools/bin/var/old.so timeout -k 10 120 python3 -u tools/epoch_adaptive_ab.py --variants "fk_device_loop=1" --rounds 1 --reps 3 2>&1 | grep round | sed "s/^/old /" | tee -a $O/ab.txt || exit 3
  timeout -k 10 120 python3 -u tools/epoch_adaptive_ab.py --variants "fk_device_loop=1" --rounds 1 --reps 3 2>&1 | grep round | sed "s/^/new /" | tee -a $O/ab.txt || exit 3
done
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_fk_e2e.py tests/test_gpu_native_solve.py -k "device_loop or fused_finish or e2e or fk" > $O/pytest.txt 2>&1
rc=$?
tail -2 $O/pytest.txt
grep -E "^FAILED|^ERROR" $O/pytest.txt
exit $rc
