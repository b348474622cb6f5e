set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_pp.py tests/test_gpu_fk.py tests/test_gpu_ode.py -x -q > gpurun_out/pp_tests.log 2>&1; rc=$?
tail -5 gpurun_out/pp_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/pp_variants.sh
