set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_pp.py tests/test_gpu_fk.py -x -q > gpurun_out/pp_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pp_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/pp_grid.sh || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp4 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-vjp --steps 100 > gpurun_out/pp4.log 2>&1
