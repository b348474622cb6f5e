set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_pp.py tests/test_gpu_fk.py -x -q > gpurun_out/vjp_tests.log 2>&1; rc=$?
tail -15 gpurun_out/vjp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/vjp_bench.json || exit 3
python3 -c "import json; d=json.load(open('gpurun_out/vjp_bench.json')); print('rhs us', round(d['roofline']['kernel_ms']*1e3,1), 'vjp us', round(d['vjp']['ms_per_step']*1e3,1))"
bash tools/gpu_vjp_prof.sh
