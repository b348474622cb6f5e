set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out/grid
for g in 0 768 1024 1536 2048; do
  timeout -k 10 180 python bench.py --grid-rhs $g --no-cpu-baseline --no-vjp --steps 200 > gpurun_out/grid/g$g.json || exit 3
  python3 -c "import json; d=json.load(open('gpurun_out/grid/g$g.json')); print('grid $g', round(d['ms_per_step']*1e3,1), 'us/step', round(d['roofline']['kernel_ms']*1e3,1), 'us kern')"
done
