# Times bench.py (table path, RHS only) against each library variant in tools/bin/var.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out/var
for so in tools/bin/var/*.so; do
  n=$(basename $so .so)
  KANODE_LIB=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-vjp --steps 200 > gpurun_out/var/$n.json || exit 3
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var/$n.json')); print('$n', round(d['ms_per_step']*1e3,1), 'us/step', round(d['roofline']['kernel_ms']*1e3,1), 'us kern', '%.3e'%d['value'])"
done
