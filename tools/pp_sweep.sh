# Times bench.py's RHS step (table path) for every library variant in tools/bin/var
# at several persistent-grid sizes (bench.py --grid-rhs = KANODE_OPT_GRID_RHS; 0 = the library default).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
GRIDS=${GRIDS:-0 1536 1792}
for so in tools/bin/var/*.so; do
  n=$(basename $so .so)
  for g in $GRIDS; do
    KANODE_LIB=$PWD/$so timeout -k 10 180 python bench.py --grid-rhs $g --no-cpu-baseline --no-vjp --no-epoch \
      --steps ${STEPS:-60} ${BENCH_ARGS:-} > gpurun_out/sweep/${n}_g$g.json || exit 3
    python3 -c "import json; d=json.load(open('gpurun_out/sweep/${n}_g$g.json')); r=d['roofline']; print('$n grid $g', round(r['kernel_ms']*1e3,1), 'us/step', round(r['achieved']), 'GB/s', round(r['frac'],3))"
  done
done
