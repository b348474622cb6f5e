#!/bin/bash
# Round 4: host-sync census of the grid-sharded adjoint (HIP runtime + copy trace, no counters), then
# the PMC stall attribution of the adaptive epoch (tools/gpu/r4_pmc.sh, one counter pass per run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/sync
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- \
    python3 tools/tp_sync_trace.py --iters 2 --out $O/tp_sync_stats.json > $O/trace.log 2>&1 &&
python3 tools/hip_sync_count.py $O/trace $O/tp_sync_stats.json > $O/tp_sync_census.json &&
rm -rf $O/trace &&
bash tools/gpu/r4_pmc.sh adaptive
