#!/usr/bin/env bash
# Stall attribution of the adaptive reference-problem epoch (bench.py's epoch_adaptive leg): one --pmc
# pass per run (≤ 8 SQ, ≤ 2 GRBM counters each), kernel trace only, then the cross-pass summary.
#   bash tools/gpu/r4_pmc.sh [tag]
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/r4/pmc_${1:-adaptive}; mkdir -p $OUT
run() { # $1 = name, rest = counters
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$n -o run --output-format csv -- \
     python3 tools/prof_epoch_adaptive.py --batch 4096 --reps 1 > $OUT/$n.log 2>&1 || { echo "pass $n failed rc=$?"; tail -5 $OUT/$n.log; exit 3; }
  echo "pass $n ok"
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run p2 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run p3 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA
run p4 SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVES
python3 tools/pmc_stall.py $OUT > $OUT/stall_summary.txt && grep -A14 "fk_vjp_step_rows_kernel" $OUT/stall_summary.txt
rm -rf $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4   # the per-dispatch CSVs are tens of MB; the summary is what is kept
