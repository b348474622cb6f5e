#!/usr/bin/env bash
# PMC passes for the FK RHS kernel (each --pmc pass separate; kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-r01}; mkdir -p $OUT
WHAT=${WHAT:-fk_rhs}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() { # $1 = name, rest = counters
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$n -o run --output-format csv -- \
     python3 tools/prof_kernel.py --what $WHAT --reps 10 > $OUT/$n.log 2>&1 || { echo "pass $n failed rc=$?"; tail -5 $OUT/$n.log; exit 3; }
  echo "pass $n ok"
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run p2 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run p3 FETCH_SIZE
run p4 WRITE_SIZE
run p5 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
