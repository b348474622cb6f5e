#!/usr/bin/env bash
# PMC passes over the FK256 training epoch (rows adjoint step, forward step): one --pmc pass per run.
#   LIB=path/to/libkanode.so TAG=name tools/pmc_epoch.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out/pmc_epoch_${TAG:-base}; mkdir -p $OUT
[ -n "${LIB:-}" ] && export KANODE_LIB=$PWD/$LIB
run() { # $1 = name, rest = counters
  local n=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$n -o run --output-format csv -- \
     python3 tools/prof_epoch.py --batch 4096 --reps 1 > $OUT/$n.log 2>&1 || { echo "pass $n failed rc=$?"; tail -5 $OUT/$n.log; exit 3; }
  echo "pass $n ok"
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run p2 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run p3 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA
