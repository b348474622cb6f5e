set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
O=gpurun_out/vjpprof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/prof_kernel.py --what fk_vjp --reps 10 > $O/trace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace -d $O/pmc1 -o run --output-format csv -- python3 tools/prof_kernel.py --what fk_vjp --reps 5 > $O/pmc1.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_ANY --kernel-trace -d $O/pmc2 -o run --output-format csv -- python3 tools/prof_kernel.py --what fk_vjp --reps 5 > $O/pmc2.log 2>&1 || exit 3
python3 tools/pmc_summary.py $O
