#!/usr/bin/env bash
# Quick GPU iteration: FK parity tests, bench (no CPU leg), VALU counters.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-q}
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${TESTS:-} > $OUT/pytest_$TAG.log 2>&1; rc=$?
tail -4 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err; rc=$?
python3 -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print('value %.3e  kernel %.1f us  frac %.3f  vjp %.1f us'%(d['value'],d['roofline']['kernel_ms']*1e3,d['roofline']['frac'],d['vjp']['ms_per_step']*1e3))" || { tail -5 $OUT/bench_$TAG.err; exit 3; }
[ "${PMC:-1}" = "1" ] || exit 0
for w in fk_rhs fk_vjp; do
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F64 --kernel-trace -d $OUT/pmc_$TAG/$w -o run --output-format csv -- \
   python3 tools/prof_kernel.py --what $w --reps 5 > $OUT/pmc_$TAG.$w.log 2>&1 || { echo "pmc failed"; exit 3; }
done
python3 tools/pmc_summary.py $OUT/pmc_$TAG
