set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_r02b.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r02b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_rhs.py --batch 1048576 --grids 0 --rounds 5 tools/bin/var_s/*.so > gpurun_out/ab_stamp_1M.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/ab_rhs.py --batch 131072 --grids 0 --rounds 5 --reps 40 tools/bin/var_s/*.so > gpurun_out/ab_stamp_128k.txt 2>&1 || exit 3
cat gpurun_out/ab_stamp_1M.txt gpurun_out/ab_stamp_128k.txt
