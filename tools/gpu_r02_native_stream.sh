set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_solve.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/native_r02.log 2>&1; rc=$?
tail -5 gpurun_out/native_r02.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/bin/streambench 1048576 1024,2048,4096,8192,0 > gpurun_out/stream_1M.txt 2>&1 || exit 3
cat gpurun_out/stream_1M.txt
timeout -k 10 120 tools/bin/streambench 131072 1024,2048,0 > gpurun_out/stream_128k.txt 2>&1 || exit 3
cat gpurun_out/stream_128k.txt
