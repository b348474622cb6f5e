#!/bin/bash
# Persistent pair adjoint: correctness, phase profile (variant build), A/B against the launch path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4/persist
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    "tests/test_gpu_native_solve.py::test_persistent_pair_adjoint_matches_launch_path" > $O/pytest_persist.txt 2>&1 &&
KANODE_LIB=$R/tools/bin/var/paprof.so timeout -k 10 120 python -u tools/pair_persist_prof.py 0 > $O/prof_s8.txt 2>&1 &&
KANODE_LIB=$R/tools/bin/var/paprof.so timeout -k 10 120 python -u tools/pair_persist_prof.py 4 > $O/prof_s4.txt 2>&1 &&

timeout -k 10 200 python -u tools/pair_persist_ab.py burgers512 0 3 > $O/ab_s8.txt 2>&1
