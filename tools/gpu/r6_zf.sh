#!/bin/bash
# LV1 host-time profile (cProfile of the training iteration)
set -e
O=gpurun_out/r6_zf
mkdir -p $O
timeout -k 10 240 python3 -u tools/lv1_iter_cprofile.py --reps 300 > $O/host_profile.txt 2>&1
