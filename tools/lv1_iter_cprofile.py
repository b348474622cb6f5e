#!/usr/bin/env python3
"""cProfile of the LV1 training iteration (tools/lv1_probe.py's it_a: step, eval_loss, loss_test solve): where the
host time between the kernels goes.  python3 tools/lv1_iter_cprofile.py [--reps 300]"""
import argparse
import cProfile
import io
import os
import pstats
import runpy
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=300)
a = ap.parse_args()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [sys.argv[0], "--reps", "2", "--rounds", "1"]
g = runpy.run_path(os.path.join(ROOT, "tools", "lv1_probe.py"), run_name="lv1_probe")
it_a = g["it_a"]
import torch  # noqa: E402
for _ in range(20):
    it_a()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(a.reps):
    it_a()
torch.cuda.synchronize()
pr.disable()
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
    print(s.getvalue(), flush=True)
