#!/usr/bin/env python3
"""In-kernel shader clock of the adjoint rows step and the standalone VJP (MI355X_MICROARCH.md, DVFS give-back item
6: Δs_memtime ÷ Δs_memrealtime × 100 MHz, summed over every block's lifetime), from the diagnostic build:

    tools/build_var.sh clock "-DKAN_CLOCK_PROBE" kan_pp.hip
    KANODE_LIB=tools/bin/var/clock.so python3 tools/clock_probe.py

GRBM_GUI_ACTIVE ÷ 8 ÷ duration reads high on dispatches shorter than ~0.3 ms (the rows step is ~55 us), so this
is the measurement the rows kernel's issue floor is restated at."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402
import kanode  # noqa: E402
from kanode import _lib as L  # noqa: E402

lib = L.lib()
if not hasattr(lib, "kan_clock_probe_read"):
    raise SystemExit("not a KAN_CLOCK_PROBE build: set KANODE_LIB to tools/bin/var/clock.so")
buf = (C.c_ulonglong * 32)()


def read():
    torch.cuda.synchronize()
    assert lib.kan_clock_probe_read(buf) == 0
    return [int(x) for x in buf]


def ghz(v, slot):
    c, r = v[2 * slot], v[2 * slot + 1]
    return c / r * 0.1 if r else float("nan")


dev = torch.device("cuda:0")
out = {}
# the adaptive reference-problem epoch (fk_vjp_step_rows_loop_kernel: slot 0)
lib.kan_clock_probe_reset()
t0 = time.perf_counter()
ep = bench.epoch_adaptive_bench(dev, bench.fk_trained_like_params(), 256, 1 / 255, 0.01, 4096, 0, reps=2)
v = read()
out["rows_step_epoch_adaptive"] = {"GHz": ghz(v, 0), "clocks": v[0], "realtime_10ns": v[1], "epoch_s": ep["gpu"]}
# phases of the device-controlled loops' other kernels over the same epochs (us; s_memrealtime is 100 MHz)
nfin, nfw = max(v[6], 1), max(v[11], 1)
out["finish_loop_last_workgroup_us"] = {"launches": v[6], "reduce": v[2] / nfin / 100, "arrive_and_terms": v[3] / nfin / 100,
                                        "decide": v[4] / nfin / 100, "plan_and_state": v[5] / nfin / 100}
out["forward_dev_step_per_workgroup_us"] = {"workgroups": v[11], "decision_and_tables": v[8] / nfw / 100,
                                            "rows": v[9] / nfw / 100, "error_partial": v[10] / nfw / 100}
# the standalone VJP at 1M trajectories (fk_vjp_pp_wave_kernel: slot 1)
nx = 256
kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign"))
rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=1 / (nx - 1), D=0.01, device=dev)
p = torch.as_tensor(kan1.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
u = bench.fk_ics(1048576, nx, 1 / (nx - 1), 1, dev)
lam = torch.randn_like(u)
for _ in range(3):
    rhs.hd.vjp(p, u, lam)
lib.kan_clock_probe_reset()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    rhs.hd.vjp(p, u, lam)
torch.cuda.synchronize()
v = read()
out["vjp_1M"] = {"GHz": ghz(v, 1), "ms_per_call": (time.perf_counter() - t0) / 20 * 1e3}
# the table build with p changing every call (bench.py's headline loop): slots 12..15
p2 = p.clone()
p2[0] += 1e-3
lib.kan_clock_probe_reset()
for i in range(40):
    rhs.hd.rhs(p if i % 2 else p2, u[:131072], torch.empty_like(u[:131072]))
v = read()
nb = max(v[15], 1)
out["pp_build_per_block_us"] = {"blocks": v[15], "stamp_check": v[12] / nb / 100, "build": v[13] / nb / 100,
                                "arrival": v[14] / nb / 100}
print(json.dumps(out), flush=True)
