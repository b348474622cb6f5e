#!/usr/bin/env python3
"""Host-sync census of the grid-sharded (tp) Burgers-512 training iteration: run under
  rocprofv3 --hip-runtime-trace --memory-copy-trace --output-format csv -d DIR -- python3 tools/tp_sync_trace.py
on one GPU (a world-1 RCCL group, so the code path is the sharded one: GridShardedChainRHS + reduce_dev),
then tools/hip_sync_count.py DIR tp_sync_stats.json.  Prints the iteration's forward/adjoint step
counts as JSON (tp_sync_stats.json) so syncs can be divided by steps.
  python3 tools/tp_sync_trace.py [--iters 2] [--out FILE]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import kanode  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=2)
ap.add_argument("--out", default="tp_sync_stats.json")
a = ap.parse_args()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29631")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
c1 = kanode.LayerCfg(512, 10, 5, normalizer="softsign")
c2 = kanode.LayerCfg(10, 512, 5, normalizer="softsign")
tp = kanode.GridShardedChainRHS(c1, c2, device=dev)
chain = kanode.Chain(kanode.KDense(512, 10, 5, normalizer="softsign"), kanode.KDense(10, 512, 5, normalizer="softsign"))
p_full = torch.as_tensor(chain.setup(np.random.default_rng(0))[0].astype(np.float64), device=dev)
u0 = torch.as_tensor(bench._surrogate_problem("burgers512", 4, 5), device=dev)
saveat = [0.005 * i for i in range(201)]
target = (0.9 * u0).unsqueeze(0).expand(len(saveat), -1, -1).contiguous()
tr = kanode.Trainer(tp, u0, (0.0, 1.0), saveat, target, tp.shard_params(p_full), eta=1e-2, tp=True)
tr.step()                                   # warm-up (the census subtracts nothing: counts are per step)
torch.cuda.synchronize()
fwd = adj = 0
t_start = time.monotonic_ns()
for _ in range(a.iters):
    _, _, sol = tr.loss_and_grad()
    st = sol.stats
    fwd += st["naccept"] + st.get("nreject", 0)
    adj += st["adjoint"]["naccept"] + st["adjoint"].get("nreject", 0)
torch.cuda.synchronize()
t_end = time.monotonic_ns()
out = dict(iters=a.iters, forward_steps=fwd, adjoint_steps=adj, sensealg=tr.sensealg,
           window_monotonic_ns=[t_start, t_end], world=dist.get_world_size())
json.dump(out, open(a.out, "w"))
print(json.dumps(out), flush=True)
dist.destroy_process_group()
