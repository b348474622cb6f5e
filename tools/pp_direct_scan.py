#!/usr/bin/env python3
"""(diagnostic build) Which states make the table VJP take the direct formula: every point of a 4096 x 256 field at
one value u, for u over [-3, 1.5), at the trained-like parameters; prints the u values whose points all went direct.
    KANODE_LIB=tools/bin/var/clock.so python3 tools/pp_direct_scan.py"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd")]
import bench  # noqa: E402
import kanode  # noqa: E402
from kanode import _lib as L  # noqa: E402

dev = torch.device("cuda:0")
nx = 256
kan1 = kanode.Chain(kanode.KDense(1, 1, 10, normalizer="softsign", basis_func="rbf"))
rhs = kanode.FisherKPPRHS(kan1, nx=nx, dx=1 / 255, D=0.01, dtype=torch.float64, device=dev)
p = torch.as_tensor(bench.fk_trained_like_params(), device=dev)
buf = (C.c_ulonglong * 32)()
B = 64
lam = torch.ones(B, nx, dtype=torch.float64, device=dev)
direct = []
for u in np.arange(-3.0, 1.5, 1 / 64):
    x = torch.full((B, nx), float(u) + 1 / 128, dtype=torch.float64, device=dev)   # (the interval's centre)
    L.lib().kan_clock_probe_reset()
    rhs.hd.vjp(p, x, lam)
    torch.cuda.synchronize()
    L.lib().kan_clock_probe_read(buf)
    if buf[7]:
        direct.append(round(float(u) + 1 / 128, 5))
# the build's rejections (diagnostic slots 8..14): per function, the worst residual / tolerance, the last interval
L.lib().kan_clock_probe_reset()
rhs.hd.vjp(p * 1.0000001, x, lam)   # (a new p: every block rebuilds)
torch.cuda.synchronize()
L.lib().kan_clock_probe_read(buf)
import struct
rej = {"phi": int(buf[16]), "dphi": int(buf[17]), "swish": int(buf[18]),
       "worst_ratio": struct.unpack("<d", struct.pack("<Q", buf[19]))[0] if buf[19] else 0.0,
       "max_interval": {"dphi": int(buf[21]), "swish": int(buf[22])}}
print(json.dumps({"intervals_direct": direct, "count": len(direct), "build_rejections": rej}), flush=True)
