"""Where the D = 0 VJP sweep differs from the oracle: per configuration, the worst λᵀJ and dp points
with the scale components (KAN part, swish part, N', basis maximum).  Diagnostic only (GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kan-odes_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

import kanode
from oracle import oracle as O
from test_gpu_pp import kan_vjp_scales, rhs_for, sweep

dev = torch.device("cuda:0")
cfgs = [(n, b, G) for n in ["softsign", "tanh_fast", "tanh", "sigmoid", "sigmoid_fast", "identity"]
        for b in ["rbf", "rswaf"] for G in [2, 5, 10, 32]]
for normalizer, basis, G in cfgs:
    rng = np.random.default_rng(G * 7 + len(normalizer) * 3 + len(basis))
    spec = O.LayerSpec(1, 1, G, normalizer, basis)
    p = rng.uniform(-1, 1, G + 1)
    u = sweep()
    lam = rng.normal(size=u.shape)
    rhs = rhs_for(256, normalizer, G, basis)
    lamJ, dp = rhs.vjp(torch.as_tensor(u, device=dev), torch.as_tensor(p, device=dev),
                       torch.as_tensor(lam, device=dev))
    lamJ, dp = lamJ.cpu().numpy(), dp.cpu().numpy()
    rJ, rdp = O.fk_vjp(spec, p, 0.0, 0.01, u, lam)
    sc, _ = kan_vjp_scales(spec, p, u, lam)
    r = np.abs(lamJ - rJ) / np.maximum(1e-14 * sc, 1e-300)
    k = np.unravel_index(np.argmax(r), r.shape)
    x = u[k]
    _, dpa = O.fk_vjp(spec, p, 0.0, 0.01, u, np.abs(lam))
    rd = np.abs(dp - rdp) / np.maximum(1e-13 * np.abs(dpa), 1e-300)
    j = int(np.argmax(rd))
    print(f"{normalizer:12s} {basis:5s} G={G:2d} table={int(rhs.hd.pointwise_table)} lamJ ratio {r[k]:8.3g} "
          f"u={x:+.6e} lam={lam[k]:+.3f} err={abs(lamJ[k] - rJ[k]):.3g} scale={sc[k]:.3g} "
          f"N'={O.dact(normalizer, x):.3g} swish'={O.dact('swish', x):.3g} | dp ratio {rd[j]:8.3g} j={j} "
          f"err={abs(dp[j] - rdp[j]):.3g} sum|lam phi_j|={abs(dpa[j]):.3g} max|dpa|={np.max(np.abs(dpa)):.3g}",
          flush=True)
