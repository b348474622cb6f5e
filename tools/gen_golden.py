#!/usr/bin/env python3
"""Generate tests/golden/*.npz — golden input/output vectors for the KAN-ODE RHS + VJP.

The reference (Julia) cannot run in this image, so the
vectors come from the C oracle (oracle/kanode_ref.c), and every fixture is
accepted only if the independent numpy restatement (oracle/kanode_np.py)
agrees with it to 1e-12 relative to the term scale.  Knot constants are also
pinned against the Float32 hex values derived from Julia's LinRange semantics
(SURVEY.md §8a row A2).

Configs follow the reference drivers at their own sizes:
  lv_f64 / lv_f32      KAN [2,10,2] G=5 tanh_fast   (LV_driver_KANODE.jl:130-142,175)
  fk26 / fk256         KDense(1,1,10) softsign + periodic lap (Fisher-KPP_Source.jl:34-59,81-98)
  burgers41            KAN [41,10,41] G=5 softsign  (Burgers_Surrogate.jl:80-88)
  schrodinger402       KAN [402,10,402] G=10 softsign (Schrodinger_Surrogate.jl:86-96)
  variants             rswaf / iqf / sigmoid / identity / no-base layers
Usage: python tools/gen_golden.py  (writes tests/golden/, prints a summary)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import kanode_np as N  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

KNOT_HEX = {
    5: ["bf800000", "bf000000", "00000000", "3f000000", "3f800000"],
    10: ["bf800000", "bf471c72", "bf0e38e4", "beaaaaab", "bde38e39",
         "3de38e39", "3eaaaaab", "3f0e38e4", "3f471c72", "3f800000"],
}


def rel_err(a, b, scale=None):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    s = np.max(np.abs(b)) if scale is None else scale
    return float(np.max(np.abs(a - b)) / max(s, 1e-300))


def glorot(rng, O_, I_):
    s = np.sqrt(6.0 / (O_ + I_))
    return rng.uniform(-s, s, (O_, I_)).astype(np.float32)


def chain_params(rng, specs, scale=1.0):
    parts = []
    for s in specs:
        C = glorot(rng, s.out_dims, s.grid_len * s.in_dims)
        parts.append(C.flatten(order="F"))
        if s.use_base_act:
            parts.append(glorot(rng, s.out_dims, s.in_dims).flatten(order="F"))
    return np.concatenate(parts).astype(np.float64) * scale


def np_chain(specs):
    return N.Chain([N.Layer(s.in_dims, s.out_dims, s.grid_len, s.normalizer, s.basis, s.use_base_act,
                            s.grid_lims, s.denominator, s.iqf_reference_quirk) for s in specs])


def spec_meta(specs):
    return [dict(in_dims=s.in_dims, out_dims=s.out_dims, grid_len=s.grid_len, normalizer=s.normalizer,
                 basis=s.basis, use_base_act=s.use_base_act, grid_lims=list(s.grid_lims),
                 iqf_reference_quirk=s.iqf_reference_quirk) for s in specs]


def chain_fixture(name, specs, p, u, rng, dtype=np.float64, tol=1e-12):
    p = p.astype(dtype)
    u = u.astype(dtype)
    y = O.chain_fwd(specs, p, u)
    ybar = rng.normal(size=y.shape).astype(dtype)
    xbar, pbar = O.chain_vjp(specs, p, u, ybar)
    if dtype == np.float64:
        ch = np_chain(specs)
        yn = ch.fwd(p, u)
        xn, pn = ch.vjp(p, u, ybar)
        errs = (rel_err(y, yn), rel_err(xbar, xn), rel_err(pbar, pn))
        assert max(errs) < tol, (name, errs)
    meta = dict(kind="chain", layers=spec_meta(specs), dtype=np.dtype(dtype).name)
    return dict(meta=np.array(json.dumps(meta)), p=p, u=u, y=y, ybar=ybar, xbar=xbar, pbar=pbar)


def fk_fixture(name, nx, dx, D, B, rng, tol=1e-12):
    spec = O.LayerSpec(1, 1, 10, "softsign")
    lay = N.Layer(1, 1, 10, "softsign")
    p = chain_params(rng, [spec])
    x = np.arange(nx) * dx
    c = rng.uniform(0.3, 0.7, B)[:, None]
    dl = rng.uniform(0.1, 0.3, B)[:, None]
    amp = rng.uniform(0.5, 1.0, B)[:, None]
    # reference IC family (Fisher-KPP_Source.jl:47-49)
    u = amp * (np.tanh((x - (c - dl / 2)) / (dl / 10)) - np.tanh((x - (c + dl / 2)) / (dl / 10))) / 2
    du = O.fk_rhs(spec, p, D, dx, u)
    du_dense = O.fk_rhs(spec, p, D, dx, u, dense=True)
    assert np.array_equal(du, du_dense), name
    lam = rng.normal(size=u.shape)
    lamJ, dp = O.fk_vjp(spec, p, D, dx, u, lam)
    scale = np.max(np.abs(N.fk_lap(np.abs(u), abs(D), dx))) + np.max(np.abs(du))
    errs = (rel_err(du, N.fk_rhs(lay, p, D, dx, u), scale),
            rel_err(lamJ, N.fk_vjp(lay, p, D, dx, u, lam)[0], np.max(np.abs(lamJ)) * 10),
            rel_err(dp, N.fk_vjp(lay, p, D, dx, u, lam)[1]))
    assert max(errs) < tol, (name, errs)
    meta = dict(kind="fisher_kpp", layers=spec_meta([spec]), dtype="float64", nx=nx, dx=dx, D=D)
    return dict(meta=np.array(json.dumps(meta)), p=p, u=u, du=du, lam=lam, lamJ=lamJ, dp=dp)


def main() -> None:
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(20240417)
    fixtures = {}

    # knots (kdense.jl:90) pinned to the LinRange hex constants
    kn = {}
    for G, hx in KNOT_HEX.items():
        g = O.knots(O.LayerSpec(1, 1, G))
        assert [format(v, "08x") for v in g.view(np.uint32)] == hx, G
        assert np.array_equal(g, N.knots(G)), G
        kn[f"knots_G{G}"] = g
        kn[f"invh_G{G}"] = np.array([O.inv_h(O.LayerSpec(1, 1, G))], np.float32)
    fixtures["knots"] = kn

    lv = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
    u_lv = rng.uniform(0.5, 2.0, (64, 2))
    # the driver's initial parameters: Glorot Float32 promoted and divided by 1e5 (LV_driver_KANODE.jl:175)
    fixtures["lv_f64_init"] = chain_fixture("lv_f64_init", lv, chain_params(rng, lv, 1e-5), u_lv, rng)
    fixtures["lv_f64"] = chain_fixture("lv_f64", lv, chain_params(rng, lv, 1.0), u_lv, rng)
    fixtures["lv_f32"] = chain_fixture("lv_f32", lv, chain_params(rng, lv, 1.0), u_lv, rng, np.float32)

    fixtures["fk26"] = fk_fixture("fk26", 26, 0.04, 0.01, 4, rng)
    fixtures["fk256"] = fk_fixture("fk256", 256, 1.0 / 255, 0.01, 8, rng)

    bu = [O.LayerSpec(41, 10, 5, "softsign"), O.LayerSpec(10, 41, 5, "softsign")]
    xg = np.linspace(-1, 1, 41)
    u_bu = np.stack([-np.sin(np.pi * xg) + 0.1 * rng.normal() * np.sin(2 * np.pi * xg) for _ in range(2)])
    fixtures["burgers41"] = chain_fixture("burgers41", bu, chain_params(rng, bu), u_bu, rng)

    sc = [O.LayerSpec(402, 10, 10, "softsign"), O.LayerSpec(10, 402, 10, "softsign")]
    xs = np.linspace(-5, 5, 201)
    th = rng.uniform(0, 2 * np.pi, 2)
    u_sc = np.stack([np.concatenate([2 / np.cosh(xs) * np.cos(t), 2 / np.cosh(xs) * np.sin(t)]) for t in th])
    fixtures["schrodinger402"] = chain_fixture("schrodinger402", sc, chain_params(rng, sc), u_sc, rng)

    var = {
        "rswaf": [O.LayerSpec(3, 4, 6, "tanh", "rswaf"), O.LayerSpec(4, 3, 6, "tanh", "rswaf")],
        "iqf_quirk": [O.LayerSpec(3, 4, 6, "softsign", "iqf", iqf_reference_quirk=True),
                      O.LayerSpec(4, 3, 6, "softsign", "iqf", iqf_reference_quirk=True)],
        "iqf_exact": [O.LayerSpec(3, 4, 6, "softsign", "iqf", iqf_reference_quirk=False),
                      O.LayerSpec(4, 3, 6, "softsign", "iqf", iqf_reference_quirk=False)],
        "sigmoid": [O.LayerSpec(3, 4, 7, "sigmoid", grid_lims=(0.0, 1.0)),
                    O.LayerSpec(4, 3, 7, "sigmoid_fast", grid_lims=(0.0, 1.0))],
        "identity_nobase": [O.LayerSpec(3, 4, 8, "identity", use_base_act=False),
                            O.LayerSpec(4, 3, 8, "identity", use_base_act=False)],
        "tanh_g10": [O.LayerSpec(3, 5, 10, "tanh"), O.LayerSpec(5, 3, 10, "tanh")],
    }
    for name, specs in var.items():
        u = rng.uniform(-2.0, 2.0, (32, 3))
        fixtures[f"var_{name}"] = chain_fixture(name, specs, chain_params(rng, specs), u, rng)

    # per-edge activations (Activation_getter.jl) on the LV first layer
    pl = fixtures["lv_f64"]["p"][:lv[0].param_length()]
    act = O.edge_act(lv[0], pl, u_lv)
    assert np.max(np.abs(act.sum(axis=1) - O.layer_fwd(lv[0], pl, u_lv))) < 1e-10  # :33-36 identity
    fixtures["edge_lv1"] = dict(meta=np.array(json.dumps(dict(kind="edge", layers=spec_meta(lv[:1])))),
                                p=pl, u=u_lv, act=act)

    total = 0
    for name, d in fixtures.items():
        path = os.path.join(OUT, f"{name}.npz")
        np.savez(path, **d)
        total += os.path.getsize(path)
        print(f"{name:22s} {os.path.getsize(path) / 1024:8.1f} KiB")
    print(f"total {total / 1024:.1f} KiB")




def gen_lv_truth() -> None:
    """LV ground truth (LV_driver_KANODE.jl:110-127): lotka!(u, p=[1.5,1,1,3]) from u0=[1,1]
    over (0, 14), saveat 0.1 (141 samples; the first 35 are the training cut), solved with
    scipy DOP853 at rtol=atol=1e-12 (the driver uses Tsit5 at 1e-12)."""
    from scipy.integrate import solve_ivp
    a, b, c, d = 1.5, 1.0, 1.0, 3.0

    def lotka(t, u):
        return [a * u[0] - b * u[0] * u[1], c * u[0] * u[1] - d * u[1]]

    t = np.round(np.arange(0, 141) * 0.1, 10)
    sol = solve_ivp(lotka, (0.0, 14.0), [1.0, 1.0], method="DOP853", t_eval=t, rtol=1e-12, atol=1e-12)
    np.savez(os.path.join(OUT, "lv_truth.npz"), t=t, X=sol.y, end_index=np.array(35))
    print("lv_truth: X", sol.y.shape)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "lv_truth":
    gen_lv_truth()


if __name__ == "__main__" and len(sys.argv) == 1:
    main()
