"""KDense chain RHS / VJP / single layer / edge activations on the GPU vs the oracle.
(Lotka-Volterra/src/kdense.jl:109-130, utils.jl:8-62, Activation_getter.jl:3-63)"""
import numpy as np
import pytest
import torch

from gpu_util import RTOL, assert_close, cfgs_from_specs, chain_scale, device, specs_from_meta, t
from oracle import oracle as O

import kanode

pytestmark = pytest.mark.gpu

CHAIN_FIXTURES = ["lv_f64_init", "lv_f64", "lv_f32", "var_rswaf", "var_iqf_quirk", "var_iqf_exact",
                  "var_sigmoid", "var_identity_nobase", "var_tanh_g10"]


def _handle(specs, dtype):
    return kanode.KanodeHandle(cfgs_from_specs(specs), dtype=dtype, rhs_kind="chain", device=device())


def _dt(meta):
    return torch.float32 if meta["dtype"] == "float32" else torch.float64


@pytest.mark.parametrize("name", CHAIN_FIXTURES)
def test_chain_rhs_vjp_golden(golden, name):
    d = golden(name)
    specs = specs_from_meta(d["meta"])
    dt = _dt(d["meta"])
    hd = _handle(specs, dt)
    p, u, yb = t(d["p"], dt), t(d["u"], dt), t(d["ybar"], dt)
    y = hd.rhs(p, u)
    p64, u64 = d["p"].astype(np.float64), d["u"].astype(np.float64)
    sc = chain_scale(specs, p64, u64)
    assert_close(y, d["y"], sc, RTOL[dt], f"{name} y")
    xb, pb = hd.vjp(p, u, yb)
    # pullback scale: the oracle pullback evaluated with |p|, |ȳ| (Σ|terms| proxy) + magnitude floor
    xs, ps = O.chain_vjp(specs, np.abs(p64), u64, np.abs(d["ybar"].astype(np.float64)))
    fl = 1e3 if dt == torch.float32 else 1e2
    assert_close(xb, d["xbar"], np.abs(xs) * fl + np.max(np.abs(xs)) * 1e-2, RTOL[dt], f"{name} xbar")
    assert_close(pb, d["pbar"], np.abs(ps) * fl + np.max(np.abs(ps)) * 1e-2, RTOL[dt], f"{name} pbar")


@pytest.mark.parametrize("name", ["lv_f64", "lv_f32", "var_rswaf", "var_tanh_g10"])
def test_single_layer_forward_vjp(golden, name):
    d = golden(name)
    specs = specs_from_meta(d["meta"])
    dt = _dt(d["meta"])
    hd = _handle(specs, dt)
    off = 0
    x = d["u"]
    for li, s in enumerate(specs):
        n = s.param_length()
        pl = d["p"][off:off + n]
        y = hd.layer_forward(li, t(pl, dt), t(x, dt))
        ry = O.layer_fwd(s, pl, x)
        sc = np.abs(O.layer_fwd(s, np.abs(pl.astype(np.float64)), x.astype(np.float64)))
        assert_close(y, ry, sc + np.max(sc) * 1e-3, RTOL[dt], f"layer {li} y")
        yb = np.random.default_rng(li).normal(size=ry.shape).astype(x.dtype)
        xb, pb = hd.layer_vjp(li, t(pl, dt), t(x, dt), t(yb, dt))
        rxb, rpb = O.layer_vjp(s, pl, x, yb)
        xs, ps = O.layer_vjp(s, np.abs(pl.astype(np.float64)), x.astype(np.float64), np.abs(yb.astype(np.float64)))
        assert_close(xb, rxb, np.abs(xs) * 1e2 + np.max(np.abs(xs)) * 1e-2, RTOL[dt], f"layer {li} xbar")
        assert_close(pb, rpb, np.abs(ps) * 1e2 + np.max(np.abs(ps)) * 1e-2, RTOL[dt], f"layer {li} pbar")
        x = ry
        off += n


def test_edge_activations_golden_and_identity(golden):
    d = golden("edge_lv1")
    specs = specs_from_meta(d["meta"])
    lay = kanode.KDense(2, 10, 5, normalizer="tanh_fast")
    act = lay.edge_activations(t(d["u"]), t(d["p"]))
    sc = np.abs(O.edge_act(specs[0], np.abs(d["p"]), d["u"]))
    assert_close(act, d["act"], sc + 1e-3 * np.max(sc), RTOL[torch.float64], "act")
    y, _ = lay(t(d["u"]), t(d["p"]), None)
    # Activation_getter.jl:33-36: Σ over inputs == layer output within 1e-10
    assert torch.max(torch.abs(act.sum(dim=1) - y)).item() < 1e-10


def test_lv_batched_random_ics_f32():
    """LV, 4096 batched random ICs, fp32 (BASELINE config 2) vs the oracle in fp32."""
    rng = np.random.default_rng(42)
    specs = [O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")]
    P = sum(s.param_length() for s in specs)
    p = rng.uniform(-0.5, 0.5, P).astype(np.float32)
    u = rng.uniform(0.5, 2.0, (4096, 2)).astype(np.float32)
    hd = _handle(specs, torch.float32)
    y = hd.rhs(t(p, torch.float32), t(u, torch.float32))
    ry = O.chain_fwd(specs, p, u)
    sc = chain_scale(specs, p.astype(np.float64), u.astype(np.float64))
    assert_close(y, ry, sc, RTOL[torch.float32], "lv4k y")


def test_autograd_through_chain_matches_vjp(golden):
    d = golden("lv_f64")
    chain = kanode.Chain(kanode.KDense(2, 10, 5, normalizer="tanh_fast"),
                         kanode.KDense(10, 2, 5, normalizer="tanh_fast"))
    p = t(d["p"]).requires_grad_(True)
    u = t(d["u"]).requires_grad_(True)
    y, _ = chain(u, p, None)
    (y * t(d["ybar"])).sum().backward()
    specs = specs_from_meta(d["meta"])
    xs, ps = O.chain_vjp(specs, np.abs(d["p"]), d["u"], np.abs(d["ybar"]))
    assert_close(u.grad, d["xbar"], np.abs(xs) * 1e2 + np.max(np.abs(xs)) * 1e-2, 1e-13, "u.grad")
    assert_close(p.grad, d["pbar"], np.abs(ps) * 1e2 + np.max(np.abs(ps)) * 1e-2, 1e-13, "p.grad")


def test_layer_knots_match_linrange(golden):
    g = golden("knots")
    for G in (5, 10):
        hd = _handle([O.LayerSpec(2, 2, G, "tanh_fast")], torch.float64)
        assert np.array_equal(hd.knots(0), g[f"knots_G{G}"])


def test_chain_empty_batch():
    hd = _handle([O.LayerSpec(2, 10, 5, "tanh_fast"), O.LayerSpec(10, 2, 5, "tanh_fast")], torch.float64)
    p = t(np.zeros(hd.P))
    assert hd.rhs(p, torch.empty((0, 2), dtype=torch.float64, device=device())).shape == (0, 2)


@pytest.mark.parametrize("name", CHAIN_FIXTURES)
def test_fused_chain_equals_layer_by_layer(golden, name):
    """The one-launch chain kernel (kd_chain_col_kernel, small layers: the layer's input sums run as a
    lane butterfly instead of a sequential loop) equals the composition of kanode_layer_forward calls
    to rounding (the stated RTOL of the dtype against the |terms| scale)."""
    d = golden(name)
    specs = specs_from_meta(d["meta"])
    dt = _dt(d["meta"])
    hd = _handle(specs, dt)
    p = t(d["p"], dt)
    x = t(np.tile(d["u"], (97, 1)), dt)          # 97 x rows: several blocks and a ragged tail
    y = hd.rhs(p, x)
    cur, off = x, 0
    for li, s in enumerate(specs):
        n = s.param_length()
        cur = hd.layer_forward(li, p[off:off + n].contiguous(), cur)
        off += n
    sc = chain_scale(specs, d["p"].astype(np.float64), np.tile(d["u"], (97, 1)).astype(np.float64))
    assert_close(y, cur.cpu().numpy(), sc, RTOL[dt], name)
