"""Full-field surrogate chains on the GPU vs the oracle
(PDE examples/Burgers_Surrogate.jl:85-97, Schrodinger_Surrogate.jl:93-104; kdense.jl:109-130)."""
import numpy as np
import pytest
import torch

from gpu_util import RTOL, assert_close, cfgs_from_specs, chain_scale, device, specs_from_meta, t
from oracle import oracle as O

import kanode

pytestmark = pytest.mark.gpu


def _check_chain(specs, p, u, ybar, dt=torch.float64, y_ref=None, xbar_ref=None, pbar_ref=None):
    hd = kanode.KanodeHandle(cfgs_from_specs(specs), dtype=dt, rhs_kind="chain", device=device())
    y = hd.rhs(t(p, dt), t(u, dt))
    y_ref = O.chain_fwd(specs, p, u) if y_ref is None else y_ref
    assert_close(y, y_ref, chain_scale(specs, p, u), RTOL[dt], "y")
    xb, pb = hd.vjp(t(p, dt), t(u, dt), t(ybar, dt))
    if xbar_ref is None:
        xbar_ref, pbar_ref = O.chain_vjp(specs, p, u, ybar)
    xs, ps = O.chain_vjp(specs, np.abs(p), u, np.abs(ybar))
    assert_close(xb, xbar_ref, np.abs(xs) * 1e2 + np.max(np.abs(xs)) * 1e-2, RTOL[dt], "xbar")
    assert_close(pb, pbar_ref, np.abs(ps) * 1e2 + np.max(np.abs(ps)) * 1e-2, RTOL[dt], "pbar")
    return hd


@pytest.mark.parametrize("name", ["burgers41", "schrodinger402"])
def test_surrogate_golden(golden, name):
    d = golden(name)
    specs = specs_from_meta(d["meta"])
    _check_chain(specs, d["p"], d["u"], d["ybar"], y_ref=d["y"], xbar_ref=d["xbar"], pbar_ref=d["pbar"])


def _glorot_params(rng, specs):
    parts = []
    for s in specs:
        lim = np.sqrt(6.0 / (s.out_dims + s.grid_len * s.in_dims))
        parts.append(rng.uniform(-lim, lim, s.out_dims * s.grid_len * s.in_dims))
        lim = np.sqrt(6.0 / (s.out_dims + s.in_dims))
        parts.append(rng.uniform(-lim, lim, s.out_dims * s.in_dims))
    return np.concatenate(parts)


@pytest.mark.parametrize("N,G,B", [(512, 5, 4), (2048, 10, 8), (300, 7, 3), (2048, 10, 1), (64, 5, 11),
                                   (512, 5, 200), (96, 5, 133)])
def test_surrogate_baseline_sizes(N, G, B):
    """BU512: KAN [512,10,512] G=5; SC1024: KAN [2048,10,2048] G=10 (state [Re; Im]); odd sizes,
    a column count that is not a multiple of the 8-column tile, and batches past the 128-column
    basis staging of the wide-out parameter pullback (kan_wide.hip kWOPK)."""
    rng = np.random.default_rng(N + G + B)
    specs = [O.LayerSpec(N, 10, G, "softsign"), O.LayerSpec(10, N, G, "softsign")]
    p = _glorot_params(rng, specs)
    x = np.linspace(-1, 1, N)
    u = np.stack([-np.sin(np.pi * x) + 0.3 * rng.normal() * np.sin(2 * np.pi * x) for _ in range(B)])
    ybar = rng.normal(size=u.shape)
    _check_chain(specs, p, u, ybar)


def test_surrogate_single_layers_and_kinds():
    """Each wide layer through the single-layer entry points (one Lux KDense call each)."""
    rng = np.random.default_rng(3)
    specs = [O.LayerSpec(512, 10, 5, "softsign"), O.LayerSpec(10, 512, 5, "softsign")]
    p = _glorot_params(rng, specs)
    hd = kanode.KanodeHandle(cfgs_from_specs(specs), dtype=torch.float64, rhs_kind="chain", device=device())
    x = rng.uniform(-1, 1, (4, 512))
    off = 0
    for li, s in enumerate(specs):
        n = s.param_length()
        pl = p[off:off + n]
        y = hd.layer_forward(li, t(pl), t(x))
        ry = O.layer_fwd(s, pl, x)
        sc = np.abs(O.layer_fwd(s, np.abs(pl), x))
        assert_close(y, ry, sc + 1e-3 * np.max(sc), RTOL[torch.float64], f"layer {li}")
        yb = rng.normal(size=ry.shape)
        xb, pb = hd.layer_vjp(li, t(pl), t(x), t(yb))
        rxb, rpb = O.layer_vjp(s, pl, x, yb)
        xs, ps = O.layer_vjp(s, np.abs(pl), x, np.abs(yb))
        assert_close(xb, rxb, np.abs(xs) * 1e2 + np.max(np.abs(xs)) * 1e-2, RTOL[torch.float64], f"layer {li} xbar")
        assert_close(pb, rpb, np.abs(ps) * 1e2 + np.max(np.abs(ps)) * 1e-2, RTOL[torch.float64], f"layer {li} pbar")
        x = ry
        off += n


def test_surrogate_f32():
    rng = np.random.default_rng(5)
    specs = [O.LayerSpec(512, 10, 5, "softsign"), O.LayerSpec(10, 512, 5, "softsign")]
    p = _glorot_params(rng, specs).astype(np.float32)
    u = rng.uniform(-1, 1, (4, 512)).astype(np.float32)
    hd = kanode.KanodeHandle(cfgs_from_specs(specs), dtype=torch.float32, rhs_kind="chain", device=device())
    y = hd.rhs(t(p, torch.float32), t(u, torch.float32))
    sc = chain_scale(specs, p.astype(np.float64), u.astype(np.float64))
    assert_close(y, O.chain_fwd(specs, p, u), sc, RTOL[torch.float32], "y f32")


@pytest.mark.parametrize("N,G,B", [(512, 5, 1), (2048, 10, 8), (300, 7, 11)])
def test_surrogate_pair_launches_equal_layer_by_layer(N, G, B):
    """KAN [N, 10, N]: the fused chain path (wide-out reading the wide-in chunk partials; merged
    dot + parameter launch) is bitwise equal to the layer-by-layer calls through
    kanode_layer_forward / kanode_layer_vjp, which materialise the hidden layer."""
    rng = np.random.default_rng(N * G + B)
    specs = [O.LayerSpec(N, 10, G, "softsign"), O.LayerSpec(10, N, G, "softsign")]
    p = t(_glorot_params(rng, specs))
    u = t(rng.uniform(-1, 1, (B, N)))
    lam = t(rng.normal(size=(B, N)))
    hd = kanode.KanodeHandle(cfgs_from_specs(specs), dtype=torch.float64, rhs_kind="chain", device=device())
    P0 = hd.layers[0].param_length
    p0, p1 = p[:P0].contiguous(), p[P0:].contiguous()
    h = hd.layer_forward(0, p0, u)
    y_ref = hd.layer_forward(1, p1, h)
    assert torch.equal(hd.rhs(p, u), y_ref)
    hbar, pb1 = hd.layer_vjp(1, p1, h, lam)
    xbar, pb0 = hd.layer_vjp(0, p0, u, hbar)
    lamJ, dp = hd.vjp(p, u, lam)
    with hd.options(pair_vjp=0):     # the four-launch pullback is the layer-by-layer one, bitwise
        lamJ, dp = hd.vjp(p, u, lam)
        assert torch.equal(lamJ, xbar)
        assert torch.equal(dp, torch.cat([pb0, pb1]))
        # the VJP without λᵀJ (dp only) and without dp (λᵀJ only)
        lamJ2, _ = hd.vjp(p, u, lam, accumulate_dp=False)
        assert torch.equal(lamJ2, xbar)
        _, dp2 = hd.vjp(p, u, lam, want_lamJ=False)
        assert torch.equal(dp2, dp)


@pytest.mark.parametrize("N,G,B", [(512, 5, 4), (2048, 10, 8), (300, 7, 3)])
def test_surrogate_pair_stages_form_their_inputs_in_the_wide_in_kernel(N, G, B):
    """kanode_rhs_stage / kanode_vjp_stage on a KAN [N, 10, N]: the wide-in forward forms the stage
    input y = u + Σ c_j k_j and the adjoint stage input λs = λ + Σ lc_j lk_j itself and the parameter
    cotangents are written with = (no combination or memset launches).  Against the plain RHS / VJP
    evaluated at the y and λs the stages wrote out: bitwise equal; y and λs against torch's
    combination to rounding; dp accumulates onto a given vector."""
    rng = np.random.default_rng(N + G + B)
    specs = [O.LayerSpec(N, 10, G, "softsign"), O.LayerSpec(10, N, G, "softsign")]
    p = t(_glorot_params(rng, specs))
    hd = kanode.KanodeHandle(cfgs_from_specs(specs), dtype=torch.float64, rhs_kind="chain", device=device())
    u = t(rng.uniform(-1, 1, (B, N)))
    ks = [t(rng.normal(size=(B, N))) for _ in range(3)]
    c = [0.1, -0.05, 0.02]
    y = torch.empty_like(u)
    sumsq = torch.zeros(1, dtype=torch.float64, device=device())
    du = hd.rhs_stage(p, u, ks, c, y_out=y, error=([0.01, -0.02, 0.03, 0.04], 1e-6, 1e-3, sumsq))
    y_ref = u + c[0] * ks[0] + c[1] * ks[1] + c[2] * ks[2]
    assert (y - y_ref).abs().max().item() <= 1e-15 * max(1.0, y_ref.abs().max().item())
    assert torch.equal(du, hd.rhs(p, y))
    e = 0.01 * ks[0] - 0.02 * ks[1] + 0.03 * ks[2] + 0.04 * du
    sk = 1e-6 + 1e-3 * torch.maximum(u.abs(), y.abs())
    assert abs(sumsq.item() - ((e / sk) ** 2).sum().item()) <= 1e-12 * ((e / sk) ** 2).sum().item()
    lam = t(rng.normal(size=(B, N)))
    lks = [t(rng.normal(size=(B, N))) for _ in range(2)]
    lc = [0.3, -0.2]
    ls = torch.empty_like(u)
    lamJ, dp = hd.vjp_stage(p, u, ks, c, lam, lks, lc, lam_out=ls)
    assert (ls - (lam + lc[0] * lks[0] + lc[1] * lks[1])).abs().max().item() <= 1e-15 * ls.abs().max().item()
    lamJ_ref, dp_ref = hd.vjp(p, y, ls)
    assert torch.equal(lamJ, lamJ_ref) and torch.equal(dp, dp_ref)   # the same (two-launch) pullback
    dp0 = t(rng.normal(size=p.shape))
    _, dp2 = hd.vjp_stage(p, u, ks, c, lam, lks, lc, dp=dp0.clone())
    assert (dp2 - (dp0 + dp_ref)).abs().max().item() <= 1e-15 * (dp0.abs() + dp_ref.abs()).max().item()


@pytest.mark.parametrize("N,G,B", [(512, 5, 4), (2048, 10, 8), (300, 7, 11), (512, 5, 64), (41, 5, 2)])
def test_pair_vjp_two_launches_equal_four(N, G, B):
    """KANODE_OPT_PAIR_VJP: the surrogate pullback in two launches (the wide-in forward blocks also form
    the wide-out dot products' chunk partials; the wide-out parameter cotangents beside the wide-in
    pullback, which forms the hidden layer's cotangent per block) against the four-launch path, for the
    plain VJP and for an adjoint stage (stage inputs formed in the kernels, dp assigned / accumulated):
    y and λs bitwise, λᵀJ and dp to the summation order of the dot products (1e-13 of Σ|terms|), and
    bitwise reproducible run to run."""
    rng = np.random.default_rng(7 * N + G + B)
    specs = [O.LayerSpec(N, 10, G, "softsign"), O.LayerSpec(10, N, G, "softsign")]
    p = t(_glorot_params(rng, specs))
    hd = kanode.KanodeHandle(cfgs_from_specs(specs), dtype=torch.float64, rhs_kind="chain", device=device())
    assert hd.get_option("pair_vjp") == 1
    u = t(rng.uniform(-1, 1, (B, N)))
    lam = t(rng.normal(size=(B, N)))
    ks = [t(rng.normal(size=(B, N)) * 0.1) for _ in range(7)]
    c = [0.01 * w for w in kanode.ode.interp_weights(0.4)]
    lks = [t(rng.normal(size=(B, N))) for _ in range(5)]
    lc = [0.02 * a for a in kanode.ode.A[4]]
    dp0 = t(rng.normal(size=p.shape))
    out = {}
    for pair in (1, 0):
        with hd.options(pair_vjp=pair):
            lamJ, dp = hd.vjp(p, u, lam)
            ls = torch.empty_like(u)
            sJ, sdp = hd.vjp_stage(p, u, ks, c, lam, lks, lc, lam_out=ls)
            _, sdp2 = hd.vjp_stage(p, u, ks, c, lam, lks, lc, dp=dp0.clone())
            out[pair] = (lamJ, dp, sJ, sdp, ls, sdp2)
    assert torch.equal(out[1][4], out[0][4])                      # λs: the same combination
    with hd.options(pair_vjp=1):
        again = hd.vjp(p, u, lam)
    assert torch.equal(again[0], out[1][0]) and torch.equal(again[1], out[1][1])
    for a, b in zip(out[1], out[0]):
        sc = b.abs().max().item()
        assert (a - b).abs().max().item() <= 1e-13 * max(sc, 1e-300)
    # and against the oracle at the stage inputs (the four-launch path's own parity)
    y = u.clone()
    for cj, kj in zip(c, ks):
        y = torch.addcmul(y, kj, torch.full_like(kj, cj))
    rJ, rdp = O.chain_vjp(specs, p.cpu().numpy(), y.cpu().numpy(), out[1][4].cpu().numpy())
    xs, ps = O.chain_vjp(specs, np.abs(p.cpu().numpy()), y.cpu().numpy(), np.abs(out[1][4].cpu().numpy()))
    assert_close(out[1][2], rJ, np.abs(xs) * 1e2 + np.max(np.abs(xs)) * 1e-2, RTOL[torch.float64], "stage lamJ")
    assert_close(out[1][3], rdp, np.abs(ps) * 1e2 + np.max(np.abs(ps)) * 1e-2, RTOL[torch.float64], "stage dp")
