"""Fisher-KPP RHS + VJP on the GPU vs the CPU oracle (PDE examples/Fisher-KPP_Source.jl:95-98)."""
import numpy as np
import pytest
import torch

from gpu_util import RTOL, assert_close, device, fk_scale, specs_from_meta, t
from oracle import oracle as O

import kanode

pytestmark = pytest.mark.gpu

SPEC = O.LayerSpec(1, 1, 10, "softsign")


def make_rhs(nx, dx, D=0.01, normalizer="softsign", G=10, dtype=torch.float64):
    kan1 = kanode.Chain(kanode.KDense(1, 1, G, normalizer=normalizer, basis_func="rbf"))
    return kanode.FisherKPPRHS(kan1, nx=nx, dx=dx, D=D, dtype=dtype, device=device())


def ics(rng, B, nx, dx):
    x = np.arange(nx) * dx
    c = rng.uniform(0.3, 0.7, (B, 1))
    dl = rng.uniform(0.1, 0.3, (B, 1))
    amp = rng.uniform(0.5, 1.0, (B, 1))
    return amp * (np.tanh((x - (c - dl / 2)) / (dl / 10)) - np.tanh((x - (c + dl / 2)) / (dl / 10))) / 2


@pytest.mark.parametrize("name", ["fk26", "fk256"])
def test_fk_golden(golden, name):
    d = golden(name)
    m = d["meta"]
    rhs = make_rhs(m["nx"], m["dx"], m["D"])
    p, u, lam = t(d["p"]), t(d["u"]), t(d["lam"])
    du = rhs.rhs(u, p)
    sc = fk_scale(d["p"], m["D"], m["dx"], d["u"])
    assert_close(du, d["du"], sc, RTOL[torch.float64], "du")
    lamJ, dp = rhs.vjp(u, p, lam)
    # λᵀJ scale: |D lap| |λ| + |λ| Σ_j |C_j| |z_j φ_j| s + ... bounded by the FD-style magnitude below
    scJ = fk_scale(np.abs(d["p"]) * 10, m["D"], m["dx"], np.abs(d["lam"])) * (1 + np.abs(d["u"]))
    assert_close(lamJ, d["lamJ"], scJ, RTOL[torch.float64], "lamJ")
    _, dpa = O.fk_vjp(SPEC, d["p"], m["D"], m["dx"], d["u"], np.abs(d["lam"]))
    assert_close(dp, d["dp"], np.abs(dpa) + 1e-300, 1e-12, "dp")


@pytest.mark.parametrize("nx", [1, 2, 3, 7, 26, 255, 256, 300])
@pytest.mark.parametrize("B", [1, 5])
def test_fk_rhs_shapes(nx, B):
    rng = np.random.default_rng(nx * 10 + B)
    dx = 1.0 / max(nx - 1, 1)
    p = rng.uniform(-1, 1, 11)
    u = rng.uniform(-0.5, 1.5, (B, nx))
    rhs = make_rhs(nx, dx)
    du = rhs.rhs(t(u), t(p))
    assert_close(du, O.fk_rhs(SPEC, p, 0.01, dx, u), fk_scale(p, 0.01, dx, u), RTOL[torch.float64], "du")
    lam = rng.normal(size=u.shape)
    lamJ, dp = rhs.vjp(t(u), t(p), t(lam))
    rJ, rdp = O.fk_vjp(SPEC, p, 0.01, dx, u, lam)
    scJ = fk_scale(np.abs(p) * 10, 0.01, dx, np.abs(lam)) * (1 + np.abs(u))
    assert_close(lamJ, rJ, scJ, RTOL[torch.float64], "lamJ")
    _, dpa = O.fk_vjp(SPEC, p, 0.01, dx, u, np.abs(lam))
    assert_close(dp, rdp, np.abs(dpa), 1e-12, "dp")


@pytest.mark.parametrize("normalizer", ["identity", "tanh", "sigmoid", "tanh_fast"])
def test_fk_other_normalizers(normalizer):
    """identity forces the per-knot (direct) path; the others the recurrence."""
    rng = np.random.default_rng(7)
    nx, dx, B = 64, 1.0 / 63, 3
    spec = O.LayerSpec(1, 1, 10, normalizer)
    p = rng.uniform(-1, 1, 11)
    u = rng.uniform(-1.0, 1.0, (B, nx))
    rhs = make_rhs(nx, dx, normalizer=normalizer)
    du = rhs.rhs(t(u), t(p))
    assert_close(du, O.fk_rhs(spec, p, 0.01, dx, u), fk_scale(p, 0.01, dx, u), RTOL[torch.float64], normalizer)


def test_fk_vjp_accumulates_dp():
    rng = np.random.default_rng(11)
    nx, dx = 32, 1 / 31
    p, u, lam = rng.uniform(-1, 1, 11), rng.uniform(0, 1, (4, nx)), rng.normal(size=(4, nx))
    rhs = make_rhs(nx, dx)
    dp = t(np.ones(11))
    rhs.vjp(t(u), t(p), t(lam), dp=dp)
    _, rdp = O.fk_vjp(SPEC, p, 0.01, dx, u, lam)
    assert np.allclose(dp.cpu().numpy(), 1.0 + rdp, rtol=1e-12, atol=1e-12)


def test_fk_large_batch_properties():
    """At the bench size: trajectory independence (a batch equals its shards, bitwise),
    VJP linearity in λ, and a random subsample against the oracle."""
    dev = device()
    rng = np.random.default_rng(5)
    nx, dx, B = 256, 1.0 / 255, 16384
    p = rng.uniform(-1, 1, 11)
    u = ics(rng, B, nx, dx)
    rhs = make_rhs(nx, dx)
    pt, ut = t(p), t(u)
    du = rhs.rhs(ut, pt)
    du_a = rhs.rhs(ut[: B // 2].contiguous(), pt)
    du_b = rhs.rhs(ut[B // 2:].contiguous(), pt)
    assert torch.equal(du, torch.cat([du_a, du_b]))
    idx = rng.choice(B, 32, replace=False)
    assert_close(du[idx], O.fk_rhs(SPEC, p, 0.01, dx, u[idx]), fk_scale(p, 0.01, dx, u[idx]),
                 RTOL[torch.float64], "du subsample")
    l1 = torch.randn(B, nx, dtype=torch.float64, device=dev)
    l2 = torch.randn(B, nx, dtype=torch.float64, device=dev)
    j1, d1 = rhs.vjp(ut, pt, l1)
    j2, d2 = rhs.vjp(ut, pt, l2)
    j3, d3 = rhs.vjp(ut, pt, (2 * l1 - 3 * l2).contiguous())
    assert torch.allclose(j3, 2 * j1 - 3 * j2, rtol=1e-11, atol=1e-9)
    assert torch.allclose(d3, 2 * d1 - 3 * d2, rtol=1e-9, atol=1e-6)
    # deterministic reduction: same inputs, same bits
    j4, d4 = rhs.vjp(ut, pt, l1)
    assert torch.equal(j4, j1) and torch.equal(d4, d1)


def test_fk_empty_batch():
    rhs = make_rhs(16, 1 / 15)
    u = torch.empty((0, 16), dtype=torch.float64, device=device())
    p = t(np.zeros(11))
    assert rhs.rhs(u, p).shape == (0, 16)


def test_fk_host_variants(golden):
    import ctypes as C
    d = golden("fk26")
    m = d["meta"]
    rhs = make_rhs(m["nx"], m["dx"], m["D"])
    lib = kanode.lib()
    du = np.zeros_like(d["u"])
    ptr = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    assert lib.kanode_rhs_host(rhs.hd._h, ptr(d["p"]), ptr(d["u"]), ptr(du), d["u"].shape[0]) == 0
    ref = rhs.rhs(t(d["u"]), t(d["p"])).cpu().numpy()
    assert np.array_equal(du, ref)
    lamJ = np.zeros_like(d["u"])
    dp = np.zeros(11)
    assert lib.kanode_vjp_host(rhs.hd._h, ptr(d["p"]), ptr(d["u"]), ptr(d["lam"]), ptr(lamJ), ptr(dp),
                               d["u"].shape[0]) == 0
    rJ, rdp = rhs.vjp(t(d["u"]), t(d["p"]), t(d["lam"]))
    assert np.array_equal(lamJ, rJ.cpu().numpy()) and np.array_equal(dp, rdp.cpu().numpy())


def test_fk_graph_capture():
    dev = device()
    nx, dx, B = 256, 1 / 255, 512
    rng = np.random.default_rng(9)
    rhs = make_rhs(nx, dx)
    p, u = t(rng.uniform(-1, 1, 11)), t(rng.uniform(0, 1, (B, nx)))
    rhs.hd.reserve(B)
    out = torch.empty_like(u)
    ref = rhs.rhs(u, p)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        rhs.rhs(u, p, out)  # warm
        with torch.cuda.graph(g, stream=s):
            rhs.rhs(u, p, out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("nx,dx", [(21, 0.05), (256, 1.0 / 255)])
def test_allen_cahn_source_rhs(nx, dx):
    """The Allen-Cahn twin of the source-term KAN-ODE (PDE examples/Allen-Cahn_Source.jl:36-40,
    90-93; dx = 0.05 there): du = -1e-4·lap·u + KAN(u) is the Fisher-KPP handle with D = -1e-4;
    RHS and VJP against the oracle."""
    rng = np.random.default_rng(nx)
    D = -1e-4
    p = rng.uniform(-1, 1, 11)
    u = rng.uniform(-1.2, 1.2, (3, nx))
    rhs = make_rhs(nx, dx, D=D)
    du = rhs.rhs(t(u), t(p))
    assert_close(du, O.fk_rhs(SPEC, p, D, dx, u), fk_scale(p, D, dx, u), RTOL[torch.float64], "du")
    lam = rng.normal(size=u.shape)
    lamJ, dp = rhs.vjp(t(u), t(p), t(lam))
    rJ, rdp = O.fk_vjp(SPEC, p, D, dx, u, lam)
    scJ = fk_scale(np.abs(p) * 10, D, dx, np.abs(lam)) * (1 + np.abs(u))
    assert_close(lamJ, rJ, scJ, RTOL[torch.float64], "lamJ")
    _, dpa = O.fk_vjp(SPEC, p, D, dx, u, np.abs(lam))
    assert_close(dp, rdp, np.abs(dpa) + 1e-300, 1e-12, "dp")
