"""Pin the CPU oracle (test infrastructure) before trusting it.

The reference holds no numeric fixtures for the KAN path,
so the oracle is pinned by: the LinRange knot constants, two independent
restatements (C and numpy) agreeing, an mpmath high-precision evaluation,
finite-difference checks of every pullback, the NNlib tanh_fast coefficients
reproducing tanh to its documented accuracy, and the Activation_getter identity.
"""
import math

import mpmath as mp
import numpy as np
import pytest

from oracle import kanode_np as N
from oracle import oracle as O


def specs_from_meta(meta):
    return [O.LayerSpec(l["in_dims"], l["out_dims"], l["grid_len"], l["normalizer"], l["basis"],
                        l["use_base_act"], tuple(l["grid_lims"]), None, l["iqf_reference_quirk"])
            for l in meta["layers"]]


def test_knots_linrange_hex(golden):
    g = golden("knots")
    assert [format(v, "08x") for v in g["knots_G10"].view(np.uint32)] == [
        "bf800000", "bf471c72", "bf0e38e4", "beaaaaab", "bde38e39",
        "3de38e39", "3eaaaaab", "3f0e38e4", "3f471c72", "3f800000"]
    assert g["knots_G5"].tolist() == [-1.0, -0.5, 0.0, 0.5, 1.0]
    for G in (5, 10):
        assert np.array_equal(O.knots(O.LayerSpec(1, 1, G)), g[f"knots_G{G}"])
    # Float32 1/h (utils.jl:9): 2.0f0 for G=5, 4.5f0 for G=10
    assert g["invh_G5"][0] == np.float32(2.0) and g["invh_G10"][0] == np.float32(4.5)


def test_float32_step_accumulation_differs_from_linrange():
    # LinRange interpolates in Float64 then rounds; accumulating a Float32 step
    # (lo + j*h in Float32) gives different knots at G=10 — the grid must come
    # from the Float64 lerp (kdense.jl:90).
    h = np.float32(2.0 / 9.0)
    acc = np.array([np.float32(-1.0) + np.float32(j) * h for j in range(10)], np.float32)
    assert not np.array_equal(acc, N.knots(10))


@pytest.mark.parametrize("dtype,tol", [(np.float64, 2.3e-16), (np.float32, 5 * 2.0 ** -23)])
def test_tanh_fast_matches_tanh(dtype, tol):
    xs = np.concatenate([np.linspace(-12, 12, 4001), np.linspace(-0.2, 0.2, 401), [0.0, 35.0, -40.0]])
    err = max(abs(O.act("tanh_fast", float(x), dtype) - math.tanh(float(dtype(x)))) for x in xs)
    assert err <= tol


@pytest.mark.parametrize("which", ["tanh_fast", "tanh", "softsign", "sigmoid", "sigmoid_fast", "swish"])
def test_activation_rrules_fd(which):
    for x in np.linspace(-5, 5, 40):  # even count: skip the |x| kink at 0
        h = 1e-6
        fd = (O.act(which, x + h) - O.act(which, x - h)) / (2 * h)
        assert abs(O.dact(which, x) - fd) < 1e-8 * max(1.0, abs(fd))


def test_swish_sigmoid_definitions():
    for x in np.linspace(-30, 30, 121):
        s = 1.0 / (1.0 + math.exp(-x))
        assert abs(O.act("sigmoid", x) - s) < 1e-15
        assert abs(O.act("swish", x) - x * s) < 1e-13 * max(1, abs(x))
        assert O.act("softsign", x) == x / (1 + abs(x))


@pytest.mark.parametrize("name", ["lv_f64_init", "lv_f64", "burgers41", "var_rswaf", "var_iqf_quirk",
                                  "var_iqf_exact", "var_sigmoid", "var_identity_nobase", "var_tanh_g10"])
def test_oracle_reproduces_golden_and_numpy(golden, name):
    d = golden(name)
    specs = specs_from_meta(d["meta"])
    y = O.chain_fwd(specs, d["p"], d["u"])
    xb, pb = O.chain_vjp(specs, d["p"], d["u"], d["ybar"])
    sy = np.max(np.abs(d["y"]))
    assert np.max(np.abs(y - d["y"])) <= 1e-14 * sy
    assert np.max(np.abs(xb - d["xbar"])) <= 1e-13 * np.max(np.abs(d["xbar"]))
    assert np.max(np.abs(pb - d["pbar"])) <= 1e-13 * np.max(np.abs(d["pbar"]))
    ch = N.Chain([N.Layer(s.in_dims, s.out_dims, s.grid_len, s.normalizer, s.basis, s.use_base_act,
                          s.grid_lims, None, s.iqf_reference_quirk) for s in specs])
    assert np.max(np.abs(ch.fwd(d["p"], d["u"]) - y)) <= 1e-12 * sy


def test_oracle_f32_close_to_f64(golden):
    d = golden("lv_f32")
    specs = specs_from_meta(d["meta"])
    y32 = O.chain_fwd(specs, d["p"], d["u"])
    y64 = O.chain_fwd(specs, d["p"].astype(np.float64), d["u"].astype(np.float64))
    assert np.array_equal(y32, d["y"])
    assert np.max(np.abs(y32 - y64)) < 1e-5 * np.max(np.abs(y64))


def _mp_layer(spec, p, x):
    """High-precision KDense forward (mpmath, 40 digits) — independent of both restatements."""
    mp.mp.dps = 40
    G, I, Ox = spec.grid_len, spec.in_dims, spec.out_dims
    grid = [mp.mpf(float(v)) for v in N.knots(G)]
    invh = mp.mpf(float(N.inv_h(N.default_denominator(G))))
    nC = Ox * G * I
    C = lambda o, c: mp.mpf(float(p[o + Ox * c]))  # noqa: E731
    W = lambda o, i: mp.mpf(float(p[nC + o + Ox * i]))  # noqa: E731

    def norm(v):
        if spec.normalizer in ("tanh", "tanh_fast"):
            return mp.tanh(v)
        return v / (1 + abs(v))

    out = []
    for o in range(Ox):
        s = mp.mpf(0)
        for i in range(I):
            xv = mp.mpf(float(x[i]))
            n = norm(xv)
            for g in range(G):
                s += C(o, g + G * i) * mp.exp(-((n - grid[g]) * invh) ** 2)
            s += W(o, i) * xv / (1 + mp.exp(-xv))
        out.append(s)
    return out


def test_oracle_vs_mpmath(golden):
    d = golden("lv_f64")
    spec = specs_from_meta(d["meta"])[0]
    pl = d["p"][:spec.param_length()]
    y = O.layer_fwd(spec, pl, d["u"][:6])
    for k in range(6):
        ref = _mp_layer(spec, pl, d["u"][k])
        for o in range(spec.out_dims):
            # tanh_fast vs exact tanh differs by ~1 ulp in the normalised input only
            assert abs(float(ref[o]) - y[k, o]) < 1e-13 * max(1.0, abs(float(ref[o])))


@pytest.mark.parametrize("name", ["lv_f64", "var_rswaf", "var_iqf_exact", "var_sigmoid", "var_tanh_g10"])
def test_chain_vjp_finite_differences(golden, name):
    d = golden(name)
    specs = specs_from_meta(d["meta"])
    p, u, yb = d["p"], d["u"][:8], d["ybar"][:8]
    xb, pb = O.chain_vjp(specs, p, u, yb)
    rng = np.random.default_rng(1)
    h = 1e-6
    dpv = rng.normal(size=p.shape)
    fd = (np.sum(O.chain_fwd(specs, p + h * dpv, u) * yb) - np.sum(O.chain_fwd(specs, p - h * dpv, u) * yb)) / (2 * h)
    assert abs(fd - pb @ dpv) < 1e-6 * max(1, abs(fd))
    dxv = rng.normal(size=u.shape)
    fd = (np.sum(O.chain_fwd(specs, p, u + h * dxv) * yb) - np.sum(O.chain_fwd(specs, p, u - h * dxv) * yb)) / (2 * h)
    assert abs(fd - np.sum(xb * dxv)) < 1e-6 * max(1, abs(fd))


def test_iqf_reference_quirk_is_not_the_derivative(golden):
    """utils.jl:59's IQF pullback is -2·x·y·ȳ (y = 1/(1+x²)); the true derivative is -2·x·y²·ȳ."""
    d = golden("var_iqf_quirk")
    specs = specs_from_meta(d["meta"])
    p, u, yb = d["p"], d["u"][:8], d["ybar"][:8]
    _, pb = O.chain_vjp(specs, p, u, yb)
    rng = np.random.default_rng(2)
    dpv = rng.normal(size=p.shape)
    h = 1e-6
    fd = (np.sum(O.chain_fwd(specs, p + h * dpv, u) * yb) - np.sum(O.chain_fwd(specs, p - h * dpv, u) * yb)) / (2 * h)
    assert abs(fd - pb @ dpv) > 1e-4 * abs(fd)


@pytest.mark.parametrize("nx", [1, 2, 3, 4, 26, 256])
def test_fk_dense_equals_stencil(nx):
    spec = O.LayerSpec(1, 1, 10, "softsign")
    rng = np.random.default_rng(nx)
    p = rng.uniform(-1, 1, 11)
    u = rng.uniform(0, 1, (3, nx))
    assert np.array_equal(O.fk_rhs(spec, p, 0.01, 1.0 / max(nx - 1, 1), u),
                          O.fk_rhs(spec, p, 0.01, 1.0 / max(nx - 1, 1), u, dense=True))


@pytest.mark.parametrize("name", ["fk26", "fk256"])
def test_fk_golden_and_fd(golden, name):
    d = golden(name)
    m = d["meta"]
    spec = specs_from_meta(m)[0]
    du = O.fk_rhs(spec, d["p"], m["D"], m["dx"], d["u"])
    assert np.array_equal(du, d["du"])
    lamJ, dp = O.fk_vjp(spec, d["p"], m["D"], m["dx"], d["u"], d["lam"])
    assert np.array_equal(lamJ, d["lamJ"]) and np.array_equal(dp, d["dp"])
    rng = np.random.default_rng(3)
    h = 1e-7
    dv = rng.normal(size=d["u"].shape)
    f = lambda uu: np.sum(O.fk_rhs(spec, d["p"], m["D"], m["dx"], uu) * d["lam"])  # noqa: E731
    fd = (f(d["u"] + h * dv) - f(d["u"] - h * dv)) / (2 * h)
    assert abs(fd - np.sum(lamJ * dv)) < 1e-5 * max(1, abs(fd))


def test_activation_getter_identity(golden):
    """Σ_i act[k, i, o] == KDense layer output (Activation_getter.jl:33-36, 55-61; tolerance 1e-10)."""
    d = golden("edge_lv1")
    spec = specs_from_meta(d["meta"])[0]
    act = O.edge_act(spec, d["p"], d["u"])
    assert np.array_equal(act, d["act"])
    assert np.max(np.abs(act.sum(axis=1) - O.layer_fwd(spec, d["p"], d["u"]))) < 1e-10
    assert np.max(np.abs(act - N.Layer(2, 10, 5, "tanh_fast").edge_act(d["p"], d["u"]))) < 1e-13
