"""Host-side mirror of the Lux / KolmogorovArnold.jl interface (no GPU needed)."""
import numpy as np
import pytest

from oracle import oracle as O

import kanode


def test_kdense_defaults_follow_reference():
    l = kanode.KDense(2, 10, 5)
    assert l.normalizer == "tanh_fast"            # fast_act(tanh) (kdense.jl:25,57-61)
    assert l.grid_lims == (-1.0, 1.0)
    assert l.denominator == float(np.float32(0.5))
    assert l.parameterlength() == 2 * 10 * 5 + 2 * 10   # kdense.jl:98-107
    assert l.statelength() == 5
    assert kanode.KDense(2, 10, 5, use_base_act=False).parameterlength() == 100
    assert kanode.KDense(1, 1, 10, normalizer="tanh", allow_fast_activation=False).normalizer == "tanh"
    with pytest.raises(NotImplementedError):
        kanode.KDense(2, 2, 5, base_act="relu")


def test_chain_setup_matches_lv_driver():
    chain = kanode.Chain(kanode.KDense(2, 10, 5), kanode.KDense(10, 2, 5))
    p, st = chain.setup(np.random.default_rng(0))
    assert p.shape == (240,) and p.dtype == np.float32   # LV KAN [2,10,2] G=5: 240 params
    assert [s["grid"].tolist() for s in st] == [[-1.0, -0.5, 0.0, 0.5, 1.0]] * 2
    pm = chain.unflatten(p)
    assert pm[0]["C"].shape == (10, 10) and pm[0]["W"].shape == (10, 2)
    assert pm[1]["C"].shape == (2, 50) and pm[1]["W"].shape == (2, 10)
    assert np.array_equal(chain.flatten(pm), p)
    assert chain.layer_offsets() == [0, 120]


@pytest.mark.parametrize("G,lo,hi", [(5, -1, 1), (10, -1, 1), (7, 0, 1), (13, -2.5, 3.0)])
def test_initialstates_grid_matches_oracle_linrange(G, lo, hi):
    g = kanode.KDense(1, 1, G, grid_lims=(lo, hi)).initialstates()["grid"]
    assert np.array_equal(g, O.knots(O.LayerSpec(1, 1, G, grid_lims=(lo, hi))))


def test_glorot_uniform_bounds():
    w = kanode.glorot_uniform(np.random.default_rng(0), 10, 50)
    assert w.dtype == np.float32 and w.shape == (10, 50)
    assert np.max(np.abs(w)) <= np.sqrt(6 / 60) + 1e-7


def test_fisher_kpp_dense_laplacian_matches_reference_form():
    lap = kanode.fisher_kpp_laplacian(26, 0.04)
    assert lap[0, -1] == lap[-1, 0] == 1 / 0.04 ** 2
    assert lap[3, 3] == -2 / 0.04 ** 2 and lap[3, 4] == 1 / 0.04 ** 2
