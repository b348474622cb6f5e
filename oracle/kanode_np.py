"""Independent numpy restatement of the reference KDense / Fisher-KPP math —
test infrastructure only (cross-checks oracle/kanode_ref.c; generates goldens).

Written separately from the C oracle (vectorised, different code path) so the
two restatements check each other.  Citations as in oracle/kanode_ref.h:
  kdense.jl:20-130, utils.jl:2-62, Fisher-KPP_Source.jl:55-59,95-98,
  NNlib 0.9.24 activations (Manifest.toml:1776).
Shapes: x (K, I) [== Julia x[i, k]], p flat in ComponentArray order.
"""
from __future__ import annotations

import numpy as np


def knots(G: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """Julia LinRange{Float32}: T((1-t)*a + t*b), t = j/(G-1) in Float64 (kdense.jl:90)."""
    a, b = float(np.float32(lo)), float(np.float32(hi))
    t = np.arange(G, dtype=np.float64) / (G - 1)
    return ((1.0 - t) * a + t * b).astype(np.float32)


def default_denominator(G: int) -> np.float32:
    return np.float32(2.0 / (G - 1))  # kdense.jl:27


def inv_h(den) -> np.float32:
    return np.float32(1.0) / np.float32(den)  # Float32 1/h (utils.jl:9)


def tanh_fast(x):
    x = np.asarray(x)
    if x.dtype == np.float32:
        x2 = x * x
        n = np.polyval(np.array([1.587199e-8, 2.2332108e-5, 0.0035974074, 0.1346604, 1.0], np.float32), x2)
        d = np.polyval(np.array([8.7767893e-7, 0.0003453992, 0.026262015, 0.4679937, 1.0], np.float32), x2)
        return np.where(x2 < np.float32(66), x * (n / d), np.sign(x)).astype(np.float32)
    x2 = x * x
    e = np.exp(np.minimum(x + x, 700.0))
    y = (e - 1.0) / (e + 1.0)
    yp = x * np.polyval([-0.008697141630499953, 0.02186660872609521, -0.05396823125794372,
                         0.13333333325511604, -0.33333333333324583, 1.0], x2)
    return np.where(x2 > 900.0, np.sign(x), np.where(x2 < 0.017, yp, y))


def sigmoid(x):
    t = np.exp(-np.abs(x))
    return np.where(x >= 0, 1 / (1 + t), t / (1 + t))


def swish(x):
    return x * sigmoid(x)


def softsign(x):
    return x / (1 + np.abs(x))


NORMS = {
    "tanh_fast": tanh_fast,
    "tanh": np.tanh,
    "softsign": softsign,
    "sigmoid": sigmoid,
    "sigmoid_fast": sigmoid,
    "identity": lambda x: x,
}


def dnorm(name, x, om):
    if name in ("tanh_fast", "tanh"):
        return 1 - om * om
    if name == "softsign":
        return (1 - np.abs(om)) ** 2
    if name in ("sigmoid", "sigmoid_fast"):
        return om * (1 - om)
    return np.ones_like(x)


def dswish(x):
    s = sigmoid(x)
    return s + x * s * (1 - s)


class Layer:
    def __init__(self, I, O, G, normalizer="tanh", basis="rbf", use_base_act=True,
                 grid_lims=(-1.0, 1.0), denominator=None, iqf_reference_quirk=True):
        self.I, self.O, self.G = I, O, G
        self.normalizer, self.basis, self.use_base_act = normalizer, basis, use_base_act
        self.grid = knots(G, *grid_lims)
        self.den = default_denominator(G) if denominator is None else np.float32(denominator)
        self.invh = inv_h(self.den)
        self.iqf_reference_quirk = iqf_reference_quirk

    @property
    def P(self):
        return self.O * self.G * self.I + (self.O * self.I if self.use_base_act else 0)

    def split(self, p):
        nC = self.O * self.G * self.I
        C = p[:nC].reshape(self.G * self.I, self.O).T  # column-major [O, G*I]
        W = p[nC:self.P].reshape(self.I, self.O).T if self.use_base_act else None
        return C, W

    def _basis(self, x):
        dt = x.dtype
        n = NORMS[self.normalizer](x)                                   # (K, I)
        y = (n[:, :, None] - self.grid.astype(dt)[None, None, :]) * dt.type(self.invh)  # (K, I, G)
        if self.basis == "rbf":
            phi = np.exp(-(y * y))
        elif self.basis == "rswaf":
            phi = 1 - np.tanh(y) ** 2
        else:
            phi = 1 / (1 + y * y)
        return n, y, phi

    def fwd(self, p, x):
        C, W = self.split(p.astype(x.dtype))
        _, _, phi = self._basis(x)
        K = x.shape[0]
        basis = phi.reshape(K, self.I * self.G)      # column index g + G*i
        y = basis @ C.T
        if self.use_base_act:
            y = y + swish(x) @ W.T
        return y

    def vjp(self, p, x, ybar):
        C, W = self.split(p.astype(x.dtype))
        n, y, phi = self._basis(x)
        K = x.shape[0]
        basis = phi.reshape(K, self.I * self.G)
        Cbar = ybar.T @ basis                         # [O, G*I]
        bbar = (ybar @ C).reshape(K, self.I, self.G)
        if self.basis == "rbf":
            zbar = -2 * y * phi * bbar
        elif self.basis == "rswaf":
            zbar = -2 * np.tanh(y) * phi * bbar
        else:
            zbar = (-2 * y * phi * bbar) if self.iqf_reference_quirk else (-2 * y * phi * phi * bbar)
        nbar = (zbar * x.dtype.type(self.invh)).sum(axis=2)
        xbar = nbar * dnorm(self.normalizer, x, n)
        parts = [Cbar.T.reshape(-1)]
        if self.use_base_act:
            xbar = xbar + (ybar @ W) * dswish(x)
            parts.append((ybar.T @ swish(x)).T.reshape(-1))
        return xbar, np.concatenate(parts)

    def edge_act(self, p, x):
        C, W = self.split(p.astype(x.dtype))
        _, _, phi = self._basis(x)                   # (K, I, G)
        Cr = C.reshape(self.O, self.I, self.G)
        a = np.einsum("kig,oig->kio", phi, Cr)
        if self.use_base_act:
            a = a + swish(x)[:, :, None] * W.T[None, :, :]
        return a


class Chain:
    def __init__(self, layers):
        self.layers = layers

    @property
    def P(self):
        return sum(l.P for l in self.layers)

    def fwd(self, p, x):
        off = 0
        for l in self.layers:
            x = l.fwd(p[off:off + l.P], x)
            off += l.P
        return x

    def vjp(self, p, x, ybar):
        acts, offs, off = [x], [], 0
        for l in self.layers:
            offs.append(off)
            acts.append(l.fwd(p[off:off + l.P], acts[-1]))
            off += l.P
        pbar = np.zeros(self.P, x.dtype)
        g = ybar
        for li in range(len(self.layers) - 1, -1, -1):
            l = self.layers[li]
            g, pb = l.vjp(p[offs[li]:offs[li] + l.P], acts[li], g)
            pbar[offs[li]:offs[li] + l.P] += pb
        return g, pbar


def fk_coeffs(D, dx):
    dx2 = dx * dx
    return D * (-2.0 / dx2), D * (1.0 / dx2)


def fk_lap(u, D, dx):
    cd, co = fk_coeffs(D, dx)
    return co * np.roll(u, 1, axis=1) + cd * u + co * np.roll(u, -1, axis=1)


def fk_rhs(layer: Layer, p, D, dx, u):
    """u (B, Nx) -> du (B, Nx): D*lap*u + KAN(u) pointwise (Fisher-KPP_Source.jl:95-98)."""
    B, Nx = u.shape
    kan = layer.fwd(p, u.reshape(-1, 1)).reshape(B, Nx)
    return fk_lap(u, D, dx) + kan


def fk_vjp(layer: Layer, p, D, dx, u, lam):
    B, Nx = u.shape
    xb, pb = layer.vjp(p, u.reshape(-1, 1), lam.reshape(-1, 1))
    return fk_lap(lam, D, dx) + xb.reshape(B, Nx), pb
