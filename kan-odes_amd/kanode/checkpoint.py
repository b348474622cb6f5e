"""`.mat` checkpoints in the reference drivers' format.

LV driver (LV_driver_KANODE.jl:252-272): keys p_list [N_epochs, P, 1], loss, loss_test,
kan_pred_t, kan_pred_u1, kan_pred_u2, size_KAN = [num_layers, layer_width, grid_size];
restart reads p_list[end, :, 1], loss, loss_test (:146-160).
PDE drivers (Fisher-KPP_Source.jl:112-128): p_list, loss.
The flat p rows are the ComponentArray order the C-ABI consumes (include/kanode.h).
"""
from __future__ import annotations

import numpy as np
import scipy.io


def save_lv(path: str, p_list, loss, loss_test=None, pred_t=None, pred_u=None, size_kan=None) -> None:
    P = np.asarray(p_list, dtype=np.float64)
    if P.ndim == 2:
        P = P[:, :, None]
    d = {"p_list": P, "loss": np.asarray(loss, np.float64).reshape(-1)}
    if loss_test is not None:
        d["loss_test"] = np.asarray(loss_test, np.float64).reshape(-1)
    if pred_t is not None:
        d["kan_pred_t"] = np.asarray(pred_t, np.float64)
    if pred_u is not None:
        pu = np.asarray(pred_u, np.float64)
        d["kan_pred_u1"], d["kan_pred_u2"] = pu[0], pu[1]
    if size_kan is not None:
        d["size_KAN"] = np.asarray(size_kan, np.float64)
    scipy.io.savemat(path, d)


def save_pde(path: str, p_list, loss) -> None:
    P = np.asarray(p_list, dtype=np.float64)
    if P.ndim == 2:
        P = P[:, :, None]
    scipy.io.savemat(path, {"p_list": P, "loss": np.asarray(loss, np.float64).reshape(-1)})


def load(path: str) -> dict:
    """matread + the driver's restart unpacking: {'p': last row, 'p_list': [...], 'loss', ...}."""
    m = scipy.io.loadmat(path)
    P = m["p_list"]
    out = {k: np.asarray(v).reshape(-1) for k, v in m.items() if not k.startswith("__") and k != "p_list"}
    out["p_list"] = [P[j, :, 0] for j in range(P.shape[0])]
    out["p"] = P[-1, :, 0]
    return out
