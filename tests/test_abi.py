"""CPU-side checks of the drop-in boundary: libkanode.so loads, exports every
symbol include/kanode.h declares, and rejects invalid specs (validation runs
before any device call, so it is testable without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

import kanode
from kanode import _lib as L

HEADER = os.path.join(ROOT, "include", "kanode.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kanode_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("kanode_create", "kanode_destroy", "kanode_rhs", "kanode_vjp", "kanode_layer_forward",
                 "kanode_layer_vjp", "kanode_edge_activations", "kanode_last_error", "kanode_rhs_host",
                 "kanode_vjp_host", "kanode_reserve", "kanode_knots", "kanode_param_length"):
        assert must in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", kanode.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\sT\s+(kanode_\w+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    # the Python binding covers exactly the declared set
    assert sorted(n for n, _, _ in L.SIGNATURES) == declared_functions()


def test_option_ids_match_the_header():
    """kanode_option enum values == the Python binding's OPTIONS table (names lower-cased)."""
    src = open(HEADER).read()
    body = re.search(r"typedef enum \{([^}]*)\} kanode_option;", src, flags=re.S).group(1)
    ids = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"KANODE_OPT_(\w+)\s*=\s*(\d+)", body)}
    assert ids == L.OPTIONS
    body = re.search(r"typedef enum \{([^}]*)\} kanode_adjoint_path;", src, flags=re.S).group(1)
    paths = {m.group(1): int(m.group(2)) for m in re.finditer(r"KANODE_ADJ_(\w+)\s*=\s*(\d+)", body)}
    assert paths == {n: getattr(L, "ADJ_" + n) for n in paths} and len(paths) == 5


def test_library_has_no_environment_knobs():
    """Launch-time behaviour comes from kanode_set_option, never from getenv in the hot path."""
    out = subprocess.run(["nm", "-D", "--undefined-only", kanode.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert not re.search(r"\bgetenv\b", out)


def test_library_loads_and_reports_version():
    lib = kanode.lib()
    assert lib.kanode_abi_version() == 1
    assert lib.kanode_status_string(L.ERR_UNSUPPORTED) == b"unsupported configuration"


@pytest.mark.parametrize("cname,cls", [("kanode_stage", L.StageC), ("kanode_solver_options", L.SolverOptsC),
                                        ("kanode_solve_stats", L.SolveStatsC)])
def test_struct_layout_matches_c_compiler(tmp_path, cname, cls):
    """Struct offsets as gcc lays them out from include/kanode.h vs the ctypes mirror."""
    fields = [f[0] for f in cls._fields_]
    src = tmp_path / "probe.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "kanode.h"\nint main(void) {\n'
                   + "".join(f'  printf("%zu\\n", offsetof({cname}, {f}));\n' for f in fields)
                   + f'  printf("%zu\\n", sizeof({cname}));\n  return 0;\n}}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got[:-1] == [getattr(cls, f).offset for f in fields]
    assert got[-1] == C.sizeof(cls)


def test_solver_option_defaults():
    """kanode_solver_options_default == kanode.Tsit5Options() (OrdinaryDiffEq defaults)."""
    o = L.SolverOptsC()
    kanode.lib().kanode_solver_options_default(C.byref(o))
    d = kanode.Tsit5Options().to_c()
    for f, _ in L.SolverOptsC._fields_:
        assert getattr(o, f) == getattr(d, f), f
    assert (o.abstol, o.reltol, o.adaptive, o.qmin, o.qmax) == (1e-6, 1e-3, 1, 0.2, 10.0)


def test_struct_layout_matches_header():
    # kanode_layer_spec: 6 int32 + 3 float + 1 int32 = 40 bytes; kanode_spec holds 8 of them
    assert C.sizeof(L.LayerSpecC) == 40
    assert L.SpecC.layers.offset == 4
    assert L.SpecC.nx.offset % 8 == 0


def _create(spec):
    h = C.c_void_p()
    st = kanode.lib().kanode_create(C.byref(spec), C.byref(h))
    msg = kanode.lib().kanode_last_error(h).decode() if h.value else ""
    kanode.lib().kanode_destroy(h)
    return st, msg


def _spec(layers, **kw):
    s = L.SpecC()
    s.n_layers = len(layers)
    for i, l in enumerate(layers):
        s.layers[i] = l
    s.dtype = kw.get("dtype", L.F64)
    s.rhs_kind = kw.get("rhs_kind", L.RHS_CHAIN)
    s.nx = kw.get("nx", 0)
    s.diffusion = 0.01
    s.dx = kw.get("dx", 0.04)
    return s


def _layer(I, O, G, norm=0, basis=0, lo=-1.0, hi=1.0):
    return L.LayerSpecC(I, O, G, norm, basis, 1, lo, hi, 0.0, 1)


@pytest.mark.parametrize("bad,code,frag", [
    (dict(layers=[_layer(2, 10, 1)]), L.ERR_UNSUPPORTED, "grid_len"),
    (dict(layers=[_layer(2, 10, 64)]), L.ERR_UNSUPPORTED, "grid_len"),
    (dict(layers=[_layer(0, 10, 5)]), L.ERR_INVALID_ARG, "in_dims"),
    (dict(layers=[_layer(2, 10, 5, norm=9)]), L.ERR_INVALID_ARG, "normalizer"),
    (dict(layers=[_layer(2, 10, 5, basis=7)]), L.ERR_INVALID_ARG, "basis"),
    (dict(layers=[_layer(2, 10, 5, lo=1.0, hi=-1.0)]), L.ERR_INVALID_ARG, "grid_lims"),
    (dict(layers=[_layer(2, 10, 5), _layer(3, 2, 5)]), L.ERR_INVALID_ARG, "in_dims"),
    (dict(layers=[_layer(2, 2, 5)], rhs_kind=L.RHS_POINTWISE_PERIODIC_LAPLACIAN, nx=16), L.ERR_INVALID_ARG,
     "KDense(1, 1, G)"),
    (dict(layers=[_layer(1, 1, 10)], rhs_kind=L.RHS_POINTWISE_PERIODIC_LAPLACIAN, nx=0), L.ERR_INVALID_ARG, "nx"),
    (dict(layers=[_layer(1, 1, 10)], rhs_kind=L.RHS_POINTWISE_PERIODIC_LAPLACIAN, nx=8, dx=0.0),
     L.ERR_INVALID_ARG, "dx"),
    (dict(layers=[_layer(1, 1, 10)], dtype=7), L.ERR_INVALID_ARG, "dtype"),
])
def test_create_rejects_invalid_specs(bad, code, frag):
    layers = bad.pop("layers")
    st, msg = _create(_spec(layers, **bad))
    assert st == code
    assert frag in msg


def test_null_arguments():
    lib = kanode.lib()
    assert lib.kanode_create(None, None) == L.ERR_INVALID_ARG
    assert lib.kanode_rhs(None, None, None, None, 1, None) == L.ERR_INVALID_ARG
    assert lib.kanode_vjp(None, None, None, None, None, None, 1, None) == L.ERR_INVALID_ARG
    assert lib.kanode_param_length(None) == -1
    lib.kanode_destroy(None)


def test_product_package_does_not_import_oracle():
    pkg = os.path.join(ROOT, "kan-odes_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"(import\s+oracle|from\s+oracle|oracle/|liboracle|kref_)", src), f
