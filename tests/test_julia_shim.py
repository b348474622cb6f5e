"""Textual check of the Julia binding julia/KANODEHip.jl against include/kanode.h (Julia is not in
this image, so the shim is not executed): every symbol it ccalls is declared in the header, and
every struct it mirrors has the C struct's fields, in order, with matching scalar types."""
import os
import re

from conftest import ROOT

JL = open(os.path.join(ROOT, "julia", "KANODEHip.jl")).read()
HDR = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "kanode.h")).read(), flags=re.S)

C2JL = {"int32_t": "Int32", "int64_t": "Int64", "float": "Float32", "double": "Float64"}
PAIRS = {"LayerSpec": "kanode_layer_spec", "Spec": "kanode_spec", "SolverOptions": "kanode_solver_options",
         "SolveStats": "kanode_solve_stats"}


def c_struct(name):
    m = re.search(r"typedef struct\s*\{([^{}]*)\}\s*" + name + r"\s*;", HDR)
    assert m, name
    fields = []
    for decl in m.group(1).split(";"):
        decl = decl.strip()
        if not decl:
            continue
        ty, rest = decl.split(None, 1)
        for v in rest.split(","):
            v = v.strip()
            arr = re.match(r"(\w+)\[(\w+)\]", v)
            if arr:
                fields.append((arr.group(1), f"{ty}[{arr.group(2)}]"))
            else:
                fields.append((v, ty))
    return fields


def jl_struct(name):
    m = re.search(r"\nstruct " + name + r"\b(.*?)\nend", JL, flags=re.S)
    assert m, name
    return re.findall(r"(\w+)::([\w{},]+)", m.group(1))


def test_every_ccall_symbol_is_declared():
    used = set(re.findall(r":(kanode_\w+)", JL))
    declared = set(re.findall(r"\b(kanode_[a-z0-9_]+)\s*\(", HDR))
    assert used, "no ccall found"
    assert used <= declared, used - declared


def test_mirrored_structs_match_the_header():
    for jname, cname in PAIRS.items():
        c, j = c_struct(cname), jl_struct(jname)
        assert [n for n, _ in c] == [n for n, _ in j], (jname, c, j)
        for (n, ct), (_, jt) in zip(c, j):
            if "[" in ct:
                assert jt.startswith("NTuple{"), (jname, n, jt)
            else:
                assert C2JL[ct] == jt, (jname, n, ct, jt)
