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


def _strip(src):
    """Julia source without comments, docstrings and string literals (for structural checks)."""
    src = re.sub(r'"""[\s\S]*?"""', '""', src)
    src = re.sub(r'"(?:\\.|[^"\\])*"', '""', src)
    return "\n".join(line.split("#", 1)[0] for line in src.splitlines())


def _functions(src):
    """name -> body of every `function name(...) ... end` block (top level, indentation 0)."""
    out = {}
    for m in re.finditer(r"^function ([\w.]+)\(.*?^end\b", src, flags=re.S | re.M):
        out.setdefault(m.group(1), []).append(m.group(0))
    return out


def test_blocks_balance():
    """Every block opener has its `end` (Julia is absent, so this stands in for the parser): `end`
    inside an index expression (x[end]) is not counted."""
    s = _strip(JL)
    while True:
        t = re.sub(r"\[[^\[\]]*\]", "[]", s)
        if t == s:
            break
        s = t
    s = re.sub(r"\bmutable struct\b", "struct", s)
    # block keywords open a statement (line start); generator `for`s inside calls and short-circuit
    # guards (`cond || throw(...)`) open nothing; `do` opens a block wherever it stands
    openers = len(re.findall(r"^\s*(?:function|struct|module|if|for|while|let|begin|try|quote|macro)\b", s, re.M))
    openers += len(re.findall(r"\bdo\b", s))
    assert openers == len(re.findall(r"\bend\b", s))
    assert s.count("(") == s.count(")")


def test_enum_values_match_the_header():
    def enum(prefix):
        return {m.group(1).lower(): int(m.group(2)) for m in re.finditer(prefix + r"(\w+)\s*=\s*(\d+)", HDR)}
    norm, basis = enum("KANODE_NORM_"), enum("KANODE_BASIS_")
    jl_norm = dict(re.findall(r":(\w+) => (\d+)", re.search(r"const NORM = Dict\((.*?)\)\n", JL, re.S).group(1)))
    jl_basis = dict(re.findall(r":(\w+) => (\d+)", re.search(r"const BASIS = Dict\((.*?)\)\n", JL, re.S).group(1)))
    for k, v in norm.items():
        assert int(jl_norm[k]) == v, k
    for k, v in basis.items():
        assert int(jl_basis[k]) == v, k
    assert "Float32 => Int32(0)" in JL and "Float64 => Int32(1)" in JL     # kanode_dtype


def test_lux_and_chainrules_surface():
    """Lux.setup on the layer must give the reference axes (initialparameters /
    initialstates / parameterlength / statelength), and the layer, the Fisher-KPP RHS and the device
    solve must each carry an rrule."""
    s = _strip(JL)
    for pat in (r"function LuxCore\.initialparameters\(rng::AbstractRNG, l::KANChainHip\)",
                r"function LuxCore\.initialstates\(::AbstractRNG, l::KANChainHip\)",
                r"LuxCore\.parameterlength\(l::KANChainHip\)",
                r"LuxCore\.statelength\(l::KANChainHip\)",
                r"ChainRulesCore\.rrule\(l::KANChainHip,",
                r"ChainRulesCore\.rrule\(f::RCKanodeHip,",
                r"ChainRulesCore\.rrule\(::typeof\(solve_tsit5\),",
                r"glorot_uniform\(rng, Int\(s\.out_dims\), Int\(s\.grid_len\) \* Int\(s\.in_dims\)\)",
                r"Symbol\(\"layer_\", i\)"):
        assert re.search(pat, JL), pat
    # layerspec passes every kanode_layer_spec choice through, and the handle takes Float32
    m = re.search(r"function layerspec\((.*?)\)\n", s, re.S)
    for kw in ("normalizer", "basis_func", "use_base_act", "grid_lims", "denominator", "iqf_reference_quirk"):
        assert kw in m.group(1), kw
    assert re.search(r"function Handle\(ls::Vector\{LayerSpec\}; T::Type", s)


def test_every_kernel_call_checks_its_sizes():
    """The C side trusts the sizes it is given: each Julia entry that hands host arrays to the
    library checks length(p) == kanode_param_length and the state rows before the ccall."""
    fns = _functions(_strip(JL))
    for name, sym in (("rhs", "kanode_rhs_host"), ("vjp", "kanode_vjp_host"), ("solve_impl", None)):
        body = fns[name][0]
        assert "checkp(h, p)" in body and "checku(h, " in body, name
        if sym:
            assert body.index("checkp(h, p)") < body.index(sym), name
    assert "solve_impl(" in fns["solve_tsit5"][0]
    checkp = fns["checkp"][0]
    assert "length(p) == h.P" in checkp and "DimensionMismatch" in checkp
