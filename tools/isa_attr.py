#!/usr/bin/env python3
"""Static instruction attribution of one kernel in a device assembly file.

Build the assembly with line tables (the .loc directives carry the innermost source line of every
instruction after inlining):

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -gline-tables-only -I../include -Icsrc \
          --cuda-device-only -S -o /tmp/kan_pp_g.s csrc/kan_pp.hip

then

    python tools/isa_attr.py /tmp/kan_pp_g.s 'fk_vjp_step_rows_kernelILi2ELi2ELi10ELi2ELi2ELi256E' \
          --map tools/isa_attr_rows.map --per 24

Every instruction is attributed to the source line of the closest preceding .loc. A basic block is
*cold* when one of its instructions comes from a line range the map file marks cold (the direct-formula
fallback of the table path): the whole block is then excluded from the hot counts. The map file assigns
line ranges to named sections (``section file first-last``; ``cold`` is the reserved cold section); lines
outside every range are reported under ``file:line``. ``--per`` divides the hot counts (e.g. 24 = 6
stages x 4 points per lane: the kernel's stage and pair loops are fully unrolled, so the static count of
the hot blocks is the dynamic count of one wave-step).
"""
from __future__ import annotations

import argparse
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kind(mn: str) -> str:
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the kernel's mangled name")
    ap.add_argument("--map", help="section map: lines 'name file first-last'")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args(argv)

    sections = []
    scope = {}
    if a.map:
        for ln in open(a.map):
            ln = ln.split("#", 1)[0].strip()
            if not ln:
                continue
            parts = ln.split(None, 2)
            name, f = parts[0], parts[1]
            if name == "scope":   # 'scope FILE REGEX': later regex entries for FILE search from its first match on
                src = open(os.path.join(ROOT, "kan-odes_amd", "csrc", f)).read().splitlines()
                scope[f] = next(i for i, t in enumerate(src) if re.search(parts[2], t))
                continue
            if " ~~ " in parts[2]:
                # START-REGEX ~~ END-REGEX: the lines from the first match of start to the next match of end, in
                # the source as it is now (kan-odes_amd/csrc/<file>): regenerate the assembly after editing
                r0, r1 = (x.strip() for x in parts[2].split(" ~~ "))
                src = open(os.path.join(ROOT, "kan-odes_amd", "csrc", f)).read().splitlines()
                lo = next((i for i, t in enumerate(src) if i >= scope.get(f, 0) and re.search(r0, t)), None)
                hi = None if lo is None else next((i for i, t in enumerate(src) if i >= lo and re.search(r1, t)), None)
                if hi is None:
                    sys.exit(f"map entry {name}: {parts[2]} does not match {f}")
                lo, hi = lo + 1, hi + 1
            else:
                lo, hi = (int(x) for x in parts[2].split("-"))
            sections.append((name, f, lo, hi))

    files = {}
    lines = open(a.asm).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
        if start is None and re.match(r"^_Z\S*" + re.escape(a.kernel) + r"\S*:", ln):
            start = i
    if start is None:
        print("kernel not found", file=sys.stderr)
        return 1
    end = start + 1
    while end < len(lines) and not re.match(r"^\.Lfunc_end", lines[end]):
        end += 1

    def sect(f, l):
        for name, sf, lo, hi in sections:
            if sf == f and lo <= l <= hi:
                return name
        return f"{f}:{l}"

    def frames_sect(chain):
        # chain: [(file, line)] innermost first (the .loc comment's inlined-at list).  The compiler's own
        # headers (::fma, the DPP and lane builtins' wrappers) and line 0 are transparent.  Cold if any
        # frame is in a cold range; otherwise the innermost frame that a section claims, else the
        # innermost transparent-free frame.
        user = [(f, l) for f, l in chain if not (f.startswith(("__clang", "amd_")) or l == 0)]
        named = [sect(f, l) for f, l in user]
        if any(n == "cold" for n in named):
            return "cold"
        for (f, l), n in zip(user, named):
            if n != f"{f}:{l}":
                return n
        return named[0] if named else None

    blocks = []   # list of (label, [(kind, mnemonic, section)])
    cur = ("entry", [])
    loc = ("?", 0)
    for ln in lines[start + 1:end + 1]:
        s = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            chain = [(fp.split("/")[-1], int(lp)) for fp, lp in re.findall(r"([\w./+-]+):(\d+):\d+", s.split(";", 1)[-1])]
            n = frames_sect(chain) if chain else None
            if n is not None:
                loc = n
            continue
        if re.match(r"^\.LBB\S*:", s):
            blocks.append(cur)
            cur = (s[:-1], [])
            continue
        if not s or s.startswith((".", ";")):
            continue
        mn = s.split()[0]
        cur[1].append((kind(mn), mn, loc))
    blocks.append(cur)

    hot = collections.Counter()
    hot_kind = collections.Counter()
    cold_kind = collections.Counter()
    by_sec = collections.defaultdict(collections.Counter)
    ncold = 0
    for label, ins in blocks:
        is_cold = 2 * sum(sec == "cold" for _, _, sec in ins) > len(ins)
        if is_cold:
            ncold += 1
            for k, _, _ in ins:
                cold_kind[k] += 1
            continue
        for k, mn, sec in ins:
            hot_kind[k] += 1
            by_sec[sec][k] += 1
            hot[sec] += 1
    per = a.per
    print(f"kernel lines {start}-{end}; {len(blocks)} blocks, {ncold} cold")
    print("hot totals:", {k: v for k, v in hot_kind.items()}, f"(÷{per:g}:",
          {k: round(v / per, 1) for k, v in hot_kind.items()}, ")")
    print("cold totals:", dict(cold_kind))
    print(f"{'section':40s} {'valu':>8s} {'/per':>7s} {'lds':>6s} {'salu':>6s} {'smem':>5s} {'vmem':>5s}")
    rows = sorted(by_sec.items(), key=lambda kv: -kv[1]["valu"])
    for sec, c in rows[: a.top]:
        print(f"{sec:40s} {c['valu']:8d} {c['valu'] / per:7.1f} {c['lds']:6d} {c['salu']:6d} {c['smem']:5d} {c['vmem']:5d}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
