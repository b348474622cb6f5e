#!/usr/bin/env python3
"""Cross-pass stall attribution from rocprofv3 --pmc CSVs (one pass per sub-directory of ROOT):
per kernel, the per-dispatch mean of every counter, then the split of wave cycles into
active / issue-stalled / parked (MI355X_MICROARCH.md §rocprofv3 PMC slots: WAIT_ANY = parked on
s_waitcnt or a barrier, WAIT_INST_ANY = issue stall, WAIT_INST_LDS = its LDS-issue sub-bucket;
the three buckets are disjoint and sum to SQ_WAVE_CYCLES).
  python3 tools/pmc_stall.py ROOT [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
want = sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "kan::" not in name:
            continue
        short = name.split("(")[0].replace("void kan::", "")
        if want and not any(w in short for w in want):
            continue
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))

for k, d in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    n = max(len(v) for v in d.values())
    print(f"{k}  ({n} dispatches/pass)")
    print("  " + " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        parts = [(c, m[c]) for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY") if c in m]
        print("  wave-cycle split: " + "  ".join(f"{c[3:]}={v / wc:.1%}" for c, v in parts)
              + f"  (sum {sum(v for _, v in parts) / wc:.1%})")
        for c in ("SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA",
                  "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_FLAT", "SQ_INST_CYCLES_SMEM"):
            if c in m:
                print(f"    {c[3:]} = {m[c] / wc:.1%} of wave cycles")
    w = m.get("SQ_WAVES")
    if w:
        per = {c: m[c] / w for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM",
                                       "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH",
                                       "SQ_INSTS_VALU_TRANS_F64") if c in m}
        print("  per wave: " + " ".join(f"{c[9:]}={v:.1f}" for c, v in per.items()))
    if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
        print(f"  LDS bank-conflict cycles / LDS active = {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.1%}")
    if "GRBM_GUI_ACTIVE" in m:
        print(f"  GRBM_GUI_ACTIVE/8 = {m['GRBM_GUI_ACTIVE'] / 8:.4g} cycles per dispatch")
