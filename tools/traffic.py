#!/usr/bin/env python3
"""HBM bytes per launch of the FK kernels from the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly half of the bytes
of a wide coalesced streaming read (16 B/lane), so the read side is doubled; WRITE_SIZE is
exact for 16-B/lane streaming stores.  Both counters are in KiB per dispatch.
"""
import csv
import glob
import json
import os
import sys


def mean_counter(path, kernel_sub, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel_sub in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(vals) / len(vals) if vals else None


root = sys.argv[1]
NX = 256
# (pmc pass name, kernel-name substring, traffic.json key, algorithmic 8-byte words per trajectory)
PASSES = (("fk_rhs", "fk_rhs_pp_wave_kernel", "fisher_kpp_256:table", 2 * NX),
          ("fk_rhs_rec", "fk_rhs_kernel", "fisher_kpp_256:recurrence", 2 * NX),
          ("fk_vjp", "fk_vjp_pp_wave_kernel", "fisher_kpp_256_vjp", 3 * NX))
out = {}
for w, kern, key, words in PASSES:
    f = glob.glob(os.path.join(root, f"pmc_{w}_FETCH_SIZE", "**", "*counter_collection.csv"), recursive=True)
    wr = glob.glob(os.path.join(root, f"pmc_{w}_WRITE_SIZE", "**", "*counter_collection.csv"), recursive=True)
    if not f or not wr:
        continue
    fetch = mean_counter(f[0], kern, "FETCH_SIZE")
    write = mean_counter(wr[0], kern, "WRITE_SIZE")
    if fetch is None or write is None:
        continue
    batch = int(os.environ.get("BATCH", "131072"))
    alg = 8.0 * (11 + batch * words)
    hbm = (2.0 * fetch + write) * 1024.0
    out[key] = {
        "batch": batch, "kernel": kern, "fetch_size_kib": fetch, "write_size_kib": write,
        "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": hbm / alg,
        "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), WRITE_SIZE as is",
    }
print(json.dumps(out, indent=1))
