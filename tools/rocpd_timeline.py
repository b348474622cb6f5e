"""Print a window of the kernel + memory-copy timeline from a rocprofv3 rocpd database (-o run, default format):
gaps between consecutive device events show the host time of a launch-bound loop.
python tools/rocpd_timeline.py DB --anchor SUBSTR [--nth -2] [--before 12]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", required=True, help="kernel-name substring marking one iteration")
    ap.add_argument("--nth", type=int, default=-3, help="which anchor occurrence starts the window")
    ap.add_argument("--before", type=int, default=12, help="events shown before the anchor")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    ev = [(s, e, "K " + n[:70]) for s, e, n in cur.execute("select start, end, name from kernels")]
    ev += [(s, e, f"C {n} {z}") for s, e, n, z in cur.execute("select start, end, name, size from memory_copies")]
    ev.sort()
    idx = [i for i, e in enumerate(ev) if a.anchor in e[2]]
    lo, hi = idx[a.nth] - a.before, idx[a.nth + 1] - a.before
    t0, prev, busy = ev[lo][0], None, 0
    for s, e, n in ev[lo:hi]:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        busy += e - s
        print(f"{(s - t0) / 1e3:9.1f} +{gap:7.1f} dur {(e - s) / 1e3:7.1f}  {n}")
        prev = e
    span = (ev[hi][0] - t0) / 1e3
    print(f"window {span:.1f} us, device busy {busy / 1e3:.1f} us, idle {span - busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
