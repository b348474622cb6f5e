#!/usr/bin/env python3
"""Two ranks of the C-ABI communicator (kanode_comm_*) on the GPU(s) this box has: the parent (which never
touches the GPU) makes the unique id and starts two child processes; each joins as its rank on device
rank % n_gpus, all-reduces a vector of (rank + 1) and [dp; L]-shaped data, and checks the sums.
    python3 tools/comm_two_ranks.py            (exit 0: both ranks agree)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kan-odes_amd"))


def child(rank, nranks, uid_hex):
    import numpy as np
    import torch
    from kanode import comm
    ndev = torch.cuda.device_count()
    dev = rank % ndev
    torch.cuda.set_device(dev)
    c = comm.Comm(nranks, rank, bytes.fromhex(uid_hex), dev)
    x = torch.full((1000,), float(rank + 1), dtype=torch.float64, device=f"cuda:{dev}")
    c.allreduce_sum_(x)
    g = torch.as_tensor(np.random.default_rng(rank).normal(size=241), device=f"cuda:{dev}")
    tot = sum(np.random.default_rng(r).normal(size=241) for r in range(nranks))
    c.allreduce_sum_(g)
    torch.cuda.synchronize()
    ok = bool(torch.all(x == nranks * (nranks + 1) / 2)) and float((g.cpu().numpy() - tot).__abs__().max()) < 1e-12
    print(f"rank {rank} on device {dev} of {ndev}: sum ok {ok}", flush=True)
    c.close()
    return 0 if ok else 1


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        sys.exit(child(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]))
    from kanode import comm   # the id needs no device
    uid = comm.unique_id().hex()
    n = 2
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    ps = [subprocess.Popen([sys.executable, __file__, "--child", str(r), str(n), uid], env=env) for r in range(n)]
    rc = [p.wait(timeout=240) for p in ps]
    print("children exit codes", rc)
    sys.exit(0 if all(r == 0 for r in rc) else 1)


if __name__ == "__main__":
    main()
