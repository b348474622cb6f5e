"""The C-ABI gradient all-reduce (kanode_comm_*, RCCL) on the GPU: a one-rank communicator sums in place
(the identity, bitwise), on a side stream in stream order, for f32 and f64; the same [dp; L] +
kanode_adam_step sequence a Julia host runs per optimiser step."""
import numpy as np
import pytest
import torch

from gpu_util import device

import kanode
from kanode import comm

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_one_rank_allreduce_is_identity_in_stream_order(dtype):
    dev = device()
    c = comm.Comm(1, 0, comm.unique_id(), dev.index or 0)
    assert c.size == 1 and c.rank == 0
    x = torch.as_tensor(np.random.default_rng(3).normal(size=4097), dtype=dtype, device=dev)
    ref = x.clone()
    s = torch.cuda.Stream(dev)
    y = torch.empty_like(x)
    with torch.cuda.stream(s):
        y.copy_(x)                      # producer on the side stream, then the all-reduce behind it
        c.allreduce_sum_(y, stream=s.cuda_stream)
    s.synchronize()
    assert torch.equal(y, ref)
    c.allreduce_sum_(x[:0])             # empty: no-op
    with pytest.raises(ValueError):
        c.allreduce_sum_(x.cpu())
    c.close()


def test_comm_then_adam_step_matches_trainer_update():
    """[dp; L] all-reduced (one rank) then kanode_adam_step with scale = 1/nranks: the FusedAdam update."""
    dev = device()
    c = comm.Comm(1, 0, comm.unique_id(), dev.index or 0)
    rng = np.random.default_rng(4)
    p = torch.as_tensor(rng.normal(size=240), device=dev)
    g = torch.as_tensor(rng.normal(size=241), device=dev)     # [dp; L]
    c.allreduce_sum_(g)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    x = p.clone()
    st = torch.cuda.current_stream(dev).cuda_stream
    assert kanode.lib().kanode_adam_step(x.data_ptr(), m.data_ptr(), v.data_ptr(), g.data_ptr(), 240, 1,
                                         1.0 / c.size, 5e-4, 0.9, 0.999, 1e-8, 0.9, 0.999, st) == 0
    xr = p.clone()
    kanode.FusedAdam(eta=5e-4).update(xr, g, 1.0 / c.size)   # kanode.Trainer's update after its all-reduce
    torch.cuda.synchronize()
    assert torch.equal(x, xr)
    c.close()


def test_two_ranks_join_or_fail_cleanly():
    """tools/comm_two_ranks.py: two processes join one communicator and all-reduce.  With two GPUs they sum
    (rank r on device r); with one GPU RCCL refuses two ranks on the same device, and that must come back
    as an error from kanode_comm_create in both processes (no hang)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "comm_two_ranks.py")], capture_output=True,
                       text=True, timeout=240)
    out = r.stdout + r.stderr
    if torch.cuda.device_count() >= 2:
        assert r.returncode == 0 and out.count("sum ok True") == 2, out[-2000:]
    else:
        assert r.returncode != 0 and out.count("kanode_comm_create failed (status 3)") == 2, out[-2000:]
