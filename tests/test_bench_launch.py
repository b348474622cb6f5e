"""bench.py's rank launcher: `bench.py --gpus N` without an external launcher must
start N ranks itself, an external launcher's WORLD_SIZE must agree with --gpus, and a failing rank
must end the job with a non-zero status instead of hanging it.  CPU only: the children here are small
Python programs (a gloo process group where a collective is needed), not the GPU bench."""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_resolve_world_modes():
    assert bench.resolve_world(1, {}) == ("single", 1)
    assert bench.resolve_world(8, {}) == ("spawn", 8)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == ("rank", 4)
    assert bench.resolve_world(1, {"WORLD_SIZE": "1"}) == ("single", 1)
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "1"})      # torchrun started fewer ranks than asked for
    with pytest.raises(SystemExit):
        bench.resolve_world(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


_GLOO_CHILD = r"""
import os, sys, json, datetime
import torch, torch.distributed as dist
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
if dist.get_rank() == 0:
    print(json.dumps({"world": dist.get_world_size(), "sum": float(t.item()),
                      "launch": os.environ.get("KANODE_BENCH_LAUNCH"), "local": os.environ["LOCAL_RANK"]}), flush=True)
dist.destroy_process_group()
"""


def test_launch_ranks_forms_a_process_group(tmp_path):
    out = tmp_path / "out.txt"
    with open(out, "w") as f:
        # run the launcher in a child so the children's stdout lands in the file
        code = ("import sys; sys.path.insert(0, %r); import bench; "
                "sys.exit(bench.launch_ranks(3, [sys.executable, '-c', %r]))") % (ROOT, _GLOO_CHILD)
        rc = subprocess.run([sys.executable, "-c", code], stdout=f, timeout=180).returncode
    assert rc == 0
    lines = [l for l in out.read_text().splitlines() if l.startswith("{")]
    assert len(lines) == 1, lines                     # only rank 0 prints
    import json
    d = json.loads(lines[0])
    assert d["world"] == 3 and d["sum"] == 6.0 and d["launch"] == "self" and d["local"] == "0"


def test_launch_ranks_failure_stops_the_job():
    # rank 1 fails at once; ranks 0 and 2 would sleep for 10 minutes: the launcher must stop them
    child = ("import os, sys, time\n"
             "r = int(os.environ['RANK'])\n"
             "sys.exit(3) if r == 1 else time.sleep(600)\n")
    t0 = time.time()
    rc = bench.launch_ranks(3, [sys.executable, "-c", child], grace_s=5.0)
    assert rc == 3
    assert time.time() - t0 < 60


def test_launch_ranks_all_ok():
    assert bench.launch_ranks(2, [sys.executable, "-c", "import os; assert os.environ['WORLD_SIZE'] == '2'"]) == 0
