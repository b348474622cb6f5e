import sys, os
sys.path[:0] = [os.environ.get("GRAFT_REPO_ROOT", "."), os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"),
                os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "kan-odes_amd")]
import test_gpu_fk_e2e as T
for opts in ({}, {"fk_device_loop": 0}, {"pointwise_table": 0}, {"fk_device_loop": 0, "fused_step": 0}):
    try:
        sg = T._e2e(256, 3, "adaptive", seed=31, diffusion=0.0, amp=1.0, shift=-2.2, pscale=0.5, **opts)
        print(opts, "OK", sg["naccept"], sg["adjoint"]["naccept"], flush=True)
    except AssertionError as e:
        print(opts, "FAIL", repr(e)[:300], flush=True)
