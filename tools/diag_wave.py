"""Wave-level loop accounting (diagnostic build, CTR_DIAG_WAVE): per wave, RK-attempt loop
iterations and iterations that ran the divergent segment-start block."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CTR_REACH_AMD_LIB"] = os.path.join(ROOT, "gym-ctr-reach_amd", "ctr_reach_amd", "lib",
                                               "libctr_reach_amd_diag.so")
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

n = 65536
env = CtrReachVecEnv(n, device="cuda", seed=0)
env.reset()
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
for k in range(5):
    env.step(((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous())
_, st = env.forward_kinematics(env.joints, env.system, return_stats=True)
iters = st["nrej"].cpu().numpy().reshape(-1, 64).max(1)
inits = st["nseg"].cpu().numpy().reshape(-1, 64).max(1)
att = st["nstep"].cpu().numpy()
print("loop iterations per wave: mean %.2f max %d" % (iters.mean(), iters.max()))
print("iterations running the segment-start block: mean %.2f max %d (%.0f%%)" % (inits.mean(), inits.max(),
                                                                              100 * inits.mean() / iters.mean()))
print("accepted steps per env mean %.2f" % att.mean())
