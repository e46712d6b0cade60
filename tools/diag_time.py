"""In-kernel s_memtime split of the FK loop (diagnostic build CTR_DIAG_TIME): cycles in the
segment-start block, in RK stages 1-5, in K6 + error norm, and total, per lane (wave-uniform
clock, so per-wave values are what matter)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CTR_REACH_AMD_LIB"] = os.path.join(ROOT, "gym-ctr-reach_amd", "ctr_reach_amd", "lib",
                                               "libctr_reach_amd_time.so")
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
for rep in range(3):
    _, st = env.forward_kinematics(env.joints, env.system, return_stats=True)
s = np.stack([st["nfev"].cpu().numpy(), st["nstep"].cpu().numpy(), st["nrej"].cpu().numpy(),
              st["nseg"].cpu().numpy()], 1).astype(np.float64).reshape(-1, 64, 4)
w = s.max(1)          # per wave (lanes that stay longest)
tot = w[:, 3]
print("per-wave cycles: total mean %.0f max %.0f" % (tot.mean(), tot.max()))
for i, name in enumerate(["segment-start block", "stages 1-5", "K6 + error norm"]):
    print("  %-22s mean %.0f (%.1f%%)" % (name, w[:, i].mean(), 100 * w[:, i].mean() / tot.mean()))
slow = np.argmax(tot)
print("slowest wave: total %.0f, split %s" % (tot[slow], w[slow, :3]))
