"""Per-env FK work statistics at the bench workload (GPU): RHS evaluations, RK attempts and
segments per env, and how they distribute over 64-lane waves.  Writes gpurun_out/work_stats.npz."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = CtrReachVecEnv(n, device="cuda", seed=0)
env.reset()
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
stats = []
for k in range(12):
    a = ((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous()
    env.step(a)
    _, st = env.forward_kinematics(env.joints, env.system, return_stats=True)
    stats.append(torch.stack([st["nfev"], st["nstep"], st["nrej"], st["nseg"]], 1).cpu().numpy())
torch.cuda.synchronize()
S = np.stack(stats)            # [steps, n, 4]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "work_stats.npz"), stats=S)
att = S[..., 1] + S[..., 2]
seg = S[..., 3]
w = att.reshape(att.shape[0], -1, 64)
print("attempts/env mean %.2f  p50 %d  p99 %d  max %d" % (att.mean(), np.median(att), np.percentile(att, 99), att.max()))
print("segments/env mean %.2f  max %d" % (seg.mean(), seg.max()))
print("per-wave max attempts: mean %.2f  max %d ; lane efficiency %.3f" % (w.max(-1).mean(), w.max(), att.mean() / w.max(-1).mean()))
print("nfev mean %.1f" % S[..., 0].mean())

# ---- reset pool behaviour at the bench workload: resets and pool misses per step
for depth, interval in ((4, 8), (4, 16), (4, 32), (6, 32), (8, 64)):
    env = CtrReachVecEnv(n, device="cuda", seed=0, pool_depth=depth, refill_interval=interval)
    env.reset()
    resets = misses = 0
    steps = 200
    for k in range(steps):
        a = ((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous()
        env.step_raw(a)
        resets += int(env.done.sum().item())
        misses += int(env.work[1 - env._batch.work_parity].item())
    print("pool depth %d refill every %d: resets/step %.1f  misses/step %.3f" % (depth, interval, resets / steps,
                                                                             misses / steps))
