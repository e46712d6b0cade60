"""A/B bit-equality of two library builds on the same workload (run once per build, then compare).

  CTR_REACH_AMD_LIB=<lib.so> python tools/ab_bits.py run <out.npz> [envs] [steps]
      65 536 envs (default), staggered episode clocks, `steps` env steps with auto-reset and
      pooled refills (bench.py's workload), then one FK with device counters of the final
      joints; saves joints, goals, obs, rewards of every step, the FK tips and RHS counts.
  python tools/ab_bits.py cmp <a.npz> <b.npz>
      reports which arrays are bit-equal and the largest differences of those that are not.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))


def run(out, n=65536, steps=40):
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    dev = torch.device("cuda", 0)
    env = CtrReachVecEnv(n, device=dev, seed=0, refill_interval=20)
    env.reset()
    g = torch.Generator(device="cpu")
    g.manual_seed(17)
    env.t.copy_(torch.randint(0, env.max_steps_per_episode, (n,), generator=g, dtype=torch.int32))
    gd = torch.Generator(device=dev)
    gd.manual_seed(1)
    hi = torch.tensor(env.action_space.high, device=dev)
    rec = {"reward": [], "obs": [], "done": []}
    for _ in range(steps):
        a = ((torch.rand((n, 6), generator=gd, device=dev) * 2 - 1) * hi).contiguous()
        obs, rew, done, _ = env.step(a)
        rec["reward"].append(rew.cpu().numpy().copy())
        rec["obs"].append(obs["observation"].cpu().numpy().copy())
        rec["done"].append(done.cpu().numpy().copy())
    tip, st = env.forward_kinematics(env.joints, env.system, return_stats=True)
    np.savez(out, joints=env.joints.cpu().numpy(), desired_goal=env.desired_goal.cpu().numpy(),
             achieved_goal=env.achieved_goal.cpu().numpy(), t=env.t.cpu().numpy(), epoch=env.epoch.cpu().numpy(),
             fk_tip=tip.cpu().numpy(), fk_nfev=st["nfev"].cpu().numpy(),
             **{k: np.stack(v) for k, v in rec.items()})
    print("saved", out)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    for k in A.files:
        x, y = A[k], B[k]
        if x.dtype.kind == "f":
            same = np.array_equal(x.view(np.uint8), y.view(np.uint8))
        else:
            same = np.array_equal(x, y)
        if same:
            print("%-14s bit-equal %s" % (k, x.shape))
        else:
            d = np.abs(x.astype(np.float64) - y.astype(np.float64))
            print("%-14s DIFFERS: %d of %d elements, max |diff| %.3g" % (k, int((d > 0).sum()), d.size, float(np.nanmax(d))))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], *(int(v) for v in sys.argv[3:]))
    else:
        cmp(sys.argv[2], sys.argv[3])
