"""Diagnostic: k_step time (autoreset off, HIP events) with lane i = env i versus the work-aware
lane order built by ctr_sort_envs from the previous step's keys."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv, _abi  # noqa: E402

n = 65536
env = CtrReachVecEnv(n, device="cuda", seed=0, sort_interval=1000000)
env.reset()
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
for k in range(30):
    env.step_raw(acts[k % 8])
torch.cuda.synchronize()
sp = _abi.stream_ptr()


def time_steps(K=20):
    st = {k: getattr(env, k).clone() for k in ("joints", "t", "achieved_goal")}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(K):
        rc = env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % 8]), env._out, 0, sp)
        _abi.check(rc, "ctr_step")
    e1.record()
    torch.cuda.synchronize()
    for k, v in st.items():
        getattr(env, k).copy_(v)
    return e0.elapsed_time(e1) / K * 1e3


zero = torch.zeros((n, 6), device="cuda")
acts = [zero] * 8                                  # joints stay put: every timed step has the same FK work
env.step_raw(zero)
torch.cuda.synchronize()
keys = env.sort_key.cpu().numpy()
p = np.argsort(keys, kind="stable")
J = env.joints.clone()


def time_fk(qq, K=20):
    env.forward_kinematics(qq)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        env.forward_kinematics(qq)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K * 1e3


pt = torch.tensor(p.astype(np.int64), device="cuda")
print("k_fk natural %.1f us, key-sorted %.1f us" % (time_fk(J), time_fk(J[pt].contiguous())))
env.perm.copy_(torch.arange(n, dtype=torch.int32, device="cuda"))
print("k_step identity perm %.1f us" % time_steps())
env.perm.copy_(pt.to(torch.int32))
print("k_step key-sorted perm %.1f us" % time_steps())
# no divergence at all: every env gets the same (median-work) joints
med = int(p[n // 2])
Jm = J[med:med + 1].expand(n, 6).contiguous()
print("k_fk all-identical %.1f us" % time_fk(Jm))
env.perm.copy_(torch.arange(n, dtype=torch.int32, device="cuda"))
env.joints.copy_(Jm)
print("k_step all-identical %.1f us" % time_steps())
# fresh key order applied physically (identity perm, permuted state)
env.perm.copy_(torch.arange(n, dtype=torch.int32, device="cuda"))
for name in ("desired_goal", "achieved_goal", "t", "system", "epoch"):
    getattr(env, name).copy_(getattr(env, name)[pt])
env.joints.copy_(J[pt])
print("k_step physically key-sorted %.1f us" % time_steps())
env.joints.copy_(J)
print("k_step physically natural %.1f us" % time_steps())
# key order restricted to each XCD class (workgroup index mod 8): an env's rows stay in one L2
ipt = torch.argsort(pt)
for name in ("desired_goal", "achieved_goal", "t", "system", "epoch"):
    getattr(env, name).copy_(getattr(env, name)[ipt])   # undo the physical permutation
env.joints.copy_(J)
idx = np.arange(n)
cls = (idx // 256) % 8
pc = np.empty(n, np.int64)
for c in range(8):
    members = idx[cls == c]                       # lanes (= env ids) of class c, increasing
    order = members[np.argsort(keys[members], kind="stable")]
    pc[members] = order                           # k-th lane of the class runs the k-th lightest env
print("perm sorted within XCD class: keys monotone per class:",
      all((np.diff(keys[pc[cls == c]]) >= 0).all() for c in range(8)))
env.perm.copy_(torch.tensor(pc.astype(np.int32), device="cuda"))
print("k_step class-sorted perm %.1f us" % time_steps())
env.perm.copy_(torch.arange(n, dtype=torch.int32, device="cuda"))
print("k_step identity again %.1f us" % time_steps())
