"""Diagnostic: k_step time (HIP events, 100 back-to-back launches after 300 warm ones) for the
library named by CTR_REACH_AMD_LIB, with auto-reset off and with the pooled auto-reset; then the
FK operator alone (ctr_fk) on the same joints.
usage: python tools/time_step_modes.py [n_envs] [rigid|c5]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv, _abi  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
kw = {}
if len(sys.argv) > 2 and sys.argv[2] == "rigid":      # configs[1]: rigid model, RK4 at 100 steps/m
    kw = dict(integrator="rk4", rk4_steps_per_m=100, model="rigid")
if len(sys.argv) > 2 and sys.argv[2] == "c5":         # configs[4]: compliant model, RK4 at 400 steps/m
    kw = dict(integrator="rk4", rk4_steps_per_m=400, model="compliant")
env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=64, **kw)
env.reset()
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
g0 = torch.Generator(device="cpu")
g0.manual_seed(2)
env.t.copy_(torch.randint(0, 150, (n,), generator=g0, dtype=torch.int32))
stream = torch.cuda.current_stream()
sp = _abi.stream_ptr(stream)
for mode, name in ((0, "autoreset off"), (_abi.AUTORESET_POOLED, "pooled auto-reset")):
    for i in range(300):
        _abi.check(env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % 8]), env._out, mode, sp), "ctr_step")
        if mode and i % 32 == 31:
            env.refill_pool()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(100):
        _abi.check(env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % 8]), env._out, mode, sp), "ctr_step")
    e1.record(stream)
    torch.cuda.synchronize()
    print("%-20s k_step %.2f us" % (name, e0.elapsed_time(e1) / 100 * 1e3), flush=True)
# the FK operator alone (ctr_fk: k_fk) on the batch's current joints, same clocks
q = env.joints.clone()
for i in range(100):
    env.forward_kinematics(q)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for i in range(100):
    env.forward_kinematics(q)
e1.record(stream)
torch.cuda.synchronize()
print("%-20s k_fk   %.2f us" % ("FK operator", e0.elapsed_time(e1) / 100 * 1e3), flush=True)
