"""Experiment: k_step's launch time with E extra spinning workgroups of T ns appended to its grid
(tools/experiments/tail_probe.sh -> libab_tail.so; scripts/gpu.sh tailprobe; CTR_TAIL_WG = E, CTR_TAIL_NS = T), 65 536 envs,
compliant scipy RK45, auto-reset off, 32 launches after 64 untimed ones from a stepped state.
usage: CTR_REACH_AMD_LIB=.../libab_tail.so CTR_TAIL_WG=E CTR_TAIL_NS=T python tools/tail_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv, _abi  # noqa: E402

n = 65536
env = CtrReachVecEnv(n, device="cuda", seed=0, autoreset=False, record_info=False)
env.reset()
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
sp = _abi.stream_ptr(None)
q0 = None
for i in range(64):
    _abi.check(env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % 8]), env._out, 0, sp), "ctr_step")
q0 = env.joints.clone()
res = []
for rep in range(3):
    env.joints.copy_(q0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(32):
        _abi.check(env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % 8]), env._out, 0, sp), "ctr_step")
    e1.record()
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) / 32 * 1e3)
print("extra WG %5s  spin %6s ns: k_step %.2f us (reps %s)" % (os.environ.get("CTR_TAIL_WG", "0"),
      os.environ.get("CTR_TAIL_NS", "0"), min(res), ", ".join("%.2f" % r for r in res)))
