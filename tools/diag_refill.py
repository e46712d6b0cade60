"""Diagnostic: where k_refill's time goes, per wave, from the clock-stamped build
(tools/experiments/diag_refill.sh -> libab_diag.so; never the product library).  Steady state of
the headline (65 536 envs, R = 20, pool 64, refill budget from argv), then one refill with the
stamps: per phase, the mean and the slowest wave's cycles, and the phases of the wave that ends
last.  Phases: 0 start -> 1 tables staged -> 2 joints sampled -> 3 suspended state read ->
4 FK done -> 5 pool / carry stores done.
usage: CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_diag.so \
       python tools/diag_refill.py [budget]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

budget = int(sys.argv[1]) if len(sys.argv) > 1 else 6     # >= 1: the stamps need the carry lists
n, R = 65536, 20
env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=R, pool_depth=64, refill_budget=budget,
                     record_info=False)
env.reset()
g0 = torch.Generator(device="cpu")
g0.manual_seed(2)
env.t.copy_(torch.randint(0, 150, (n,), generator=g0, dtype=torch.int32))
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
for i in range(30 * R):
    env.step_raw(acts[i % 8])
for i in range(R - 1):
    env.step_raw(acts[i % 8])
env._steps_since_refill = 0
env.step_raw(acts[0])
torch.cuda.synchronize()
stamps = torch.zeros(2 * 1024 * 8 * 64, dtype=torch.int64, device="cuda")
env.carry[520:528].copy_(torch.tensor([stamps.data_ptr()], dtype=torch.int64).view(torch.uint8))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(200000)
e0.record()
env.refill_pool()
e1.record()
torch.cuda.synchronize()
d = stamps.cpu().numpy()[:1024 * 8 * 64].reshape(1024, 8, 64)[:, :, 0]      # lane 0's copy
span_us = e0.elapsed_time(e1) * 1e3
zero = (d == 0).sum(axis=0)
print("unwritten stamps per phase:", zero[:6].tolist())
d = d[(d[:, :6] != 0).all(axis=1)].astype(np.float64) / 100.0    # s_memrealtime: 100 MHz -> us
# (the counters of different XCDs are not comparable: only differences within a wave are used)
span = d[:, 5] - d[:, 0]
print("k_refill %.1f us (events); a wave spans %.2f us on average, %.2f at most" % (span_us, span.mean(), span.max()))
names = ["staging", "sampling", "state read", "FK", "stores"]
for k in range(5):
    ph = d[:, k + 1] - d[:, k]
    print("  %-10s mean %6.2f us  max %6.2f us" % (names[k], ph.mean(), ph.max()))
w = int(np.argmax(span))
print("  the longest wave (%d): %s" % (w, ", ".join("%s %.2f" % (names[k], d[w, k + 1] - d[w, k]) for k in range(5))))

# one pooled step with the stamps (k_step: 0 start -> 1 tables staged -> 2 rows read + set_action
# -> 3 FK -> 4 reward / obs / reset / stores)
env._steps_since_refill = 0
env.step_raw(acts[1])
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(200000)
e0.record()
env.step_raw(acts[2])
e1.record()
torch.cuda.synchronize()
d = stamps.cpu().numpy()[1024 * 8 * 64:].reshape(1024, 8, 64)[:, :, 0]
print("unwritten k_step stamps per phase:", (d == 0).sum(axis=0)[:5].tolist())
d = d[(d != 0).all(axis=1)].astype(np.float64) / 100.0
span = d[:, 4] - d[:, 0]
print("k_step %.1f us (events); a wave spans %.2f us on average, %.2f at most" %
      (e0.elapsed_time(e1) * 1e3, span.mean(), span.max()))
names = ["staging", "rows + set_action", "FK", "finish"]
for k in range(4):
    ph = d[:, k + 1] - d[:, k]
    print("  %-18s mean %6.2f us  max %6.2f us" % (names[k], ph.mean(), ph.max()))
w = int(np.argmax(span))
print("  the longest wave (%d): %s" % (w, ", ".join("%s %.2f" % (names[k], d[w, k + 1] - d[w, k]) for k in range(4))))
print("  staging split: tables copied %.2f, SysK derived %.2f, segment LUT %.2f (means)" %
      ((d[:, 5] - d[:, 0]).mean(), (d[:, 6] - d[:, 5]).mean(), (d[:, 1] - d[:, 6]).mean()))
app = d[:, 7] - d[:, 4]
print("  refill-queue append after the finish: mean %.2f us, max %.2f us; on the longest wave %.2f" %
      (app.mean(), app.max(), app[w]))
