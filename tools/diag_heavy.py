import os, sys, numpy as np, torch
sys.path.insert(0, "/root/repo/gym-ctr-reach_amd") if os.path.exists("/root/repo/gym-ctr-reach_amd") else None
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv
n = 65536
env = CtrReachVecEnv(n, device="cuda", seed=0)
env.reset()
g = torch.Generator(device="cuda"); g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
for k in range(20):
    env.step(((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous())
J = env.joints.clone()
_, st = env.forward_kinematics(J, return_stats=True)
att = (st["nstep"] + st["nrej"]).cpu().numpy(); seg = st["nseg"].cpu().numpy()
def t(q, K=20):
    env.forward_kinematics(q); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K): env.forward_kinematics(q)
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1) / K * 1e3
print("attempts: mean %.2f max %d; segs mean %.2f" % (att.mean(), att.max(), seg.mean()))
print("natural %.1f us" % t(J))
for name, idx in (("heaviest", int(np.argmax(att * 8 + seg))), ("median", int(np.argsort(att)[n // 2])), ("p99", int(np.argsort(att)[int(n * 0.99)]))):
    print("all = %s (att %d, seg %d): %.1f us" % (name, att[idx], seg[idx], t(J[idx:idx + 1].expand(n, 6).contiguous())))
