"""Dev tool: FK of the same joints through two library builds; prints the worst differences."""
import os, sys, subprocess, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
if len(sys.argv) > 2 and sys.argv[1] == "child":
    import torch, oracle
    from ctr_reach_amd import CtrReachVecEnv
    n = 65536
    q, _ = oracle.sample_joints(n, seed=0, stream=1)
    env = CtrReachVecEnv(1, device="cuda:0")
    tip, st = env.forward_kinematics(torch.tensor(q, device="cuda:0"), None, return_stats=True)
    np.savez(sys.argv[2], q=q, tip=tip.cpu().numpy(), nfev=st["nfev"].cpu().numpy(), nseg=st["nseg"].cpu().numpy())
    sys.exit(0)
libdir = os.path.join(ROOT, "gym-ctr-reach_amd", "ctr_reach_amd", "lib")
outs = []
for lib in sys.argv[1:3]:
    out = "/tmp/cmp_%s.npz" % lib
    subprocess.check_call([sys.executable, __file__, "child", out], env=dict(os.environ, CTR_REACH_AMD_LIB=os.path.join(libdir, lib)))
    outs.append(np.load(out))
import oracle
a, b = outs
ref = oracle.fk(a["q"])
for name, d in (("A", a), ("B", b)):
    e = np.abs(d["tip"] - ref["tip"]).max(1)
    print(name, "max %.3g  n>1e-12: %d  nfev!=oracle: %d" % (e.max(), (e > 1e-12).sum(), (d["nfev"] != ref["nfev"]).sum()))
e = np.abs(b["tip"] - ref["tip"]).max(1)
for i in np.argsort(-e)[:5]:
    print(i, e[i], a["q"][i].tolist(), "nfev A/B/oracle", a["nfev"][i], b["nfev"][i], ref["nfev"][i], "nseg", a["nseg"][i], ref["nseg"][i])
