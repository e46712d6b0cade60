"""Diagnostic: the duration of every k_step wave of one launch, from a library built with
-DCTR_DIAG_WAVETIME (each wave's lane 0 stores the kernel's start, the FK's start and end, the finish's and the appends'
end, and the kernel's end on the
100 MHz real-time clock).
Is the launch as long as its slowest wave with the others close behind (per-iteration cost is the
lever), or do a few waves trail the rest (work balance is)?

build: PATCH=tools/experiments/diag.patch EXTRA=-DCTR_DIAG_WAVETIME bash tools/experiments/build_rev.sh HEAD wavet
       (the diagnostic is a patch, not part of the product sources)
usage: CTR_REACH_AMD_LIB=.../libab_wavet.so python tools/wave_times.py [n_envs]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv, _abi  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=64)
env.reset()
lib = env.lib
lib.ctr_diag_wavetimes.argtypes = [ctypes.c_void_p, ctypes.c_int]
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
g0 = torch.Generator(device="cpu")
g0.manual_seed(2)
env.t.copy_(torch.randint(0, 150, (n,), generator=g0, dtype=torch.int32))
stream = torch.cuda.current_stream()
sp = _abi.stream_ptr(stream)
nw = n // 64
rows = []
for mode, name in ((0, "autoreset off"), (_abi.AUTORESET_POOLED, "pooled auto-reset")):
    for i in range(300):
        _abi.check(lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % 8]), env._out, mode, sp), "ctr_step")
        if mode and i % 32 == 31:
            env.refill_pool()
    durs, spans, pre, fk, post, st0, fin, app, end = [], [], [], [], [], [], [], [], []
    for rep in range(8):
        _abi.check(lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[rep % 8]), env._out, mode, sp), "ctr_step")
        torch.cuda.synchronize()
        t = np.zeros((nw, 6), dtype=np.uint64)
        _abi.check(lib.ctr_diag_wavetimes(t.ctypes.data, nw), "ctr_diag_wavetimes")
        d = (t[:, 5] - t[:, 0]).astype(np.float64) * 0.01          # us
        durs.append(d)
        pre.append((t[:, 1] - t[:, 0]).astype(np.float64) * 0.01)
        fk.append((t[:, 2] - t[:, 1]).astype(np.float64) * 0.01)
        post.append((t[:, 5] - t[:, 2]).astype(np.float64) * 0.01)
        fin.append((t[:, 3] - t[:, 2]).astype(np.float64) * 0.01)
        app.append((t[:, 4] - t[:, 3]).astype(np.float64) * 0.01)
        end.append((t[:, 5] - t[:, 4]).astype(np.float64) * 0.01)
        st0.append((t[:, 0] - t[:, 0].min()).astype(np.float64) * 0.01)
        spans.append((t[:, 5].max() - t[:, 0].min()) * 0.01)
    d = np.concatenate(durs)
    q = np.percentile(d, [0, 10, 50, 90, 99, 100])
    print("%-18s wave us: min %.1f p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f mean %.1f | launch span %.1f us "
          "| mean/max %.3f" % (name, *q, d.mean(), float(np.mean(spans)), d.mean() / q[-1]), flush=True)
    for lab, arr in (("start skew", st0), ("pre-FK", pre), ("FK", fk), ("post-FK", post), ("  finish", fin),
                     ("  appends", app), ("  to end", end)):
        a = np.concatenate(arr)
        print("    %-10s us: p50 %.2f p90 %.2f max %.2f mean %.2f" % (lab, *np.percentile(a, [50, 90, 100]), a.mean()),
              flush=True)
    # does the previous launch predict the slow waves?  (consecutive launches of the same envs)
    cor = np.mean([np.corrcoef(durs[k], durs[k + 1])[0, 1] for k in range(len(durs) - 1)])
    top = np.mean([len(set(np.argsort(durs[k])[-16:]) & set(np.argsort(durs[k + 1])[-16:])) / 16.0
                   for k in range(len(durs) - 1)])
    rank = np.mean([int((durs[k] > durs[k][int(np.argmax(durs[k + 1]))]).sum()) for k in range(len(durs) - 1)])
    print("    consecutive launches: duration correlation %.3f, top-16 overlap %.2f, the next slowest wave's "
          "rank in this launch %.1f (0 = slowest)" % (cor, top, rank), flush=True)
    sl = int(np.argmax(durs[0]))
    print("    slowest wave of launch 0: #%d  pre %.2f FK %.2f post %.2f start %.2f" % (
        sl, pre[0][sl], fk[0][sl], post[0][sl], st0[0][sl]), flush=True)
