"""Diagnostic: what would k_step gain from running each FK loop iteration at the wave's highest
*tube level* instead of always the full 3-tube RHS?

Tubes are present on [beta_i, beta_i + L_i] with beta_i <= 0, so along the backbone the set of
present tubes only shrinks: level 3 (tubes 0-2), then 2 (tubes 0-1; tube 2 absent: no
sin/cos(alpha_2 - alpha_0), no alpha_2 / u_z,2 stage sums), then 1 (tube 0 alone: no trig at all,
u_z,0 constant).  A wave executes an iteration at the highest level any of its active lanes needs
(a wave-uniform choice: lanes at a lower level compute exact zeros in the omitted terms).  This
replays every lane's per-segment attempt counts (CPU oracle, env-trajectory joints) through the
wave cost model of tools/sim_sched.py (segment-start block CI, attempt block CA per iteration)
with per-level block costs, relative to today's all-level-3 loop.

usage: python tools/sim_levels.py [n_envs] [system]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle  # noqa: E402
from sim_sched import trajectory_joints  # noqa: E402

# relative instruction counts of the attempt block (CA) and the segment-start block (CI) per level,
# from the source's operation counts ("census"): level 2 drops one table sincos + the
# angle-difference identity + 5 RHS products per RHS and the u_z,2 / alpha_2 stage, update and norm
# terms; level 1 drops both sincos, the identity and 12 of the 18 frame products per RHS and the
# u_z,1-2 / alpha_1-2 terms
CA = {3: 1.0, 2: 0.79, 1: 0.57}
CI = {3: 0.43, 2: 0.43 * 0.80, 1: 0.43 * 0.58}


def lane_levels(q, system=0):
    """Per env: list of (level, attempts) of its kept segments in integration order."""
    params = oracle.default_system_params()["ctr_%d" % system]
    L = np.array([params["tube_%d" % i]["length"] for i in range(3)])
    att = oracle.fk_segattempts(q, system=system)
    m, S = oracle.segments(q, system=system)
    out = []
    for e in range(q.shape[0]):
        beta = q[e, :3].astype(np.float64)
        seq, prev = [], 0.0
        for k in range(m[e]):
            mid = 0.5 * (prev + S[e, k])
            pres = [(beta[i] <= mid) and (mid < beta[i] + L[i]) for i in range(3)]
            lvl = 3 if pres[2] else (2 if pres[1] else 1)
            if att[e, k] > 0:
                seq.append((lvl, int(att[e, k])))
            prev = S[e, k]
        out.append(seq)
    return out


def wave_cost(lanes, levels=True):
    seg = [0] * len(lanes)
    left = [0] * len(lanes)
    done = [len(s) == 0 for s in lanes]
    cost, hist = 0.0, {1: 0, 2: 0, 3: 0}
    while not all(done):
        need_i = [i for i in range(len(lanes)) if not done[i] and left[i] == 0]
        if need_i:
            lv = max(lanes[i][seg[i]][0] for i in need_i) if levels else 3
            cost += CI[lv]
            for i in need_i:
                left[i] = lanes[i][seg[i]][1]
        runners = [i for i in range(len(lanes)) if not done[i] and left[i] > 0]
        if runners:
            lv = max(lanes[i][seg[i]][0] for i in runners) if levels else 3
            cost += CA[lv]
            hist[lv] += 1
            for i in runners:
                left[i] -= 1
                if left[i] == 0:
                    seg[i] += 1
                    if seg[i] >= len(lanes[i]):
                        done[i] = True
    return cost, hist


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    system = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    q = trajectory_joints(n, 12)
    lanes = lane_levels(q, system)
    lv_att = {1: 0, 2: 0, 3: 0}
    for s in lanes:
        for lv, a in s:
            lv_att[lv] += a
    tot = sum(lv_att.values())
    print("lane attempts by level: " + "  ".join("L%d %.1f%%" % (k, 100.0 * v / tot) for k, v in sorted(lv_att.items())))
    base, lev = [], []
    hist = {1: 0, 2: 0, 3: 0}
    for w in range(0, n, 64):
        b, _ = wave_cost(lanes[w:w + 64], levels=False)
        c, h = wave_cost(lanes[w:w + 64], levels=True)
        base.append(b)
        lev.append(c)
        for k in h:
            hist[k] += h[k]
    base, lev = np.array(base), np.array(lev)
    it = sum(hist.values())
    print("wave iterations by level: " + "  ".join("L%d %.1f%%" % (k, 100.0 * v / it) for k, v in sorted(hist.items())))
    print("wave cost today: mean %.2f  max %.2f" % (base.mean(), base.max()))
    print("with levels:     mean %.2f (%.3f)  max %.2f (%.3f)  slowest-wave ratio p99 %.3f" % (
        lev.mean(), lev.mean() / base.mean(), lev.max(), lev.max() / base.max(), np.quantile(lev / base, 0.99)))
