"""Diagnostic: wave-level cost model of k_step's FK loop under segment-start scheduling policies.

Each lane runs, per kept segment, one segment-start block (I: f0, select_initial_step's second
RHS and norms) and then that segment's RK45 attempts (A).  A wave issues a block whenever any of
its lanes needs it, so its cost is (# iterations running I) * CI + (# iterations running A) * CA.
Attempt counts per segment come from the CPU oracle on env-trajectory joints.  Policies:
  now        I whenever any lane needs it, then A in the same iteration (fk_lane today)
  batch K W  I only when >= K lanes wait for it, or a lane has waited W iterations, or no lane
             has an attempt to run; waiting lanes idle through the attempt block
`python tools/sim_sched.py sort` compares wave regroupings by predicted work instead.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402


def trajectory_joints(n, steps, seed=0):
    q, _ = oracle.sample_joints(n, seed)
    rng = np.random.default_rng(seed)
    hi = np.array([0.001, 0.001, 0.001, np.deg2rad(5), np.deg2rad(5), np.deg2rad(5)], np.float32)
    dg = np.zeros((n, 3))
    t = np.zeros(n, np.int32)
    for _ in range(steps):
        a = ((rng.random((n, 6)) * 2 - 1) * hi).astype(np.float32)
        out = oracle.step(q, a, dg, t, 0.02)
        q = out["joints"]
    return q


def lane_tasks(att_row):
    seq = []
    for a in att_row:
        if a <= 0:
            continue
        seq.append(("I", int(a)))
    return seq


def simulate(att, policy, K=1, W=0, CI=0.43, CA=1.0):
    n = att.shape[0]
    total = 0.0
    iters_tot = 0
    for w0 in range(0, n, 64):
        lanes = [lane_tasks(r) for r in att[w0:w0 + 64]]
        seg = [0] * len(lanes)
        left = [0] * len(lanes)          # attempts left in the current segment (0: needs I)
        waited = [0] * len(lanes)
        done = [len(s) == 0 for s in lanes]
        cost = 0.0
        it = 0
        while not all(done):
            need_i = [i for i in range(len(lanes)) if not done[i] and left[i] == 0]
            have_a = [i for i in range(len(lanes)) if not done[i] and left[i] > 0]
            run_i = bool(need_i) and (policy == "now" or len(need_i) >= K or not have_a or
                                      max(waited[i] for i in need_i) >= W)
            if run_i:
                cost += CI
                for i in need_i:
                    left[i] = lanes[i][seg[i]][1]
                    waited[i] = 0
            else:
                for i in need_i:
                    waited[i] += 1
            runners = [i for i in range(len(lanes)) if not done[i] and left[i] > 0]
            if runners:
                cost += CA
                for i in runners:
                    left[i] -= 1
                    if left[i] == 0:
                        seg[i] += 1
                        if seg[i] >= len(lanes[i]):
                            done[i] = True
            it += 1
        total += cost
        iters_tot += it
    return total / (n / 64), iters_tot / (n / 64)


def sort_study(n=16384, seed=3):
    """Wave regrouping by predicted work (the previous step's attempt counts): the launch is as
    long as its slowest wave (one wave per SIMD, all resident at once), so compare max, not mean."""
    q = trajectory_joints(n, 10, seed=seed)
    rng = np.random.default_rng(seed + 2)
    hi = np.array([0.001, 0.001, 0.001, np.deg2rad(5), np.deg2rad(5), np.deg2rad(5)], np.float32)
    a = ((rng.random((n, 6)) * 2 - 1) * hi).astype(np.float32)
    att_prev = oracle.fk_segattempts(q)
    att = oracle.fk_segattempts(oracle.step(q, a, np.zeros((n, 3)), np.zeros(n, np.int32), 0.02)["joints"])

    def waves(x):
        return np.array([simulate(x[w:w + 64], "now")[0] for w in range(0, len(x), 64)])

    key = att_prev.sum(1) * 16 + (att_prev > 0).sum(1)
    orders = {"natural": np.arange(n), "global, previous step": np.argsort(key, kind="stable"),
              "global, this step": np.argsort(att.sum(1) * 16 + (att > 0).sum(1), kind="stable")}
    for b in (256, 1024):
        orders["blocks of %d, previous step" % b] = np.concatenate(
            [b0 + np.argsort(key[b0:b0 + b], kind="stable") for b0 in range(0, n, b)])
    for name, o in orders.items():
        c = waves(att[o])
        print("%-28s wave cost mean %.2f  p99 %.2f  max %.2f" % (name, c.mean(), np.quantile(c, 0.99), c.max()))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "sort":
        sort_study()
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    q = trajectory_joints(n, 12)
    att = oracle.fk_segattempts(q)
    print("mean attempts %.2f, mean kept segments %.2f" % (att.sum(1).mean(), (att > 0).sum(1).mean()))
    base, it0 = simulate(att, "now")
    print("now            cost %.2f  iters %.2f" % (base, it0))
    for K in (4, 8, 16, 24, 32):
        for W in (1, 2, 3, 5, 100):
            c, it = simulate(att, "batch", K, W)
            print("batch K=%-3d W=%-3d cost %.2f (%.3f)  iters %.2f" % (K, W, c, c / base, it))
