"""Cost model: the lane-level, barrier-free tube-parallel split of one env's FK
that north_star's "wavefront shuffles for the 3x3 frame update" suggests, against today's one env
per lane.

Split form (3 tubes padded to 4 lanes, an env on a 4-lane DPP group): lane i owns u_z,i, alpha_i,
r_i and row i of R (6 of the 18 state components).  Per RHS each lane needs every alpha (two
64-bit DPP broadcasts of the others' alpha: 2 x 2 b32 moves each), computes ONE sin/cos pair of
the three angle differences (lane 0: (a1 - a0), lane 1: (a2 - a0), lane 2: (a2 - a1); the table
sincos of tools/attempt_census.py, 13 FP64 ops + 5 index / LDS instructions), gets the other
pairs its row needs (2 pairs x 2 doubles x 2 b32 moves), forms its uy_i (2 FMA) and du_z,i
(1 MUL), lane 0 forms ux_0, uy_0 and the group receives u = (ux_0, uy_0, u_z,0) (3 doubles x 2
b32 moves), and each lane forms its row of R [u]x (6 ops).  Per attempt each lane runs its
6 components' stage sums (6 x 15 FMA + 15 coefficient MUL), y_new and error sums (6 x 10), its
6 norm terms (6 x 6, with the v_rcp_f64), a 2-round DPP sum of the partial norms (2 x (2 moves +
1 add)) and the controller (inv_root10 and the step-size logic, every lane: ~40).
Today's counts come from the census of the level-3 attempt block (1 117-1 153 instructions).

Time model: every VALU instruction of a wave64 occupies its SIMD for 4 cycles (16 lanes per cycle,
FP64 FMA at full rate); one wave per SIMD (today: 368 registers per lane) issues one instruction
per 5.15 cycles on average (PMC, profiles/r03c_pmc.json: its dependent FP64 chains), while >= 2
waves per SIMD fill the pipe (4 cycles per instruction).  The iterations per wave come from the
CPU oracle's per-segment attempt counts on env-trajectory joints (tools/sim_sched.py's wave
model): 64 envs per wave today, 16 envs per wave (64 lanes / 4) in the split form.

usage: python tools/sim_split.py [n_envs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle  # noqa: E402
from sim_sched import simulate, trajectory_joints  # noqa: E402

TODAY_ATTEMPT = 1117          # census, level-3 attempt block (tools/attempt_census.py)
TODAY_START = 444             # segment-start block (select_initial_step + f0)
CPI_ONE_WAVE = 5.15           # cycles per issued instruction, one wave per SIMD (PMC)
CPI_FULL = 4.0                # a wave64 VALU instruction's SIMD occupancy


def split_counts():
    sincos = 13 + 5
    per_rhs = (2 * 4          # broadcast of the two other alphas
               + 2            # the angle differences
               + sincos       # one sin/cos pair
               + 2 * 2 * 2    # the two other pairs the row's uy_i / ux needs
               + 2 + 1        # uy_i, du_z,i
               + 2            # lane 0: ux_0 (lanes compute it redundantly)
               + 3 * 2        # u = (ux_0, uy_0, u_z,0) to the group
               + 6)           # row i of R [u]x
    stages = 6 * 15 + 15
    update = 6 * 10 + 5
    norm = 6 * 6 + 2 * 3
    control = 40
    attempt = 6 * per_rhs + stages + update + norm + control
    start = 2 * per_rhs + 6 * 8 + 2 * 3 + 60      # select_initial_step: 2 RHS, its norms, h0 / h1
    return attempt, start, per_rhs


def wave_iterations(att, env_per_wave):
    """Mean and max over waves of (iterations running the start block, running an attempt)."""
    costs = []
    for w in range(0, att.shape[0], env_per_wave):
        rows = att[w:w + env_per_wave]
        c, it = simulate(rows, "now", CI=TODAY_START / TODAY_ATTEMPT, CA=1.0)
        costs.append(c * rows.shape[0] / 64.0)      # simulate() averages over n / 64 waves
    return np.array(costs)


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    att = oracle.fk_segattempts(trajectory_joints(n, 12))
    sa, ss, pr = split_counts()
    today = wave_iterations(att, 64)            # attempt-block units per wave
    split = wave_iterations(att, 16)
    # wave instructions per wave: units x attempt-block size (the start block is folded in by CI)
    t_today = today.max() * TODAY_ATTEMPT * CPI_ONE_WAVE                 # 1 wave per SIMD
    # split: 4x the waves (4 per SIMD, resident together); a SIMD's time is the sum of its 4 waves'
    # instructions at full issue, or its slowest wave's chain at one-wave issue, whichever is longer
    per_simd = np.add.reduceat(split * sa, np.arange(0, len(split), 4))
    t_split = max(per_simd.max() * CPI_FULL, split.max() * sa * CPI_ONE_WAVE)
    print("per-lane instructions: attempt %d (today %d), segment start %d (today %d), per RHS %d" % (
        sa, TODAY_ATTEMPT, ss, TODAY_START, pr))
    print("instructions per env and attempt: split %d (4 lanes x %d) vs today %d: %.2fx the issue" % (
        4 * sa, sa, TODAY_ATTEMPT, 4 * sa / TODAY_ATTEMPT))
    print("wave iterations (attempt units), mean / max: today %.2f / %.2f (64 envs), split %.2f / %.2f (16 envs)" % (
        today.mean(), today.max(), split.mean(), split.max()))
    print("modelled launch (cycles of the slowest SIMD): today %.0f, split %.0f -> split / today = %.2f" % (
        t_today, t_split, t_split / t_today))
