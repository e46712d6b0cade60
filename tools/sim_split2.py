"""Cost model: the 2-lane env split of k_step's RK45 FK, against today's one env
per lane (tools/sim_split.py modelled the 4-lane tube-parallel form: 2.04x the issue, 1.41x slower).

Split form: an env on an adjacent lane pair (quad_perm DPP swaps, no LDS), both lanes running ONE
instruction stream on different state slots -- a wave executes every slot program for all its
lanes, so the work per lane is the larger of the two lanes' slot counts:
  lane 0: R rows 0-1 and r_0, r_1          lane 1: R row 2, r_2, u_z (3), alpha (3)
  stage inputs: r is never an RHS input, so 9 slots (lane 0: 6 used)                  9 x 15 FMA
  per RHS: lane 1 forms d10, d20 and passes d10 (2 moves); each lane runs ONE table sincos (lane 0
    sin/cos(d10), lane 1 sin/cos(d20): 13 FP64 + 5 index / LDS instructions), the pairs are
    swapped (4 moves), both lanes form c21 / s21 (4), the three uy sums, ux_0, uy_0 (10) and
    du_z (3), u_z,0 goes to lane 0 (2 moves), and each lane forms TWO row slots of R [u]x (12;
    lane 1's second slot is idle)                                                         57
  y_new 10 slots x 5, error sums 10 x 6, norm terms 10 x 4 (v_rcp_f64 scales), a 1-round DPP sum
  of the two partial norms (3), the controller on both lanes (40).
Today's counts come from the census of the level-3 attempt block (tools/attempt_census.py).

Time model (tools/sim_split.py's): a wave64 VALU instruction occupies its SIMD 4 cycles; one wave
per SIMD issues one instruction per 5.15 cycles (PMC: dependent FP64 chains); with 2 waves per
SIMD the better of full issue (4 cycles) and each wave's own chain at one-wave issue bounds the
SIMD.  Iterations per wave from the CPU oracle's per-segment attempt counts on env-trajectory
joints: 64 envs per wave today, 32 in the split form (2048 waves at 65 536 envs: 2 per SIMD, which
needs <= 256 registers per lane -- the split holds half the state).

usage: python tools/sim_split2.py [n_envs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from sim_split import CPI_FULL, CPI_ONE_WAVE, TODAY_ATTEMPT, TODAY_START, wave_iterations  # noqa: E402
from sim_sched import trajectory_joints  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402


def split2_counts():
    sincos = 13 + 5
    per_rhs = 2 + 2 + sincos + 4 + 4 + 10 + 3 + 2 + 12
    stages = 9 * 15
    update = 10 * 5 + 10 * 6
    norm = 10 * 4 + 3
    control = 40
    attempt = 6 * per_rhs + stages + update + norm + control
    start = 2 * per_rhs + 10 * 8 + 3 + 60          # select_initial_step: 2 RHS, its norms, h0 / h1
    return attempt, start, per_rhs


def model(n=8192, cpi_two=CPI_FULL):
    att = oracle.fk_segattempts(trajectory_joints(n, 12))
    sa, ss, pr = split2_counts()
    today = wave_iterations(att, 64)
    split = wave_iterations(att, 32)
    t_today = today.max() * TODAY_ATTEMPT * CPI_ONE_WAVE
    per_simd = np.add.reduceat(split * sa, np.arange(0, len(split), 2))
    t_split = max(per_simd.max() * cpi_two, split.max() * sa * CPI_ONE_WAVE)
    return dict(attempt=sa, start=ss, per_rhs=pr, issue_ratio=2 * sa / TODAY_ATTEMPT,
                today_mean=today.mean(), today_max=today.max(), split_mean=split.mean(), split_max=split.max(),
                t_today=t_today, t_split=t_split, ratio=t_split / t_today)


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    for cpi in (CPI_FULL, 4.3, 4.6):
        m = model(n, cpi)
        if cpi == CPI_FULL:
            print("per-lane instructions: attempt %d (today %d), segment start %d (today %d), per RHS %d" % (
                m["attempt"], TODAY_ATTEMPT, m["start"], TODAY_START, m["per_rhs"]))
            print("instructions per env and attempt: split %d (2 lanes x %d) vs today %d: %.2fx the issue" % (
                2 * m["attempt"], m["attempt"], TODAY_ATTEMPT, m["issue_ratio"]))
            print("wave iterations (attempt units), mean / max: today %.2f / %.2f (64 envs), split %.2f / %.2f "
                  "(32 envs)" % (m["today_mean"], m["today_max"], m["split_mean"], m["split_max"]))
        print("two waves per SIMD at %.2f cycles per instruction: slowest SIMD today %.0f, split %.0f cycles "
              "-> split / today = %.3f" % (cpi, m["t_today"], m["t_split"], m["ratio"]))
