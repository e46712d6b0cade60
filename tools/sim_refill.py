"""Diagnostic: the resumable refill in the wave cost model (tools/sim_sched.py's: a wave pays the
segment-start block CI whenever any lane starts a segment and the attempt block CA whenever any
lane attempts).  Fresh-sample FKs from the CPU oracle, 20 FK lanes per wave (a 20-step queue at
65 536 envs); with budget B a new FK runs at most B iterations and a carried one resumes (one
start-like block) and runs to its end.  Prints the slowest / mean wave of a steady-state refill
and the share of FKs suspended.  (The kernel also lets a carried FK be suspended again while its
reset is at least a refill period ahead; this model does not.)
usage: python tools/sim_refill.py [n_fks]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle  # noqa: E402
from sim_sched import lane_tasks  # noqa: E402

CI, CA = 0.43, 1.0
PER_WAVE = 20


def iterations(tasks):
    """Per loop iteration of one FK: (starts a segment, attempts)."""
    ev = []
    for _, attempts in tasks:
        ev.append((True, True))
        ev += [(False, True)] * (attempts - 1)
    return ev


def wave_cost(lanes):
    cost = 0.0
    for i in range(max((len(e) for e in lanes), default=0)):
        cost += CI * any(len(e) > i and e[i][0] for e in lanes)
        cost += CA * any(len(e) > i and e[i][1] for e in lanes)
    return cost


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 40960
    qj, _ = oracle.sample_joints(m, seed=11, stream=1)
    fks = [iterations(lane_tasks(r)) for r in oracle.fk_segattempts(qj)]
    units = np.array([len(e) + sum(s for s, _ in e) for e in fks])
    print("fresh-sample FK: %.1f iterations on average, %d at most" % (np.mean([len(e) for e in fks]),
                                                                       max(len(e) for e in fks)))
    nw = len(fks) // PER_WAVE
    base = [wave_cost(fks[w * PER_WAVE:(w + 1) * PER_WAVE]) for w in range(nw)]
    print("budget none: slowest wave %.2f, mean %.2f  (units %.1f per FK)" % (max(base), np.mean(base), units.mean()))
    for B in (6, 8, 10, 12, 14, 16):
        carried = []
        for _ in range(2):                     # the second refill sees the first one's carry
            waves = [[e[:B] for e in fks[w * PER_WAVE:(w + 1) * PER_WAVE]] for w in range(nw)]
            nxt = [e[B:] for e in fks[:nw * PER_WAVE] if len(e) > B]
            for k, e in enumerate(carried):
                waves[k % nw].append([(True, True)] + e)
            costs = [wave_cost(lanes) for lanes in waves]
            carried = nxt
        print("budget %2d: slowest wave %.2f, mean %.2f, %.0f %% suspended" %
              (B, max(costs), np.mean(costs), 100.0 * len(carried) / (nw * PER_WAVE)))


if __name__ == "__main__":
    main()
