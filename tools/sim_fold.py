"""Diagnostic: would folding the reset pool's FKs into k_step's idle lanes pay?  

Extends tools/sim_sched.py's wave cost model (a wave pays CI for every iteration in which any lane
runs the segment-start block and CA for every iteration in which any lane runs an attempt; CI/CA =
0.43 from the measured block sizes).  A lane whose env FK is done takes a reset FK ("job") when
fewer than M lanes of its wave are on jobs; starting a job costs the wave a job-start block CJ
(loading the job's joints and segment table, precomputed by the sampling launch) in that
iteration; a job that is unfinished when the wave's env lanes are all done is suspended (its
progress carries over, so the model only needs the work rate).  Segment attempts come from the CPU
oracle: env-trajectory joints for the envs, freshly sampled joints for the jobs (what resets FK).

Prints, per M: the mean and max wave cost relative to today's, and the job work the waves get done
per step against what the pool needs (~500 resets x 2 FKs per step at 65 536 envs, ~1 reset-FK
per wave and step).  The fold pays only if the cost increase stays below the refill's share of
the step (~95 us per 20 steps = 4.8 us of ~88 us: 5.4 %).
usage: python tools/sim_fold.py [n_envs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle  # noqa: E402
from sim_sched import lane_tasks, simulate, trajectory_joints  # noqa: E402


def simulate_fold(att, jobs, M, CI=0.43, CA=1.0, CJ=0.3):
    """Per wave: (cost, job_units_done); job units = attempts + segment starts of job FKs."""
    n = att.shape[0]
    out = []
    jq = 0
    for w0 in range(0, n, 64):
        lanes = [lane_tasks(r) for r in att[w0:w0 + 64]]
        L = len(lanes)
        seg, left = [0] * L, [0] * L
        done = [len(s) == 0 for s in lanes]
        job = [None] * L                 # (tasks, seg, left) of the lane's job
        cost, units = 0.0, 0
        while not all(done):
            # lanes whose env is done take a job (at most M job lanes per wave)
            n_job = sum(j is not None for j in job)
            start = False
            for i in range(L):
                if done[i] and job[i] is None and n_job < M:
                    job[i] = [lane_tasks(jobs[jq % len(jobs)]), 0, 0]
                    jq += 1
                    n_job += 1
                    start = True
            if start:
                cost += CJ
            need_i = [i for i in range(L) if not done[i] and left[i] == 0]
            job_i = [i for i in range(L) if job[i] is not None and job[i][2] == 0 and job[i][1] < len(job[i][0])]
            if need_i or job_i:
                cost += CI
                for i in need_i:
                    left[i] = lanes[i][seg[i]][1]
                for i in job_i:
                    job[i][2] = job[i][0][job[i][1]][1]
                    units += 1
            runners = [i for i in range(L) if not done[i] and left[i] > 0]
            jrun = [i for i in range(L) if job[i] is not None and job[i][2] > 0]
            if runners or jrun:
                cost += CA
                for i in runners:
                    left[i] -= 1
                    if left[i] == 0:
                        seg[i] += 1
                        if seg[i] >= len(lanes[i]):
                            done[i] = True
                for i in jrun:
                    job[i][2] -= 1
                    units += 1
                    if job[i][2] == 0:
                        job[i][1] += 1
                        if job[i][1] >= len(job[i][0]):
                            job[i] = None        # finished: the lane may take the next one
        out.append((cost, units))
    return np.array(out)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    q = trajectory_joints(n, 12)
    att = oracle.fk_segattempts(q)
    qj, _ = oracle.sample_joints(4096, seed=11, stream=1)
    jobs = oracle.fk_segattempts(qj)
    per_fk = float(((jobs > 0).sum(1) + jobs.sum(1)).mean())
    base = np.array([simulate(att[w:w + 64], "now")[0] for w in range(0, n, 64)])
    need = 1000.0 / 1024 * per_fk            # job units per wave and step the pool needs
    print("env FK: mean attempts %.2f, segments %.2f; reset FK: %.1f units (attempts + segment starts)"
          % (att.sum(1).mean(), (att > 0).sum(1).mean(), per_fk))
    print("today: wave cost mean %.2f max %.2f;  the pool needs %.1f job units per wave and step" %
          (base.mean(), base.max(), need))
    for M in (1, 2, 4, 8, 16):
        r = simulate_fold(att, jobs, M)
        print("M=%-3d wave cost mean %.2f (%+.1f %%)  max %.2f (%+.1f %%)  job units per wave %.1f (%.1fx the need)"
              % (M, r[:, 0].mean(), 100 * (r[:, 0].mean() / base.mean() - 1), r[:, 0].max(),
                 100 * (r[:, 0].max() / base.max() - 1), r[:, 1].mean(), r[:, 1].mean() / need))


if __name__ == "__main__":
    main()
