"""HER replay feed throughput at the headline size (65 536 envs, 150-step episodes, k = 4 future).

Times, with HIP events on the launch stream: ctr_her_record after each ctr_step (per step), and
ctr_her_sample of a 65 536-row batch, once the store is warm.  Prints one JSON line with the
algorithmic bytes and the achieved GB/s of each kernel.

usage: python tools/bench_her.py [--envs N] [--steps K] [--batch B]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--slots", type=int, default=4)
    args = ap.parse_args()
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    from ctr_reach_amd import _abi
    dev = torch.device("cuda", 0)
    env = CtrReachVecEnv(args.envs, device=dev, seed=0, record_info=False)
    her = env.enable_her(slots=args.slots)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    hi = torch.tensor(env.action_space.high, device=dev)
    acts = [((torch.rand((args.envs, 6), generator=g, device=dev) * 2 - 1) * hi).contiguous() for _ in range(8)]
    # warm: fill the store (the recording kernel runs inside step_raw)
    for i in range(args.steps):
        env.step_raw(acts[i % 8])
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    sp = _abi.stream_ptr(stream)
    # record alone: re-run the recorder on the last step's outputs (same bytes moved)
    K = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    saved = (her.cur_t.clone(), her.len.clone())
    e0.record(stream)
    for _ in range(K):
        her.cur_t.copy_(saved[0])
        rc = env.lib.ctr_her_record(her._h, env._batch, _abi.ptr(acts[0]), env._out, float(env.cfg.tol), sp)
        _abi.check(rc, "ctr_her_record")
    e1.record(stream)
    torch.cuda.synchronize()
    rec_ms = e0.elapsed_time(e1) / K
    # the copy_ of cur_t (256 KB) is inside the bracket: time it alone and subtract
    e0.record(stream)
    for _ in range(K):
        her.cur_t.copy_(saved[0])
    e1.record(stream)
    torch.cuda.synchronize()
    rec_ms -= e0.elapsed_time(e1) / K
    her.len.copy_(saved[1])
    # sample
    her.sample(args.batch)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(K):
        her.sample(args.batch)
    e1.record(stream)
    torch.cuda.synchronize()
    smp_ms = e0.elapsed_time(e1) / K
    # the fused path (ctr_step_her) against the same steps without recording
    def step_us(with_her):
        keep = env._her
        env._her = keep if with_her else None
        torch.cuda.synchronize()
        e0.record(stream)
        for i in range(K):
            env.step_raw(acts[i % 8])
        e1.record(stream)
        torch.cuda.synchronize()
        env._her = keep
        return e0.elapsed_time(e1) / K * 1e3
    plain_us, fused_us = step_us(False), step_us(True)
    d = env.obs_dim
    # algorithmic bytes: record reads action 24 + reward 4 + done 1 + t 4 + cur_t/epoch 8 + obs_{t+1}
    # 4d + ag 24 (+ terminal selects), writes action 24 + reward 4 + obs 4d + ag 24 + cur_t 4
    rec_bytes = args.envs * (24 + 4 + 1 + 4 + 8 + 4 * d + 24 + 24 + 4 + 4 * d + 24 + 4)
    # sample: per row ~1.05 draws x (len 4) + obs_t, obs_t+1 4d each + ag_t, ag_t+1, goal 72 + action 24
    # + reward 4 + tol 8 + dg/epoch 12; writes 2 x 4(d + 6) + 24 + 4 + 4
    smp_bytes = args.batch * (4 + 8 * d + 72 + 24 + 4 + 8 + 12 + 8 * (d + 6) + 32)
    print(json.dumps({
        "envs": args.envs, "slots": args.slots, "store_bytes": her.nbytes, "stored_rows": len(her),
        "record_us": rec_ms * 1e3, "record_bytes": rec_bytes, "record_gbs": rec_bytes / (rec_ms * 1e-3) / 1e9,
        "sample_rows": args.batch, "sample_us": smp_ms * 1e3, "sample_bytes": smp_bytes,
        "sample_gbs": smp_bytes / (smp_ms * 1e-3) / 1e9, "rows_per_s": args.batch / (smp_ms * 1e-3),
        "step_us": plain_us, "step_her_fused_us": fused_us}))


if __name__ == "__main__":
    main()
