"""Summarise a scripts/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>_*.

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-kernel PMC averages (per launch)
  profiles/traffic.json             HBM bytes per k_step launch for bench.py's roofline.traffic:
                                    FETCH_SIZE x 2 (gfx950 reports half of wide reads,
                                    MI355X_MICROARCH.md HBM section) + WRITE_SIZE, KiB -> bytes
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, tag + "_kernel_stats.csv"))

def kname(full):
    m = re.search(r"\b(k_\w+(?:<\w+>)?)\(", full)
    return m.group(1) if m else full[:60]


pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in sorted(os.listdir(src)):
    f = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        name = kname(r["Kernel_Name"])
        pmc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in pmc.items() if k.startswith("k_")}
for k, d in out.items():
    if "SQ_THREAD_CYCLES_VALU" in d and "SQ_ACTIVE_INST_VALU" in d:
        d["lane_utilisation_est"] = d["SQ_THREAD_CYCLES_VALU"] / (64.0 * d["SQ_ACTIVE_INST_VALU"])
with open(os.path.join(dst, tag + "_pmc.json"), "w") as fh:
    json.dump(out, fh, indent=1, sort_keys=True)

step = [k for k in out if "k_step" in k]
stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
avg_ns = {kname(r["Name"]): float(r["AverageNs"]) for r in stats}
if step:
    d = out[step[0]]
    fetch = d.get("FETCH_SIZE", 0.0) * 1024
    write = d.get("WRITE_SIZE", 0.0) * 1024
    envs = 65536
    t = {"envs": envs, "kernel": step[0], "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
         "bytes_per_launch": 2 * fetch + write,
         "note": "FETCH_SIZE doubled per the gfx950 calibration for wide reads; k_step reads 4-8 B/lane "
                 "AoS rows, for which the counter is uncalibrated",
         "avg_ns_rocprof": avg_ns.get(step[0])}
    with open(os.path.join(dst, "traffic.json"), "w") as fh:
        json.dump(t, fh, indent=1)
    print(json.dumps(t, indent=1))
for k, v in avg_ns.items():
    if k.startswith("k_"):
        print("%-60s %10.1f us" % (k[:60], v / 1e3))
