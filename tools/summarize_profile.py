"""Summarise a scripts/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>_*.

Writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-kernel PMC averages (per launch)
  profiles/<tag>_traffic_calibration.json  FETCH_SIZE / WRITE_SIZE against known byte counts in
                                    k_step's access shapes (tools/traffic_probe.hip)
  profiles/traffic.json             (traffic_c<config>.json for another bench config, argv[2])
                                    HBM bytes per k_step launch for bench.py's roofline.traffic:
                                    FETCH_SIZE and WRITE_SIZE scaled by the calibrated factors
                                    (KiB -> bytes)
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
# the bench config the passes ran (bench.py --config, from BENCH_ARGS): 3 (the headline) writes
# profiles/traffic.json, another config profiles/traffic_c<config>.json
config = int(sys.argv[2]) if len(sys.argv) > 2 else 3
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
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts in k_step's own access shapes
# (tools/traffic_probe.hip, scripts/profile.sh passes probe_fetch / probe_write)
cal = None
probe = {}
for sub, ctr in (("probe_fetch", "FETCH_SIZE"), ("probe_write", "WRITE_SIZE")):
    f = os.path.join(src, sub, "run_counter_collection.csv")
    if os.path.exists(f):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == ctr:
                acc[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024)
        probe[ctr] = {k: sum(v) / len(v) for k, v in acc.items()}
if "FETCH_SIZE" in probe and "WRITE_SIZE" in probe:
    logf = os.path.join(src, "probe1.log")
    known = json.loads([ln for ln in open(logf) if ln.startswith("{")][-1])
    pf, pw = probe["FETCH_SIZE"], probe["WRITE_SIZE"]
    cal = {"tool": "tools/traffic_probe.hip (scripts/profile.sh)", "known_bytes": known,
           "fetch_size_bytes": {k: pf[k] for k in ("k_rows_cold", "k_rows_warm", "k_stream_cold") if k in pf},
           "write_size_bytes": {k: pw[k] for k in ("k_rows_write", "k_rows_cold") if k in pw},
           "read_factor_rows_cold": known["read_bytes_known"] / pf["k_rows_cold"],
           "read_factor_rows_warm": known["read_bytes_known"] / pf["k_rows_warm"],
           "read_factor_stream16": known["stream_bytes_known"] / pf["k_stream_cold"],
           "write_factor_rows": known["write_bytes_known"] / pw["k_rows_write"],
           "write_factor_sink": known["sink_bytes"] / pw["k_rows_cold"]}
    with open(os.path.join(dst, tag + "_traffic_calibration.json"), "w") as fh:
        json.dump(cal, fh, indent=1)
    print(json.dumps(cal, indent=1))
if step:
    d = out[step[0]]
    fetch = d.get("FETCH_SIZE", 0.0) * 1024
    write = d.get("WRITE_SIZE", 0.0) * 1024
    envs = 65536
    rf = cal["read_factor_rows_warm"] if cal else 2.0
    wf = cal["write_factor_rows"] if cal else 1.0
    t = {"envs": envs, "config": config, "kernel": step[0], "fetch_size_bytes_raw": fetch, "write_size_bytes_raw": write,
         "read_factor": rf, "write_factor": wf,
         "bytes_per_launch": rf * fetch + wf * write,
         "read_bytes": rf * fetch, "write_bytes": wf * write,
         "note": ("FETCH_SIZE x read_factor + WRITE_SIZE x write_factor, the factors measured on known byte "
                  "counts in k_step's own row-load / row-store shapes (%s_traffic_calibration.json)" % tag)
         if cal else "FETCH_SIZE doubled per the gfx950 calibration for wide reads (uncalibrated here)",
         "avg_ns_rocprof": avg_ns.get(step[0])}
    # the bench's own k_step timing set: its last 32 launches (auto-reset off, after 256 untimed
    # ones), which bench.py brackets with one HIP event pair -- the same launches, rocprof's clock
    trace = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace):
        ks = sorted((r for r in csv.DictReader(open(trace)) if step[0] in r["Kernel_Name"]),
                    key=lambda r: int(r["Start_Timestamp"]))
        dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks]
        if len(dur) >= 32:
            t["avg_ns_rocprof_bench_timed_32"] = sum(dur[-32:]) / 32.0
            t["launches_in_trace"] = len(dur)
    with open(os.path.join(dst, "traffic.json" if config == 3 else "traffic_c%d.json" % config), "w") as fh:
        json.dump(t, fh, indent=1)
    print(json.dumps(t, indent=1))
for k, v in avg_ns.items():
    if k.startswith("k_"):
        print("%-60s %10.1f us" % (k[:60], v / 1e3))
