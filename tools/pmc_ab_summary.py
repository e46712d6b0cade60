"""Summarise scripts/pmc_ab.sh: per library variant, the per-launch PMC averages of the step kernel."""
import collections
import csv
import glob
import os
import re
import sys

tag = sys.argv[1]
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "pmcab_" + tag)
for lib in sorted(os.listdir(root)):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, lib, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if re.search(r"k_step", r["Kernel_Name"]):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d = {k: sum(v) / len(v) for k, v in acc.items()}
    w = d.get("SQ_WAVES", 1)
    print("== %s" % lib)
    for k in sorted(d):
        print("  %-26s %16.1f   per wave %12.1f" % (k, d[k], d[k] / w))
    if "SQ_THREAD_CYCLES_VALU" in d and "SQ_ACTIVE_INST_VALU" in d:
        print("  lane_utilisation_est       %.3f" % (d["SQ_THREAD_CYCLES_VALU"] / (64 * d["SQ_ACTIVE_INST_VALU"])))
    if "SQ_WAVE_CYCLES" in d and "SQ_INSTS_VALU" in d:
        print("  wave-cycles per VALU inst  %.3f" % (d["SQ_WAVE_CYCLES"] / d["SQ_INSTS_VALU"]))
