"""Quick per-launch HBM bytes of the headline kernel from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; counter_collection.csv), for A/Bs of the
state layout: FETCH x 2.00 / WRITE x 1.00 (tools/pmc_calib.hip's gfx950
correction, as tools/pmc_summary.py applies it).
usage: python tools/pmc_quick.py FETCH_DIR WRITE_DIR [kernel substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def means(d, counter, sub):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and sub in r["Kernel_Name"]:
                vals[(r["Kernel_Name"], r.get("Grid_Size", "?"))].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


sub = sys.argv[3] if len(sys.argv) > 3 else "k_step<10, 20, false, false, true, false>"
fe, wr = means(sys.argv[1], "FETCH_SIZE", sub), means(sys.argv[2], "WRITE_SIZE", sub)
for k in sorted(set(fe) | set(wr)):
    f = fe.get(k, (float("nan"), 0))[0] * 1024 * 2.0
    w = wr.get(k, (float("nan"), 0))[0] * 1024 * 1.0
    print("%s grid %s: reads %.3f MB  writes %.3f MB  total %.3f MB  (%d launches)"
          % (k[0][:60], k[1], f / 1e6, w / 1e6, (f + w) / 1e6, fe.get(k, (0, 0))[1]))
