"""Per-wave SQ counter summary (instructions, wave/wait cycles) per kernel."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for r in rows:
    k = r["Kernel_Name"].replace("st::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if not k.startswith("k_step") and not k.startswith("k_rollout"):
        continue
    agg[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k, cs in agg.items():
    med = {c: sorted(d.values())[len(d) // 2] for c, d in cs.items()}
    w = med["SQ_WAVES"]
    print(f"{k:28s} per wave: VALU {med['SQ_INSTS_VALU']/w:6.0f} SALU {med['SQ_INSTS_SALU']/w:5.0f} "
          f"LDS {med['SQ_INSTS_LDS']/w:4.0f} | wave cyc(x4) {med['SQ_WAVE_CYCLES']/w:6.0f} "
          f"wait {med['SQ_WAIT_ANY']/w:6.0f} wait_inst {med['SQ_WAIT_INST_ANY']/w:5.0f} "
          f"active {med['SQ_ACTIVE_INST_ANY']/w:6.0f}")
