#!/usr/bin/env python
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch
HBM bytes (profiles/<tag>_pmc.json, read by bench.py's roofline.traffic).

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB and
derive from the L2's memory-side requests; FETCH_SIZE under-reports wide
streaming reads by 2x on gfx950 and other widths are uncalibrated, so the
factors are measured on tools/pmc_calib.hip's 512 MiB streams with the step
kernel's own 4 B/lane shapes (factor = true bytes / (counter * 1024)).

usage: pmc_summary.py TAG FETCH_DIR WRITE_DIR CALIB_FETCH_DIR CALIB_WRITE_DIR
                      [--rollout-k K] [--bench-json PATH]

Entries are keyed like bench.launch_key: `name@grid@kK` (K = steps per
launch: the pass's --rollout-chunk for k_rollout, 1 for every other kernel),
so bench.py never prices a launch with counters of another launch shape;
--bench-json (the JSON line of the profiled bench run) adds each key's
p_lock from that run.

The summary carries bench.kernel_source_sha() of the sources it measured;
bench.py reports `traffic` only from a summary with its own sources' hash.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CALIB_BYTES = 512 << 20


def per_kernel(d, counter, by_grid=False):
    """counter values per kernel name (by_grid: per (name, grid size), so that
    the bench's 65,536-env and 4,096-env launches of one kernel stay apart)."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                key = r["Kernel_Name"]
                if by_grid:
                    key = (key, int(r.get("Grid_Size") or 0))
                vals[key].append(float(r["Counter_Value"]))
    return vals


def short(name):
    name = name.replace("st::(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].strip()


def launch_k(name, rollout_k):
    """Steps per launch of a profiled kernel (bench.launch_key's k)."""
    return rollout_k if short(name).startswith("k_rollout") else 1


def bench_p_lock(path):
    """launch_key -> p_lock from every roofline object of a bench JSON line."""
    if not path:
        return {}
    d = json.loads(open(path).read().strip().splitlines()[-1])
    out = {}
    objs = [d.get("roofline", {})] + [v.get("roofline", {}) for v in d.get("variants", {}).values()
                                       if isinstance(v, dict)]
    for r in objs:
        if r.get("launch_key") and r.get("p_lock") is not None:
            out[r["launch_key"]] = r["p_lock"]
    return out


def main():
    args = sys.argv[1:]
    rollout_k, bench_json = 100, None
    if "--rollout-k" in args:
        i = args.index("--rollout-k")
        rollout_k = int(args[i + 1])
        del args[i:i + 2]
    if "--bench-json" in args:
        i = args.index("--bench-json")
        bench_json = args[i + 1]
        del args[i:i + 2]
    tag, fdir, wdir, cfdir, cwdir = args[:5]
    pl = bench_p_lock(bench_json)
    cf = per_kernel(cfdir, "FETCH_SIZE")
    cw = per_kernel(cwdir, "WRITE_SIZE")

    def factor(vals, kname, counter):
        for k, v in vals.items():
            if short(k) == kname:
                m = sorted(v)[len(v) // 2]
                return CALIB_BYTES / (m * 1024.0), m
        raise SystemExit(f"calibration kernel {kname} missing for {counter}")

    f_rd4, raw_rd4 = factor(cf, "rd4", "FETCH_SIZE")
    f_rd16, raw_rd16 = factor(cf, "rd16", "FETCH_SIZE")
    f_wr4, raw_wr4 = factor(cw, "wr4", "WRITE_SIZE")
    fetch = per_kernel(fdir, "FETCH_SIZE", by_grid=True)
    write = per_kernel(wdir, "WRITE_SIZE", by_grid=True)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    out = {"tag": tag, "kernel_source_sha": bench.kernel_source_sha(), "rollout_k": rollout_k,
           "calibration": {"fetch_factor_4B_lane": f_rd4, "fetch_factor_16B_lane": f_rd16,
                           "write_factor_4B_lane": f_wr4, "raw_kib": {"rd4": raw_rd4, "rd16": raw_rd16,
                                                                     "wr4": raw_wr4},
                           "stream_bytes": CALIB_BYTES},
           "kernels": {}}
    for k in set(fetch) | set(write):
        fv, wv = fetch.get(k, []), write.get(k, [])
        if not fv or not wv:
            continue
        # drop the first quarter (cold caches / warm-up launches)
        fv, wv = fv[len(fv) // 4:], wv[len(wv) // 4:]
        fk = sum(fv) / len(fv)
        wk = sum(wv) / len(wv)
        rd = fk * 1024.0 * f_rd4
        wr = wk * 1024.0 * f_wr4
        name, grid = k
        ent = {"launches": len(fv), "grid_size": grid, "fetch_kib": fk, "write_kib": wk,
               "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
               "hbm_bytes_per_launch": rd + wr, "full_name": name}
        key = f"{short(name)}@{grid}@k{launch_k(name, rollout_k)}"
        ent["steps_per_launch"] = launch_k(name, rollout_k)
        if key in pl:
            ent["p_lock_profiled_run"] = pl[key]
        out["kernels"][key] = ent
    os.makedirs("profiles", exist_ok=True)
    path = os.path.join("profiles", f"{tag}_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
