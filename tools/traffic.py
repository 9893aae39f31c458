#!/usr/bin/env python3
"""HBM traffic per launch of the roofline probe from two rocprofv3 PMC passes.

FETCH_SIZE / WRITE_SIZE are read per dispatch (KB); FETCH_SIZE is doubled (gfx950: it counts
64 B per 128-B request, MI355X_MICROARCH.md HBM section).  The probe: bench.py re-runs the probed
layer phase alone 20 times after the timed region (the last launches of the process, after the
last NITI_SGD), and the probed kernel is the launch of that phase with the most dispatch time --
its FETCH / WRITE averaged over those re-runs.
usage: traffic.py <pmcF dir> <pmcW dir> [traffic.json key plan]
  key: e.g. vgg11_b256_L3_p2 (bench.py looks it up as {arch}_b{batch}_L{layer}_p{phase}); plan:
  bm,bn,splits,strategy of the probed launch.  The entry is merged into traffic.json.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, name):
    rows = []
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == name]
    return sorted(rows, key=lambda r: int(r["Dispatch_Id"]))


def probe_rows(rows):
    last = max(k for k, r in enumerate(rows) if "sgd_update_kernel" in r["Kernel_Name"])
    # (the fully connected layers' fused NITI_SGD passes follow the update launch: still the step)
    while last + 1 < len(rows) and "KtRowsU, niti::KtRowsU, 4, true" in rows[last + 1]["Kernel_Name"]:
        last += 1
    tail = rows[last + 1:]
    t = collections.defaultdict(float)
    for r in tail:
        t[(r["Kernel_Name"], r["Grid_Size"])] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    key = max(t, key=t.get)
    return key, [r for r in tail if (r["Kernel_Name"], r["Grid_Size"]) == key]


def main():
    F = load(sys.argv[1], "FETCH_SIZE")
    W = load(sys.argv[2], "WRITE_SIZE")
    for r in F:  # calibration line: a layout conversion with known bytes, when the run has one
        if "NchwToNhwc16" in r["Kernel_Name"]:
            print(f"calib NchwToNhwc16: fetch x2 = {2 * float(r['Counter_Value']):.0f} KB")
            break
    (kname, grid), fr = probe_rows(F)
    (kw, gw), wr = probe_rows(W)
    if (kname, grid) != (kw, gw):
        sys.exit("the two passes probed different launches")
    # bench.py re-runs the probed phase ISO = 20 times; a phase that is a launch pair (the row kernels'
    # speculative pair: A multiplies, B settles) shows 40 launches of the kernel -- its bytes are
    # reported per probe event (the pair), as its time is
    ISO = 20
    per = len(fr) // ISO if len(fr) % ISO == 0 and len(fr) >= ISO else 1
    fetch = sum(2 * float(r["Counter_Value"]) for r in fr) / len(fr) * 1024 * per
    write = sum(float(r["Counter_Value"]) for r in wr) / len(wr) * 1024 * per
    short = kname.split("(")[0]
    print(f"probe {short}, grid {grid} work items, {len(fr)} launches ({per} per probe event): fetch "
          f"{fetch / 1e6:.2f} MB, write {write / 1e6:.2f} MB per probe event")
    if len(sys.argv) > 5:
        path, key = sys.argv[3], sys.argv[4]
        plan = [int(v) for v in sys.argv[5].split(",")]
        tj = json.load(open(path)) if os.path.exists(path) else {}
        tj[key] = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch),
                   "write_bytes": round(write), "launches_averaged": len(fr), "launches_per_probe": per,
                   "kernel": short,
                   "grid_work_items": int(grid), "plan": plan,
                   "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE, separate passes"}
        json.dump(tj, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
