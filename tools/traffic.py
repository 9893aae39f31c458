#!/usr/bin/env python3
"""HBM traffic per launch of the roofline probe from two rocprofv3 PMC passes.

FETCH_SIZE / WRITE_SIZE are read per dispatch (KB); FETCH_SIZE is doubled (gfx950: it counts
64 B per 128-B request, MI355X_MICROARCH.md HBM section).  The probe is the VGG-11 conv4 weight
gradient launch, picked by kernel-name substring and grid (work items x, y) -- both from the
bench line's roofline block.
usage: traffic.py <pmcF dir> <pmcW dir> [out.json] [grid_x_work_items grid_y [name_substring [last_n]]]
last_n: only the last n matching dispatches (bench.py re-runs the probed phase alone 20 times at
the end, so the last 20 are the probe even when another layer's launch has the same grid)
"""
import csv
import glob
import json
import sys


def load(d, name):
    out = {}
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]))
    return out


def main():
    F = load(sys.argv[1], "FETCH_SIZE")
    W = load(sys.argv[2], "WRITE_SIZE")
    # calibration line: the input layout conversion NCHW int8 -> NHWC16 (known bytes)
    for ids in (sorted(F), ):
        for i in ids:
            if "NchwToNhwc16" in F[i][0]:
                print(f"calib NchwToNhwc16: fetch x2 = {2 * F[i][2]:.0f} KB (expect 768 KB), "
                      f"write = {W.get(i, ('', 0, 0))[2]:.0f} KB (expect 4096 KB)")
                break
    gx = int(sys.argv[4]) if len(sys.argv) > 4 else 36 * 512
    gy = int(sys.argv[5]) if len(sys.argv) > 5 else 7
    sub = sys.argv[6] if len(sys.argv) > 6 else "KtIm2colU"
    want = set()
    kname = ""
    for f in glob.glob(f"{sys.argv[1]}/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"] and int(r["Grid_Size_X"]) == gx and int(r["Grid_Size_Y"]) == gy:
                want.add(int(r["Dispatch_Id"]))
                kname = r["Kernel_Name"].split("(")[0]
    last_n = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    ids = [i for i in sorted(F) if i in want]
    wids = [i for i in sorted(W) if sub in W[i][0] and W[i][1] == gx * gy]
    if last_n:
        ids, wids = ids[-last_n:], wids[-last_n:]
    probes = [(2 * F[i][2], 0.0) for i in ids]
    wr = [W[i][2] for i in wids]
    if not probes:
        sys.exit("probe dispatches not found")
    fetch = sum(p[0] for p in probes) / len(probes) * 1024
    write = sum(wr) / max(len(wr), 1) * 1024
    print(f"probe launches {len(probes)}: fetch {fetch / 1e6:.2f} MB, write {write / 1e6:.2f} MB per launch")
    if len(sys.argv) > 3:
        out = {"vgg11_b256_L3_p2": {"hbm_bytes_per_launch": round(fetch + write),
                                    "fetch_bytes": round(fetch), "write_bytes": round(write),
                                    "launches_averaged": len(probes),
                                    "kernel": f"{kname} (conv4 weight gradient)",
                                    "grid": [gx, gy],
                                    "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE, separate passes"}}
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
