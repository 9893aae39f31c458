#!/usr/bin/env python3
"""Per-dispatch durations of the roofline probe kernel in a rocprofv3 kernel trace.

The probe is the VGG-11 conv4 weight-gradient GEMM at batch 256 (layer index 3): the KT
gemm_kernel dispatch whose grid holds the conv4 tiles x splits.  Prints its count and average
duration, to set against bench.py's HIP-event average (roofline.avg_launch_us).
usage: probe_trace.py <run_kernel_trace.csv> [grid_x_work_items grid_y]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    want = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (36 * 512, 7)
    cands = {}
    for r in rows:
        n = r["Kernel_Name"]
        if "KtRowsU" not in n or "128, 128" not in n:
            continue
        g = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))
        cands.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    for g, d in sorted(cands.items()):
        mark = " <- probe" if want == g else ""
        print(f"grid {str(g):14s}: {len(d):4d} dispatches, avg {sum(d) / len(d):8.2f} us, "
              f"min {min(d):7.2f}, max {max(d):7.2f}{mark}")


if __name__ == "__main__":
    main()
