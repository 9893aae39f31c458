#!/usr/bin/env python3
"""HBM traffic per launch of the roofline probe from two rocprofv3 PMC passes.

FETCH_SIZE / WRITE_SIZE are read per dispatch (KB); FETCH_SIZE is doubled (gfx950: it counts
64 B per 128-B request, MI355X_MICROARCH.md HBM section).  The probe is the VGG-11 conv4 weight
gradient: the KT GEMM dispatch with the layer's grid plus the split-K reduce that follows it.
usage: traffic.py <pmcF dir> <pmcW dir> [out.json]
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
    probes = []
    ids = sorted(F)
    for k, i in enumerate(ids):
        name, grid, _ = F[i]
        if "KtIm2colU" in name and "128, 128" in name and ", 3, true" in name and grid == 36 * 9 * 512:
            j = ids[k + 1] if k + 1 < len(ids) else None
            parts = [i] + ([j] if j is not None and "splitk_reduce" in F[j][0] else [])
            fetch = sum(2 * F[p][2] for p in parts)
            write = sum(W[p][2] for p in parts if p in W)
            probes.append((fetch, write))
    if not probes:
        sys.exit("probe dispatches not found")
    fetch = sum(p[0] for p in probes) / len(probes) * 1024
    write = sum(p[1] for p in probes) / len(probes) * 1024
    print(f"probe launches {len(probes)}: fetch {fetch / 1e6:.2f} MB, write {write / 1e6:.2f} MB per launch")
    if len(sys.argv) > 3:
        out = {"vgg11_b256_L3_p2": {"hbm_bytes_per_launch": round(fetch + write),
                                    "fetch_bytes": round(fetch), "write_bytes": round(write),
                                    "launches_averaged": len(probes),
                                    "kernels": "gemm_kernel<128,128,2,2,KtRowsU,KtIm2colU,SLAB,KT,8> + splitk_reduce_kernel",
                                    "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE, separate passes"}}
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
