#!/usr/bin/env python3
"""Copy tools/gpu_others.sh's results for one tag from gpurun_out/ into profiles/.

usage: collect_others.py TAG
Writes profiles/TAG_{vgg16,lenet,resnet18}_bench.json (the bench lines, with roofline and
cpu_baseline), profiles/TAG_{vgg16,lenet,resnet18}_traffic.txt (the probes' PMC bytes per launch)
and refreshes profiles/traffic.json from the run's copy.
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def line(path):
    return json.loads([x for x in open(path) if x.startswith("{")][-1])


def main():
    tag = sys.argv[1]
    for net in ("vgg16", "lenet", "resnet18"):
        src = f"{G}/{net}_{tag}.log"
        if not os.path.exists(src):
            print(f"{net}: no bench log")
            continue
        b = line(src)
        with open(f"{P}/{tag}_{net}_bench.json", "w") as f:
            json.dump(b, f)
            f.write("\n")
        r = b["roofline"]
        print(f"{net}: {b['ms_per_step']} ms/step, {b['value']} {b['unit']}, probe frac {r['frac']}, "
              f"traffic {r.get('traffic')}, bound {r.get('bound')} / {r.get('limiter')}")
        t = f"{G}/traffic_{net}_{tag}.txt"
        if os.path.exists(t):
            shutil.copy(t, f"{P}/{tag}_{net}_traffic.txt")
    tj = f"{G}/traffic_{tag}.json"
    if os.path.exists(tj):
        shutil.copy(tj, f"{P}/traffic.json")


if __name__ == "__main__":
    main()
