#!/usr/bin/env python3
"""Copy tools/gpu_others.sh's results for one tag from gpurun_out/ into profiles/.

usage: collect_others.py TAG
Writes profiles/TAG_{vgg16,lenet,resnet18}_bench.json (the bench lines, with roofline and
cpu_baseline), profiles/TAG_{vgg16,lenet,resnet18}_traffic.txt (the probes' PMC bytes per launch)
and the probes' entries of profiles/traffic.json (recomputed from the counter passes).
"""
import json
import os
import subprocess
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
        # the probe's PMC bytes, recomputed here from the two counter passes (tools/traffic.py) into
        # profiles/traffic.json under the plan the bench line probed
        pf, pw = f"{G}/pmcF_{net}_{tag}", f"{G}/pmcW_{net}_{tag}"
        if os.path.isdir(pf) and os.path.isdir(pw):
            plan = ",".join(str(r["plan"][k]) for k in ("bm", "bn", "splits", "strategy"))
            key = {"vgg16": "vgg16_b64_L3_p2", "lenet": "lenet_b256_L1_p2", "resnet18": "resnet18_b128_L1_p0"}[net]
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic.py"), pf, pw,
                                  f"{P}/traffic.json", key, plan], capture_output=True, text=True, check=True).stdout
            open(f"{P}/{tag}_{net}_traffic.txt", "w").write(out)


if __name__ == "__main__":
    main()
