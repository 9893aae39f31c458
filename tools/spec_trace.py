"""Diagnostics: the speculative pairs' record per row-kernel layer over a bench-like run.

Builds the bench's model (synthetic weights seed 17, one fixed batch of random uint8 images and
labels, keep_grads(0), the given plan set), runs --steps steps and prints, per layer and direction,
the last 6 pairs' (bit width, input scale = exponent in + weight scale, guess A used) from the slot
record (niti_model_spec_slot) -- what the hint predictor sees.

  python tools/spec_trace.py --arch resnet18 --load-plans tools/probes/plans_resnet18_r06.json
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
sys.path.insert(0, ROOT)

import niti_amd  # noqa: E402
from niti_amd.model import NitiModel  # noqa: E402
from bench import synth_weights  # noqa: E402

ARCH = {"vgg11": niti_amd.ARCH_VGG11, "vgg16": niti_amd.ARCH_VGG16, "resnet18": niti_amd.ARCH_RESNET18}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--load-plans", default="")
    ap.add_argument("--new-images", action="store_true", help="draw new images every step")
    args = ap.parse_args()
    arch = ARCH[args.arch]
    batch = args.batch or {"vgg11": 256, "vgg16": 64, "resnet18": 128}[args.arch]
    model = NitiModel(arch, batch, 0)
    model.keep_grads(False)
    for i, (w, s) in enumerate(synth_weights(model.layers, seed=17)):
        model.set_weight(i, w, s)
    l0 = model.layers[0]
    rng = np.random.default_rng(100)
    shape = (batch, l0["c_in"], l0["h"], l0["w"])
    x = torch.from_numpy(rng.integers(0, 256, shape).astype(np.uint8)).cuda()
    classes = 10 if args.arch == "vgg11" else 1000
    labels = torch.from_numpy(rng.integers(0, classes, batch).astype(np.int32)).cuda()
    model.train_step_images(x, labels)
    if args.load_plans:
        for k, p in json.load(open(args.load_plans)).items():
            layer, phase = (int(v) for v in k.split(","))
            model.set_plan(layer, phase, p)
    for _ in range(args.steps):
        if args.new_images:
            x = torch.from_numpy(rng.integers(0, 256, shape).astype(np.uint8)).cuda()
        model.train_step_images(x, labels)
    torch.cuda.synchronize()
    for i in range(len(model.layers)):
        for d in (0, 1):
            w = model.spec_slot(i, d)
            n = w[7]
            if n == 0:
                continue
            recs = [w[26 + (j % 6)] for j in range(max(0, n - 6), n)]
            bws = [r & 0xFF for r in recs]
            esc = [((r >> 8) & 0xFFF) - 256 for r in recs]
            used = [(r >> 20) - 1 for r in recs]
            miss = sum(1 for b, u in zip(bws, used) if b != u)
            print(f"layer {i:2d} {'dgrad' if d else 'fwd  '} pairs {n:3d} redone {w[2]:3d} last6 miss {miss:2d}")
            print("   bw    ", " ".join(f"{b:3d}" for b in bws))
            print("   escale", " ".join(f"{e:3d}" for e in esc))
            print("   K      ", " ".join(f"{b + e:3d}" for b, e in zip(bws, esc)))
            print("   guess ", " ".join(f"{u:3d}" for u in used))


if __name__ == "__main__":
    main()
