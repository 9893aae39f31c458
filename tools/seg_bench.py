"""Per-layer A/B of the row-segment register-fed conv (niti_conv_fwd_rows / _dgrad_rows, modes 1 + 2:
range, then recompute-and-requantise) against the implicit-GEMM path (niti_conv_{fwd,dgrad}_phase1/2:
range-or-store, then requantise) on VGG-16's (batch 64) and ResNet-18's (batch 128) stride-1 3x3
layers at 224 px input.  HIP events on the current stream, mean of `reps` back-to-back pairs.

    python tools/seg_bench.py [--reps 5] [--net vgg16|resnet18|both]
"""
import argparse
import os
import sys

import numpy as np
import torch

os.environ.setdefault("NITI_SEG_MAX_CIN", "1024")  # every width on the row-segment form, for the A/B
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
from niti_amd import ops  # noqa: E402

PEAK = 256 * 4 * 2048 * 2.4e9 / 1e12
VGG16 = [(64, 64, 224), (64, 128, 112), (128, 128, 112), (128, 256, 56), (256, 256, 56), (256, 512, 28),
         (512, 512, 28), (512, 512, 14)]
RESNET = [(64, 64, 56), (128, 128, 28), (256, 256, 14)]


def timeit(f, reps):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--net", default="both")
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    nets = []
    if args.net in ("vgg16", "both"):
        nets.append(("VGG-16", 64, VGG16))
    if args.net in ("resnet18", "both"):
        nets.append(("ResNet-18", 128, RESNET))
    for name, n, layers in nets:
        print(f"{name}, batch {n}: us per conv (both launches), fraction of int8 peak")
        for ci, co, h in layers:
            g = ops.geom(n, ci, h, h, co, 3, pad=1)
            ops_n = 2 * n * h * h * ci * co * 9
            x = torch.from_numpy(rng.integers(-127, 128, (n, h, h, ci)).astype(np.int8)).cuda()
            w = torch.from_numpy(rng.integers(-127, 128, (co, ci, 3, 3)).astype(np.int8)).cuda()
            x16 = ops.nchw_to_nhwc16(x.permute(0, 3, 1, 2).contiguous())
            w16 = ops.oihw_to_ohwi16(w)
            wt16 = ops.ohwi16_to_ihwo16(w16, ci)
            dy = torch.from_numpy(rng.integers(-127, 128, (n, co, h, h)).astype(np.int8)).cuda()
            dy16 = ops.nchw_to_nhwc16(dy)
            amax = ops.new_range()
            res = []
            # forward
            xc = ops.nhwc16_to_c32(x16, ci)
            wf = ops.weights_to_wf(w16, ci)

            def rows_f():
                ops.conv_fwd_rows(g, xc, wf, amax, mode=1, relu=True)
                ops.conv_fwd_rows(g, xc, wf, amax, mode=2, relu=True)

            def gemm_f():
                ops.conv_fwd_requant(g, x16, w16, amax, relu=True)
            # input gradient
            dyc = ops.nhwc16_to_c32(dy16, co)
            wft = ops.weights_to_wf(w16, ci, transpose=True)

            def rows_d():
                ops.conv_dgrad_rows(g, dyc, wft, amax, mode=1)
                ops.conv_dgrad_rows(g, dyc, wft, amax, mode=2)

            def gemm_d():
                ops.conv_dgrad_requant(g, dy16, wt16, amax)
            for lab, f in (("fwd rows", rows_f), ("fwd gemm", gemm_f), ("dgrad rows", rows_d), ("dgrad gemm", gemm_d)):
                us = timeit(f, args.reps)
                res.append(f"{lab} {us:8.1f} ({ops_n / us / 1e6 / PEAK:.3f})")
            print(f"  {ci:4d}->{co:4d} @{h:3d}: " + "  ".join(res), flush=True)
            del x, w, x16, w16, wt16, dy, dy16, xc, wf, dyc, wft
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
