#!/usr/bin/env python3
"""Split-K / tile sweep of one weight-gradient GEMM (diagnostic, GPU box, run under rocprofv3
--kernel-trace; tools/sweep_summary.py then groups the GEMM dispatches by grid).
python3 tools/wgrad_sweep.py --layer 3 --splits 1,2,4,7,14 --tiles 0,6464"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))

import torch  # noqa: E402

import niti_amd._lib as L  # noqa: E402
from niti_amd import ops  # noqa: E402

LAYERS = [(3, 64, 32), (64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4),
          (512, 512, 2), (512, 512, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--splits", default="1,2,3,4,5,7,9,14,18,28")
    ap.add_argument("--tiles", default="0")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--op", type=int, default=2)
    ap.add_argument("--notaps", action="store_true", help="generic K-major GEMM only (NITI_DIAG_NO_TAPS)")
    args = ap.parse_args()
    if args.notaps:
        os.environ["NITI_DIAG_NO_TAPS"] = "1"
    lib = L.lib()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ci, co, h = LAYERS[args.layer]
    n = args.batch
    g = ops.geom(n, ci, h, h, co, 3, pad=1)
    dev = "cuda"
    x = torch.randint(-127, 128, (n * h * h, g.cip), dtype=torch.int8, device=dev)
    dy = torch.randint(-127, 128, (n * g.oh * g.ow, g.cop), dtype=torch.int8, device=dev)
    w = torch.randint(-127, 128, (g.cop, 9, g.cip), dtype=torch.int8, device=dev)
    amax = torch.zeros(2048, dtype=torch.int32, device=dev)
    ws = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for t in args.tiles.split(","):
        if t != "0":
            os.environ["NITI_DIAG_TILE"] = t
        else:
            os.environ.pop("NITI_DIAG_TILE", None)
        for sp in args.splits.split(","):
            os.environ["NITI_DIAG_SPLITS"] = sp
            if args.op == 2:
                acc = torch.empty((g.cop, 9 * g.cip), dtype=torch.int32, device=dev)
                f = lambda: lib.niti_conv_wgrad_acc(C.byref(g), x.data_ptr(), dy.data_ptr(), acc.data_ptr(),  # noqa
                                                    amax.data_ptr(), ws.data_ptr(), ws.numel(), s)
            else:
                acc = torch.empty((n * g.oh * g.ow, g.cop), dtype=torch.int32, device=dev)
                f = lambda: lib.niti_conv_fwd_acc(C.byref(g), x.data_ptr(), w.data_ptr(), acc.data_ptr(),  # noqa
                                                  amax.data_ptr(), ws.data_ptr(), ws.numel(), s)
            for _ in range(args.reps):
                assert f() == 0
            torch.cuda.synchronize()
            print(f"tile {t} splits {sp} done", flush=True)


if __name__ == "__main__":
    main()
