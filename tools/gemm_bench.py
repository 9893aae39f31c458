#!/usr/bin/env python3
"""Per-op GEMM timing for the VGG-11 layers (batch 256) and a few square matmuls.

Times conv_fwd_acc / conv_dgrad_acc / conv_wgrad_acc (GEMM + any split-K reduce) with HIP
events on the launching stream, and prints us / TOPS / fraction of int8 peak per op.
Diagnostic tool only (GPU box): python3 tools/gemm_bench.py [--reps 20]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))

import torch  # noqa: E402

import niti_amd._lib as L  # noqa: E402
from niti_amd import ops  # noqa: E402

PEAK = 5033.2


def timed(fn, reps):
    st = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--only", default="")
    ap.add_argument("--sweep", action="store_true", help="K sweep of a 16384x256 matmul (256 tiles, no split)")
    args = ap.parse_args()
    lib = L.lib()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    n = args.batch
    if args.sweep:
        amax = torch.zeros(2048, dtype=torch.int32, device="cuda")
        for (m, o) in ((16384, 256), (32768, 256), (16384, 512)):
            for k in (128, 256, 512, 1024, 2048, 4096, 8192):
                B = torch.randint(-127, 128, (m, k), dtype=torch.int8, device="cuda")
                A = torch.randint(-127, 128, (o, k), dtype=torch.int8, device="cuda")
                acc = torch.empty((m, o), dtype=torch.int32, device="cuda")
                f = lambda: lib.niti_matmul_acc(m, o, k, B.data_ptr(), k, A.data_ptr(), k, acc.data_ptr(), o,  # noqa
                                                amax.data_ptr(), None, 0, s)
                assert f() == 0
                us = timed(f, args.reps)
                t = 2 * m * o * k / us / 1e6
                print(f"sweep {m}x{o}x{k:5d}  {us:8.2f} us  {t:8.1f} TOPS  {t / PEAK:6.3f}", flush=True)
        return
    layers = [(3, 64, 32), (64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4),
              (512, 512, 2), (512, 512, 2)]
    dev = "cuda"
    amax = torch.zeros(2048, dtype=torch.int32, device=dev)
    rows = []
    for li, (ci, co, h) in enumerate(layers):
        if args.only and str(li) not in args.only.split(","):
            continue
        g = ops.geom(n, ci, h, h, co, 3, pad=1)
        x = torch.randint(-127, 128, (n * h * h, g.cip), dtype=torch.int8, device=dev)
        dy = torch.randint(-127, 128, (n * g.oh * g.ow, g.cop), dtype=torch.int8, device=dev)
        w = torch.randint(-127, 128, (g.cop, 9, g.cip), dtype=torch.int8, device=dev)
        wt = torch.randint(-127, 128, (g.cip, 9, g.cop), dtype=torch.int8, device=dev)
        ops_n = 2 * n * g.oh * g.ow * co * ci * 9
        for name, op in (("fwd", 0), ("dgrad", 1), ("wgrad", 2)):
            if op == 1 and li == 0:
                continue
            ws, nb = ops.conv_workspace(g, op, dev)
            if op == 0:
                acc = torch.empty((n * g.oh * g.ow, g.cop), dtype=torch.int32, device=dev)
                f = lambda: lib.niti_conv_fwd_acc(C.byref(g), x.data_ptr(), w.data_ptr(), acc.data_ptr(),  # noqa
                                                  amax.data_ptr(), ops._ptr(ws), nb, s)
            elif op == 1:
                acc = torch.empty((n * h * h, g.cip), dtype=torch.int32, device=dev)
                f = lambda: lib.niti_conv_dgrad_acc(C.byref(g), dy.data_ptr(), wt.data_ptr(), acc.data_ptr(),  # noqa
                                                    amax.data_ptr(), ops._ptr(ws), nb, s)
            else:
                acc = torch.empty((g.cop, 9 * g.cip), dtype=torch.int32, device=dev)
                f = lambda: lib.niti_conv_wgrad_acc(C.byref(g), x.data_ptr(), dy.data_ptr(), acc.data_ptr(),  # noqa
                                                    amax.data_ptr(), ops._ptr(ws), nb, s)
            assert f() == 0
            us = timed(f, args.reps)
            t = ops_n / us / 1e6
            rows.append((f"L{li} {name}", us, t))
            print(f"L{li} {name:6s} ci={ci:4d} co={co:4d} h={h:3d}  {us:8.2f} us  {t:8.1f} TOPS  {t / PEAK:6.3f}",
                  flush=True)
    # square matmuls: C[m][o] = A[m][k] . B[o][k]
    for (m, o, k) in ((4096, 4096, 4096), (8192, 8192, 8192), (16384, 256, 2304)):
        B = torch.randint(-127, 128, (m, k), dtype=torch.int8, device=dev)  # acc[m][o] = B[m][:] . A[o][:]
        A = torch.randint(-127, 128, (o, k), dtype=torch.int8, device=dev)
        acc = torch.empty((m, o), dtype=torch.int32, device=dev)
        f = lambda: lib.niti_matmul_acc(m, o, k, B.data_ptr(), k, A.data_ptr(), k, acc.data_ptr(), o,  # noqa
                                        amax.data_ptr(), None, 0, s)
        assert f() == 0
        us = timed(f, max(3, args.reps // 4))
        t = 2 * m * o * k / us / 1e6
        print(f"matmul {m}x{o}x{k}  {us:8.2f} us  {t:8.1f} TOPS  {t / PEAK:6.3f}", flush=True)
    print("total conv GEMM us (b=%d): %.1f" % (n, sum(r[1] for r in rows)))


if __name__ == "__main__":
    main()
