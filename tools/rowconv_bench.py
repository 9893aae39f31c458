"""Time the register-fed forward conv (niti_conv_fwd_rows) per mode on the VGG-11 batch-256 3x3
layers: mode 1 (GEMM + range only), mode 2 (GEMM + requantise epilogue), mode 0 (GEMM, in-kernel
grid barrier, epilogue) -- HIP events on the current stream, mean of `reps` launches."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
from niti_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--layer", type=int, default=-1, help="only this VGG-11 layer index (1..7)")
ap.add_argument("--modes", default="1,2,0")
ap.add_argument("--stamps", action="store_true", help="per-wave in-kernel stamps (cycles) of one extra launch per mode")
ap.add_argument("--dgrad", default="", help="time the layer's input gradient instead: 'fused' (the previous layer's "
                "relu / pool gradient as in VGG-11) or 'plain' (requantised dx only)")
args = ap.parse_args()
PEAK = 256 * 4 * 2048 * 2.4e9 / 1e12
layers = [(64, 128, 16, 1), (128, 256, 8, 0), (256, 256, 8, 1), (256, 512, 4, 0), (512, 512, 4, 1),
          (512, 512, 2, 0), (512, 512, 2, 1)]
rng = np.random.default_rng(0)
st = ops.RowConvState()
for li, (ci, co, h, pool) in enumerate(layers, start=1):
    if args.layer > 0 and li != args.layer:
        continue
    n = args.batch
    g = ops.geom(n, ci, h, h, co, 3, pad=1)
    x = torch.from_numpy(rng.integers(-127, 128, (n, ci, h, h)).astype(np.int8)).cuda()
    w = torch.from_numpy(rng.integers(-127, 128, (co, ci, 3, 3)).astype(np.int8)).cuda()
    xc = ops.nhwc16_to_c32(ops.nchw_to_nhwc16(x), ci)
    wf = ops.weights_to_wf(ops.oihw_to_ohwi16(w), ci)
    amax = ops.new_range()
    res = {}
    if args.dgrad:
        prev_pool = li in (1, 2, 4, 6)  # conv0, conv1, conv3, conv5 pool
        dyc = ops.nhwc16_to_c32(ops.nchw_to_nhwc16(torch.from_numpy(
            rng.integers(-127, 128, (n, co, h, h)).astype(np.int8)).cuda()), co)
        wft = ops.weights_to_wf(ops.oihw_to_ohwi16(w), ci, transpose=True)
        hp = 2 * h if prev_pool else h
        px = torch.from_numpy(np.maximum(rng.integers(-2, 6, (n, hp, hp, ci)), 0).astype(np.int8)).cuda()
        py = torch.from_numpy(np.maximum(rng.integers(-2, 6, (n, h, h, ci)), 0).astype(np.int8)).cuda()
        kw = {}
        if args.dgrad == "fused":
            kw = dict(pool_x=px, pool_y=py, pool_relu=True) if prev_pool else dict(relu_mask=px)
    for mode in [int(v) for v in args.modes.split(",")]:
        if args.dgrad:
            f = lambda: ops.conv_dgrad_rows(g, dyc, wft, amax, mode=mode, state=st, dx_c32=True,  # noqa
                                            dx_p16=args.dgrad == "fused", **kw)
        else:
            f = lambda: ops.conv_fwd_rows(g, xc, wf, amax, mode=mode, state=st, relu=True, pool=bool(pool),  # noqa
                                          next_c32=True)
        try:
            f()
        except Exception:  # the P16 dy copy is not fused for this shape (the model converts it)
            f = lambda: ops.conv_dgrad_rows(g, dyc, wft, amax, mode=mode, state=st, dx_c32=True, **kw)  # noqa
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[mode] = e0.elapsed_time(e1) * 1e3 / args.reps
        if args.stamps:
            import ctypes as C
            from niti_amd import _lib as L
            buf = torch.zeros(16 * 4 * 2048, dtype=torch.int64, device="cuda")
            L.lib().niti_diag_rowconv_stamps(C.c_void_p(buf.data_ptr()))
            f()
            torch.cuda.synchronize()
            L.lib().niti_diag_rowconv_stamps(None)
            t = buf.view(-1, 16).cpu().numpy()
            rt = t[::4, 8:10].astype(np.float64)  # wave 0 of each workgroup
            rt = rt[rt[:, 0] > 0]
            t = t[t[:, 0] > 0].astype(np.float64)
            d = lambda k0, k1: np.median(t[:, k1] - t[:, k0])  # noqa: E731  (per-wave deltas: s_memtime is per XCD)
            print(f"    mode {mode} waves {len(t)}: prologue {d(0, 1):.0f}  K loop {d(1, 3):.0f}  "
                  f"(waits {np.median(t[:, 6]):.0f}, issuing loads {np.median(t[:, 2]):.0f}, fragment reads "
                  f"{np.median(t[:, 7]) - np.median(t[:, 2]):.0f})  to max/barrier {d(3, 4) if mode == 0 else 0:.0f}  "
                  f"epilogue {d(4, 5) if mode == 0 else 0:.0f}  total {d(0, 5) if mode != 2 else 0:.0f} cycles", flush=True)
            if mode == 0 and len(rt):
                arr, rel_ = rt[:, 0], rt[:, 1]
                print(f"      grid barrier (us): arrivals spread {(arr.max() - arr.min()) / 100:.2f}, median wait "
                      f"{np.median(rel_ - arr) / 100:.2f}, last arrival -> last release {(rel_.max() - arr.max()) / 100:.2f}",
                      flush=True)
    ops_ = 2 * n * h * h * co * ci * 9
    print(f"{ci:4d}->{co:4d} @{h:2d} pool={pool}: " + "  ".join(f"mode {m} {t:6.2f} us ({ops_ / t / 1e6 / PEAK:.3f})"
                                                                 for m, t in res.items()), flush=True)
print("barrier timeouts:", int(st.err.item()))
