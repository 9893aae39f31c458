"""Weight gradient timing: the NHWC16 kernels (wgrad_taps_kernel + split-K reduce, or the GEMM) vs
the P16 kernel (niti_wgrad.hip) on the VGG-11 batch-256 layer shapes.  Run under
`rocprofv3 --kernel-trace --stats` for per-kernel durations; prints HIP-event times per launch too.
"""
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from niti_amd import ops  # noqa: E402

LAYERS = {"conv2": (256, 64, 16, 128), "conv3": (256, 128, 8, 256), "conv4": (256, 256, 8, 256),
          "conv5": (256, 256, 4, 512), "conv6": (256, 512, 4, 512), "conv7": (256, 512, 2, 512)}


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return b.elapsed_time(e) / reps * 1000.0


def main():
    names = sys.argv[1:] or list(LAYERS)
    rng = np.random.default_rng(0)
    for name in names:
        n, ci, h, co = LAYERS[name]
        g = ops.geom(n, ci, h, h, co, 3, stride=1, pad=1)
        x16 = torch.from_numpy(rng.integers(-127, 128, (n, h, h, ci), dtype=np.int16).astype(np.int8)).cuda()
        d16 = torch.from_numpy((rng.integers(-127, 128, (n, h, h, co), dtype=np.int16) *
                                (rng.random((n, h, h, co)) < 0.3)).astype(np.int8)).cuda()
        xP, dP = ops.nhwc16_to_p16(x16), ops.nhwc16_to_p16(d16)
        amax = ops.new_range()
        gop = 2.0 * n * h * h * ci * co * 9 / 1e9
        old = timeit(lambda: ops.conv_wgrad_acc(g, x16, d16, amax))
        line = [f"{name}: {gop:.2f} GOP  nhwc16 {old:7.2f} us"]
        for s in (0, 1, 2, 4, 8):
            ws, _ = ops.wgrad_p16_workspace(g, s)
            t = timeit(lambda: ops.conv_wgrad_p16_acc(g, xP, dP, amax, splits=s, ws=ws))
            line.append(f"p16 s{s} {t:7.2f} us ({gop / t * 1e3:6.0f} TOPS)")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
