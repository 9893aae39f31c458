"""Per-block stamp report of the P16 weight-gradient kernel (NITI_WG_STAMPS builds, tools/wg_diag.sh):
mean cycles of prologue / K loop (and per region step) / K-group exchange / output, plus event time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import niti_amd._lib as L  # noqa: E402
from niti_amd import ops  # noqa: E402
from wg_bench import LAYERS  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "conv4"
    splits = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "1,4").split(",")]
    n, ci, h, co = LAYERS[name]
    rng = np.random.default_rng(0)
    g = ops.geom(n, ci, h, h, co, 3, stride=1, pad=1)
    x16 = torch.from_numpy(rng.integers(-127, 128, (n, h, h, ci), dtype=np.int16).astype(np.int8)).cuda()
    d16 = torch.from_numpy(rng.integers(-127, 128, (n, h, h, co), dtype=np.int16).astype(np.int8)).cuda()
    xP, dP = ops.nhwc16_to_p16(x16), ops.nhwc16_to_p16(d16)
    amax = ops.new_range()
    kg_total = n * h * h // 32
    tiles = (co // 32) * (ci // 32)
    for s in splits:
        ws, _ = ops.wgrad_p16_workspace(g, s)
        st = torch.zeros(tiles * s * 16, dtype=torch.int64, device="cuda")
        for _ in range(3):
            ops.conv_wgrad_p16_acc(g, xP, dP, amax, splits=s, ws=ws)
        torch.cuda.synchronize()
        L.lib().niti_diag_wgrad_stamps(C_ptr(st))
        b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b.record()
        ops.conv_wgrad_p16_acc(g, xP, dP, amax, splits=s, ws=ws)
        e.record()
        torch.cuda.synchronize()
        L.lib().niti_diag_wgrad_stamps(None)
        allst = st.cpu().numpy().astype(np.int64)
        a = allst[:tiles * s * 8].reshape(-1, 8)
        wv = allst[tiles * s * 8:].reshape(-1, 4, 2)  # [block][wave][start, loop end]
        steps = -(-((kg_total + s - 1) // s) // 4)  # K groups per wave (4 waves)
        last = a[:, 5] > a[:, 0]  # blocks that wrote the output (last arrivers / all)
        clk = np.median((a[last, 5] - a[last, 0]) / np.maximum(a[last, 7] - a[last, 6], 1) * 100.0)
        d = np.diff(a[:, :6], axis=1).astype(np.float64)
        d[:, 3:] = np.where(last[:, None], d[:, 3:], np.nan)
        m = np.nanmean(d, axis=0)
        spread = (a[:, 6].max() - a[:, 6].min()) / 100.0  # block starts, us (s_memrealtime: 100 MHz)
        wall = (a[last, 7].max() - a[:, 6].min()) / 100.0
        # wall-clock (us) from the first block start: when the last K loop ends, when the last
        # partial tile is in the slab, when the last output is written
        t0w = a[:, 6].min()
        loop_end = ((a[:, 6] + (a[:, 2] - a[:, 0]) / (clk / 100.0)) - t0w).max() / 100.0
        print(f"{name} splits {s}: {tiles * s} blocks x {steps} K groups per wave, event {b.elapsed_time(e) * 1e3:.1f} us; "
              f"cycles prologue {m[0]:.0f} loop {m[1]:.0f} ({m[1] / steps:.0f}/K group) slowest wave {m[2]:.0f} "
              f"LDS adds {m[3]:.0f} output {m[4]:.0f}; start spread {spread:.2f} us, first start to last end {wall:.2f} us, "
              f"clock {clk:.0f} MHz; last K loop ends at {loop_end:.2f} us", flush=True)
        if wv[:, :, 0].min() > 0:
            ws0 = wv[:, :, 0] - wv[:, :1, 0]
            we = wv[:, :, 1] - wv[:, :1, 1]
            dur = wv[:, :, 1] - wv[:, :, 0]
            print(f"  per wave (cycles, mean over blocks): start - wave0 {ws0.mean(0).round()}, loop end - wave0 "
                  f"{we.mean(0).round()}, duration {dur.mean(0).round()}; end spread in a block mean "
                  f"{(wv[:, :, 1].max(1) - wv[:, :, 1].min(1)).mean():.0f} max {(wv[:, :, 1].max(1) - wv[:, :, 1].min(1)).max():.0f}; "
                  f"slowest wave id histogram {np.bincount(wv[:, :, 1].argmax(1), minlength=4)}", flush=True)


def C_ptr(t):
    return t.data_ptr()


if __name__ == "__main__":
    main()
