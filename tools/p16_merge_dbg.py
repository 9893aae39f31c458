"""Where does the P16 weight gradient differ from the oracle (rows / taps / columns)?"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from niti_amd import ops  # noqa: E402
import niti_oracle as O  # noqa: E402

n, ci, h, co = int(os.environ.get("DBG_N", "2")), 32, 8, 32
rng = np.random.default_rng(0)
x = rng.integers(-127, 128, (n, ci, h, h)).astype(np.int8)
dy = rng.integers(-127, 128, (n, co, h, h)).astype(np.int8)
g = O.geom(n, ci, h, h, co, 3, pad=1)
ref, _ = O.conv_wgrad_acc(g, x, dy)  # [co][ci][3][3]
gg = ops.geom(n, ci, h, h, co, 3, pad=1)
xP = ops.nhwc16_to_p16(ops.nchw_to_nhwc16(torch.from_numpy(x).cuda()))
dP = ops.nhwc16_to_p16(ops.nchw_to_nhwc16(torch.from_numpy(dy).cuda()))
acc = ops.conv_wgrad_p16_acc(gg, xP, dP, splits=1).cpu().numpy()  # [co][3][3][cip]
got = acc[..., :ci].transpose(0, 3, 1, 2)
bad = np.argwhere(got != ref)
print("mismatches", len(bad), "of", ref.size)
if len(bad):
    rows = sorted(set(bad[:, 0].tolist()))
    print("rows", rows)
    print("taps", sorted(set((b[2] * 3 + b[3]) for b in bad.tolist())))
    print("cols", sorted(set(bad[:, 1].tolist()))[:40])
    r = rows[0]
    print("row", r, "got", got[r, :4, 1, 1], "ref", ref[r, :4, 1, 1], "ratio", got[r, 0, 1, 1] / max(ref[r, 0, 1, 1], 1))
