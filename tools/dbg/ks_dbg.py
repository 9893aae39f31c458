import sys, os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import niti_oracle as O
from niti_amd import ops
for seed, (n, ci, co) in [(921, (33, 256, 64)), (5, (8, 512, 32)), (6, (16, 128, 32))]:
    rng = np.random.default_rng(seed)
    h = 2
    g = O.geom(n, ci, h, h, co, 3, pad=1)
    x = rng.integers(-127, 128, (n, ci, h, h)).astype(np.int8)
    w = rng.integers(-127, 128, (co, ci, 3, 3)).astype(np.int8)
    acc, _ = O.conv_fwd_acc(g, x, w)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    gg = ops.geom(n, ci, h, h, co, 3, pad=1)
    xc = ops.nhwc16_to_c32(ops.nchw_to_nhwc16(dev(x)), ci)
    wf = ops.weights_to_wf(ops.oihw_to_ohwi16(dev(w)), ci)
    for mode in (0, 1):
        amax = ops.new_range(); st = ops.RowConvState()
        if mode == 0:
            out, _, _ = ops.conv_fwd_rows(gg, xc, wf, amax, mode=0, state=st, relu=False)
        else:
            ops.conv_fwd_rows(gg, xc, wf, amax, mode=1, relu=False)
            out, _, _ = ops.conv_fwd_rows(gg, xc, wf, amax, mode=2, relu=False)
        torch.cuda.synchronize()
        y, _, _, _ = O.conv_fwd(g, x, w, 0, 0)
        got = out.cpu().numpy()[..., :co].transpose(0, 3, 1, 2)
        bad = np.argwhere(got != y)
        print(seed, n, ci, co, "mode", mode, "range", ops.range_max(amax), "true max", int(np.abs(acc).max()), "bad", len(bad), bad[:12].tolist())
