"""Is the VGG-11 batch-256 step host-bound?  Times the host's enqueue of K steps (no sync) against
the wall time until the GPU finishes them, with and without the weight-gradient side stream."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "mandheling-dsp-training_amd")
from bench import synth_weights  # noqa: E402  (bench puts the package on the path)
import niti_amd  # noqa: E402
from niti_amd.model import NitiModel  # noqa: E402
from bench import synth_weights  # noqa: E402


def run(overlap, p16, K=40):
    m = NitiModel(niti_amd.ARCH_VGG11, 256)
    m.set_overlap(overlap)
    for i, (w, s) in enumerate(synth_weights(m.layers, seed=17)):
        m.set_weight(i, w, s)
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.integers(0, 256, (256, 3, 32, 32)).astype(np.uint8)).cuda()
    lab = torch.from_numpy(rng.integers(0, 10, 256).astype(np.int32)).cuda()
    p16_default = {i: p for (i, ph), p in m.plans().items() if ph == 2 and p[:2] == (16, 16)}
    m.train_step_images(x, lab)
    m.autotune()
    if p16:
        for i, p in p16_default.items():
            m.set_plan(i, 2, p)
    for _ in range(5):
        m.train_step_images(x, lab)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        m.train_step_images(x, lab)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    NitiModel.reset_plans()
    print(f"overlap={overlap} p16={p16}: host enqueue {1e6 * (t1 - t0) / K:7.1f} us/step, "
          f"wall {1e6 * (t2 - t0) / K:7.1f} us/step", flush=True)


for ov in (True, False):
    for p16 in (False, True):
        run(ov, p16)
