"""2^24-guard and float32-accumulation change counts at ImageNet size, at the bench batch, on a sampled
layer set: VGG-16 224 px batch 64 (BASELINE cfg 4 per GPU) and ResNet-18 224 px
batch 128 (cfg 5 per GPU, its stem).

One device step (uint8 images through the on-device quantiser, as bench.py) records every layer's
input, output, output gradient and int8 weight gradient; for sampled outputs of a few layers the
oracle (niti_ref_sample_stats) computes the exact sum, sum|p| and the sum the reference's float32
unit would produce (Int8FunctionsOpt.cpp:211-226, product by product in its K order).  Reported per
layer and op: outputs sampled, how many have sum|p| >= 2^24 (where the float32 accumulation is not
guaranteed exact), how many int32 sums the float32 order changes, and how many int8 outputs change
under the layer's shift (inferred from the device's own int8 outputs on the samples).

    python tools/guard_sample.py [--arch vgg16|resnet18|both] [--samples 4096] [--wsamples 128]
"""
import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mandheling-dsp-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import niti_oracle as O  # noqa: E402


def psto(a, s):
    """NITI_MNNPstoShiftInt32 (CommonOptFunction.cpp:1595-1627) on int64 arrays, clipped to +-127."""
    a = np.asarray(a, np.int64)
    if s <= 0:
        return np.clip(a, -127, 127)
    ua = np.abs(a)
    q = ua >> s
    prob = ua & ((1 << s) - 1)
    h = s >> 1
    qp = prob >> h
    pr = prob & ((1 << h) - 1)
    if s & 1:
        pr = pr << 1
    r = np.minimum(q + (qp > pr), 127)
    return np.where(a < 0, -r, r)


def act_rule(a, s):
    """the forward / input-gradient rule for shift s = bw - 7: raw int8 cast, or PSTO(max(s, 2))"""
    a = np.asarray(a, np.int64)
    if s <= 0:
        return ((a + 128) % 256 - 128)
    return psto(a, max(s, 2))


def infer(fn, exact, dev, lo, hi):
    for s in range(lo, hi):
        if np.array_equal(fn(exact, s), dev):
            return s
    return None


def stats(g, kind, a, b, idx, threads):
    chunks = np.array_split(idx, max(1, min(threads, idx.size)))
    with ThreadPoolExecutor(len(chunks)) as ex:
        parts = list(ex.map(lambda c: O.sample_stats(g, kind, a, b, c), chunks))
    return tuple(np.concatenate([p[k] for p in parts]) for k in range(3))


def report(name, op, g, kind, a, b, dev, idx, threads, relu=False, rule="act"):
    t = time.time()
    ex, sa, f = stats(g, kind, a, b, idx, threads)
    guard = int((sa >= (1 << 24)).sum())
    ch32 = int((f.astype(np.int64) != ex).sum())
    line = f"  {name:<18} {op:<15} sampled {idx.size:>6}  sum|p| >= 2^24: {guard:>6}  float32 changes {ch32:>4} int32 sums"
    if dev is not None:
        dv = dev.ravel()[idx].astype(np.int64)
        if rule == "act":
            fn = (lambda v, s: np.maximum(act_rule(v, s), 0)) if relu else act_rule
            s = infer(fn, ex, dv, -8, 31)
        else:
            fn = psto
            s = infer(fn, ex, dv, 0, 31)
        if s is None:
            line += " / int8: shift not inferred (device != exact on the samples)"
        else:
            line += f" / {int((fn(f, s) != fn(ex, s)).sum())} int8 outputs (shift {s}; device == exact on every sample)"
    print(line + f"  [{time.time() - t:.1f} s]", flush=True)


def run_vgg16(args, T, threads):
    import niti_amd
    import niti_model_ref as R
    from niti_amd.model import NitiModel
    batch = 64
    layers = R.vgg16_layers(224)
    W, S = R.init_weights(layers, seed=7)
    m = NitiModel(niti_amd.ARCH_VGG16, batch)
    for i, (w, s) in enumerate(zip(W, S)):
        m.set_weight(i, w, s)
    rng = np.random.default_rng(7)
    img = T.from_numpy(rng.integers(0, 256, (batch, 3, 224, 224), dtype=np.uint8)).cuda()
    lab = T.from_numpy(rng.integers(0, 1000, batch).astype(np.int32)).cuda()
    m.keep_grads(True)
    m.train_step_images(img, lab)
    T.cuda.synchronize()
    print(f"VGG-16 224x224, batch {batch}, one device step from uint8 images (seed 7)", flush=True)
    x0, _ = m.input()
    srng = np.random.default_rng(1)
    for i in (0, 1, 4, 13):
        l = layers[i]
        if i == 0:
            x = x0
        elif i == 13:  # the first FC layer: the flattened pooled last conv output as a 1x1 map
            x = O.maxpool(m.tap(12, 0)).reshape(batch, -1, 1, 1)
        else:
            prev = m.tap(i - 1, 0)
            x = O.maxpool(prev) if layers[i - 1]["pool"] else prev
        y = m.tap(i, 0)
        dy = m.tap(i, 2)
        dw = m.tap(i, 1)
        h = l["h"]
        g = O.geom(batch, l["ci"], h, h, l["co"], l["k"], pad=l["pad"])
        name = f"layer {i} {l['ci']}->{l['co']}@{h}"
        ny = batch * l["co"] * g.oh * g.ow
        report(name, "forward", g, 0, x, W[i], y, srng.choice(ny, min(args.samples, ny), replace=False), threads,
               relu=bool(l["relu"]))
        nw = l["co"] * l["ci"] * l["k"] * l["k"]
        report(name, "weight gradient", g, 1, x, dy, dw, srng.choice(nw, min(args.wsamples, nw), replace=False),
               threads, rule="grad")
        if i > 0 and l["k"] == 3:
            nx = batch * l["ci"] * h * h
            report(name, "input gradient", g, 2, dy, W[i], None, srng.choice(nx, min(args.samples, nx), replace=False),
                   threads)
        del x, y, dy


def run_resnet18(args, T, threads):
    """The stem (7x7 / 2 over 224 px, the ResNet-18 layer with the largest K and the most guard
    passes) on the C++ step driver: its input is the quantised batch (model.input()); the other
    layers' inputs are not exposed as taps by niti_model_get_tap."""
    import niti_amd
    from niti_amd.model import NitiModel
    batch = 128
    net = NitiModel(niti_amd.ARCH_RESNET18, batch, 224, 1000)
    rng = np.random.default_rng(11)
    W = []
    for i in range(len(net.layers)):
        w, s = O.synth_w(rng, net.weight_shape(i))
        net.set_weight(i, w, s)
        W.append(w)
    img = T.from_numpy(rng.integers(0, 256, (batch, 3, 224, 224), dtype=np.uint8)).cuda()
    lab = T.from_numpy(rng.integers(0, 1000, batch).astype(np.int32)).cuda()
    net.train_step_images(img, lab)
    T.cuda.synchronize()
    print(f"ResNet-18 224x224, batch {batch}, one device step from uint8 images (seed 11), the stem", flush=True)
    srng = np.random.default_rng(2)
    l = net.layers[0]
    x, _ = net.input()
    y, dy, dw = net.tap(0, 0), net.tap(0, 2), net.tap(0, 1)
    g = O.geom(batch, l["c_in"], l["h"], l["w"], l["c_out"], l["kh"], stride=l["stride"], pad=l["pad"])
    name = f"stem {l['c_in']}->{l['c_out']}@{l['h']}"
    ny = batch * l["c_out"] * g.oh * g.ow
    report(name, "forward", g, 0, x, W[0], y, srng.choice(ny, min(args.samples, ny), replace=False), threads,
           relu=bool(l["relu"]))
    nw = l["c_out"] * l["c_in"] * l["kh"] * l["kw"]
    report(name, "weight gradient", g, 1, x, dy, dw, srng.choice(nw, min(args.wsamples, nw), replace=False),
           threads, rule="grad")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="both", choices=["vgg16", "resnet18", "both"])
    ap.add_argument("--samples", type=int, default=4096)
    ap.add_argument("--wsamples", type=int, default=96)
    args = ap.parse_args()
    import torch as T
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    print(f"oracle threads {threads}; samples per forward / input gradient {args.samples}, per weight gradient "
          f"{args.wsamples}", flush=True)
    if args.arch in ("vgg16", "both"):
        run_vgg16(args, T, threads)
    if args.arch in ("resnet18", "both"):
        run_resnet18(args, T, threads)


if __name__ == "__main__":
    main()
