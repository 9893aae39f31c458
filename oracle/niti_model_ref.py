"""One NITI_SGD training step on the CPU oracle (TEST INFRASTRUCTURE ONLY).

Restates the reference's NITIInt8Train step op by op with the oracle primitives:
  forward  NITIInt8::onForward            tools/train/source/demo/mnistTrain.cpp:159-181
  loss     NITI_LOSS_Grad_Int8            source/backend/cpu/NITI_CPULossGrad_Int8.cpp:81-200
  backward grad/NITI_Conv_Int8_Grad.cpp:16-197, NITI_Pool_Int8_Grad, NITI_ReluGrad_Int8
  update   NITI_SGD::onGetNextParameter   tools/train/source/optimizer/NITI_SGD.hpp:20-54
Parity unpinned (see niti_oracle.h).
"""
from __future__ import annotations

import numpy as np

import niti_oracle as O


def lenet_layers():
    # mnistTrain.cpp:131-157 / :159-181
    return [
        dict(ci=1, co=20, k=5, pad=0, h=28, relu=1, pool=1, flatten=0),
        dict(ci=20, co=52, k=5, pad=0, h=12, relu=1, pool=1, flatten=1),
        dict(ci=832, co=500, k=1, pad=0, h=1, relu=1, pool=0, flatten=0),
        dict(ci=500, co=12, k=1, pad=0, h=1, relu=0, pool=0, flatten=0),
    ]


def vgg11_layers():
    L = []
    for ci, co, h, pool in [(3, 64, 32, 1), (64, 128, 16, 1), (128, 256, 8, 0), (256, 256, 8, 1),
                            (256, 512, 4, 0), (512, 512, 4, 1), (512, 512, 2, 0), (512, 512, 2, 1)]:
        L.append(dict(ci=ci, co=co, k=3, pad=1, h=h, relu=1, pool=pool, flatten=0))
    L.append(dict(ci=512, co=12, k=1, pad=0, h=1, relu=0, pool=0, flatten=0))
    return L


def vgg16_layers(hw=224):
    """VGG-16 (configuration D) with the 4096-4096-1000 head; hw a multiple of 32."""
    L = []
    h = hw
    cfg = [(3, 64, 0), (64, 64, 1), (64, 128, 0), (128, 128, 1), (128, 256, 0), (256, 256, 0), (256, 256, 1),
           (256, 512, 0), (512, 512, 0), (512, 512, 1), (512, 512, 0), (512, 512, 0), (512, 512, 1)]
    for i, (ci, co, pool) in enumerate(cfg):
        L.append(dict(ci=ci, co=co, k=3, pad=1, h=h, relu=1, pool=pool, flatten=int(i == 12)))
        if pool:
            h //= 2
    L.append(dict(ci=512 * h * h, co=4096, k=1, pad=0, h=1, relu=1, pool=0, flatten=0))
    L.append(dict(ci=4096, co=4096, k=1, pad=0, h=1, relu=1, pool=0, flatten=0))
    L.append(dict(ci=4096, co=1000, k=1, pad=0, h=1, relu=0, pool=0, flatten=0))
    return L


def init_weights(layers, seed=17):
    rng = np.random.default_rng(seed)
    W, S = [], []
    for l in layers:
        w, s = O.synth_w(rng, (l["co"], l["ci"], l["k"], l["k"]))
        W.append(w)
        S.append(s)
    return W, S


def onehot(labels, classes=10):
    oh = np.zeros((len(labels), classes), np.int32)
    oh[np.arange(len(labels)), labels] = 1
    return oh


def train_step(layers, W, S, x, exp_in, labels, classes=10, impl="naive", threads=1, wgrad_stats=False,
               acc_mode=None):
    """Returns (new weights, record) where record holds logits, exponents and per-layer taps.

    impl "naive": the exact NCHW restatement; "mnn": the reference-structured one (C4 layout,
    16x4 GEMM unit, the grad graph's transposes / LeftPoolGrad / rot180), exact accumulation, on
    `threads` pthreads (acc_mode O.ACC_F32_SEQ: the reference's float32 accumulation, as the CPU
    baseline runs it; default exact).  wgrad_stats: record per layer, for the weight gradient
    ("wstats"), the forward ("fstats") and the input gradient ("dstats"), the 2^24-guard and int32
    overflow counts (naive pass) and how many int32 sums / int8 outputs / exponents the reference's
    float32 accumulation (Int8FunctionsOpt.cpp:211-226) would change on the same exact inputs (mnn
    pass, ACC_F32_SEQ; the forward pass exposes no int32 tensor, so its int32 count is absent)."""
    n = x.shape[0]
    rec = dict(inp=[], y=[], r=[], p=[], exp=[], dw=[], dy=[], geom=[], wstats=[], fstats=[], dstats=[])
    mnn = impl == "mnn"
    am = O.ACC_EXACT if acc_mode is None else acc_mode
    a = x
    exp = exp_in
    for i, l in enumerate(layers):
        g = O.geom(n, l["ci"], l["h"], l["h"], l["co"], l["k"], pad=l["pad"])
        rec["geom"].append(g)
        rec["inp"].append(a)
        if mnn:
            y, exp, _ = O.mnn_conv_fwd(g, a, W[i], exp, S[i], am, threads)
        else:
            y, exp, _, st = O.conv_fwd(g, a, W[i], exp, S[i])
            assert st.overflow == 0
        if wgrad_stats:
            _, st = O.conv_fwd_acc(g, a, W[i])
            yf, ef, _ = O.mnn_conv_fwd(g, a, W[i], rec["exp"][-1] if i else exp_in, S[i], O.ACC_F32_SEQ, threads)
            rec["fstats"].append(dict(layer=i, outputs=int(y.size), guard=int(st.guard), overflow=int(st.overflow),
                                      f32_int8_diff=int((yf != y).sum()), exp_diff=int(ef != exp)))
        r = O.relu(y) if l["relu"] else y
        rec["y"].append(y)
        rec["r"].append(r)
        rec["exp"].append(exp)
        if l["pool"]:
            p = O.maxpool(r)
            rec["p"].append(p)
            a = p
        else:
            rec["p"].append(None)
            a = r
        if l["flatten"]:
            a = a.reshape(n, -1, 1, 1)
    last = layers[-1]
    logits = rec["r"][-1].reshape(n, last["co"])
    d = O.loss_grad(logits, rec["exp"][-1], onehot(labels, classes)).reshape(n, last["co"], 1, 1)
    dy = [None] * len(layers)
    dy[-1] = d
    newW = list(W)
    for i in range(len(layers) - 1, -1, -1):
        g = rec["geom"][i]
        if mnn:
            dw, bw, acc = O.mnn_conv_wgrad(g, rec["inp"][i], dy[i], am, threads)
        else:
            dw, bw, acc, _ = O.conv_wgrad(g, rec["inp"][i], dy[i])
        if wgrad_stats:
            _, st = O.conv_wgrad_acc(g, rec["inp"][i], dy[i])
            dwf, bwf, accf = O.mnn_conv_wgrad(g, rec["inp"][i], dy[i], O.ACC_F32_SEQ, threads)
            rec["wstats"].insert(0, dict(layer=i, outputs=int(acc.size), guard=int(st.guard),
                                         overflow=int(st.overflow), f32_int32_diff=int((accf != acc).sum()),
                                         f32_int8_diff=int((dwf != dw).sum()), bw=bw, bw_f32=bwf))
        rec["dw"].insert(0, dw)
        if i > 0:
            if mnn:
                dx, dinc, dacc = O.mnn_conv_dgrad(g, dy[i], W[i], am, threads)
            else:
                dx, dinc, dacc, _ = O.conv_dgrad(g, dy[i], W[i])
            if wgrad_stats:
                _, st = O.conv_dgrad_acc(g, dy[i], W[i])
                dxf, dincf, daccf = O.mnn_conv_dgrad(g, dy[i], W[i], O.ACC_F32_SEQ, threads)
                rec["dstats"].insert(0, dict(layer=i, outputs=int(dx.size), guard=int(st.guard),
                                             overflow=int(st.overflow), f32_int32_diff=int((daccf != dacc).sum()),
                                             f32_int8_diff=int((dxf != dx).sum()), exp_diff=int(dincf != dinc)))
            pl = layers[i - 1]
            if pl["flatten"]:
                dx = dx.reshape(rec["p"][i - 1].shape)
            if pl["pool"]:
                dx = O.maxpool_grad(rec["r"][i - 1], rec["p"][i - 1], dx)
            if pl["relu"]:
                dx = O.relu_grad(rec["y"][i - 1], dx)
            dy[i - 1] = dx
        newW[i] = O.sgd_update(W[i], dw)
    rec["dy"] = dy
    rec["logits"] = logits
    return newW, rec
