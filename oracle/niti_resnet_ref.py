"""One NITI_SGD training step of ResNet-18 on the CPU oracle (TEST INFRASTRUCTURE ONLY).

BASELINE.json config 5 names ResNet-18, but the reference has no ResNet NITI model and no residual
rule: NITI_Eltwise_Int8 is an empty stub (execution-engine/source/backend/cpu/NITI_Eltwise_Int8.cpp:20-28).
The rules below are this project's, built only from the reference's NITI pieces:
  conv / relu / max pool / loss / weight update: the NITIInt8Train ops as niti_model_ref.py restates
    them (NITI_Conv_Int8.cpp:255-307 forward and input-gradient requantisation, NITI_SGD.hpp:20-54);
  residual add (forward block output, and the gradient sum at a block input): residual_add() below,
    then the forward requantisation (range estimate, PSTO(bitwidth - 7), exponent + inc);
  global pool: the sum over the pixels, then the same requantisation; its gradient broadcasts dy;
  gradient exponents: the loss gradient has exponent 0, an input gradient e_dy + wscale + inc (the
    forward rule applied to NITI_DeConv_Int8's output), and pooling / relu gradients keep theirs --
    so the two gradients meeting at a block input can be aligned like the forward add.
Parity unpinned (no reference ResNet exists to pin it against).
"""
from __future__ import annotations

import numpy as np

import niti_oracle as O
from niti_model_ref import onehot


def resnet18_convs(hw=224, classes=1000):
    """The 21 parameter layers in parameter order: conv1, then per basic block conv a, conv b and
    (first block of stages 2-4) the 1x1 stride-2 projection, then the fc head (a 1x1 conv).
    Each: dict(name, ci, co, k, stride, pad, h (input size))."""
    L = [dict(name="conv1", ci=3, co=64, k=7, stride=2, pad=3, h=hw)]
    h = (hw + 6 - 7) // 2 + 1          # conv1 output
    h = (h + 2 - 3) // 2 + 1           # 3x3 / 2 max pool, pad 1
    ci = 64
    for stage, co in enumerate((64, 128, 256, 512)):
        for blk in range(2):
            s = 2 if stage > 0 and blk == 0 else 1
            L.append(dict(name=f"layer{stage + 1}.{blk}.a", ci=ci, co=co, k=3, stride=s, pad=1, h=h))
            ho = (h + 2 - 3) // s + 1
            L.append(dict(name=f"layer{stage + 1}.{blk}.b", ci=co, co=co, k=3, stride=1, pad=1, h=ho))
            if s != 1 or ci != co:
                L.append(dict(name=f"layer{stage + 1}.{blk}.proj", ci=ci, co=co, k=1, stride=s, pad=0, h=h))
            ci, h = co, ho
    L.append(dict(name="fc", ci=512, co=classes, k=1, stride=1, pad=0, h=1))
    return L


def blocks(convs):
    """[(index of conv a, conv b, projection or None)] of the 8 basic blocks."""
    out, i = [], 1
    while i < len(convs) - 1:
        proj = i + 2 if convs[i + 2]["name"].endswith("proj") else None
        out.append((i, i + 1, proj))
        i += 3 if proj else 2
    return out


def init_weights(convs, seed=18):
    rng = np.random.default_rng(seed)
    W, S = [], []
    for l in convs:
        w, s = O.synth_w(rng, (l["co"], l["ci"], l["k"], l["k"]))
        W.append(w)
        S.append(s)
    return W, S


def _e8(v):
    return int(np.int8(np.int32(v).astype(np.int8)))


def residual_add(a, ea, b, eb):
    """z = hi * 2^d + (lo >> r) (int32), d = min(|ea - eb|, 23), r = |ea - eb| - d, hi the operand
    with the larger exponent (a on ties); returns (z, e_hi - d)."""
    a_hi = ea >= eb
    hi, lo = (a, b) if a_hi else (b, a)
    diff = abs(int(ea) - int(eb))
    d = min(diff, 23)
    r = diff - d
    z = hi.astype(np.int32) * (1 << d) + (lo.astype(np.int32) >> min(r, 31))
    return z.astype(np.int32), int((ea if a_hi else eb) - d)


def requant(z, e):
    """The forward requantisation of an int32 tensor with exponent e: (int8, exponent)."""
    q, inc = O.requant_fwd(z)
    return q, _e8(e + inc)


def _conv(l, n):
    return O.geom(n, l["ci"], l["h"], l["h"], l["co"], l["k"], stride=l["stride"], pad=l["pad"])


def train_step(convs, W, S, x, exp_in, labels, classes=1000):
    """Returns (new weights, record): record['fwd'][i] / ['dy'][i] / ['dw'][i] per parameter layer
    (the requantised pre-relu conv output, its output gradient, the int8 weight gradient),
    'logits' with 'exp_logits', and the block outputs with their exponents."""
    n = x.shape[0]
    rec = dict(fwd=[None] * len(convs), exp=[None] * len(convs), inp=[None] * len(convs), dy=[None] * len(convs),
               dw=[None] * len(convs), blk_out=[], blk_exp=[])
    G = [_conv(l, n) for l in convs]

    def conv_fwd(i, a, ea):
        y, e, _, st = O.conv_fwd(G[i], a, W[i], ea, S[i])
        assert st.overflow == 0
        rec["fwd"][i], rec["exp"][i], rec["inp"][i] = y, e, a
        return y, e

    # stem: conv1 + relu, 3x3 / 2 max pool (pad 1)
    y, e = conv_fwd(0, x, exp_in)
    r0 = O.relu(y)
    p0 = O.maxpool(r0, 3, 2, 1)
    u, eu = p0, e
    BL = blocks(convs)
    saved = []
    for (ia, ib, ip) in BL:
        ya, ea = conv_fwd(ia, u, eu)
        h = O.relu(ya)
        yb, eb = conv_fwd(ib, h, ea)
        if ip is not None:
            sc, es = conv_fwd(ip, u, eu)
        else:
            sc, es = u, eu
        z, ez = residual_add(yb, eb, sc, es)
        q, eo = requant(z, ez)
        out = O.relu(q)
        saved.append(dict(u=u, eu=eu, h=h, ya=ya, q=q))
        rec["blk_out"].append(out)
        rec["blk_exp"].append(eo)
        u, eu = out, eo
    # global sum pool + requantisation, fc head (1x1 conv on 1x1 images)
    gsum = u.astype(np.int32).sum(axis=(2, 3)).astype(np.int32)
    g8, eg = requant(gsum, eu)
    rec["pool"], rec["pool_exp"] = g8, eg
    fc = len(convs) - 1
    logits4, el = conv_fwd(fc, g8.reshape(n, -1, 1, 1), eg)
    logits = logits4.reshape(n, classes)
    rec["logits"], rec["exp_logits"] = logits, el
    d = O.loss_grad(logits, el, onehot(labels, classes)).reshape(n, classes, 1, 1)
    ed = 0

    newW = list(W)
    dW = [None] * len(convs)

    def wgrad(i, dy):
        dw, _, _, _ = O.conv_wgrad(G[i], rec["inp"][i], dy)
        rec["dy"][i], rec["dw"][i] = dy, dw
        dW[i] = dw

    def dgrad(i, dy, edy):
        dx, inc, _, _ = O.conv_dgrad(G[i], dy, W[i])
        return dx, _e8(edy + S[i] + inc)

    wgrad(fc, d)
    dg, edg = dgrad(fc, d, ed)
    hh = u.shape[2]
    du = np.broadcast_to(dg.reshape(n, -1, 1, 1), (n, dg.shape[1], hh, hh)).astype(np.int8).copy()
    edu = edg
    for k in range(len(BL) - 1, -1, -1):
        ia, ib, ip = BL[k]
        s = saved[k]
        dz = O.relu_grad(s["q"], du)                  # block-output relu
        wgrad(ib, dz)
        dh, edh = dgrad(ib, dz, edu)
        dh = O.relu_grad(s["ya"], dh)                 # relu after conv a
        wgrad(ia, dh)
        dua, edua = dgrad(ia, dh, edh)
        if ip is not None:
            wgrad(ip, dz)
            dus, edus = dgrad(ip, dz, edu)
        else:
            dus, edus = dz, edu
        zsum, ez = residual_add(dua, edua, dus, edus)
        du, edu = requant(zsum, ez)
    # stem backward: max pool, relu, conv1 weight gradient
    dp = O.maxpool_grad(r0, p0, du, 3, 2, 1)
    d0 = O.relu_grad(rec["fwd"][0], dp)
    wgrad(0, d0)
    for i in range(len(convs)):
        newW[i] = O.sgd_update(W[i], dW[i])
    return newW, rec
