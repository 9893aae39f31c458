#!/usr/bin/env python3
"""Generate tests/golden/niti_golden.npz: fixed input/output vectors of the NITI int8 path.

Produced by the CPU oracle (oracle/, a restatement of the reference's CPU int8 path; parity
unpinned): the reference holds no fixture of its own for this path and running
it was denied, so these vectors pin the oracle against drift and give the HIP path fixed cases
to match.  Cases:
  * PSTO shift over a table of values and every shift 0..31, range estimates
  * conv forward / weight gradient / input gradient (+ requant, exponents) on three geometries
    (stride 1 pad 1, stride 2 pad 1 with odd sizes, 5x5 valid with ragged channels)
  * NITI_Matmul_Int8, relu / max pool / pool gradient / loss gradient
  * one whole LeNet NITI_SGD training step at batch 4 (updated weights stored as new - old)
Run from the repository root: python3 tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import niti_model_ref as R  # noqa: E402
import niti_oracle as O  # noqa: E402

GEOMS = [  # n, ci, h, co, k, stride, pad
    (2, 8, 8, 16, 3, 1, 1),
    (3, 6, 9, 8, 3, 2, 1),
    (2, 5, 12, 12, 5, 1, 0),
]


def main():
    rng = np.random.default_rng(2024)
    out = {}
    vals = np.array([0, 1, -1, 2, -2, 3, -3, 5, -5, 127, -127, 128, -128, 255, -255, 1000, -1000, 65535,
                     -65535, 1 << 20, -(1 << 20), 2147483647, -2147483647], np.int32)
    shifts = np.arange(0, 32, dtype=np.int32)
    out["psto_vals"] = vals
    out["psto_shifts"] = shifts
    out["psto_out"] = np.stack([O.psto(vals, int(s)) for s in shifts])
    rs = [np.array(v, np.int32) for v in ([0], [1], [2], [3], [-4], [5, -9], [127, 128], [1 << 20, 1], [-2147483647])]
    out["range_cases"] = np.array([O.range_estimate(a) for a in rs], np.int32)
    out["range_lens"] = np.array([len(a) for a in rs], np.int32)
    out["range_vals"] = np.concatenate(rs)
    for gi, (n, ci, h, co, k, s, p) in enumerate(GEOMS):
        g = O.geom(n, ci, h, h, co, k, stride=s, pad=p)
        x = O.synth_x(rng, (n, ci, h, h))
        w, ws = O.synth_w(rng, (co, ci, k, k))
        dy = O.synth_dy(rng, (n, co, g.oh, g.ow))
        y, e, _, _ = O.conv_fwd(g, x, w, -7, ws)
        dw, bw, _, _ = O.conv_wgrad(g, x, dy)
        dx, inc, _, _ = O.conv_dgrad(g, dy, w)
        out.update({f"g{gi}_x": x, f"g{gi}_w": w, f"g{gi}_dy": dy, f"g{gi}_wscale": np.int32(ws),
                    f"g{gi}_y": y, f"g{gi}_exp": np.int32(e), f"g{gi}_dw": dw, f"g{gi}_bw": np.int32(bw),
                    f"g{gi}_dx": dx, f"g{gi}_dinc": np.int32(inc)})
    B = rng.integers(-127, 128, (24, 40)).astype(np.int8)
    A = rng.integers(-127, 128, (12, 40)).astype(np.int8)
    dwT, bw, _, _ = O.matmul(B, A)
    out.update({"mm_B": B, "mm_A": A, "mm_dwT": dwT, "mm_bw": np.int32(bw)})
    x = rng.integers(-127, 128, (2, 4, 6, 6)).astype(np.int8)
    y = O.maxpool(x)
    dyp = rng.integers(-127, 128, y.shape).astype(np.int8)
    out.update({"pool_x": x, "pool_y": y, "pool_dy": dyp, "pool_dx": O.maxpool_grad(x, y, dyp),
                "relu_y": O.relu(x), "relu_dx": O.relu_grad(x, O.relu(x))})
    logits = rng.integers(-127, 128, (5, 12)).astype(np.int8)
    labels = rng.integers(0, 10, 5).astype(np.int32)
    out.update({"loss_logits": logits, "loss_labels": labels, "loss_ascale": np.int32(-4),
                "loss_grad": O.loss_grad(logits, -4, R.onehot(labels, 12))})
    layers = R.lenet_layers()
    W, S = R.init_weights(layers, seed=31)
    xb = rng.integers(-127, 128, (4, 1, 28, 28)).astype(np.int8)
    lb = rng.integers(0, 10, 4).astype(np.int32)
    newW, rec = R.train_step(layers, W, S, xb, -3, lb)
    out.update({"lenet_x": xb, "lenet_labels": lb, "lenet_exp_in": np.int32(-3),
                "lenet_logits": rec["logits"], "lenet_exp_out": np.int32(rec["exp"][-1])})
    for i in range(len(layers)):
        out[f"lenet_w{i}"] = W[i]
        out[f"lenet_s{i}"] = np.int32(S[i])
        out[f"lenet_delta{i}"] = (newW[i].astype(np.int16) - W[i].astype(np.int16)).astype(np.int8)  # new - old
    path = os.path.join(HERE, "niti_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
