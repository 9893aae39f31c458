"""Parameter snapshots for the NITI step.

The reference snapshots the trainable Variables with `Variable::save(model->parameters(), path)`
at the end of each epoch (`EE/tools/train/source/demo/mnistTrain.cpp:375-376`); the NITI
weights are int8 OIHW tensors whose power-of-two scale `wscale` lives beside them as a
fixed int8 chosen at init (`EE/tools/train/source/nn/NN.cpp:1108-1134`, never updated by
NITI_SGD, `NITI_SGD.hpp:20-54`).  A snapshot here holds exactly that state:

    layer{i}.weight  int8 [C_out, C_in, KH, KW]  (OIHW, the reference's parameter layout)
    layer{i}.wscale  int8 [1]                    (the side-car the MNN file does not carry)

stored as safetensors (no code executes on load) with `arch` / `num_layers` metadata.  The
MNN flatbuffer container itself is not reproduced: `Variable::load` of that format needs
the MNN schema, which is outside the hot path; the tensors and their order are the same.
"""
from __future__ import annotations

import numpy as np
from safetensors.numpy import load_file, save_file

FORMAT = "niti-int8-params-v1"


def save_params(path: str, weights, wscales, arch: int, in_hw: int = 0) -> None:
    """Write per-layer int8 OIHW weights and their int8 wscale side-car."""
    if len(weights) != len(wscales):
        raise ValueError(f"{len(weights)} weights but {len(wscales)} wscales")
    tensors = {}
    for i, (w, s) in enumerate(zip(weights, wscales)):
        w = np.asarray(w)
        if w.dtype != np.int8 or w.ndim != 4:
            raise ValueError(f"layer {i}: expected int8 OIHW weight, got {w.dtype} {w.shape}")
        if not -128 <= int(s) <= 127:
            raise ValueError(f"layer {i}: wscale {s} does not fit int8")
        tensors[f"layer{i}.weight"] = np.ascontiguousarray(w)
        tensors[f"layer{i}.wscale"] = np.array([int(s)], np.int8)
    save_file(tensors, path, metadata={"format": FORMAT, "arch": str(int(arch)), "num_layers": str(len(weights)),
                                       "in_hw": str(int(in_hw))})


def load_params(path: str):
    """Read a snapshot back: (weights, wscales, arch).  Raises ValueError on a malformed file."""
    from safetensors import safe_open

    with safe_open(path, framework="numpy") as f:
        meta = f.metadata() or {}
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} snapshot (format={meta.get('format')!r})")
    try:
        n = int(meta["num_layers"])
        arch = int(meta["arch"])
    except (KeyError, ValueError, TypeError) as e:
        raise ValueError(f"{path}: malformed snapshot metadata ({e!r})") from None
    if n <= 0:
        raise ValueError(f"{path}: num_layers {n}")
    t = load_file(path)
    weights, wscales = [], []
    for i in range(n):
        w, s = t.get(f"layer{i}.weight"), t.get(f"layer{i}.wscale")
        if w is None or s is None or w.dtype != np.int8 or s.dtype != np.int8 or s.shape != (1,):
            raise ValueError(f"{path}: layer {i} missing or malformed")
        weights.append(w)
        wscales.append(int(s[0]))
    return weights, wscales, arch
