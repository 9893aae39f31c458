"""MNN's tensor fixture text format and its layouts on the host.

The reference's tools exchange tensors as whitespace-separated decimal values in the tensor's
element order: `createTensor` reads `elementSize()` values with `stream >> double`
(execution-engine/tools/cpp/testModel.cpp:43-56), the express demo reads `input_0.txt` the same way
and writes `output.txt` one value per line (demo/exec/expressDemo.cpp:84-101), and `checkFile`
compares two such files value by value against a tolerance (tools/cpp/checkFile.cpp:32-50).  The
element order is the tensor's own layout: the reference's fixtures hold NHWC images
(resource/model/MobileNet/qnt_input.txt: 224 x 224 lines of 3 values) and MNN C4 tensors
(resource/model/SqueezeNet/input.txt: [C/4][N][H][W][4] with the pad lane 0).

On the device the same layouts go through niti_tensor_convert (C4 / NCHW / NHWC <-> NHWC16, the
Execution boundary); these host helpers read and write the files and restate the C4 order so a
fixture can be fed to either.
"""
from __future__ import annotations

import math

import numpy as np


def read_txt(path: str, count: int | None = None, dtype=np.float64) -> np.ndarray:
    """Values of a fixture file in file order, as `stream >> v` reads them: whitespace-separated
    decimals, stopping at the first token that is not a number (or after `count` values).  With
    `count`, a file holding fewer values raises ValueError (createTensor would leave the rest
    unset)."""
    vals = []
    with open(path) as f:
        for line in f:
            for tok in line.split():
                try:
                    v = float(tok)
                except ValueError:
                    return _finish(vals, count, dtype, path)
                vals.append(v)
                if count is not None and len(vals) == count:
                    return _finish(vals, count, dtype, path)
    return _finish(vals, count, dtype, path)


def _finish(vals, count, dtype, path):
    if count is not None and len(vals) < count:
        raise ValueError(f"{path}: {len(vals)} values, want {count}")
    a = np.asarray(vals, dtype=np.float64)
    if np.issubdtype(np.dtype(dtype), np.integer):
        info = np.iinfo(dtype)
        if a.size and (a.min() < info.min or a.max() > info.max or not np.array_equal(a, np.round(a))):
            raise ValueError(f"{path}: values do not fit {np.dtype(dtype).name}")
    return a.astype(dtype)


def write_txt(path: str, a) -> None:
    """One value per line in the array's element order (expressDemo's output.txt)."""
    a = np.asarray(a).reshape(-1)
    with open(path, "w") as f:
        if np.issubdtype(a.dtype, np.integer):
            f.writelines(f"{int(v)}\n" for v in a)
        else:
            f.writelines(f"{float(v):g}\n" for v in a)


def check_file(path1: str, path2: str, tolerance: float = 0.001):
    """checkFile.cpp: walk both files in step while the first has values; returns the
    (position, v1, v2) pairs that differ by more than `tolerance`."""
    a = read_txt(path1)
    b = read_txt(path2)
    bad = []
    for pos, v1 in enumerate(a):
        if pos >= b.size:
            break
        if abs(v1 - b[pos]) > tolerance:
            bad.append((pos, float(v1), float(b[pos])))
    return bad


def c4_to_nchw(flat, n: int, c: int, h: int, w: int) -> np.ndarray:
    """MNN NC4HW4 element order [ceil(C/4)][N][H][W][4] (CPUTensorConvert.cpp:98-178) -> NCHW."""
    c4 = math.ceil(c / 4)
    t = np.asarray(flat).reshape(c4, n, h, w, 4)
    return t.transpose(1, 0, 4, 2, 3).reshape(n, c4 * 4, h, w)[:, :c].copy()


def nchw_to_c4(x) -> np.ndarray:
    """NCHW -> the NC4HW4 element order, pad lanes zero."""
    x = np.asarray(x)
    n, c, h, w = x.shape
    c4 = math.ceil(c / 4)
    p = np.zeros((n, c4 * 4, h, w), dtype=x.dtype)
    p[:, :c] = x
    return p.reshape(n, c4, 4, h, w).transpose(1, 0, 3, 4, 2).copy()


def nhwc_to_nchw(flat, n: int, c: int, h: int, w: int) -> np.ndarray:
    return np.asarray(flat).reshape(n, h, w, c).transpose(0, 3, 1, 2).copy()
