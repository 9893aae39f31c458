"""ctypes/numpy front end of the CPU oracle (oracle/niti_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  The product path never imports it.

Parity unpinned: the reference ships no fixture or test for any NITI op and
running it was denied; see niti_oracle.h for how the
restatement is anchored instead.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libniti_oracle.so")
_lib = None

ACC_EXACT = 0
ACC_F32_SEQ = 1


class Geom(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "n", "c_in", "h", "w", "c_out", "kh", "kw", "stride_h", "stride_w",
        "pad_t", "pad_l", "pad_b", "pad_r", "dilate_h", "dilate_w", "oh", "ow")]


class Stats(C.Structure):
    _fields_ = [("guard", C.c_int64), ("overflow", C.c_int64)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _declare(_lib)
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _declare(L):
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    gp = C.POINTER(Geom)
    sig = {
        "niti_ref_int8_clip": (i32, [i32]),
        "niti_ref_sign": (i32, [i32]),
        "niti_ref_pow2": (i32, [i32]),
        "niti_ref_range_estimate": (i32, [vp, i64]),
        "niti_ref_range_estimate_libm": (i32, [vp, i64]),
        "niti_ref_psto1": (i32, [i32, i32]),
        "niti_ref_psto_shift": (None, [vp, i32, vp, i64]),
        "niti_ref_requant_fwd": (i32, [vp, i64, vp]),
        "niti_ref_requant_wgrad": (i32, [vp, i64, vp]),
        "niti_ref_requant_matmul": (i32, [vp, i64, vp]),
        "niti_ref_geom_finalize": (C.c_int, [gp]),
        "niti_ref_conv_fwd_acc": (None, [gp, vp, vp, vp, vp]),
        "niti_ref_conv_wgrad_acc": (None, [gp, vp, vp, vp, vp]),
        "niti_ref_conv_dgrad_acc": (None, [gp, vp, vp, vp, vp]),
        "niti_ref_matmul_acc": (None, [C.c_int, C.c_int, C.c_int, vp, vp, vp, vp]),
        "niti_ref_nchw_to_c4": (None, [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]),
        "niti_ref_c4_to_nchw": (None, [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]),
        "niti_ref_c4_to_nchw_i32": (None, [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]),
        "niti_ref_mnn_conv_core": (None, [gp, vp, vp, vp, C.c_int, C.c_int]),
        "niti_ref_mnn_conv_fwd": (i32, [gp, vp, vp, i32, i32, vp, C.c_int, C.c_int]),
        "niti_ref_mnn_conv_wgrad": (i32, [gp, vp, vp, vp, vp, C.c_int, C.c_int]),
        "niti_ref_mnn_conv_dgrad": (i32, [gp, vp, vp, vp, vp, C.c_int, C.c_int]),
        "niti_ref_relu": (None, [vp, i64, vp]),
        "niti_ref_relu_grad": (None, [vp, vp, i64, vp]),
        "niti_ref_maxpool": (None, [vp] + [C.c_int] * 7 + [vp, C.c_int, C.c_int]),
        "niti_ref_maxpool_grad": (None, [vp, vp, vp] + [C.c_int] * 9 + [vp]),
        "niti_ref_loss_grad": (None, [vp, C.c_int, C.c_int, i32, vp, C.c_int, vp]),
        "niti_ref_sgd_update": (None, [vp, vp, i64]),
        "niti_ref_quantize_input": (i32, [vp, i64, i64, vp]),
        "niti_ref_quantize_input_lanes": (i32, [vp, i64, i64, C.c_int, vp]),
        "niti_ref_sample_stats": (None, [gp, C.c_int, vp, vp, vp, i64, vp, vp, vp]),
        "niti_ref_image_stats": (None, [vp, i64, vp]),
        "niti_ref_set_threads": (None, [C.c_int]),
        "niti_ref_image_quantize": (i32, [vp, i64, vp, i64, i64, vp]),
        "niti_ref_layer_step": (C.c_int, [gp, vp, vp, vp, vp, vp, vp, C.c_int, C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


# ----------------------------------------------------------------------------- geometry
def geom(n, c_in, h, w, c_out, kh, kw=None, stride=1, pad=0, dilate=1, pads=None) -> Geom:
    kw = kh if kw is None else kw
    if pads is None:
        pads = (pad, pad, pad, pad)  # t, l, b, r
    g = Geom(n, c_in, h, w, c_out, kh, kw, stride, stride, pads[0], pads[1], pads[2], pads[3],
             dilate, dilate, 0, 0)
    if lib().niti_ref_geom_finalize(C.byref(g)) != 0:
        raise ValueError("invalid convolution geometry")
    return g


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


# ----------------------------------------------------------------------------- scalars
def psto(a, shift):
    a = _c(a, np.int32)
    out = np.empty_like(a)
    lib().niti_ref_psto_shift(_p(a), int(shift), _p(out), a.size)
    return out


def range_estimate(a):
    a = _c(a, np.int32)
    return int(lib().niti_ref_range_estimate(_p(a), a.size))


def range_estimate_libm(a):
    a = _c(a, np.int32)
    return int(lib().niti_ref_range_estimate_libm(_p(a), a.size))


def requant_fwd(acc):
    acc = _c(acc, np.int32)
    out = np.empty(acc.shape, np.int8)
    inc = lib().niti_ref_requant_fwd(_p(acc), acc.size, _p(out))
    return out, int(inc)


def requant_wgrad(acc):
    acc = _c(acc, np.int32)
    out = np.empty(acc.shape, np.int8)
    bw = lib().niti_ref_requant_wgrad(_p(acc), acc.size, _p(out))
    return out, int(bw)


def requant_matmul(acc):
    acc = _c(acc, np.int32)
    out = np.empty(acc.shape, np.int8)
    bw = lib().niti_ref_requant_matmul(_p(acc), acc.size, _p(out))
    return out, int(bw)


# ----------------------------------------------------------------------------- naive exact
def set_threads(n: int):
    """pthreads of the naive restatement (results independent of it)."""
    lib().niti_ref_set_threads(int(n))


def conv_fwd_acc(g: Geom, x, w):
    x, w = _c(x, np.int8), _c(w, np.int8)
    acc = np.empty((g.n, g.c_out, g.oh, g.ow), np.int32)
    st = Stats()
    lib().niti_ref_conv_fwd_acc(C.byref(g), _p(x), _p(w), _p(acc), C.byref(st))
    return acc, st


def conv_wgrad_acc(g: Geom, x, dy):
    x, dy = _c(x, np.int8), _c(dy, np.int8)
    acc = np.empty((g.c_out, g.c_in, g.kh, g.kw), np.int32)
    st = Stats()
    lib().niti_ref_conv_wgrad_acc(C.byref(g), _p(x), _p(dy), _p(acc), C.byref(st))
    return acc, st


def conv_dgrad_acc(g: Geom, dy, w):
    dy, w = _c(dy, np.int8), _c(w, np.int8)
    acc = np.empty((g.n, g.c_in, g.h, g.w), np.int32)
    st = Stats()
    lib().niti_ref_conv_dgrad_acc(C.byref(g), _p(dy), _p(w), _p(acc), C.byref(st))
    return acc, st


def matmul_acc(B, A):
    """C[m][o] = sum_k B[m][k] * A[o][k]  (NITI_Matmul_Int8)."""
    B, A = _c(B, np.int8), _c(A, np.int8)
    m, k = B.shape
    o = A.shape[0]
    acc = np.empty((m, o), np.int32)
    st = Stats()
    lib().niti_ref_matmul_acc(m, o, k, _p(B), _p(A), _p(acc), C.byref(st))
    return acc, st


# ----------------------------------------------------------------------------- full ops (naive)
def conv_fwd(g, x, w, exp_in=-7, wscale=-7):
    acc, st = conv_fwd_acc(g, x, w)
    y, inc = requant_fwd(acc)
    return y, int(np.int8(np.int32(exp_in + wscale + inc).astype(np.int8))), acc, st


def conv_wgrad(g, x, dy):
    acc, st = conv_wgrad_acc(g, x, dy)
    dw, bw = requant_wgrad(acc)
    return dw, bw, acc, st


def conv_dgrad(g, dy, w):
    acc, st = conv_dgrad_acc(g, dy, w)
    dx, inc = requant_fwd(acc)
    return dx, inc, acc, st


def matmul(B, A):
    """NITI_Matmul_Int8: returns dw [o][m] (the geometry's transpose back), bw, acc [m][o]."""
    acc, st = matmul_acc(B, A)
    q, bw = requant_matmul(acc)
    return np.ascontiguousarray(q.T), bw, acc, st


# ----------------------------------------------------------------------------- C4 / structured
def nchw_to_c4(x):
    x = _c(x, np.int8)
    n, c, h, w = x.shape
    out = np.empty(((c + 3) // 4, n, h, w, 4), np.int8)
    lib().niti_ref_nchw_to_c4(_p(x), n, c, h, w, _p(out))
    return out


def c4_to_nchw(x4, c):
    x4 = _c(x4, np.int8)
    cq, n, h, w, _ = x4.shape
    out = np.empty((n, c, h, w), np.int8)
    lib().niti_ref_c4_to_nchw(_p(x4), n, c, h, w, _p(out))
    return out


def mnn_conv_fwd(g, x_nchw, w, exp_in=-7, wscale=-7, acc_mode=ACC_EXACT, threads=1):
    x4 = nchw_to_c4(x_nchw)
    w = _c(w, np.int8)
    y4 = np.empty(((g.c_out + 3) // 4, g.n, g.oh, g.ow, 4), np.int8)
    e = lib().niti_ref_mnn_conv_fwd(C.byref(g), _p(x4), _p(w), exp_in, wscale, _p(y4), acc_mode, threads)
    return c4_to_nchw(y4, g.c_out), int(e), y4


def mnn_conv_wgrad(g, x, dy, acc_mode=ACC_EXACT, threads=1):
    x, dy = _c(x, np.int8), _c(dy, np.int8)
    dw = np.empty((g.c_out, g.c_in, g.kh, g.kw), np.int8)
    acc = np.empty((g.c_out, g.c_in, g.kh, g.kw), np.int32)
    bw = lib().niti_ref_mnn_conv_wgrad(C.byref(g), _p(x), _p(dy), _p(dw), _p(acc), acc_mode, threads)
    return dw, int(bw), acc


def mnn_conv_dgrad(g, dy, w, acc_mode=ACC_EXACT, threads=1):
    dy, w = _c(dy, np.int8), _c(w, np.int8)
    dx = np.empty((g.n, g.c_in, g.h, g.w), np.int8)
    acc = np.empty((g.n, g.c_in, g.h, g.w), np.int32)
    inc = lib().niti_ref_mnn_conv_dgrad(C.byref(g), _p(dy), _p(w), _p(dx), _p(acc), acc_mode, threads)
    return dx, int(inc), acc


# ----------------------------------------------------------------------------- rest of step
def relu(x):
    x = _c(x, np.int8)
    y = np.empty_like(x)
    lib().niti_ref_relu(_p(x), x.size, _p(y))
    return y


def relu_grad(x, dy):
    x, dy = _c(x, np.int8), _c(dy, np.int8)
    out = np.empty_like(x)
    lib().niti_ref_relu_grad(_p(x), _p(dy), x.size, _p(out))
    return out


def pool_out(h, k, s, p):
    return (h + 2 * p - min(k, h)) // s + 1


def maxpool(x, k=2, s=2, p=0):
    x = _c(x, np.int8)
    n, c, h, w = x.shape
    oh, ow = pool_out(h, k, s, p), pool_out(w, k, s, p)
    y = np.empty((n, c, oh, ow), np.int8)
    lib().niti_ref_maxpool(_p(x), n, c, h, w, k, s, p, _p(y), oh, ow)
    return y


def maxpool_grad(x, y, dy, k=2, s=2, p=0):
    x, y, dy = _c(x, np.int8), _c(y, np.int8), _c(dy, np.int8)
    n, c, h, w = x.shape
    oh, ow = y.shape[2], y.shape[3]
    dx = np.empty_like(x)
    lib().niti_ref_maxpool_grad(_p(x), _p(y), _p(dy), n, c, h, w, k, s, p, oh, ow, _p(dx))
    return dx


def maxpool_grad_ref806(x, y, dy, out, kx=2, ky=2, sx=2, sy=2):
    """NITI_DSP_MAXPOOLGRAD_REF_Int8 (NITI_DSPMaxPoolGradRef_Int8.cpp:17-80), its loops restated
    in Python (small sizes only).  x and out are raw NHWC [N][H][W][C] buffers read as
    [ih = N][iw = H][ib * ic] (:23-28); y / dy are flat buffers indexed at
    (offset * bc) // kx // ky (:54-55).  out is updated in place and returned: bytes no window
    visits keep their value (the op never zeroes its output)."""
    x = np.ascontiguousarray(x).reshape(-1)
    y = np.ascontiguousarray(y).reshape(-1)
    dy = np.ascontiguousarray(dy).reshape(-1)
    shp = out.shape
    o = np.ascontiguousarray(out).reshape(-1).copy()
    ih, iw, bc = shp[0], shp[1], shp[2] * shp[3]
    for i in range(0, ih, sx):                       # :36
        for j in range(0, iw, sy):                   # :37
            offset = i * iw + j                      # :39
            for m in range(bc // 128):               # :43
                base = offset * bc // kx // ky + m * 128
                yb, db = y[base:base + 128], dy[base:base + 128]
                finish = np.zeros(128, bool)
                for a in range(ky):                  # :59
                    for b in range(kx):              # :61
                        ko = (offset + a * iw + b) * bc + m * 128
                        same = x[ko:ko + 128] == yb
                        take = same & ~finish
                        o[ko:ko + 128] = np.where(take, db, 0)
                        finish |= take
    return o.reshape(shp)


def loss_grad(logits, ascale, onehot):
    logits = _c(logits, np.int8)
    onehot = _c(onehot, np.int32)
    b, classes = logits.shape
    out = np.empty_like(logits)
    lib().niti_ref_loss_grad(_p(logits), b, classes, int(ascale), _p(onehot), onehot.shape[1], _p(out))
    return out


def sgd_update(w, g):
    w = _c(w, np.int8).copy()
    g = _c(g, np.int8)
    lib().niti_ref_sgd_update(_p(w), _p(g), w.size)
    return w


MNIST_VAR_PIXELS = 28 * 28  # MnistUtils.cpp:86 divides the variance by batchSize * 28 * 28, literally


def quantize_input(x, lanes=1):
    """x float [n][...]: the float restatement of MnistUtils.cpp:83-93, its two full reductions
    summed in `lanes` interleaved partials (1 = the C source's sequential loop; 4 / 8 / 16 = the
    vector orders -ffast-math lets the compiler choose, niti_ref_quantize_input_lanes)."""
    x = _c(x, np.float32)
    out = np.empty(x.shape, np.int8)
    a = lib().niti_ref_quantize_input_lanes(_p(x), x.size, x.shape[0] * MNIST_VAR_PIXELS, int(lanes), _p(out))
    return out, int(a)


def sample_stats(g, kind, a, b, idx):
    """Per sampled output (flat indices idx): exact sum, sum|p|, reference-order float32 sum as int32
    (niti_ref_sample_stats; kind 0 forward (x, w), 1 weight gradient (x, dy), 2 stride-1 input
    gradient (dy, w); NCHW / OIHW int8)."""
    a, b = _c(a, np.int8), _c(b, np.int8)
    idx = np.ascontiguousarray(idx, np.int64)
    ex = np.empty(idx.size, np.int64)
    sa = np.empty(idx.size, np.uint64)
    f = np.empty(idx.size, np.int32)
    lib().niti_ref_sample_stats(C.byref(g), int(kind), _p(a), _p(b), _p(idx), idx.size, _p(ex), _p(sa), _p(f))
    return ex, sa, f


def image_stats(images):
    """{S1, S2, xmax, 255 - xmin} (uint64) of uint8 pixels (niti_ref_image_stats)."""
    img = _c(images, np.uint8)
    st = np.zeros(4, np.uint64)
    lib().niti_ref_image_stats(_p(img), img.size, _p(st))
    return st


def quantize_images(images, stats=None, count=None):
    """MnistUtils.cpp:83-93 over exact integer statistics: (x int8 same shape, ascale).  stats /
    count default to this batch's own (data-parallel ranks pass the global ones).  The variance
    divisor is the reference's literal batchSize * 28 * 28 for the global batch (count / image
    pixels images), whatever the image size."""
    img = _c(images, np.uint8)
    st = image_stats(img) if stats is None else np.ascontiguousarray(stats, np.uint64)
    out = np.empty(img.shape, np.int8)
    count = int(count or img.size)
    per_image = int(np.prod(img.shape[1:]))
    var_count = (count // per_image) * MNIST_VAR_PIXELS
    a = lib().niti_ref_image_quantize(_p(img), img.size, _p(st), count, var_count, _p(out))
    return out, int(a)


def layer_step(g, x, w, dy, threads=1, with_dgrad=True):
    x, w, dy = _c(x, np.int8), _c(w, np.int8), _c(dy, np.int8)
    y4 = np.empty(((g.c_out + 3) // 4, g.n, g.oh, g.ow, 4), np.int8)
    dw = np.empty((g.c_out, g.c_in, g.kh, g.kw), np.int8)
    dx = np.empty((g.n, g.c_in, g.h, g.w), np.int8)
    lib().niti_ref_layer_step(C.byref(g), _p(x), _p(w), _p(dy), _p(y4), _p(dw), _p(dx), threads,
                              1 if with_dgrad else 0)
    return y4, dw, dx


# ----------------------------------------------------------------------------- synthetic inputs
def synth_x(rng, shape, zero_frac=0.5):
    """Parity set: post-ReLU-like x ~ U{0..127} with 50 % zeros."""
    x = rng.integers(0, 128, size=shape, dtype=np.int16)
    x[rng.random(shape) < zero_frac] = 0
    return x.astype(np.int8)


def synth_dy(rng, shape, zero_frac=0.7):
    d = rng.integers(-127, 128, size=shape, dtype=np.int16)
    d[rng.random(shape) < zero_frac] = 0
    return d.astype(np.int8)


def synth_w(rng, shape):
    """niti_normal_int8 (nn/Distributions.cpp:26-51) with a fixed seed instead of gettimeofday."""
    fan_in = int(np.prod(shape[1:]))
    fan_out = shape[0] * int(np.prod(shape[2:]))
    std = np.sqrt(2.0 / (fan_in + fan_out))
    t = rng.normal(0.0, std, size=shape).astype(np.float32)
    rng_ = float(np.abs(t).max())
    wscale = int(np.ceil(np.log2(rng_))) - 7
    return np.round(t / rng_ * 127).astype(np.int8), wscale


def synth_stress(rng, shape):
    """Stress set: U{-127..127} everywhere (exercises the 2^24 guard)."""
    return rng.integers(-127, 128, size=shape, dtype=np.int16).astype(np.int8)
