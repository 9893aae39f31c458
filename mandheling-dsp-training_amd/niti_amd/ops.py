"""Thin torch-facing wrappers over the C ABI (include/niti_hip.h).

torch supplies device memory and the stream; every byte of compute runs in
libniti_hip.so.  Section 1 (the MNN Execution-shaped drop-in) is exposed as
`NITIExecution`; section 2 (native split primitives) as plain functions.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L
from ._lib import check


def _stream(stream=None):
    if stream is not None:
        return stream
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def tensor(t: torch.Tensor, dims, fmt=L.FORMAT_NCHW) -> L.Tensor:
    """niti_tensor view of `t`; the view keeps `t` alive (the C side only holds the pointer)."""
    d = list(dims) + [1] * (4 - len(dims))
    v = L.Tensor(t.data_ptr(), (C.c_int * 4)(*d), fmt)
    v._keep = t
    return v


def convert(src: L.Tensor, dst: L.Tensor, stream=None) -> int:
    """CPUTensorConverter::convert (CPUTensorConvert.cpp:98-210): int8 NCHW / NHWC / NC4HW4."""
    s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
    return L.lib().niti_tensor_convert(C.byref(src), C.byref(dst), C.c_void_p(s))


def conv_common(kernel, stride=1, pad=0, dilate=1, pads=None, pad_mode=L.PAD_CAFFE, input_count=0,
                output_count=0, group=1) -> L.ConvCommon:
    kx, ky = (kernel, kernel) if isinstance(kernel, int) else kernel
    c = L.ConvCommon()
    c.kernel_x, c.kernel_y = kx, ky
    c.stride_x = c.stride_y = stride
    c.dilate_x = c.dilate_y = dilate
    c.pad_x = c.pad_y = pad
    if pads is not None:
        c.has_pads = 1
        c.pads = (C.c_int * 4)(*pads)
    c.pad_mode = pad_mode
    c.input_count, c.output_count, c.group = input_count, output_count, group
    return c


class NITIExecution:
    """One MNN Execution (Creator::onCreate + onResize + onExecute) for `op_type`."""

    def __init__(self, op_type: int, common: L.ConvCommon | None = None):
        self._lib = L.lib()
        h = C.c_void_p()
        check(self._lib.niti_create_execution(op_type, C.byref(common) if common is not None else None,
                                              C.byref(h)), f"create op {op_type}")
        self._h = h

    @staticmethod
    def _arr(ts):
        arr = (L.Tensor * len(ts))(*ts)
        return arr, len(ts)

    def resize(self, inputs, outputs):
        i, ni = self._arr(inputs)
        o, no = self._arr(outputs)
        return self._lib.niti_execution_resize(self._h, i, ni, o, no)

    def execute(self, inputs, outputs, stream=None):
        i, ni = self._arr(inputs)
        o, no = self._arr(outputs)
        return self._lib.niti_execution_execute(self._h, i, ni, o, no, _stream(stream))

    def status(self, stream=None):
        """The asynchronous path's ErrorCode (niti_execution_status): synchronizes `stream`, then
        NO_EXECUTION if a launch since the last check flagged invalid results."""
        return self._lib.niti_execution_status(self._h, _stream(stream))

    @property
    def workspace_bytes(self):
        return int(self._lib.niti_execution_workspace_bytes(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.niti_destroy_execution(h)
            self._h = None


# ------------------------------------------------------------------------------------ native
def geom(n, c_in, h, w, c_out, kh, kw=None, stride=1, pad=0, dilate=1, pads=None) -> L.Geom:
    kw = kh if kw is None else kw
    pt, pl, pb, pr = pads if pads is not None else (pad,) * 4
    g = L.Geom(n, c_in, h, w, c_out, kh, kw, stride, stride, pt, pl, pb, pr, dilate, dilate, 0, 0, 0, 0, 0)
    check(L.lib().niti_geom_finalize(C.byref(g)), "geometry")
    return g


def r16(x):
    return (x + 15) // 16 * 16


def nchw_to_nhwc16(x: torch.Tensor, stream=None):
    n, c, h, w = x.shape
    out = torch.empty((n, h, w, r16(c)), dtype=torch.int8, device=x.device)
    check(L.lib().niti_nchw_to_nhwc16(_ptr(x), n, c, h * w, r16(c), _ptr(out), _stream(stream)), "nchw->nhwc16")
    return out


def nchw_to_chwn16(x: torch.Tensor, stream=None):
    n, c, h, w = x.shape
    out = torch.empty((r16(c), h, w, r16(n)), dtype=torch.int8, device=x.device)
    check(L.lib().niti_nchw_to_chwn16(_ptr(x), n, c, h * w, r16(c), r16(n), _ptr(out), _stream(stream)),
          "nchw->chwn16")
    return out


def nhwc16_to_nchw(x16: torch.Tensor, c: int, stream=None):
    n, h, w, cp = x16.shape
    out = torch.empty((n, c, h, w), dtype=torch.int8, device=x16.device)
    check(L.lib().niti_nhwc16_to_nchw(_ptr(x16), n, c, h * w, cp, _ptr(out), _stream(stream)), "nhwc16->nchw")
    return out


def oihw_to_ohwi16(w: torch.Tensor, stream=None):
    co, ci, kh, kw = w.shape
    out = torch.empty((co, kh, kw, r16(ci)), dtype=torch.int8, device=w.device)
    check(L.lib().niti_oihw_to_ohwi16(_ptr(w), co, ci, kh * kw, r16(ci), _ptr(out), _stream(stream)), "oihw->ohwi16")
    return out


def ohwi16_to_ihwo16(w16: torch.Tensor, ci: int, stream=None):
    co, kh, kw, cip = w16.shape
    out = torch.empty((ci, kh, kw, r16(co)), dtype=torch.int8, device=w16.device)
    check(L.lib().niti_ohwi16_to_ihwo16(_ptr(w16), co, ci, kh * kw, cip, r16(co), _ptr(out), _stream(stream)),
          "ohwi16->ihwo16")
    return out


def ohwi16_to_oihw(w16: torch.Tensor, ci: int, stream=None):
    co, kh, kw, cip = w16.shape
    out = torch.empty((co, ci, kh, kw), dtype=torch.int8, device=w16.device)
    check(L.lib().niti_ohwi16_to_oihw(_ptr(w16), co, ci, kh * kw, cip, _ptr(out), _stream(stream)), "ohwi16->oihw")
    return out


def nhwc16_to_chwn16(x16: torch.Tensor, stream=None):
    n, h, w, cp = x16.shape
    out = torch.empty((cp, h, w, r16(n)), dtype=torch.int8, device=x16.device)
    check(L.lib().niti_nhwc16_to_chwn16(_ptr(x16), n, h * w, cp, r16(n), _ptr(out), _stream(stream)),
          "nhwc16->chwn16")
    return out


def conv_plan_set(g: L.Geom, op: int, plan=None):
    """Force the GEMM plan (bm, bn, splits, strategy) of a conv phase (op 0 / 1 / 2); None: default."""
    arr = (C.c_int * 4)(*plan) if plan is not None else None
    check(L.lib().niti_conv_plan_set(C.byref(g), op, arr), "conv_plan_set")


def conv_workspace(g: L.Geom, op: int, device="cuda"):
    n = C.c_size_t()
    check(L.lib().niti_conv_workspace_bytes(C.byref(g), op, C.byref(n)), "workspace")
    return torch.empty(max(int(n.value), 16), dtype=torch.uint8, device=device), int(n.value)


def conv_fwd_acc(g: L.Geom, x16, w16, amax, stream=None):
    acc = torch.empty((g.n * g.oh * g.ow, g.cop), dtype=torch.int32, device=x16.device)
    ws, nb = conv_workspace(g, 0, x16.device)
    check(L.lib().niti_conv_fwd_acc(C.byref(g), _ptr(x16), _ptr(w16), _ptr(acc), _ptr(amax), _ptr(ws), nb,
                                    _stream(stream)), "conv_fwd_acc")
    return acc


def conv_dgrad_acc(g: L.Geom, dy16, wt16, amax, stream=None):
    acc = torch.empty((g.n * g.h * g.w, g.cip), dtype=torch.int32, device=dy16.device)
    ws, nb = conv_workspace(g, 1, dy16.device)
    check(L.lib().niti_conv_dgrad_acc(C.byref(g), _ptr(dy16), _ptr(wt16), _ptr(acc), _ptr(amax), _ptr(ws), nb,
                                      _stream(stream)), "conv_dgrad_acc")
    return acc


def _conv_requant(op, g: L.Geom, a, b, amax, exp_in, wscale, exp_out, relu, relu_mask, between, stream):
    rows, ld = (g.n * g.oh * g.ow, g.cop) if op == 0 else (g.n * g.h * g.w, g.cip)
    acc = torch.empty((rows, ld), dtype=torch.int32, device=a.device)
    out = torch.empty((rows, ld), dtype=torch.int8, device=a.device)
    ws, nb = conv_workspace(g, op, a.device)
    lib = L.lib()
    p1, p2 = (lib.niti_conv_fwd_phase1, lib.niti_conv_fwd_phase2) if op == 0 else \
        (lib.niti_conv_dgrad_phase1, lib.niti_conv_dgrad_phase2)
    check(p1(C.byref(g), _ptr(a), _ptr(b), _ptr(acc), _ptr(amax), _ptr(ws), nb, _stream(stream)), "conv phase 1")
    if between is not None:  # e.g. the data-parallel MAX all-reduce of the range
        between(amax)
    check(p2(C.byref(g), _ptr(a), _ptr(b), _ptr(acc), _ptr(amax), _ptr(exp_in), _ptr(wscale), _ptr(exp_out),
             1 if relu else 0, _ptr(relu_mask), _ptr(out), nb, _stream(stream)), "conv phase 2")
    return out


ROWCONV_STATE_WORDS = 1216


def conv_rows_ok(g: L.Geom) -> bool:
    return bool(L.lib().niti_conv_rows_ok(C.byref(g)))


def nhwc16_to_c32(x16: torch.Tensor, c: int, stream=None, out=None):
    """NHWC16 [n][h][w][cp] -> C32 [n][ceil(c/32)][h][w][32] (the register-fed conv's activations)."""
    n, h, w, cp = x16.shape
    cb = (c + 31) // 32
    if out is None:
        out = torch.empty((n, cb, h, w, 32), dtype=torch.int8, device=x16.device)
    check(L.lib().niti_nhwc16_to_c32(_ptr(x16), n, h * w, cp, c, _ptr(out), _stream(stream)), "nhwc16->c32")
    return out


def weights_to_wf(w16: torch.Tensor, ci: int, transpose=False, stream=None, out=None):
    """OHWI16 [co][kh][kw][cip] (3x3) -> WF fragment-major weights (transpose: the input gradient's);
    out: a persistent buffer to rewrite in place."""
    co, cip = w16.shape[0], w16.shape[-1]
    ob, ib = ((ci if transpose else co) + 31) // 32, ((co if transpose else ci) + 31) // 32
    if out is None:
        out = torch.empty(ob * ib * 9 * 1024, dtype=torch.int8, device=w16.device)
    check(L.lib().niti_weights_to_wf(_ptr(w16), co, ci, cip, int(transpose), _ptr(out), _stream(stream)), "wf")
    return out


class RowConvState:
    """Grid-barrier state of the fused register-fed conv (mode 0) and its epoch counter; the
    speculative pair's (modes 3 / 4) hint slots live in it too."""

    def __init__(self, device="cuda"):
        self.state = torch.zeros(ROWCONV_STATE_WORDS, dtype=torch.int32, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.epoch = 0

    def spec_offset(self, dgrad=False):
        """Word offset in `state` of the speculative pair's forward / input-gradient slot."""
        return (L.lib().niti_rows_spec_slot(_ptr(self.state), 1 if dgrad else 0) - self.state.data_ptr()) // 4

    def spec_slot(self, dgrad=False):
        """(hint, guess used, misses) of the speculative pair's forward / input-gradient slot."""
        off = self.spec_offset(dgrad)
        return tuple(int(v) for v in self.state[off:off + 3].cpu())


ROWS_X_NHWC16 = 0x100  # NITI_ROWS_X_NHWC16


def rows_nhwc_ok(g: L.Geom, dgrad=False, preferred=False) -> bool:
    """Whether the row kernel takes its input as NHWC16 in place (row-segment maps, cip % 32 == 0);
    preferred: whether that is the faster choice too (64-channel inputs)."""
    return bool(L.lib().niti_conv_rows_nhwc_ok(C.byref(g), (1 if dgrad else 0) | (2 if preferred else 0)))


def conv_fwd_rows(g: L.Geom, xc32, wf, amax, mode=0, state: RowConvState | None = None, exp_in=None, wscale=None,
                  exp_out=None, relu=False, pool=False, next_c32=False, x_nhwc=False, stream=None, outs=None):
    """The register-fed forward (niti_conv_fwd_rows): (out NHWC16, pooled NHWC16 or None,
    next C32 or None).  mode 0 fused (state required), 1 range only, 2 requantise with amax;
    3 / 4 the speculative pair (state required; mode 4 takes mode 3's outputs as `outs`).
    x_nhwc: xc32 is the NHWC16 input itself (rows_nhwc_ok)."""
    dev = xc32.device
    if outs is not None:
        out, pout, nxt = outs
    else:
        out = None if mode == 1 else torch.empty((g.n, g.oh, g.ow, g.cop), dtype=torch.int8, device=dev)
        pout = torch.empty((g.n, g.oh // 2, g.ow // 2, g.cop), dtype=torch.int8, device=dev) if pool and mode != 1 else None
        nxt = None
        if next_c32 and mode != 1:
            hh, ww = (g.oh // 2, g.ow // 2) if pool else (g.oh, g.ow)
            nxt = torch.empty((g.n, g.cop // 32, hh, ww, 32), dtype=torch.int8, device=dev)
    st_ptr = err_ptr = None
    epoch = 0
    if mode == 0:
        # the launch's epoch; state.epoch advances only when the launch happened (a NOT_SUPPORT
        # return launches nothing, and a skipped epoch would reuse the previous launch's barrier words)
        epoch, st_ptr, err_ptr = state.epoch + 1, _ptr(state.state), _ptr(state.err)
    elif mode >= 3:
        st_ptr = _ptr(state.state)
    check(L.lib().niti_conv_fwd_rows(C.byref(g), _ptr(xc32), _ptr(wf), _ptr(exp_in), _ptr(wscale), _ptr(exp_out),
                                     1 if relu else 0, _ptr(out), _ptr(pout), _ptr(nxt),
                                     mode | (ROWS_X_NHWC16 if x_nhwc else 0), _ptr(amax), st_ptr,
                                     epoch, err_ptr, _stream(stream)), "conv_fwd_rows")
    if mode == 0:
        state.epoch = epoch
    return out, pout, nxt


def conv_dgrad_rows(g: L.Geom, dyc32, wft, amax, mode=0, state: RowConvState | None = None, relu_mask=None,
                    pool_x=None, pool_y=None, pool_relu=False, dx_c32=False, dx_p16=False, exp_in=None, wscale=None,
                    exp_out=None, x_nhwc=False, stream=None, outs=None):
    """The input gradient on the register-fed kernel (niti_conv_dgrad_rows) for the layer of
    geometry g: (dx NHWC16, dx C32 or None, dx P16 or None).  dx is [n][h][w][cip], or
    [n][2h][2w][cip] routed through the previous layer's 2x2 max pool when pool_x / pool_y are
    given.  Modes as conv_fwd_rows."""
    dev = dyc32.device
    hh, ww = (2 * g.h, 2 * g.w) if pool_x is not None else (g.h, g.w)
    if outs is not None:
        dx, nxt, p16 = outs
    else:
        dx = None if mode == 1 else torch.empty((g.n, hh, ww, g.cip), dtype=torch.int8, device=dev)
        nxt = torch.empty((g.n, g.cip // 32, hh, ww, 32), dtype=torch.int8, device=dev) if dx_c32 and mode != 1 else None
        p16 = torch.empty((g.n * hh * ww // 16, g.cip, 16), dtype=torch.int8, device=dev) if dx_p16 and mode != 1 else None
    st_ptr = err_ptr = None
    epoch = 0
    if mode == 0:
        # the launch's epoch; state.epoch advances only when the launch happened (a NOT_SUPPORT
        # return launches nothing, and a skipped epoch would reuse the previous launch's barrier words)
        epoch, st_ptr, err_ptr = state.epoch + 1, _ptr(state.state), _ptr(state.err)
    elif mode >= 3:
        st_ptr = _ptr(state.state)
    check(L.lib().niti_conv_dgrad_rows(C.byref(g), _ptr(dyc32), _ptr(wft), _ptr(relu_mask), _ptr(pool_x),
                                       _ptr(pool_y), 1 if pool_relu else 0, _ptr(dx), _ptr(nxt), _ptr(p16),
                                       _ptr(exp_in), _ptr(wscale), _ptr(exp_out),
                                       mode | (ROWS_X_NHWC16 if x_nhwc else 0),
                                       _ptr(amax), st_ptr, epoch, err_ptr, _stream(stream)), "conv_dgrad_rows")
    if mode == 0:
        state.epoch = epoch
    return dx, nxt, p16


def conv_fwd_requant(g: L.Geom, x16, w16, amax, exp_in=None, wscale=None, exp_out=None, relu=False,
                     relu_mask=None, between=None, stream=None):
    """The forward conv with its NITI requantisation in two phases (range, [between(amax)],
    requantise; small-K GEMMs recompute instead of storing int32): int8 [n*oh*ow][cop]."""
    return _conv_requant(0, g, x16, w16, amax, exp_in, wscale, exp_out, relu, relu_mask, between, stream)


def conv_dgrad_requant(g: L.Geom, dy16, wt16, amax, exp_in=None, wscale=None, exp_out=None, relu=False,
                       relu_mask=None, between=None, stream=None):
    """The input gradient with its requantisation in two phases: int8 [n*h*w][cip]."""
    return _conv_requant(1, g, dy16, wt16, amax, exp_in, wscale, exp_out, relu, relu_mask, between, stream)


def conv_plan(g: L.Geom, op: int, ws_bytes: int | None = None):
    """(bm, bn, splits, strategy) the conv GEMM `op` (0 fwd, 1 dgrad, 2 wgrad) runs with."""
    if ws_bytes is None:
        n = C.c_size_t(0)
        check(L.lib().niti_conv_workspace_bytes(C.byref(g), op, C.byref(n)), "workspace")
        ws_bytes = int(n.value)
    info = (C.c_int * 4)()
    check(L.lib().niti_conv_plan_info(C.byref(g), op, ws_bytes, info), "conv_plan_info")
    return tuple(info)


def wgrad_taps_ok(g: L.Geom) -> bool:
    """Whether the weight gradient of g runs on the tap-sharing kernel (wgrad_taps_kernel)."""
    return conv_plan(g, 2)[0] == 32


def conv_wgrad_acc(g: L.Geom, xT, dyT, amax=None, stream=None):
    acc = torch.empty((g.c_out, g.kh, g.kw, g.cip), dtype=torch.int32, device=xT.device)
    ws, nb = conv_workspace(g, 2, xT.device)
    check(L.lib().niti_conv_wgrad_acc(C.byref(g), _ptr(xT), _ptr(dyT), _ptr(acc), _ptr(amax), _ptr(ws), nb,
                                      _stream(stream)), "conv_wgrad_acc")
    return acc


def nhwc16_to_p16(x16: torch.Tensor, stream=None):
    """NHWC16 [N][H][W][Cp] -> P16 pixel blocks [N*H*W/16][Cp][16]."""
    cp = x16.shape[-1]
    px = x16.numel() // cp
    out = torch.empty((px // 16, cp, 16), dtype=torch.int8, device=x16.device)
    check(L.lib().niti_nhwc16_to_p16(_ptr(x16), px, cp, _ptr(out), _stream(stream)), "nhwc16->p16")
    return out


def wgrad_p16_workspace(g: L.Geom, splits: int = 0, device="cuda"):
    n = C.c_size_t()
    check(L.lib().niti_conv_wgrad_p16_workspace(C.byref(g), splits, C.byref(n)), "p16 workspace")
    return torch.zeros(max(int(n.value), 16), dtype=torch.uint8, device=device), int(n.value)


def conv_wgrad_p16_acc(g: L.Geom, xP, dyP, amax=None, splits: int = 0, ws=None, stream=None):
    """Weight gradient acc[co][kh][kw][cip] from P16 operands (niti_wgrad.hip); rows >= c_out stay 0."""
    acc = torch.zeros((g.c_out, g.kh, g.kw, g.cip), dtype=torch.int32, device=xP.device)
    if ws is None:
        ws, nb = wgrad_p16_workspace(g, splits, xP.device)
    else:
        nb = ws.numel()
    check(L.lib().niti_conv_wgrad_p16_acc(C.byref(g), _ptr(xP), _ptr(dyP), _ptr(acc), _ptr(amax), _ptr(ws), nb,
                                          splits, _stream(stream)), "conv_wgrad_p16_acc")
    return acc


def matmul_acc(B16, A16, ldc, amax=None, use_workspace=True, stream=None):
    m, k16 = B16.shape
    o = A16.shape[0]
    acc = torch.empty((m, ldc), dtype=torch.int32, device=B16.device)
    n = C.c_size_t(0)
    if use_workspace:
        check(L.lib().niti_matmul_workspace_bytes(m, ldc, k16, C.byref(n)), "workspace")
    ws = torch.empty(max(int(n.value), 16), dtype=torch.uint8, device=B16.device)
    check(L.lib().niti_matmul_acc(m, o, k16, _ptr(B16), k16, _ptr(A16), k16, _ptr(acc), ldc, _ptr(amax), _ptr(ws),
                                  int(n.value), _stream(stream)), "matmul_acc")
    return acc


MAX_WORDS = 2048  # NITI_MAX_WORDS: words per range-estimate buffer (64 slots, one per 128 B)


def new_range(device="cuda"):
    """A zeroed range-estimate buffer (NITI_MAX_WORDS uint32 words, held as int32)."""
    return torch.zeros(MAX_WORDS, dtype=torch.int32, device=device)


def range_max(amax) -> int:
    """max|acc| recorded in a range buffer: the max over its words."""
    return int(amax.view(-1, MAX_WORDS).max(dim=1).values.max().item())


def absmax(acc, amax, stream=None):
    check(L.lib().niti_absmax_i32(_ptr(acc), acc.numel(), _ptr(amax), _stream(stream)), "absmax")


def requant_act(acc, amax, exp_in=None, wscale=None, exp_out=None, relu=False, relu_mask=None, stream=None):
    rows, ldc = acc.shape
    out = torch.empty((rows, ldc), dtype=torch.int8, device=acc.device)
    check(L.lib().niti_requant_act(_ptr(acc), rows, ldc, _ptr(amax), _ptr(exp_in), _ptr(wscale), _ptr(exp_out),
                                   1 if relu else 0, _ptr(relu_mask), _ptr(out), _stream(stream)), "requant_act")
    return out


def requant_grad(acc, amax, rule=2, w_update=None, stream=None):
    g = torch.empty(acc.shape, dtype=torch.int8, device=acc.device)
    check(L.lib().niti_requant_grad(_ptr(acc), acc.numel(), _ptr(amax), rule, _ptr(g), _ptr(w_update),
                                    _stream(stream)), "requant_grad")
    return g


def sgd_update(acc, amax, w16, ci, rule=2, stream=None, wT=None, g=None, wf=None, wft=None):
    """acc [co][kh][kw][cip] int32, w16 OHWI16 int8 (updated in place) -> (wT IHWO16, g OHWI16);
    wT / g may be given (written in place, e.g. persistent buffers of a captured step)."""
    co, kh, kw, cip = acc.shape
    cop = r16(co)
    if wT is None:
        wT = torch.zeros((ci, kh, kw, cop), dtype=torch.int8, device=acc.device)
    if g is None:
        g = torch.empty(acc.shape, dtype=torch.int8, device=acc.device)
    assert wT.shape == (ci, kh, kw, cop) and g.shape == acc.shape
    if wf is not None or wft is not None:  # the row kernels' fragment-major copies in the same pass
        check(L.lib().niti_sgd_update_wf(_ptr(acc), _ptr(amax), rule, co, ci, kh * kw, cip, cop, _ptr(w16), _ptr(wT),
                                         _ptr(g), _ptr(wf), _ptr(wft), _stream(stream)), "sgd_update_wf")
        return wT, g
    check(L.lib().niti_sgd_update(_ptr(acc), _ptr(amax), rule, co, ci, kh * kw, cip, cop, _ptr(w16), _ptr(wT), _ptr(g),
                                  _stream(stream)), "sgd_update")
    return wT, g


def residual_add(a, ea, b, eb, amax, stream=None, ez=None):
    """Exponent-aligned int32 sum of two int8 tensors (niti_resnet.hip) -> (z int32, ez int8 [1])."""
    assert a.shape == b.shape and a.dtype == b.dtype == torch.int8
    z = torch.empty(a.shape, dtype=torch.int32, device=a.device)
    if ez is None:
        ez = torch.zeros(1, dtype=torch.int8, device=a.device)
    check(L.lib().niti_residual_add(_ptr(a), _ptr(ea), _ptr(b), _ptr(eb), a.numel(), _ptr(z), _ptr(ez), _ptr(amax),
                                    _stream(stream)), "residual_add")
    return z, ez


def residual_range(a, ea, b, eb, amax, stream=None):
    """max|z| of the residual add into amax, z not stored (the fused form's first pass)."""
    assert a.shape == b.shape and a.dtype == b.dtype == torch.int8
    check(L.lib().niti_residual_add(_ptr(a), _ptr(ea), _ptr(b), _ptr(eb), a.numel(), None, None, _ptr(amax),
                                    _stream(stream)), "residual_range")


def residual_requant(a, ea, b, eb, amax, ez=None, exp_out=None, relu=False, relu_mask=None, stream=None):
    """int8 requant(aligned a + b) with the range in amax; the residual and output exponents into ez /
    exp_out (device int8 [1], created when None) -> (out, ez, exp_out).  relu_mask (same shape):
    then the next op's relu gradient, out = relu_mask > 0 ? q : 0 (no relu)."""
    assert a.shape == b.shape and a.dtype == b.dtype == torch.int8
    out = torch.empty(a.shape, dtype=torch.int8, device=a.device)
    if ez is None:
        ez = torch.zeros(1, dtype=torch.int8, device=a.device)
    if exp_out is None:
        exp_out = torch.zeros(1, dtype=torch.int8, device=a.device)
    if relu_mask is not None:
        assert not relu and relu_mask.numel() == a.numel() and relu_mask.dtype == torch.int8
        check(L.lib().niti_residual_requant_relu_grad(_ptr(a), _ptr(ea), _ptr(b), _ptr(eb), a.numel(), _ptr(amax),
                                                      _ptr(ez), _ptr(exp_out), _ptr(relu_mask), _ptr(out),
                                                      _stream(stream)), "residual_requant_relu_grad")
        return out, ez, exp_out
    check(L.lib().niti_residual_requant(_ptr(a), _ptr(ea), _ptr(b), _ptr(eb), a.numel(), _ptr(amax), _ptr(ez),
                                        _ptr(exp_out), 1 if relu else 0, _ptr(out), _stream(stream)),
          "residual_requant")
    return out, ez, exp_out


def sum_pool(x16, amax, stream=None):
    """Global sum pool of x NHWC16 [n][h][w][cp] -> acc int32 [n][cp]."""
    n, h, w, cp = x16.shape
    acc = torch.empty((n, cp), dtype=torch.int32, device=x16.device)
    check(L.lib().niti_sum_pool(_ptr(x16), n, h * w, cp, _ptr(acc), _ptr(amax), _stream(stream)), "sum_pool")
    return acc


def im2col(g: L.Geom, x16, kp, stream=None, nchw=False):
    """im2col of a shallow NHWC16 input (c_in <= 4; nchw: an int8 NCHW input) -> xcol int8
    [n * oh * ow][kp], column (ky * kw + kx) * c_in + c (niti_im2col / niti_im2col_nchw)."""
    xcol = torch.empty((g.n * g.oh * g.ow, kp), dtype=torch.int8, device=x16.device)
    f = L.lib().niti_im2col_nchw if nchw else L.lib().niti_im2col
    check(f(C.byref(g), _ptr(x16), kp, _ptr(xcol), _stream(stream)), "im2col")
    return xcol


def sum_pool_grad(dy16, h, w, stream=None):
    """dx [n][h][w][cp] = dy [n][cp] at every pixel."""
    n, cp = dy16.shape
    dx = torch.empty((n, h, w, cp), dtype=torch.int8, device=dy16.device)
    check(L.lib().niti_sum_pool_grad(_ptr(dy16), n, h * w, cp, _ptr(dx), _stream(stream)), "sum_pool_grad")
    return dx


def maxpool(x16, k=2, s=2, p=0, stream=None):
    n, h, w, cp = x16.shape
    oh = (h + 2 * p - min(k, h)) // s + 1
    ow = (w + 2 * p - min(k, w)) // s + 1
    y = torch.empty((n, oh, ow, cp), dtype=torch.int8, device=x16.device)
    check(L.lib().niti_maxpool(_ptr(x16), n, h, w, cp, k, s, p, _ptr(y), oh, ow, _stream(stream)), "maxpool")
    return y


def maxpool_grad(x16, y16, dy16, k=2, s=2, p=0, relu=False, stream=None, two_pass=None):
    """dx of the max pool (first max wins), relu mask optional.  Overlapping windows (k > s) run the
    two-pass form over a workspace (niti_maxpool_grad_ws) unless two_pass=False."""
    n, h, w, cp = x16.shape
    oh, ow = y16.shape[1], y16.shape[2]
    dx = torch.empty_like(x16)
    if two_pass is None:
        two_pass = k > s
    if two_pass:
        ws = torch.empty_like(y16)
        check(L.lib().niti_maxpool_grad_ws(_ptr(x16), _ptr(y16), _ptr(dy16), n, h, w, cp, k, s, p, oh, ow,
                                           1 if relu else 0, _ptr(ws), _ptr(dx), _stream(stream)), "maxpool_grad_ws")
    else:
        check(L.lib().niti_maxpool_grad(_ptr(x16), _ptr(y16), _ptr(dy16), n, h, w, cp, k, s, p, oh, ow,
                                        1 if relu else 0, _ptr(dx), _stream(stream)), "maxpool_grad")
    return dx


def relu_grad(x, dy, stream=None):
    out = torch.empty_like(x)
    check(L.lib().niti_relu_grad(_ptr(x), _ptr(dy), x.numel(), _ptr(out), _stream(stream)), "relu_grad")
    return out


def loss_grad(logits, classes, ascale_dev, labels, stream=None):
    b, ld = logits.shape
    out = torch.empty_like(logits)
    check(L.lib().niti_loss_grad(_ptr(logits), b, classes, ld, _ptr(ascale_dev), _ptr(labels), _ptr(out),
                                 _stream(stream)), "loss_grad")
    return out


def image_stats(images: torch.Tensor, stream=None):
    """{sum p, sum p^2, max p, 255 - min p} (int64 device [4], u64 values) of a uint8 image batch
    (the input quantiser's statistics, MnistUtils.cpp:83-93; SUM / MAX over DP ranks)."""
    assert images.dtype == torch.uint8 and images.is_contiguous()
    stats = torch.zeros(4, dtype=torch.int64, device=images.device)  # u64 values < 2^63
    check(L.lib().niti_image_stats(_ptr(images), images.numel(), _ptr(stats), _stream(stream)), "image_stats")
    return stats


def image_quantize(images: torch.Tensor, stats: torch.Tensor, count: int | None = None, stream=None):
    """x int8 NCHW and its exponent (device int8 [1]) from uint8 images [n][c][h][w] and the
    statistics over `count` pixels (default: this batch's)."""
    assert images.dtype == torch.uint8 and images.is_contiguous() and images.dim() == 4
    n, c, h, w = images.shape
    out = torch.empty(images.shape, dtype=torch.int8, device=images.device)
    ascale = torch.zeros(1, dtype=torch.int8, device=images.device)
    check(L.lib().niti_image_quantize(_ptr(images), n, c, h * w, _ptr(stats), int(count or images.numel()),
                                      _ptr(out), _ptr(ascale), _stream(stream)), "image_quantize")
    return out, ascale


def image_quantize_nhwc16(images: torch.Tensor, stats: torch.Tensor, count: int | None = None, stream=None):
    """image_quantize with x written as NHWC16 [n][h][w][16 * ceil(c / 16)] (a conv input)."""
    assert images.dtype == torch.uint8 and images.is_contiguous() and images.dim() == 4
    n, c, h, w = images.shape
    out = torch.empty((n, h, w, r16(c)), dtype=torch.int8, device=images.device)
    ascale = torch.zeros(1, dtype=torch.int8, device=images.device)
    check(L.lib().niti_image_quantize_nhwc16(_ptr(images), n, c, h * w, r16(c), _ptr(stats),
                                             int(count or images.numel()), _ptr(out), _ptr(ascale), _stream(stream)),
          "image_quantize_nhwc16")
    return out, ascale
