"""ResNet-18 NITI int8 training step on the HIP ops (BASELINE.json config 5).

The reference has no ResNet NITI model and its NITI_Eltwise_Int8 is an empty stub
(execution-engine/source/backend/cpu/NITI_Eltwise_Int8.cpp:20-28); the residual and pooling rules
are this library's (csrc/niti_resnet.hip, restated in oracle/niti_resnet_ref.py).  Every op runs on
the device through the C ABI (niti_amd.ops): the convs on the int8 MFMA GEMMs with their range
estimate and requantisation, the 7x7 / 2 stem, the 3x3 / 2 max pool, the 1x1 / 2 projections, the
exponent-aligned residual adds, the global sum pool, the 1000-way head and NITI_SGD.  Activations
stay in HBM as NHWC16 and every exponent stays a device int8 scalar: a step never synchronises the
host.  Data parallel (comm = niti_amd.dp.TorchComm / ThreadComm): the exact protocol of
SURVEY.md §8(e) -- every range estimate MAX-reduced over the ranks before its requantisation, every
int32 weight gradient SUM-reduced before its range and NITI_SGD, the input quantiser's statistics
SUM / MAX-reduced -- so each rank is bit-identical to one device running the global batch.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import ops
from ._lib import NitiError


def resnet18_convs(hw=224, classes=1000):
    """The 21 parameter layers in parameter order (conv1; per basic block conv a, conv b and the
    1x1 / 2 projection of the first block of stages 2-4; the fc head as a 1x1 conv)."""
    L = [dict(name="conv1", ci=3, co=64, k=7, stride=2, pad=3, h=hw)]
    h = (hw + 6 - 7) // 2 + 1
    h = (h + 2 - 3) // 2 + 1
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
    for l in L:
        l["oh"] = (l["h"] + 2 * l["pad"] - l["k"]) // l["stride"] + 1
    return L


def _blocks(convs):
    out, i = [], 1
    while i < len(convs) - 1:
        proj = i + 2 if convs[i + 2]["name"].endswith("proj") else None
        out.append((i, i + 1, proj))
        i += 3 if proj else 2
    return out


class ResNet18:
    STEM_KP = 160  # the stem's im2col columns: 7 * 7 * 3 = 147, padded to whole 32-byte chunks

    def __init__(self, batch: int, in_hw: int = 224, classes: int = 1000, device="cuda", comm=None):
        """batch: images per rank; comm: data-parallel collectives (niti_amd.dp), None for one device."""
        if in_hw % 16 or in_hw < 32:
            raise ValueError("in_hw must be a multiple of 16, at least 32")
        self.batch, self.in_hw, self.classes, self.dev = batch, in_hw, classes, device
        self.comm = comm
        self.convs = resnet18_convs(in_hw, classes)
        self.blocks = _blocks(self.convs)
        n = batch
        self.geoms = [ops.geom(n, l["ci"], l["h"], l["h"], l["co"], l["k"], stride=l["stride"], pad=l["pad"])
                      for l in self.convs]
        # the 7x7 / 2 stem runs as a 1x1 conv over its im2col (STEM_KP columns, k = (ky * 7 + kx) * 3
        # + c; ops.im2col): the implicit-GEMM forms gather 3 useful bytes of every 16-byte input pixel
        # per tap and ran the stem's forward + weight gradient at ~2 % of peak.  Its weight is kept
        # in that column order ([64][1][1][STEM_KP]); get_weight / set_weight / taps map OIHW.
        s0 = self.convs[0]
        self.stem_geom = self.geoms[0]
        self.geoms[0] = ops.geom(n, self.STEM_KP, s0["oh"], s0["oh"], s0["co"], 1, stride=1, pad=0)
        self._xcol = None
        self.w16 = [None] * len(self.convs)
        self.wT = [None] * len(self.convs)
        self.wscale = [None] * len(self.convs)
        self.ws_dev = [None] * len(self.convs)
        # stride-1 3x3 layers over 56 / 28 / 14-px maps run on the register-fed row-segment kernels
        # (csrc/niti_rowconv.hip: range + requantise launches, or one fused launch where the grid is
        # resident; no int32 tensor where the GEMM is shallow), their fragment-major weight copies
        # rewritten after every update; use_rows = False keeps every conv on the GEMM path
        self.rows = [ops.conv_rows_ok(g) for g in self.geoms]
        self.rows_nhwc = [(r and ops.rows_nhwc_ok(g, preferred=True), r and ops.rows_nhwc_ok(g, dgrad=True, preferred=True))
                          for r, g in zip(self.rows, self.geoms)]
        self.use_rows = True
        self.wf = [None] * len(self.convs)
        self.wft = [None] * len(self.convs)
        self.rstate = [ops.RowConvState(device) if r else None for r in self.rows]
        self.fwd_recompute = set()  # forward GEMM shapes the autotuner put on the two-phase recompute form
        self.record = False
        self.rec = {}
        # range buffers and exponent scalars of one step, allocated once and handed out in order
        # (one memset clears every range; exponents are always written before they are read)
        self._ranges = torch.zeros((160, ops.MAX_WORDS), dtype=torch.int32, device=device)
        self._exps = torch.zeros(160, dtype=torch.int8, device=device)
        self._ri = self._ei = 0

    def _range(self):
        r = self._ranges[self._ri]
        self._ri += 1
        return r

    def _exp(self):
        e = self._exps[self._ei:self._ei + 1]
        self._ei += 1
        return e

    def _global_range(self, amax):  # NITI_RangeEstimate over the global batch
        if self.comm is not None:
            self.comm.all_max(amax)

    @property
    def layers(self):
        return self.convs

    def _ci(self, i):  # input channels of the conv as it runs (the stem: its im2col columns)
        return self.STEM_KP if i == 0 else self.convs[i]["ci"]

    def _stem_cols(self, w):  # OIHW [co][3][7][7] -> [co][STEM_KP][1][1], column (ky * 7 + kx) * 3 + c
        co, ci, k, _ = w.shape
        wc = np.zeros((co, self.STEM_KP), dtype=np.int8)
        wc[:, :k * k * ci] = w.transpose(0, 2, 3, 1).reshape(co, k * k * ci)
        return wc.reshape(co, self.STEM_KP, 1, 1)

    def _stem_oihw(self, wc):  # [co][STEM_KP] (any int dtype) -> OIHW [co][3][7][7]
        l = self.convs[0]
        k, ci = l["k"], l["ci"]
        return wc[:, :k * k * ci].reshape(-1, k, k, ci).transpose(0, 3, 1, 2).copy()

    def weight_shape(self, i):
        l = self.convs[i]
        return (l["co"], l["ci"], l["k"], l["k"])

    def set_weight(self, i, w: np.ndarray, wscale: int):
        w = np.asarray(w)
        if w.dtype != np.int8 or tuple(w.shape) != self.weight_shape(i):
            raise ValueError(f"layer {i}: weight {w.dtype} {tuple(w.shape)}, want int8 {self.weight_shape(i)}")
        if i == 0:
            w = self._stem_cols(w)
        w16 = ops.oihw_to_ohwi16(torch.from_numpy(np.ascontiguousarray(w)).to(self.dev))
        wT = ops.ohwi16_to_ihwo16(w16, self._ci(i))
        if self.w16[i] is None:
            self.w16[i], self.wT[i] = w16, wT
        else:  # in place: a captured step holds these addresses
            self.w16[i].copy_(w16)
            self.wT[i].copy_(wT)
        self._refresh_wf(i)
        self.wscale[i] = int(wscale)
        if self.ws_dev[i] is None:
            self.ws_dev[i] = torch.tensor([wscale], dtype=torch.int8, device=self.dev)
        else:
            self.ws_dev[i].fill_(int(wscale))

    def _refresh_wf(self, i):
        if self.rows[i]:
            ci = self.convs[i]["ci"]
            self.wf[i] = ops.weights_to_wf(self.w16[i], ci, out=self.wf[i])
            self.wft[i] = ops.weights_to_wf(self.w16[i], ci, transpose=True, out=self.wft[i])

    def _rows(self, fwd, i, xc, amax, **kw):
        """One row-kernel conv: the fused launch where it is possible (one device, not capturing, the
        grid resident), else the speculative pair (modes 3, [global MAX], 4) or range, [global
        MAX], recompute-or-stored requantise."""
        f = ops.conv_fwd_rows if fwd else ops.conv_dgrad_rows
        g, wf = self.geoms[i], self.wf[i] if fwd else self.wft[i]
        if self.comm is None and not torch.cuda.is_current_stream_capturing():
            try:
                return f(g, xc, wf, amax, mode=0, state=self.rstate[i], **kw)[0]
            except NitiError as e:
                if e.code != 2:  # NOT_SUPPORT: the grid is not resident
                    raise
        if os.environ.get("NITI_RC_SPEC2", "1") != "0":
            # the speculative pair: requantised with the layer's previous bit width, redone only
            # where the (global) max's bit width differs
            outs = f(g, xc, wf, amax, mode=3, state=self.rstate[i], **kw)
            self._global_range(amax)
            return f(g, xc, wf, amax, mode=4, state=self.rstate[i], outs=outs, **kw)[0]
        f(g, xc, wf, amax, mode=1, **kw)
        self._global_range(amax)
        return f(g, xc, wf, amax, mode=2, **kw)[0]

    def rowconv_error(self) -> int:
        """1 if a fused row-kernel launch's grid barrier timed out (its results are invalid): the OR
        of every row layer's error word."""
        errs = [s.err for s in self.rstate if s is not None]
        return int(torch.stack(errs).max().item()) if errs else 0

    def get_weight(self, i) -> np.ndarray:
        w = ops.ohwi16_to_oihw(self.w16[i], self._ci(i)).cpu().numpy()
        return self._stem_oihw(w[:, :, 0, 0]) if i == 0 else w

    # ---------------------------------------------------------------- pieces
    def _nchw(self, t16, c):  # [n, h, w, cp] NHWC16 -> NCHW int8 (host, records only)
        return t16.cpu().numpy()[..., :c].transpose(0, 3, 1, 2).copy()

    # The convs store int32 and requantise in a separate pass (ops.conv_*_acc + requant_act): with
    # the planner's default plans (no autotuning on this path) the two-phase form, which recomputes
    # small-K GEMMs instead of storing them (ops.conv_fwd_requant), ran the step 9 % slower on
    # MI355X (5.40 vs 4.94 ms at batch 128, 224x224).
    def _fwd(self, i, x16, e_in, relu):
        l, g = self.convs[i], self.geoms[i]
        amax = self._range()
        if self.use_rows and self.rows[i]:
            # the row-segment maps read NHWC16 in place, the others a C32 copy
            xn = self.rows_nhwc[i][0]
            xc = x16 if xn else ops.nhwc16_to_c32(x16.view(self.batch, l["h"], l["h"], -1), l["ci"])
            e_out = self._exp()
            y = self._rows(True, i, xc, amax, exp_in=e_in, wscale=self.ws_dev[i], exp_out=e_out, relu=relu, x_nhwc=xn)
        else:
            xg = x16
            if i == 0:  # the stem: its im2col (from NCHW or NHWC16), kept for the weight gradient
                self._xcol = ops.im2col(self.stem_geom, x16, self.STEM_KP, nchw=x16.dim() == 4 and x16.shape[1] == 3)
                xg = self._xcol
            e_out = self._exp()
            if self._fwd_key(i) in self.fwd_recompute:  # autotune: the two-phase recompute form is faster
                y = ops.conv_fwd_requant(g, xg, self.w16[i], amax, exp_in=e_in, wscale=self.ws_dev[i], exp_out=e_out,
                                         relu=relu, between=self._global_range)
            else:
                acc = ops.conv_fwd_acc(g, xg, self.w16[i], amax)
                self._global_range(amax)
                y = ops.requant_act(acc, amax, exp_in=e_in, wscale=self.ws_dev[i], exp_out=e_out, relu=relu)
        y = y.view(self.batch, l["oh"], l["oh"], -1)
        if self.record:
            self.rec.setdefault("fwd", {})[i] = (y, relu)
            self.rec.setdefault("in", {})[i] = x16
        return y, e_out

    def _dgrad(self, i, dy16, e_dy, relu_mask=None):
        """The input gradient (exponent e_dy + wscale + inc), then the previous op's relu gradient
        where relu_mask (its output) is given -- fused into the row kernel's epilogue there."""
        l, g = self.convs[i], self.geoms[i]
        amax = self._range()
        e_dx = self._exp()
        if self.use_rows and self.rows[i]:
            xn = self.rows_nhwc[i][1]
            dyc = dy16 if xn else ops.nhwc16_to_c32(dy16.view(self.batch, l["oh"], l["oh"], -1), l["co"])
            m = None if relu_mask is None else relu_mask.view(self.batch, l["h"], l["h"], -1)
            dx = self._rows(False, i, dyc, amax, relu_mask=m, exp_in=e_dy, wscale=self.ws_dev[i], exp_out=e_dx,
                            x_nhwc=xn)
            return dx.view(self.batch, l["h"], l["h"], -1), e_dx
        acc = ops.conv_dgrad_acc(g, dy16, self.wT[i], amax)
        self._global_range(amax)
        dx = ops.requant_act(acc, amax, exp_in=e_dy, wscale=self.ws_dev[i], exp_out=e_dx)
        dx = dx.view(self.batch, l["h"], l["h"], -1)
        if relu_mask is not None:
            dx = ops.relu_grad(relu_mask, dx)
        return dx, e_dx

    def _wgrad_update(self, i, x16, dy16):
        amax = self._range()
        acc = ops.conv_wgrad_acc(self.geoms[i], self._xcol if i == 0 else x16, dy16, amax)
        if self.comm is not None:  # the global batch's gradient, then its range
            self.comm.all_sum(acc)
            amax.zero_()
            ops.absmax(acc, amax)
        # the transposed copy is rewritten in place (its input gradient above read it first), so a
        # captured step keeps reading the same buffer
        # the row kernels' fragment-major copies are rewritten by the update itself
        rw = self.rows[i] and self.wf[i] is not None and self.convs[i]["ci"] % 32 == 0 and self.convs[i]["co"] % 32 == 0
        _, g8 = ops.sgd_update(acc, amax, self.w16[i], self._ci(i), rule=2, wT=self.wT[i],
                               wf=self.wf[i] if rw else None, wft=self.wft[i] if rw else None)
        if not rw:
            self._refresh_wf(i)
        if self.record:
            self.rec.setdefault("dy", {})[i] = dy16
            self.rec.setdefault("dw", {})[i] = g8

    def _add(self, a, ea, b, eb, relu, relu_mask=None):
        # fused residual requantisation: a range pass without the int32 z, then z recomputed from
        # the int8 operands while requantising (2 x 2 int8 reads instead of an int32 write + read);
        # relu_mask: the next op's relu gradient applied in the same pass (backward)
        amax = self._range()
        ops.residual_range(a, ea, b, eb, amax)
        self._global_range(amax)
        ez, e_out = self._exp(), self._exp()
        q, _, _ = ops.residual_requant(a, ea, b, eb, amax, ez=ez, exp_out=e_out, relu=relu, relu_mask=relu_mask)
        return q, e_out

    # ---------------------------------------------------------------- plans
    def _fwd_key(self, i, op=0):  # the autotuner's per-shape key of layer i's GEMM `op`
        g = self.geoms[i]
        return (op, g.n, g.c_in, g.h, g.w, g.c_out, g.kh, g.stride_h if hasattr(g, "stride_h") else 0, g.oh, g.ow)

    def autotune(self, reps=3):
        """Per-shape plan autotuning of the GEMM-path convs (what niti_model_autotune does for the C++
        Model): every candidate tile / K-split plan of each forward, input-gradient and weight-gradient
        GEMM (and the tap-sharing weight gradient where it applies) timed on this batch's shapes with
        dummy operands, the fastest forced (ops.conv_plan_set: per process, keyed by GEMM shape; the
        results are plan-independent).  Returns {(layer, op): (plan, us)}."""
        dev, n = self.dev, self.batch
        tiles = [(128, 128), (128, 64), (64, 128), (64, 64), (256, 128), (128, 256)]
        splits = [2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64]
        done, out = set(), {}
        amax = torch.zeros(ops.MAX_WORDS, dtype=torch.int32, device=dev)

        def timed(f):
            f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = float("inf")
            for _ in range(reps):
                e0.record()
                f()
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1000.0)
            return best

        for i, l in enumerate(self.convs):
            g = self.geoms[i]
            rows = self.use_rows and self.rows[i]
            phases = ([] if rows else [0]) + ([1] if i > 0 and not rows else []) + [2]
            x16 = torch.randint(-8, 8, (g.n * g.h * g.w, g.cip), dtype=torch.int8, device=dev)
            dy16 = torch.randint(-8, 8, (g.n * g.oh * g.ow, g.cop), dtype=torch.int8, device=dev)
            w16 = torch.randint(-8, 8, (g.c_out, g.kh, g.kw, g.cip), dtype=torch.int8, device=dev)
            wT = torch.randint(-8, 8, (g.c_in, g.kh, g.kw, g.cop), dtype=torch.int8, device=dev)
            for op in phases:
                key = self._fwd_key(i, op)
                if key in done:
                    continue
                done.add(key)
                run = {0: lambda: ops.conv_fwd_acc(g, x16, w16, amax),
                       1: lambda: ops.conv_dgrad_acc(g, dy16, wT, amax),
                       2: lambda: ops.conv_wgrad_acc(g, x16, dy16, amax)}[op]
                ops.conv_plan_set(g, op, None)
                best_plan, best_us = None, timed(run)
                M, N = {0: (g.n * g.oh * g.ow, g.cop), 1: (g.n * g.h * g.w, g.cip),
                        2: (g.c_out, g.kh * g.kw * g.cip)}[op]
                # K splits only where the tiles alone leave the chip idle (their int32 slabs are M x N each)
                cands = [(bm, bn, 1, 0) for bm, bn in tiles] + [
                    (bm, bn, sp, 2) for bm, bn in tiles for sp in splits
                    if -(-M // bm) * -(-N // bn) < 256 and -(-M // bm) * -(-N // bn) * sp <= 4096]
                if op == 2 and ops.wgrad_taps_ok(g):
                    cands += [(32, 32, 1, 0)] + [(32, 32, sp, 2) for sp in splits]
                for plan in cands:
                    try:
                        ops.conv_plan_set(g, op, plan)
                        us = timed(run)
                    except NitiError:
                        continue
                    if us < best_us:
                        best_plan, best_us = plan, us
                ops.conv_plan_set(g, op, best_plan)
                out[(i, op)] = (best_plan, best_us)
                if op == 0:
                    # the forward with its requantisation: int32 stored + requant_act, or the two-phase
                    # form recomputing the GEMM (strategy 1: no int32 round trip; the stem's K = 160
                    # GEMM moves 257 MB of im2col against 411 MB of int32 out and back)
                    bm, bn = best_plan[:2] if best_plan else ops.conv_plan(g, 0)[:2]
                    e8 = torch.zeros(1, dtype=torch.int8, device=dev)
                    t_acc = timed(lambda: ops.requant_act(run(), amax, exp_in=e8, wscale=e8, exp_out=e8))
                    try:
                        ops.conv_plan_set(g, 0, (bm, bn, 1, 1))
                        t_rc = timed(lambda: ops.conv_fwd_requant(g, x16, w16, amax, exp_in=e8, wscale=e8, exp_out=e8))
                    except NitiError:
                        t_rc = float("inf")
                    if t_rc < t_acc:
                        self.fwd_recompute.add(key)
                        out[(i, "fwd_recompute")] = ((bm, bn, 1, 1), t_rc)
                    else:
                        ops.conv_plan_set(g, 0, best_plan)
        return out

    # ---------------------------------------------------------------- step
    def train_step(self, x: torch.Tensor, exp_in: int, labels: torch.Tensor):
        """One NITI_SGD step on x int8 NCHW [n][3][hw][hw] (device) with exponent exp_in (an int or
        a device int8 [1], e.g. the input quantiser's ascale)."""
        n = self.batch
        if x.dtype != torch.int8 or tuple(x.shape) not in ((n, 3, self.in_hw, self.in_hw),
                                                            (n, self.in_hw, self.in_hw, 16)):
            raise ValueError(f"x must be int8 NCHW {(n, 3, self.in_hw, self.in_hw)} or NHWC16")
        if any(w is None for w in self.w16):
            raise ValueError("set every layer's weight first")
        self.rec = {}
        self._ranges.zero_()
        self._ri = self._ei = 0
        x0 = x  # NCHW int8 or NHWC16: only the stem's im2col reads it
        e0 = exp_in if isinstance(exp_in, torch.Tensor) else torch.tensor([exp_in], dtype=torch.int8, device=self.dev)
        saved_in = {}
        # stem
        r0, e = self._fwd(0, x0, e0, relu=True)
        saved_in[0] = x0
        p0 = ops.maxpool(r0, 3, 2, 1)
        u, eu = p0, e
        saved = []
        for (ia, ib, ip) in self.blocks:
            h, eh = self._fwd(ia, u, eu, relu=True)
            yb, eb = self._fwd(ib, h, eh, relu=False)
            saved_in[ia], saved_in[ib] = u, h
            if ip is not None:
                sc, es = self._fwd(ip, u, eu, relu=False)
                saved_in[ip] = u
            else:
                sc, es = u, eu
            out, eo = self._add(yb, eb, sc, es, relu=True)
            saved.append((h, out))
            u, eu = out, eo
        # global sum pool, head, loss gradient
        amax = self._range()
        gsum = ops.sum_pool(u, amax)
        self._global_range(amax)
        eg = self._exp()
        g8 = ops.requant_act(gsum, amax, exp_in=eu, exp_out=eg).view(n, 1, 1, -1)
        fc = len(self.convs) - 1
        saved_in[fc] = g8
        logits, el = self._fwd(fc, g8, eg, relu=False)
        logits = logits.view(n, -1)
        d = ops.loss_grad(logits, self.classes, el, labels).view(n, 1, 1, -1)
        ed = self._exp()
        ed.zero_()
        if self.record:
            self.rec.update(logits=logits, exp_logits=el, pool=g8)
        # backward: each layer's input gradient reads the old weights before its update
        dg, edg = self._dgrad(fc, d, ed)
        self._wgrad_update(fc, g8, d)
        hh = u.shape[1]
        du, edu = ops.sum_pool_grad(dg.view(n, -1), hh, hh), edg
        for k in range(len(self.blocks) - 1, -1, -1):
            ia, ib, ip = self.blocks[k]
            h, out = saved[k]
            # block k's output relu gradient: fused into block k + 1's backward residual sum, except
            # for the last block (after the sum pool's gradient)
            dz = ops.relu_grad(out, du) if k == len(self.blocks) - 1 else du
            dh, edh = self._dgrad(ib, dz, edu, relu_mask=h)  # conv a's relu gradient rides along
            self._wgrad_update(ib, h, dz)
            dua, edua = self._dgrad(ia, dh, edh)
            self._wgrad_update(ia, saved_in[ia], dh)
            if ip is not None:
                dus, edus = self._dgrad(ip, dz, edu)
                self._wgrad_update(ip, saved_in[ip], dz)
            else:
                dus, edus = dz, edu
            du, edu = self._add(dua, edua, dus, edus, relu=False,
                                relu_mask=saved[k - 1][1].view(dua.shape) if k > 0 else None)
        dp = ops.maxpool_grad(r0, p0, du, 3, 2, 1)
        d0 = ops.relu_grad(r0, dp)
        self._wgrad_update(0, x0, d0)

    def train_step_images(self, images: torch.Tensor, labels: torch.Tensor):
        """NITIInt8Train's input quantiser (MnistUtils.cpp:83-93) on uint8 images [n][3][hw][hw],
        straight into the stem's NHWC16 input, then the step."""
        stats = ops.image_stats(images)
        count = images.numel()
        if self.comm is not None:  # batch statistics over every rank's images
            self.comm.all_sum(stats[:2])
            self.comm.all_max(stats[2:])
            count *= self.comm.world
        x, a = ops.image_quantize(images, stats, count)  # NCHW: the stem's im2col reads its planes
        self.train_step(x, a, labels)

    def taps(self):
        """Host copies of the last recorded step (record = True): per parameter layer the
        requantised forward output (pre-relu values where relu follows are not kept: relu'd
        outputs), its output gradient and int8 weight gradient, NCHW / OIHW; logits + exponent."""
        out = {"fwd": {}, "dy": {}, "dw": {}}
        for i, (y, _) in self.rec.get("fwd", {}).items():
            out["fwd"][i] = self._nchw(y, self.convs[i]["co"])
        for i, dy in self.rec.get("dy", {}).items():
            out["dy"][i] = self._nchw(dy, self.convs[i]["co"])
        for i, g8 in self.rec.get("dw", {}).items():
            g = g8.cpu().numpy()
            out["dw"][i] = (self._stem_oihw(g[:, 0, 0, :]) if i == 0
                            else g[..., :self.convs[i]["ci"]].transpose(0, 3, 1, 2).copy())
        if "logits" in self.rec:
            out["logits"] = self.rec["logits"].cpu().numpy()[:, :self.classes].copy()
            out["exp_logits"] = int(self.rec["exp_logits"].item())
        return out

    def input_tap(self, i):
        """Host copy (NCHW) of parameter layer i's input in the last recorded step."""
        x16 = self.rec["in"][i]
        if x16.dim() == 4 and x16.shape[1] == 3 and i == 0:  # the stem's NCHW input
            return x16.cpu().numpy().copy()
        return self._nchw(x16.view(self.batch, self.convs[i]["h"], self.convs[i]["h"], -1), self.convs[i]["ci"])

    def step_macs(self) -> int:
        """MACs of one step, counted as the VGG driver counts them (niti_model_step_macs): every
        layer's forward and weight gradient, and the input gradient of every layer but the stem
        (train_step never computes the stem's, as the lazy reference graph skips conv1's)."""
        s = 0
        for i, l in enumerate(self.convs):
            f = self.batch * l["oh"] * l["oh"] * l["co"] * l["ci"] * l["k"] * l["k"]
            s += 2 * f + (f if i > 0 else 0)
        return s
