"""Device-resident NITI training step (section 3 of include/niti_hip.h)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib as L
from ._lib import check
from .ops import _stream


class NitiModel:
    """NITIInt8Train's model + NITI_SGD step, on one GPU (optionally one rank of a DP group)."""

    def __init__(self, arch: int, batch: int, in_hw: int = 0, classes: int = 0):
        """arch: niti_amd.ARCH_*; in_hw: the input size (0: the architecture's); classes: the head's
        class count (0: the architecture's; ResNet-18 only)."""
        self._lib = L.lib()
        h = C.c_void_p()
        check(self._lib.niti_model_create3(arch, batch, int(in_hw), int(classes), C.byref(h)), "model_create")
        self._h = h
        self.arch, self.batch = arch, batch
        self._wscale = {}
        self.layers = []
        for i in range(self._lib.niti_model_num_layers(h)):
            info = (C.c_int * 12)()
            check(self._lib.niti_model_layer_info(h, i, info), "layer_info")
            keys = ("c_in", "c_out", "kh", "kw", "h", "w", "oh", "ow", "pad", "stride", "relu", "pool")
            self.layers.append(dict(zip(keys, list(info))))

    def weight_shape(self, i):
        l = self.layers[i]
        return (l["c_out"], l["c_in"], l["kh"], l["kw"])

    def set_weight(self, i, w: np.ndarray, wscale: int):
        if not 0 <= i < len(self.layers):
            raise ValueError(f"layer {i} out of range (model has {len(self.layers)})")
        w = np.asarray(w)
        if w.dtype != np.int8 or tuple(w.shape) != self.weight_shape(i):
            # checked here, not by an assert: the C ABI copies weight_shape(i) bytes from w
            raise ValueError(f"layer {i}: weight {w.dtype} {tuple(w.shape)}, want int8 {self.weight_shape(i)}")
        w = np.ascontiguousarray(w)
        check(self._lib.niti_model_set_weight(self._h, i, w.ctypes.data_as(C.c_void_p), int(wscale)), "set_weight")
        self._wscale[i] = int(wscale)

    def save(self, path: str):
        """Snapshot the device weights + wscales (mnistTrain.cpp:375-376 `Variable::save`)."""
        from .checkpoint import save_params
        if len(self._wscale) != len(self.layers):
            raise ValueError("save() before every layer's weight was set")
        save_params(path, [self.get_weight(i) for i in range(len(self.layers))],
                    [self._wscale[i] for i in range(len(self.layers))], self.arch,
                    in_hw=self.layers[0]["h"])

    def load(self, path: str):
        """Restore a snapshot written by save() into this model's device weights."""
        from .checkpoint import load_params
        weights, wscales, arch = load_params(path)
        if arch != self.arch or len(weights) != len(self.layers):
            raise ValueError(f"snapshot is arch {arch} with {len(weights)} layers, model is arch {self.arch}")
        # every layer's shape before any device write (a VGG-16 snapshot taken at another input
        # size has the same arch and layer count but a different first FC layer)
        for i, w in enumerate(weights):
            if tuple(w.shape) != self.weight_shape(i):
                raise ValueError(f"snapshot layer {i} is {tuple(w.shape)}, model layer is {self.weight_shape(i)}")
        for i, (w, s) in enumerate(zip(weights, wscales)):
            self.set_weight(i, w, s)

    def save_mnn(self, path: str):
        """The reference's own snapshot: `Variable::save(model->parameters(), path)` -- an MNN Net
        flatbuffer of one TrainableParam Blob per layer weight (int8 OIHW, express/Expr.cpp:833-965)
        -- plus `path.wscale.json` with the weight scales the NITI modules keep outside their
        parameters.  `Variable::load` + `Module::loadParameters` read the .mnn unchanged."""
        from . import mnn_snapshot
        if len(self._wscale) != len(self.layers):
            raise ValueError("save_mnn() before every layer's weight was set")
        mnn_snapshot.save(path, [self.get_weight(i) for i in range(len(self.layers))],
                          [self._wscale[i] for i in range(len(self.layers))],
                          meta={"arch": int(self.arch), "in_hw": int(self.layers[0]["h"])})

    def load_mnn(self, path: str):
        """`Module::loadParameters(Variable::load(path))` (mnistTrain.cpp:375-376): the weights in
        file order; the wscales from the side-car when there is one, otherwise the model keeps its
        own (as the reference's modules do).  Every shape is checked before any device write."""
        from . import mnn_snapshot
        weights, wscales, _ = mnn_snapshot.load(path)
        if len(weights) != len(self.layers):
            raise ValueError(f"{path}: {len(weights)} parameters, model has {len(self.layers)} layers")
        for i, w in enumerate(weights):
            if tuple(w.shape) != self.weight_shape(i):
                raise ValueError(f"snapshot parameter {i} is {tuple(w.shape)}, model layer is {self.weight_shape(i)}")
        if wscales is None:
            if len(self._wscale) != len(self.layers):
                raise ValueError(f"{path}: no wscale side-car and the model's scales are not set")
            wscales = [self._wscale[i] for i in range(len(self.layers))]
        for i, (w, s) in enumerate(zip(weights, wscales)):
            self.set_weight(i, w, s)

    def get_weight(self, i) -> np.ndarray:
        w = np.empty(self.weight_shape(i), np.int8)
        check(self._lib.niti_model_get_weight(self._h, i, w.ctypes.data_as(C.c_void_p)), "get_weight")
        return w

    def train_step(self, x: torch.Tensor, exp_in: int, labels: torch.Tensor, stream=None):
        assert x.dtype == torch.int8 and x.is_contiguous() and labels.dtype == torch.int32
        check(self._lib.niti_model_train_step(self._h, C.c_void_p(x.data_ptr()), int(exp_in),
                                              C.c_void_p(labels.data_ptr()), _stream(stream)), "train_step")

    def train_step_images(self, images: torch.Tensor, labels: torch.Tensor, stream=None):
        """One step from uint8 images [batch][C][H][W]: the input quantiser (MnistUtils.cpp:83-93)
        runs on device and supplies x and its exponent."""
        assert images.dtype == torch.uint8 and images.is_contiguous() and labels.dtype == torch.int32
        check(self._lib.niti_model_train_step_images(self._h, C.c_void_p(images.data_ptr()),
                                                     C.c_void_p(labels.data_ptr()), _stream(stream)),
              "train_step_images")

    def input(self, stream=None):
        """The last step's quantised input x (NCHW int8) and its exponent."""
        l0 = self.layers[0]
        out = np.empty((self.batch, l0["c_in"], l0["h"], l0["w"]), np.int8)
        e = C.c_int()
        check(self._lib.niti_model_get_input(self._h, out.ctypes.data_as(C.c_void_p), C.byref(e), _stream(stream)),
              "get_input")
        return out, int(e.value)

    def logits(self, stream=None):
        last = self.layers[-1]
        out = np.empty((self.batch, last["c_out"]), np.int8)
        e = C.c_int()
        check(self._lib.niti_model_get_logits(self._h, out.ctypes.data_as(C.c_void_p), C.byref(e),
                                              _stream(stream)), "get_logits")
        return out, int(e.value)

    def tap(self, i, which, stream=None):
        l = self.layers[i]
        if which == 1:
            shape = (l["c_out"], l["c_in"], l["kh"], l["kw"])
        else:
            shape = (self.batch, l["c_out"], l["oh"], l["ow"])
        out = np.empty(shape, np.int8)
        check(self._lib.niti_model_get_tap(self._h, i, which, out.ctypes.data_as(C.c_void_p), out.nbytes,
                                           _stream(stream)), "get_tap")
        return out

    def autotune(self, reps: int = 5, stream=None):
        """Time candidate GEMM plans per layer phase and keep the fastest (niti_model_autotune).
        Call after one train_step; plans never change results."""
        check(self._lib.niti_model_autotune(self._h, int(reps), _stream(stream)), "autotune")

    def plan(self, layer: int, phase: int):
        """(bm, bn, splits, strategy) of one layer phase; 32x32 = the tap-sharing weight gradient,
        16x16 = the P16 weight gradient."""
        info = (C.c_int * 4)()
        check(self._lib.niti_model_plan_info(self._h, layer, phase, info), "plan_info")
        return tuple(info)

    def plans(self):
        """{(layer, phase): (bm, bn, splits, strategy)}; phase 0 fwd / 1 input grad / 2 weight grad,
        strategy 0 store / 1 recompute / 2 split-K / 3 the speculative pair / 4 fused: one launch with the
        rescale behind an in-kernel grid barrier (forward / input gradient)."""
        out = {}
        for i in range(len(self.layers)):
            for ph in (0, 1, 2):
                if ph == 1 and i == 0:
                    continue
                out[(i, ph)] = self.plan(i, ph)
        return out

    def set_plan(self, layer: int, phase: int, plan=None):
        """Force (bm, bn, splits, strategy) for one layer phase; None restores the default."""
        arr = None if plan is None else (C.c_int * 4)(*[int(v) for v in plan])
        check(self._lib.niti_model_plan_set(self._h, layer, phase, arr), "plan_set")

    @staticmethod
    def reset_plans():
        """Drop every plan override in this process."""
        L.lib().niti_plan_reset()

    def set_overlap(self, enable: bool):
        """Weight gradients on a second stream overlapping the input gradients (default on)."""
        check(self._lib.niti_model_set_overlap(self._h, int(enable)), "set_overlap")

    def set_graph(self, enable: bool):
        """Replay the step as a hipGraph or launch its kernels directly (default)."""
        check(self._lib.niti_model_set_graph(self._h, int(enable)), "set_graph")

    def keep_grads(self, enable: bool):
        """Store each step's int8 weight gradient for tap(layer, 1) (default) or not: the SGD
        kernel then updates the weights without writing the copy."""
        check(self._lib.niti_model_keep_grads(self._h, int(enable)), "keep_grads")

    def set_rowconv(self, enable: bool):
        """Forward convs and input gradients of the stride-1 pad-1 3x3 layers on the register-fed
        kernel with the fused rescale (default) or on the GEMM + requantisation passes; identical
        results."""
        check(self._lib.niti_model_set_rowconv(self._h, int(enable)), "set_rowconv")

    def rowconv_error(self) -> int:
        """1 if an in-kernel grid barrier of the register-fed forward ever timed out."""
        return int(self._lib.niti_model_rowconv_error(self._h))

    def spec_stats(self):
        """Per layer: (fwd hint, fwd launches redone, fwd pairs stored, dgrad hint, dgrad redone,
        dgrad stored) of the speculative row-kernel pairs (niti_model_spec_stats)."""
        n = len(self.layers)
        buf = (C.c_uint32 * (6 * n))()
        check(self._lib.niti_model_spec_stats(self._h, buf, n), "spec_stats")
        return [tuple(buf[6 * i:6 * i + 6]) for i in range(n)]

    def set_probe(self, layer: int, phase: int, max_launches: int = 256):
        check(self._lib.niti_model_set_probe(self._h, layer, phase, max_launches), "set_probe")

    def spec_slot(self, layer: int, dgrad: int):
        """The 32 words of one row-kernel layer's speculative slot (diagnostics)."""
        out = (C.c_uint32 * 32)()
        check(self._lib.niti_model_spec_slot(self._h, int(layer), int(dgrad), out), "spec_slot")
        return list(out)

    def probe_pause(self, paused: bool):
        """Skip (True) or time again (False) the armed probe's launches; host-side only."""
        check(self._lib.niti_model_probe_pause(self._h, 1 if paused else 0), "probe_pause")

    def probe_read(self):
        t = C.c_double()
        n = C.c_int()
        check(self._lib.niti_model_probe_read(self._h, C.byref(t), C.byref(n)), "probe_read")
        return float(t.value), int(n.value)

    def run_phase(self, layer: int, phase: int, stream=None):
        """One layer phase of the last step again (0 fwd, 1 input grad, 2 weight grad), alone."""
        check(self._lib.niti_model_run_phase(self._h, int(layer), int(phase), _stream(stream)), "run_phase")

    def probe_read_span(self):
        """(summed ms, launches) of the weight-gradient probe's in-kernel spans (device wall clock)."""
        t, n = C.c_double(0), C.c_int(0)
        check(self._lib.niti_model_probe_read_span(self._h, C.byref(t), C.byref(n)), "probe_read_span")
        return t.value, n.value

    def step_macs(self) -> int:
        return int(self._lib.niti_model_step_macs(self._h))

    def attach_comm(self, unique_id: bytes, rank: int, world: int, exact: bool = True):
        check(self._lib.niti_model_attach_comm(self._h, unique_id, rank, world, 1 if exact else 0), "attach_comm")

    def attach_local(self, group: "LocalGroup", rank: int, exact: bool = True):
        """Join an in-process rank group on this device (one host thread per rank)."""
        check(self._lib.niti_model_attach_local(self._h, group._h, rank, 1 if exact else 0), "attach_local")
        self._group = group  # keep the group alive as long as the model

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(L.lib().niti_dp_get_unique_id(buf), "unique_id")
        return buf.raw

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.niti_model_destroy(h)
            self._h = None


class LocalGroup:
    """niti_local_group: `world` ranks of the data-parallel protocol on ONE device, one host
    thread per rank, collectives reduced on the device (include/niti_hip.h)."""

    def __init__(self, world: int):
        self._lib = L.lib()
        h = C.c_void_p()
        check(self._lib.niti_local_group_create(int(world), C.byref(h)), "local_group_create")
        self._h = h
        self.world = world

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._lib.niti_local_group_destroy(h)
            self._h = None
