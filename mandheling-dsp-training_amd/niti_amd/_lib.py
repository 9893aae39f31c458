"""ctypes binding of libniti_hip.so (the C ABI declared in include/niti_hip.h).

There is no fallback: if the HIP library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# NITI_HIP_LIB selects another build of the same library (diagnostic variants under tools/)
LIB_PATH = os.environ.get("NITI_HIP_LIB") or os.path.join(_HERE, "_lib", "libniti_hip.so")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "niti_hip.h")

# MNN::ErrorCode names (include/MNN/ErrorCode.hpp:17-30)
ERROR_NAMES = {0: "NO_ERROR", 1: "OUT_OF_MEMORY", 2: "NOT_SUPPORT", 3: "COMPUTE_SIZE_ERROR",
               4: "NO_EXECUTION", 5: "INVALID_VALUE", 10: "INPUT_DATA_ERROR", 11: "CALL_BACK_STOP"}

OP_CONV_INT8 = 700
OP_DECONV_INT8 = 701
OP_RELU_INT8 = 703
OP_RELUGRAD_INT8 = 704
OP_MAXPOOL_INT8 = 705
OP_POOLGRAD_INT8 = 706
OP_LOSS_GRAD_INT8 = 711
OP_MATMUL_INT8 = 713
OP_PAD_INT8 = 714
OP_LEFTPOOLGRAD_INT8 = 718
OP_GRADIENT_CONV_INT8 = 715
OP_DSP_CONV_INT8 = 800
OP_DSP_RELU_INT8 = 801
OP_DSP_MAXPOOL_INT8 = 802
OP_DSP_RESHAPE_INT8 = 803
OP_DSP_LOSSGRAD_INT8 = 804
OP_DSP_RELUGRAD_INT8 = 805
OP_DSP_MAXPOOLGRAD_INT8 = 807
OP_DSP_TRANSPOSE_INT8 = 808
OP_DSP_WEIGHTROTATE180_INT8 = 809
OP_DSP_RESHAPEGRAD_INT8 = 813
OP_DSP_LEFTPOOLGRAD_DECONV_INT8 = 814
OP_DSP_LEFTPOOLGRAD_GRADIENT_INT8 = 815
OP_DSP_NOP_INT8 = 817
OP_DSP_DECONV_INT8 = 811
OP_DSP_MATMUL_GRADIENT_INT8 = 818
OP_DSP_PARALLEL_GRADIENTCONV_INT8 = 820
OP_DSP_GRADIENT_SPLITBATCHCONV_INT8 = 821
OP_DSP_TRANSPOSEGRADIENT_CONV_INT8 = 822
FORMAT_NCHW, FORMAT_NHWC, FORMAT_NC4HW4 = 0, 1, 2
PAD_CAFFE, PAD_VALID, PAD_SAME = 0, 1, 2
ARCH_LENET, ARCH_VGG11, ARCH_VGG16, ARCH_RESNET18 = 1, 2, 3, 4


class NitiError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {ERROR_NAMES.get(code, code)}")


class Tensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("dims", C.c_int * 4), ("format", C.c_int)]


class ConvCommon(C.Structure):
    _fields_ = [("kernel_x", C.c_int), ("kernel_y", C.c_int), ("stride_x", C.c_int), ("stride_y", C.c_int),
                ("dilate_x", C.c_int), ("dilate_y", C.c_int), ("pad_x", C.c_int), ("pad_y", C.c_int),
                ("has_pads", C.c_int), ("pads", C.c_int * 4), ("pad_mode", C.c_int),
                ("input_count", C.c_int), ("output_count", C.c_int), ("group", C.c_int)]


class Geom(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "n", "c_in", "h", "w", "c_out", "kh", "kw", "stride_h", "stride_w", "pad_t", "pad_l", "pad_b",
        "pad_r", "dilate_h", "dilate_w", "oh", "ow", "cip", "cop", "np")]


_lib = None


def header_functions():
    """Every function the public header declares (name -> None)."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\*?(niti_[a-z0-9_]+)\s*\(", src, flags=re.M)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libniti_hip.so not built ({LIB_PATH}); run __graft_entry__.build() or "
                          f"make -C mandheling-dsp-training_amd/csrc")
    # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's).  Load torch first so
    # this library binds to the runtime torch uses; loaded the other way round, torch is bound to
    # /opt/rocm's copy and the first allocation in the process fails (seen on the GPU box).
    import torch  # noqa: F401
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, ci = C.c_void_p, C.c_int32, C.c_int64, C.c_int
    tp = C.POINTER(Tensor)
    sig = {
        "niti_version": (C.c_char_p, []),
        "niti_create_execution": (ci, [ci, C.POINTER(ConvCommon), C.POINTER(vp)]),
        "niti_execution_resize": (ci, [vp, tp, ci, tp, ci]),
        "niti_execution_execute": (ci, [vp, tp, ci, tp, ci, vp]),
        "niti_destroy_execution": (None, [vp]),
        "niti_execution_workspace_bytes": (C.c_size_t, [vp]),
        "niti_execution_status": (ci, [vp, vp]),
        "niti_diag_rowconv_barrier": (None, [C.c_uint32, C.c_uint32]),
        "niti_diag_rowconv_speculate": (None, [C.c_int]),
        "niti_diag_gemm_speculate": (None, [C.c_int]),
        "niti_diag_gemm_fused_launches": (C.c_ulonglong, []),
        "niti_diag_head_chain_launches": (C.c_ulonglong, []),
        "niti_diag_head_chain": (None, [C.c_int]),
        "niti_diag_p16_jobs_cap": (None, [C.c_int]),
        "niti_tensor_convert": (ci, [tp, tp, vp]),
        "niti_geom_finalize": (ci, [C.POINTER(Geom)]),
        "niti_conv_workspace_bytes": (ci, [C.POINTER(Geom), ci, C.POINTER(C.c_size_t)]),
        "niti_matmul_workspace_bytes": (ci, [ci, ci, ci, C.POINTER(C.c_size_t)]),
        "niti_conv_plan_info": (ci, [C.POINTER(Geom), ci, C.c_size_t, C.POINTER(C.c_int)]),
        "niti_conv_fwd_acc": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, C.c_size_t, vp]),
        "niti_conv_dgrad_acc": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, C.c_size_t, vp]),
        "niti_conv_wgrad_acc": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, C.c_size_t, vp]),
        "niti_conv_fwd_phase1": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, C.c_size_t, vp]),
        "niti_conv_rows_ok": (ci, [C.POINTER(Geom)]),
        "niti_nhwc16_to_c32": (ci, [vp, ci, ci, ci, ci, vp, vp]),
        "niti_weights_to_wf": (ci, [vp, ci, ci, ci, ci, vp, vp]),
        "niti_conv_fwd_rows": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, ci, vp, vp, vp, ci, vp, vp, C.c_uint32, vp,
                                    vp]),
        "niti_conv_dgrad_rows": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, ci, vp, vp, vp, vp, vp, vp, ci, vp, vp, C.c_uint32, vp, vp]),
        "niti_rows_spec_slot": (vp, [vp, ci]),
        "niti_conv_fwd_phase2": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, vp, vp, ci, vp, vp, C.c_size_t, vp]),
        "niti_conv_dgrad_phase1": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, C.c_size_t, vp]),
        "niti_conv_dgrad_phase2": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, vp, vp, ci, vp, vp, C.c_size_t, vp]),
        "niti_nhwc16_to_p16": (ci, [vp, i64, ci, vp, vp]),
        "niti_diag_wgrad_stamps": (None, [vp]),
        "niti_diag_rowconv_stamps": (None, [vp]),
        "niti_conv_wgrad_p16_workspace": (ci, [C.POINTER(Geom), ci, C.POINTER(C.c_size_t)]),
        "niti_conv_wgrad_p16_acc": (ci, [C.POINTER(Geom), vp, vp, vp, vp, vp, C.c_size_t, ci, vp]),
        "niti_matmul_acc": (ci, [ci, ci, ci, vp, i64, vp, i64, vp, i64, vp, vp, C.c_size_t, vp]),
        "niti_absmax_i32": (ci, [vp, i64, vp, vp]),
        "niti_requant_act": (ci, [vp, i64, ci, vp, vp, vp, vp, ci, vp, vp, vp]),
        "niti_requant_grad": (ci, [vp, i64, vp, ci, vp, vp, vp]),
        "niti_sgd_update": (ci, [vp, vp, ci, ci, ci, ci, ci, ci, vp, vp, vp, vp]),
        "niti_nhwc16_to_chwn16": (ci, [vp, ci, ci, ci, ci, vp, vp]),
        "niti_ohwi16_to_ihwo16": (ci, [vp, ci, ci, ci, ci, ci, vp, vp]),
        "niti_nchw_to_nhwc16": (ci, [vp, ci, ci, ci, ci, vp, vp]),
        "niti_nchw_to_chwn16": (ci, [vp, ci, ci, ci, ci, ci, vp, vp]),
        "niti_nhwc16_to_nchw": (ci, [vp, ci, ci, ci, ci, vp, vp]),
        "niti_oihw_to_ohwi16": (ci, [vp, ci, ci, ci, ci, vp, vp]),
        "niti_ohwi16_to_oihw": (ci, [vp, ci, ci, ci, ci, vp, vp]),
        "niti_residual_add": (ci, [vp, vp, vp, vp, i64, vp, vp, vp, vp]),
        "niti_residual_requant": (ci, [vp, vp, vp, vp, i64, vp, vp, vp, ci, vp, vp]),
        "niti_residual_requant_relu_grad": (ci, [vp, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]),
        "niti_sum_pool": (ci, [vp, ci, ci, ci, vp, vp, vp]),
        "niti_sum_pool_grad": (ci, [vp, ci, ci, ci, vp, vp]),
        "niti_im2col": (ci, [C.POINTER(Geom), vp, ci, vp, vp]),
        "niti_im2col_nchw": (ci, [C.POINTER(Geom), vp, ci, vp, vp]),
        "niti_sgd_update_wf": (ci, [vp, vp, ci, ci, ci, ci, ci, ci, vp, vp, vp, vp, vp, vp]),
        "niti_conv_rows_nhwc_ok": (ci, [C.POINTER(Geom), ci]),
        "niti_conv_plan_set": (ci, [C.POINTER(Geom), ci, vp]),
        "niti_maxpool": (ci, [vp] + [ci] * 7 + [vp, ci, ci, vp]),
        "niti_maxpool_grad": (ci, [vp, vp, vp] + [ci] * 10 + [vp, vp]),
        "niti_maxpool_grad_ws": (ci, [vp, vp, vp] + [ci] * 10 + [vp, vp, vp]),
        "niti_relu_grad": (ci, [vp, vp, i64, vp, vp]),
        "niti_loss_grad": (ci, [vp, ci, ci, ci, vp, vp, vp, vp]),
        "niti_model_create": (ci, [ci, ci, C.POINTER(vp)]),
        "niti_model_create2": (ci, [ci, ci, ci, C.POINTER(vp)]),
        "niti_model_create3": (ci, [ci, ci, ci, ci, C.POINTER(vp)]),
        "niti_model_destroy": (None, [vp]),
        "niti_model_num_layers": (ci, [vp]),
        "niti_model_layer_info": (ci, [vp, ci, C.POINTER(ci)]),
        "niti_model_set_weight": (ci, [vp, ci, vp, ci]),
        "niti_model_get_weight": (ci, [vp, ci, vp]),
        "niti_model_train_step": (ci, [vp, vp, ci, vp, vp]),
        "niti_model_get_logits": (ci, [vp, vp, C.POINTER(ci), vp]),
        "niti_model_get_tap": (ci, [vp, ci, ci, vp, C.c_size_t, vp]),
        "niti_model_step_macs": (i64, [vp]),
        "niti_model_set_graph": (ci, [vp, ci]),
        "niti_model_set_rowconv": (ci, [vp, ci]),
        "niti_model_keep_grads": (ci, [vp, ci]),
        "niti_model_rowconv_error": (ci, [vp]),
        "niti_model_spec_stats": (ci, [vp, vp, ci]),
        "niti_model_autotune": (ci, [vp, ci, vp]),
        "niti_model_set_overlap": (ci, [vp, ci]),
        "niti_model_plan_info": (ci, [vp, ci, ci, C.POINTER(ci)]),
        "niti_model_plan_set": (ci, [vp, ci, ci, C.POINTER(ci)]),
        "niti_plan_reset": (None, []),
        "niti_model_set_probe": (ci, [vp, ci, ci, ci]),
        "niti_model_probe_read": (ci, [vp, C.POINTER(C.c_double), C.POINTER(ci)]),
        "niti_model_probe_pause": (ci, [vp, ci]),
        "niti_model_spec_slot": (ci, [vp, ci, ci, C.POINTER(C.c_uint32)]),
        "niti_model_run_phase": (ci, [vp, ci, ci, vp]),
        "niti_model_probe_read_span": (ci, [vp, C.POINTER(C.c_double), C.POINTER(ci)]),
        "niti_dp_get_unique_id": (ci, [C.c_char_p]),
        "niti_model_attach_comm": (ci, [vp, C.c_char_p, ci, ci, ci]),
        "niti_image_stats": (ci, [vp, i64, vp, vp]),
        "niti_image_quantize": (ci, [vp, ci, ci, ci, vp, i64, vp, vp, vp]),
        "niti_image_quantize_nhwc16": (ci, [vp, ci, ci, ci, ci, vp, i64, vp, vp, vp]),
        "niti_model_train_step_images": (ci, [vp, vp, vp, vp]),
        "niti_model_get_input": (ci, [vp, vp, C.POINTER(ci), vp]),
        "niti_local_group_create": (ci, [ci, C.POINTER(vp)]),
        "niti_local_group_destroy": (None, [vp]),
        "niti_model_attach_local": (ci, [vp, vp, ci, ci]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(code, what=""):
    if code != 0:
        raise NitiError(code, what)
