"""niti_amd -- MI355X-native NITI int8 training backend (Python side of the C ABI).

The compute lives in libniti_hip.so (hand-written gfx950 HIP kernels, see ../csrc);
this package only binds it.  Importing it without the built library raises.
"""
from ._lib import (ARCH_LENET, ARCH_RESNET18, ARCH_VGG11, ARCH_VGG16, FORMAT_NC4HW4, FORMAT_NCHW, FORMAT_NHWC, LIB_PATH,  # noqa: F401
                   OP_CONV_INT8, OP_DECONV_INT8, OP_DSP_CONV_INT8, OP_DSP_DECONV_INT8,
                   OP_DSP_GRADIENT_SPLITBATCHCONV_INT8, OP_DSP_MATMUL_GRADIENT_INT8, OP_DSP_PARALLEL_GRADIENTCONV_INT8,
                   OP_DSP_TRANSPOSEGRADIENT_CONV_INT8, OP_GRADIENT_CONV_INT8,
                   OP_MATMUL_INT8, PAD_CAFFE, PAD_SAME, PAD_VALID, NitiError, check, header_functions, lib)

lib()  # fail loudly if the HIP library is missing
