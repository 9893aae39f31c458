/*
 * niti_hip.h -- C ABI of the MI355X (gfx950) NITI int8 training backend.
 *
 * This is the drop-in boundary for the reference's NITI int8 hot path.  The reference
 * exposes that path through MNN's operator interface:
 *
 *   Creator  : CPUBackend::Creator::onCreate(inputs, outputs, const MNN::Op*, Backend*)
 *              execution-engine/source/backend/cpu/CPUBackend.hpp:85-91, registered per
 *              OpType by REGISTER_CPU_OP_CREATOR (:179-182)
 *   Execution: onResize(inputs, outputs) / onExecute(inputs, outputs)
 *              execution-engine/source/core/Execution.hpp:24-82
 *   Errors   : MNN::ErrorCode, execution-engine/include/MNN/ErrorCode.hpp:17-30
 *
 * Section 1 mirrors that interface one to one (niti_create_execution / _resize / _execute /
 * niti_destroy_execution), keyed by the same OpType values, taking the same input and output
 * tensors in the same layouts; an MNN maintainer binds it with a ~40-line Creator (see
 * INTEGRATION.md).  Section 2 is the native split interface the device-resident training
 * driver and data parallelism use (accumulate -> [RCCL] -> requantise).  Section 3 is the
 * whole-step driver (NITIInt8Train's step, execution-engine/tools/train/source/demo/
 * MnistUtils.cpp:68-147, on device) with an optional RCCL communicator.
 *
 * All pointers are device (HBM) pointers unless stated; `stream` is a hipStream_t passed as
 * void*.  No call synchronises the stream or allocates on the execute path.  Handles are not
 * thread safe (as MNN Executions are not re-entrant).
 */
#ifndef NITI_HIP_H
#define NITI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes: MNN::ErrorCode (include/MNN/ErrorCode.hpp:17-30) ------------------------ */
enum niti_error_code {
    NITI_NO_ERROR = 0,
    NITI_OUT_OF_MEMORY = 1,
    NITI_NOT_SUPPORT = 2,
    NITI_COMPUTE_SIZE_ERROR = 3,
    NITI_NO_EXECUTION = 4,
    NITI_INVALID_VALUE = 5,
    NITI_INPUT_DATA_ERROR = 10,
    NITI_CALL_BACK_STOP = 11
};

/* ---- OpType keys (schema/default/MNN.fbs:189-233) ------------------------------------------ */
enum niti_op_type {
    NITI_OP_CONV_INT8 = 700,               /* NITI_CONV_Int8          -> NITI_Conv_Int8.cpp:162-310 */
    NITI_OP_DECONV_INT8 = 701,             /* NITI_DeCONV_Int8        -> NITI_DeConv_Int8.cpp:187-332 */
    NITI_OP_RELU_INT8 = 703,               /* NITI_Relu_Int8          -> NITI_CPURelu_Int8.cpp:28-61 */
    NITI_OP_RELUGRAD_INT8 = 704,           /* NITI_ReluGrad_Int8      -> NITI_CPUReluGrad_Int8.cpp:28-62 */
    NITI_OP_MAXPOOL_INT8 = 705,            /* NITI_Maxpool_Int8       -> NITI_Maxpool_Int8.cpp:24-175 */
    NITI_OP_POOLGRAD_INT8 = 706,           /* NITI_PoolGrad_Int8      -> NITI_CPUPoolGrad_Int8.cpp:21-77 */
    NITI_OP_LOSS_GRAD_INT8 = 711,          /* NITI_LOSS_Grad_Int8     -> NITI_CPULossGrad_Int8.cpp:81-200 */
    NITI_OP_MATMUL_INT8 = 713,             /* NITI_MatMul_Int8        -> NITI_Matmul_Int8.cpp:140-231 */
    NITI_OP_PAD_INT8 = 714,                /* NITI_PAD_Int8           -> NITI_Pad_Int8.cpp:24-62 */
    NITI_OP_GRADIENT_CONV_INT8 = 715,      /* NITI_GradientCONV_Int8  -> NITI_GradientConv_Int8.cpp:165-298 */
    NITI_OP_LEFTPOOLGRAD_INT8 = 718,       /* NITI_LeftPoolGrad_Int8  -> NITI_CPULeftPoolGrad_Int8.cpp:18-52 */
    NITI_OP_DSP_CONV_INT8 = 800,           /* NITI_DSP_CONV_Int8      -> NITI_DSPConv_Int8.cpp:160-455 */
    NITI_OP_DSP_RELU_INT8 = 801,           /* NITI_DSP_RELU_Int8      -> NITI_DSPRelu_Int8.cpp */
    NITI_OP_DSP_MAXPOOL_INT8 = 802,        /* NITI_DSP_MAXPOOL_Int8   -> NITI_DSPMaxpool_Int8.cpp */
    NITI_OP_DSP_RESHAPE_INT8 = 803,        /* NITI_DSP_RESHAPE_Int8   -> NITI_DSPReshape_Int8.cpp */
    NITI_OP_DSP_LOSSGRAD_INT8 = 804,       /* NITI_DSP_LOSSGRAD_Int8  -> NITI_DSPLossGrad_Int8.cpp */
    NITI_OP_DSP_RELUGRAD_INT8 = 805,       /* NITI_DSP_RELUGRAD_Int8  -> NITI_DSPReluGrad_Int8.cpp */
    NITI_OP_DSP_MAXPOOLGRAD_REF_INT8 = 806, /* NITI_DSP_MAXPOOLGRAD_REF_Int8 -> NITI_DSPMaxPoolGradRef_Int8.cpp:17-80 */
    NITI_OP_DSP_MAXPOOLGRAD_INT8 = 807,    /* NITI_DSP_MAXPOOLGRAD_Int8 -> NITI_DSPMaxPoolGrad_Int8.cpp */
    NITI_OP_DSP_TRANSPOSE_INT8 = 808,      /* NITI_DSP_TRANSPOSE_Int8 -> NITI_DSPTranspose_Int8.cpp */
    NITI_OP_DSP_WEIGHTROTATE180_INT8 = 809, /* NITI_DSP_WEIGHTROTATE180_REF_Int8 -> NITI_DSPWeightRotateRef_Int8.cpp */
    NITI_OP_DSP_DECONV_INT8 = 811,         /* NITI_DSP_DECONV_Int8    -> NITI_DSPDeConv_Int8.cpp */
    NITI_OP_DSP_GRADIENTCONV_INT8 = 810,   /* NITI_DSP_GRADIENTCONV_Int8 -> NITI_DSPGradientConv_Int8.cpp (818's tensors) */
    NITI_OP_DSP_PAD_INT8 = 812,            /* NITI_DSP_PAD_Int8       -> NITI_DSPPAD_Int8.cpp */
    NITI_OP_DSP_RESHAPEGRAD_INT8 = 813,    /* NITI_DSP_RESHAPEGrad_Int8 -> NITI_DSPReshapeGrad_Int8.cpp */
    NITI_OP_DSP_LEFTPOOLGRAD_DECONV_INT8 = 814,   /* -> NITI_DSPLeftPoolGrad_Int8.cpp */
    NITI_OP_DSP_LEFTPOOLGRAD_GRADIENT_INT8 = 815, /* -> NITI_DSPLeftPoolGrad_Int8.cpp */
    NITI_OP_DSP_NOP_INT8 = 817,            /* NITI_DSP_NOP_Int8       -> NITI_DSPNop_Int8.cpp */
    NITI_OP_DSP_MATMUL_GRADIENT_INT8 = 818, /* NITI_DSP_MATMUL_GRADIENT_Int8 -> NITI_DSPMatmulGradientConv_Int8.cpp:105-553 */
    NITI_OP_DSP_MATMUL_INT8 = 819,         /* NITI_DSP_MATMUL_Int8    -> NITI_DSPMatmul_Int8.cpp (818's tensors) */
    NITI_OP_DSP_PARALLEL_GRADIENTCONV_INT8 = 820,   /* -> NITI_DSPParallelGradientConv_Int8.cpp (818's tensors) */
    NITI_OP_DSP_GRADIENT_SPLITBATCHCONV_INT8 = 821, /* -> NITI_DSPGradientSplitBatchConv_Int8.cpp (822's tensors) */
    NITI_OP_DSP_TRANSPOSEGRADIENT_CONV_INT8 = 822 /* -> NITI_DSPTransposeGradientConv_Int8.cpp:137-440 */
};

/* ---- tensor formats: MNN_DATA_FORMAT (schema/default/Tensor.fbs:12-18) ---------------------- */
enum niti_format { NITI_FORMAT_NCHW = 0, NITI_FORMAT_NHWC = 1, NITI_FORMAT_NC4HW4 = 2 };

/* ---- pad modes: PadMode (schema/default/CaffeOp.fbs:3-7) ----------------------------------- */
enum niti_pad_mode { NITI_PAD_CAFFE = 0, NITI_PAD_VALID = 1, NITI_PAD_SAME = 2 };

/* A tensor as an Execution sees it: Tensor::host<T>() + batch/channel/height/width +
 * TensorUtils::getDescribe()->dimensionFormat.  dims are the logical N, C, H, W in every
 * format (for NHWC data, dims still list N, C, H, W).  2-D tensors use dims {rows, cols, 1, 1}. */
typedef struct niti_tensor {
    void* data;
    int dims[4];
    int format;
} niti_tensor;

/* The parts of Convolution2DCommon (schema/default/CaffeOp.fbs) the NITI ops read
 * (NeuralNetWorkOp.cpp:1857-1880). pads = {top, left, bottom, right} when has_pads. */
typedef struct niti_conv2d_common {
    int kernel_x, kernel_y;
    int stride_x, stride_y;
    int dilate_x, dilate_y;
    int pad_x, pad_y;
    int has_pads;
    int pads[4];
    int pad_mode;
    int input_count, output_count;
    int group;
} niti_conv2d_common;

/* ============================ 1. Execution-shaped drop-in ============================== */
typedef struct niti_execution* niti_execution_t;

/* CPUBackend::Creator::onCreate for `op_type`.  common may be NULL for NITI_OP_MATMUL_INT8.
 * Returns NITI_NOT_SUPPORT for an op type or parameter the backend does not implement
 * (group != 1; dilation != 1 on a gradient op). */
int niti_create_execution(int op_type, const niti_conv2d_common* common, niti_execution_t* out);

/* Execution::onResize: shape checks + workspace (device memory owned by the handle).
 *  NITI_OP_CONV_INT8          in {x NC4HW4 [N,Ci,H,W], w NCHW [Co,Ci,KH,KW], exp_in int8[1], wscale int8[1]}
 *                             out{y NC4HW4 [N,Co,OH,OW], exp_out int8[1]}
 *  NITI_OP_DECONV_INT8        in {dy' NC4HW4 [N,Co,H',W'] (already padded/dilated by the graph),
 *                                 w^T NCHW [Ci,Co,KH,KW], exp int8[1]}     out{dx NC4HW4 [N,Ci,H,W]}
 *  NITI_OP_GRADIENT_CONV_INT8 in {C4(x^T) NC4HW4 [Ci,N,H,W], dy^T NCHW [Co,N,OH',OW'], ...}
 *                             out{dw NC4HW4 [Ci,Co,KH,KW]}
 *  NITI_OP_MATMUL_INT8        in {B [M,K], A [Co,K]} (2-D, row major)      out{C [M,Co]}
 *  NITI_OP_DSP_MATMUL_GRADIENT_INT8
 *                             in {x NHWC [N,Ci,H,W], dy NHWC [N,Co,OH,OW]} out{dw HWIO [KH,KW,Ci,Co] as
 *                                 dims {KH,KW,Ci,Co}}
 *  NITI_OP_DSP_CONV_INT8, NITI_OP_DSP_DECONV_INT8
 *                             in {x NHWC [N,Ci,H,W], w HWIO as dims {KH,KW,Ci,Co}, exp_in int8[1],
 *                                 wscale int8[1]}                         out{y NHWC [N,Co,OH,OW], exp_out int8[1]}
 *                             (the deconv slot gets the graph's padded/dilated dy and rotated weights)
 *  NITI_OP_DSP_GRADIENTCONV_INT8, NITI_OP_DSP_MATMUL_INT8, NITI_OP_DSP_PARALLEL_GRADIENTCONV_INT8
 *                             as NITI_OP_DSP_MATMUL_GRADIENT_INT8, KH x KW from dw's dims
 *  NITI_OP_RELU_INT8, NITI_OP_RELUGRAD_INT8, NITI_OP_MAXPOOL_INT8, NITI_OP_POOLGRAD_INT8: as the DSP
 *                             slots below, on NC4HW4 (relu / relu grad also NCHW or NHWC) tensors
 *  NITI_OP_DSP_RELU_INT8 / NITI_OP_DSP_NOP_INT8 in {x NHWC} out{y NHWC}; NITI_OP_DSP_RELUGRAD_INT8
 *                             in {x, dy} out{dx}; common may be NULL for these three
 *  NITI_OP_DSP_MAXPOOL_INT8   in {x NHWC, ascale int8[1]} out{y NHWC, ascale int8[1]}; the pool's
 *                             kernel / stride / pad in the common's kernel_x/y, stride_x/y, pad_x/y
 *  NITI_OP_DSP_MAXPOOLGRAD_INT8 in {x, y, dy} NHWC out{dx NHWC}
 *  NITI_OP_DSP_MAXPOOLGRAD_REF_INT8 (806) in {x, y, dy} NHWC out{dx NHWC}: the reference's literal
 *                             walk (x read as [batch][height][width * channel], y / dy at
 *                             (offset * bc) / kernelX / kernelY, untouched bytes kept); kernel /
 *                             stride in the common; NOT_SUPPORT for stride < kernel or windows
 *                             past the tensor (order-dependent / out of bounds in the reference)
 *  NITI_OP_DSP_TRANSPOSE_INT8 in {x, perm int32[4] (device)} out{x permuted}; WEIGHTROTATE180 in {w}
 *                             out{w, raw axes 2, 3 reversed}; RESHAPE / RESHAPEGRAD in {x} out{same bytes};
 *                             all on the stored axis order ([N][H][W][C] for NHWC), common may be NULL
 *  NITI_OP_DSP_PAD_INT8       in {x NHWC} out{NHWC with a zero border of common.pad_x pixels}
 *  NITI_OP_PAD_INT8 (NCHW), NITI_OP_LEFTPOOLGRAD_INT8 (NC4HW4): the CPU graph's pad and stride
 *                             dilation, parameters as the DSP slots'
 *  NITI_OP_DSP_LEFTPOOLGRAD_DECONV_INT8 / _GRADIENT_INT8 in {dy NHWC} out{NHWC, dy[i][j] at
 *                             (stride_y*i, stride_x*j), zeros elsewhere}; stride in the common
 *  NITI_OP_LOSS_GRAD_INT8, NITI_OP_DSP_LOSSGRAD_INT8 (common may be NULL)
 *                             in {logits int8 [batch, classes], ascale int8[1], target int32 one-hot
 *                                 [batch, tc], dy (unused)} out{grad int8 [batch, classes]}; classes <= 2048
 *  NITI_OP_DSP_TRANSPOSEGRADIENT_CONV_INT8, NITI_OP_DSP_GRADIENT_SPLITBATCHCONV_INT8 (stride 1; the graph
 *                             dilates dy for stride 2)
 *                             in {x^T NHWC [Ci,N,H,W], dy NHWC [N,Co,OH,OW], 0, 0}
 *                             out{dw NHWC [Ci,Co,KH,KW] (kernel size from the shapes), exp_out int8[1] (optional)}
 * Output channel counts must be multiples of 4 on NC4HW4 outputs (the reference sizes its
 * int32 accumulator N*C*H*W but its GEMM writes ceil(C/4)*4 channels): NITI_NOT_SUPPORT. */
int niti_execution_resize(niti_execution_t e, const niti_tensor* inputs, int n_in, const niti_tensor* outputs,
                          int n_out);
/* Execution::onExecute on `stream`: asynchronous for device tensors; with any host tensor it stages
 * them and returns when the host outputs are written, and then also returns NITI_NO_EXECUTION if a
 * launch flagged its results invalid (the fused row kernel's grid barrier timed out: the grid was
 * not resident).  Replaces Execution::onExecute (execution-engine/source/core/Execution.hpp:24-82),
 * codes as ErrorCode.hpp:17-30. */
int niti_execution_execute(niti_execution_t e, const niti_tensor* inputs, int n_in, const niti_tensor* outputs,
                           int n_out, void* stream);
/* the asynchronous path's status: synchronizes `stream`, then NITI_NO_EXECUTION (and the flag
 * cleared) if a launch since the last check flagged invalid results, else NITI_NO_ERROR */
int niti_execution_status(niti_execution_t e, void* stream);
void niti_destroy_execution(niti_execution_t e);
/* bytes of device workspace the handle holds after resize */
size_t niti_execution_workspace_bytes(niti_execution_t e);
/* CPUTensorConverter::convert (source/backend/cpu/CPUTensorConvert.cpp:98-210) for int8 device
 * tensors: NCHW <-> NHWC <-> NC4HW4 (MNN CPU layout [ceil(C/4)][N][H][W][4], pad lanes written as
 * zero).  src and dst have the same logical dims {N, C, H, W}; asynchronous on `stream`.
 * COMPUTE_SIZE_ERROR on a dims mismatch, NOT_SUPPORT on another format, INVALID_VALUE on NULL or
 * in-place buffers. */
int niti_tensor_convert(const niti_tensor* src, const niti_tensor* dst, void* stream);

/* ============================ 2. native split primitives ============================== */
/* A range estimate (max|acc| of one tensor, NITI_RangeEstimate's input, CommonOptFunction.cpp:
 * 1565-1576) is carried in a buffer of NITI_MAX_WORDS uint32 words that the caller zeroes before
 * the producing call.  Producers atomically max into one of 64 slots (one per 128-byte line,
 * word 32*i), spreading the atomics; the value is the max over the slots, which is what every
 * consumer below reads.  An all-reduce (MAX) over the whole buffer of every rank gives the
 * global range in data-parallel exact mode. */
#define NITI_MAX_WORDS 2048
/* Native layouts (padded lanes zero): NHWC16 [N][H][W][round16(C)]; CHWN16 [round16(C)][H][W]
 * [round16(N)]; OHWI16 weights [Co][KH][KW][round16(Ci)]; IHWO16 [Ci][KH][KW][round16(Co)]. */
typedef struct niti_geom {
    int n, c_in, h, w, c_out, kh, kw;
    int stride_h, stride_w, pad_t, pad_l, pad_b, pad_r, dilate_h, dilate_w;
    int oh, ow, cip, cop, np; /* filled by niti_geom_finalize */
} niti_geom;

int niti_geom_finalize(niti_geom* g);

/* Device workspace (bytes) an op needs to split K over workgroups when its output has too
 * few tiles for 256 CUs (op 0 forward, 1 input gradient, 2 weight gradient).  Passing less
 * (or NULL) is allowed: the op then runs unsplit. */
int niti_conv_workspace_bytes(const niti_geom* g, int op, size_t* bytes);
/* The plan a conv GEMM of geometry g runs with under a workspace of ws_bytes (op 0 forward,
 * 1 input gradient, 2 weight gradient): info = {bm, bn, splits, strategy}; bm = bn = 32 is the
 * tap-sharing weight-gradient kernel (stride-1 3x3, Cip % 32 == 0, Cop % 64 == 0). */
int niti_conv_plan_info(const niti_geom* g, int op, size_t ws_bytes, int info[4]);
/* Force the plan a conv GEMM of geometry g runs with (op 0 forward, 1 input gradient, 2 weight
 * gradient; plan as niti_model_plan_set, NULL restores the default); niti_conv_workspace_bytes then
 * reports the workspace the forced plan needs.  Per process, keyed by GEMM shape (what the host-
 * driven ResNet-18 step's autotuner uses). */
int niti_conv_plan_set(const niti_geom* g, int op, const int plan[4]);
int niti_matmul_workspace_bytes(int m, int ldc, int k16, size_t* bytes);
/* acc[n*oh*ow][cop] int32 = conv(x, w); if amax (NITI_MAX_WORDS words): range max-ed in */
int niti_conv_fwd_acc(const niti_geom* g, const int8_t* x_nhwc16, const int8_t* w_ohwi16, int32_t* acc,
                      uint32_t* amax, void* workspace, size_t workspace_bytes, void* stream);
/* acc[n*h*w][cip] int32 = input gradient of the conv for dy (NHWC16) and w^T (IHWO16) */
int niti_conv_dgrad_acc(const niti_geom* g, const int8_t* dy_nhwc16, const int8_t* wt_ihwo16, int32_t* acc,
                        uint32_t* amax, void* workspace, size_t workspace_bytes, void* stream);
/* Two-phase forward / input-gradient conv with the NITI requantisation (NITI_Conv_Int8.cpp:255-307,
 * NITI_DeConv_Int8.cpp:294-329), the training step's path: phase 1 puts max|acc| into amax (zeroed
 * by the caller) -- materialising acc, or, for small K, computing the range only; a data-parallel
 * caller all-reduces amax (MAX) between the phases; phase 2 writes out_nhwc16 = requant(acc) (+ relu,
 * relu_mask as niti_requant_act) and exp_out, recomputing the GEMM where phase 1 stored nothing.
 * acc ([rows][cop] / [rows][cip] int32) and the workspace size must be the same in both calls. */
int niti_conv_fwd_phase1(const niti_geom* g, const int8_t* x_nhwc16, const int8_t* w_ohwi16, int32_t* acc,
                         uint32_t* amax, void* workspace, size_t workspace_bytes, void* stream);
int niti_conv_fwd_phase2(const niti_geom* g, const int8_t* x_nhwc16, const int8_t* w_ohwi16, const int32_t* acc,
                         const uint32_t* amax, const int8_t* exp_in, const int8_t* wscale, int8_t* exp_out, int relu,
                         const int8_t* relu_mask, int8_t* out_nhwc16, size_t workspace_bytes, void* stream);
int niti_conv_dgrad_phase1(const niti_geom* g, const int8_t* dy_nhwc16, const int8_t* wt_ihwo16, int32_t* acc,
                           uint32_t* amax, void* workspace, size_t workspace_bytes, void* stream);
int niti_conv_dgrad_phase2(const niti_geom* g, const int8_t* dy_nhwc16, const int8_t* wt_ihwo16, const int32_t* acc,
                           const uint32_t* amax, const int8_t* exp_in, const int8_t* wscale, int8_t* exp_out,
                           int relu, const int8_t* relu_mask, int8_t* out_nhwc16, size_t workspace_bytes,
                           void* stream);
/* Register-fed forward conv of stride-1 pad-1 3x3 layers with the NITI rescale fused
 * (niti_rowconv.hip; square images of 2, 4, 8 or 16 pixels, c_out padded to 16 a multiple of 32):
 * activations in C32 [n][ceil(C/32)][H][W][32], weights in WF [Co/32][Ci/32][9][2][32][16] (one
 * 1 KiB MFMA fragment per co block, ci block and tap).  mode 0: one launch, max|y| reduced by an
 * in-kernel grid barrier (state: NITI_ROWCONV_STATE_WORDS u32 zeroed once; epoch 1, 2, 3, ... one per
 * call in stream order; err u32 set to 1 if the barrier ever timed out); mode 1: max|y| into amax
 * (zeroed by the caller); mode 2: recompute and requantise with amax (a data-parallel caller
 * all-reduces amax between modes 1 and 2).  Outputs: out_nhwc16 [n][H][W][cop] = relu?(requant(y)),
 * pool_out_nhwc16 (may be NULL) its 2x2 max pool, next_c32 (may be NULL) the (pooled) output as the
 * next layer's C32 input; exp_out = exp_in + wscale + inc.  Modes 3 and 4, the speculative pair
 * (state required; both calls with the same outputs and amax): mode 3 multiplies, requantises with
 * the bit width this state's layer had at its previous mode-4 call and publishes max|y| into amax;
 * mode 4 (after the caller's all-reduce of amax, if any) writes exp_out and redoes the launch only
 * if max|y|'s bit width differs from that guess -- the results are modes 1 + 2's, at one GEMM pass
 * when the bit width holds from step to step. */
#define NITI_ROWCONV_STATE_WORDS 1216
/* the speculative pair's slot of a state (dgrad 0 forward, 1 input gradient): u32 [0] the hint (the
 * bit width on the input's scale: bw + 1 + exp_in + wscale + 512, 0 none), [1] the guess (bw + 1) the
 * last mode-3 call used, [2] the mode-4 calls that redid */
uint32_t* niti_rows_spec_slot(uint32_t* state, int dgrad);
int niti_conv_rows_ok(const niti_geom* g);
int niti_nhwc16_to_c32(const int8_t* in_nhwc16, int n, int hw, int cp, int c, int8_t* out_c32, void* stream);
int niti_weights_to_wf(const int8_t* w_ohwi16, int co, int ci, int cip, int transpose, int8_t* out_wf,
                       void* stream);
/* mode | NITI_ROWS_X_NHWC16 (niti_conv_fwd_rows / niti_conv_dgrad_rows): the input (x, or dy) is NHWC16
 * [n][H][W][cip] instead of C32 -- the row-segment maps (niti_conv_rows_nhwc_ok: 14-px multiples
 * above 16 px, or 14 px; cip % 32 == 0) read it in place, with no C32 copy */
#define NITI_ROWS_X_NHWC16 0x100
/* flags bit 0: the input gradient's input (dy) instead of the forward's x; bit 1: whether the
 * library's own step prefers it over a C32 copy (64-channel inputs), not only whether it works */
int niti_conv_rows_nhwc_ok(const niti_geom* g, int flags);
int niti_conv_fwd_rows(const niti_geom* g, const int8_t* x_c32, const int8_t* wf, const int8_t* exp_in,
                       const int8_t* wscale, int8_t* exp_out, int relu, int8_t* out_nhwc16, int8_t* pool_out_nhwc16,
                       int8_t* next_c32, int mode, uint32_t* amax, uint32_t* state, uint32_t epoch, uint32_t* err,
                       void* stream);
/* The input gradient of that conv on the same kernel (NITI_DeConv_Int8.cpp:294-329 with the next
 * op's backward fused): g is the LAYER's geometry; dy_c32 its output gradient in C32, wft the
 * rotated transposed weights (niti_weights_to_wf with transpose = 1); the int32 gradient is
 * requantised by the forward rule (no exponent, no relu) and then either masked by the previous
 * layer's relu (relu_mask NHWC16 [n][H][W][cip]: dx = mask > 0 ? q : 0) into dx_nhwc16, or -- pool_x
 * non-NULL -- routed through the previous layer's 2x2 max pool (pool_x [n][2H][2W][cip] its input,
 * pool_y [n][H][W][cip] its output; pool_relu: zero where pool_x <= 0) into dx_nhwc16 at 2H x 2W.
 * dx_c32 (may be NULL) is the same gradient in C32 (the previous layer's dy_c32), dx_p16 (may be NULL)
 * in the weight gradient's P16 layout [pixels/16][cip][16] (NITI_NOT_SUPPORT where a launch's pixels
 * do not make whole 16-pixel blocks: 4x4 images without the pool at small batches).  exp_out (may be
 * NULL) = exp_in + wscale + the rule's increment, as the forward (NITI_DeConv_Int8 has no exponent
 * output; callers that track gradient exponents, e.g. a residual network, read it here).  mode, amax,
 * state, epoch and err as niti_conv_fwd_rows. */
int niti_conv_dgrad_rows(const niti_geom* g, const int8_t* dy_c32, const int8_t* wft, const int8_t* relu_mask,
                         const int8_t* pool_x, const int8_t* pool_y, int pool_relu, int8_t* dx_nhwc16, int8_t* dx_c32,
                         int8_t* dx_p16, const int8_t* exp_in, const int8_t* wscale, int8_t* exp_out, int mode,
                         uint32_t* amax, uint32_t* state, uint32_t epoch, uint32_t* err, void* stream);
/* acc[co][kh][kw][cip] int32 = weight gradient for x (NHWC16) and dy (NHWC16): a K-major GEMM
 * over the pixels whose operand tiles are transposed in LDS (ds_read_b64_tr_b8) */
int niti_conv_wgrad_acc(const niti_geom* g, const int8_t* x_nhwc16, const int8_t* dy_nhwc16, int32_t* acc,
                        uint32_t* amax, void* workspace, size_t workspace_bytes, void* stream);
/* P16 pixel blocks: an activation of P pixels (P % 16 == 0) and Cp channels as [P/16][Cp][16], so the
 * 16 consecutive pixels of one channel are 16 contiguous bytes -- the MFMA operand fragment of the
 * weight gradient, loaded straight into registers. */
int niti_nhwc16_to_p16(const int8_t* in_nhwc16, int64_t pixels, int cp, int8_t* out_p16, void* stream);
/* Weight gradient on P16 operands (3x3, stride 1, pad 1, Cip % 32 == 0, Cop % 32 == 0, n*oh*ow % 32 == 0,
 * ow in {2, 4, 8, 16} with oh = ow for 2 and 4, oh even for 8):
 * acc[co][kh][kw][cip] int32 (rows < c_out written) and, if amax, its range.  splits <= 0 picks the
 * default.  The workspace holds the split-K partials (niti_conv_wgrad_p16_workspace bytes, 0 without a
 * split).  NOT_SUPPORT for other geometries. */
int niti_conv_wgrad_p16_workspace(const niti_geom* g, int splits, size_t* bytes);
/* diagnostics: device buffer (8 u64 per block) for the per-block stamps of stamp builds; NULL disarms */
void niti_diag_wgrad_stamps(void* buf);
/* diagnostics: device buffer (8 u64 per wave) for the register-fed conv's per-wave stamps; NULL disarms */
void niti_diag_rowconv_stamps(void* buf);
/* diagnostics: the fused row kernel's barrier poll limit (0 = default) and a number of arrivals it
 * waits for that never come (> 0 forces a timeout, to test the error plumbing) for later launches */
void niti_diag_rowconv_barrier(uint32_t spin_limit, uint32_t expect_extra);
/* the fused row kernel's speculative epilogue for later launches: 1 on (the previous launch's bit width
 * is applied while the grid barrier completes, the epilogue redone if it differs), 0 off (default:
 * measured slower), 2 always guess wrong (every launch redoes its epilogue).  Results are identical
 * in every mode. */
void niti_diag_rowconv_speculate(int mode);
/* diagnostics: launch A of every GEMM speculative pair (plan strategy 3) guesses the layer's previous
 * bit width + bias: +-1 makes launch B settle from an alternate, 2 makes it redo the GEMM (tests);
 * 0 (default) off.  Results are the rule's whatever the bias. */
void niti_diag_gemm_speculate(int bias);
/* diagnostics: implicit-GEMM launches of this process that ran with the rescale fused behind the
 * in-kernel grid barrier (plan strategy 4) */
unsigned long long niti_diag_gemm_fused_launches(void);
/* diagnostics: launches of the classifier head's one-launch chain (forward, loss gradient, weight and
 * input gradient) in this process */
unsigned long long niti_diag_head_chain_launches(void);
/* diagnostics: VGG-11's classifier head as one launch (forward, loss gradient, weight gradient, input
 * gradient through the pool routes; niti_head.hip) instead of four; 0 (default, measured slower) off.
 * Also NITI_HEAD_CHAIN=1.  Results identical either way. */
void niti_diag_head_chain(int on);
/* jobs per P16 input-copy launch of a model step for later steps (<= 0: the default 16); a small
 * cap sends a step down its more-than-one-launch branches.  Results are identical for every cap. */
void niti_diag_p16_jobs_cap(int cap);
int niti_conv_wgrad_p16_acc(const niti_geom* g, const int8_t* x_p16, const int8_t* dy_p16, int32_t* acc,
                            uint32_t* amax, void* workspace, size_t workspace_bytes, int splits, void* stream);
/* acc[m][ldc] = sum_k B[m][k] A[o][k] (columns o..ldc = 0); K zero padded to k16; ldb/lda bytes */
int niti_matmul_acc(int m, int o, int k16, const int8_t* B, int64_t ldb, const int8_t* A, int64_t lda,
                    int32_t* acc, int64_t ldc, uint32_t* amax, void* workspace, size_t workspace_bytes,
                    void* stream);
int niti_absmax_i32(const int32_t* acc, int64_t n, uint32_t* amax, void* stream);
/* forward/deconv rule (NITI_Conv_Int8.cpp:260-307) on acc[rows][ldc]; exp_out = exp_in + wscale + inc
 * (any exponent pointer may be NULL); relu fuses NITI_Relu_Int8; relu_mask (NHWC16) fuses
 * NITI_ReluGrad_Int8.  out_nhwc16 [rows][ldc]. */
int niti_requant_act(const int32_t* acc, int64_t rows, int ldc, const uint32_t* amax, const int8_t* exp_in,
                     const int8_t* wscale, int8_t* exp_out, int relu, const int8_t* relu_mask, int8_t* out_nhwc16,
                     void* stream);
/* gradient rules: rule 2 = NITI_GradientConv_Int8 (bw-2), rule 3 = NITI_Matmul_Int8 (bw-3);
 * g_out optional; w_update optional fused NITI_SGD step w <- clip(w - g, +-127). */
int niti_requant_grad(const int32_t* acc, int64_t n, const uint32_t* amax, int rule, int8_t* g_out,
                      int8_t* w_update, void* stream);
/* Fused NITI_SGD step for one layer: g = rule(acc [co][kk][cip], amax), w <- clip(w - g, +-127)
 * on the OHWI16 weights, the updated weights also written to wt (IHWO16, may be NULL) and g to
 * g_out (OHWI16, may be NULL). */
int niti_sgd_update(const int32_t* acc, const uint32_t* amax, int rule, int co, int ci, int kk, int cip, int cop,
                    int8_t* w_ohwi16, int8_t* wt_ihwo16, int8_t* g_out, void* stream);
/* the same, also rewriting the row kernels' fragment-major copies of a 3x3 layer (niti_weights_to_wf:
 * wf the forward's, wft the input gradient's; either may be NULL; ci, co multiples of 32) in the same
 * pass -- no separate weights_to_wf launches after the update */
int niti_sgd_update_wf(const int32_t* acc, const uint32_t* amax, int rule, int co, int ci, int kk, int cip, int cop,
                       int8_t* w_ohwi16, int8_t* wt_ihwo16, int8_t* g_out, int8_t* wf, int8_t* wft, void* stream);
/* layout helpers */
int niti_nhwc16_to_chwn16(const int8_t* in, int n, int hw, int cp, int np, int8_t* out, void* stream);
int niti_ohwi16_to_ihwo16(const int8_t* w, int co, int ci, int kk, int cip, int cop, int8_t* wt, void* stream);
int niti_nchw_to_nhwc16(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, void* stream);
int niti_nchw_to_chwn16(const int8_t* x, int n, int c, int hw, int cp, int np, int8_t* out, void* stream);
int niti_nhwc16_to_nchw(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, void* stream);
int niti_oihw_to_ohwi16(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, void* stream);
int niti_ohwi16_to_oihw(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, void* stream);
/* rest of the step, NHWC16 */
/* ResNet pieces (niti_resnet.hip; the reference's NITI_Eltwise_Int8 is an empty stub,
 * NITI_Eltwise_Int8.cpp:20-28, so the rule is this library's): z = hi * 2^d + (lo >> r) with
 * d = min(|ea - eb|, 23), r = |ea - eb| - d, hi the operand of the larger exponent (a on ties);
 * *ez = e_hi - d; max|z| into amax.  n % 16 == 0; requantise z with niti_requant_act. */
int niti_residual_add(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n, int32_t* z,
                      int8_t* ez, uint32_t* amax, void* stream);
/* the fused form: with z = NULL above (range only; a data-parallel caller MAX-reduces amax next),
 * out[n] int8 = the forward rule on z recomputed from a and b (+ relu), exactly as niti_requant_act
 * on the stored z; *ez = e_hi - d and *exp_out = *ez + inc (either may be NULL). */
int niti_residual_requant(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                          const uint32_t* amax, int8_t* ez, int8_t* exp_out, int relu, int8_t* out, void* stream);
/* the same (no relu), followed by the next op's relu gradient: out = relu_mask > 0 ? q : 0 (the
 * backward residual sum of a block, masked by the previous block's output, NITI_ReluGrad_Int8) */
int niti_residual_requant_relu_grad(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                                    const uint32_t* amax, int8_t* ez, int8_t* exp_out, const int8_t* relu_mask,
                                    int8_t* out, void* stream);
/* global sum pool: acc[img][c] = sum over hw pixels of x NHWC16 [n][hw][cp] (+ max into amax) */
int niti_sum_pool(const int8_t* x, int n, int hw, int cp, int32_t* acc, uint32_t* amax, void* stream);
/* its gradient: dx[img][p][c] = dy[img][c] */
int niti_sum_pool_grad(const int8_t* dy, int n, int hw, int cp, int8_t* dx, void* stream);
/* im2col of a shallow NHWC16 input (c_in <= 4; the ResNet-18 stem) for a conv run as a 1x1 conv over
 * kp columns (kp % 16 == 0, kp >= kh * kw * c_in): xcol [n * oh * ow][kp], column k = (ky * kw + kx) *
 * c_in + c, zero beyond kh * kw * c_in and outside the image (the weight [co][kp] in the same order). */
int niti_im2col(const niti_geom* g, const int8_t* x, int kp, int8_t* xcol, void* stream);
/* the same from an int8 NCHW input [n][c_in][h][w] (niti_image_quantize's output) */
int niti_im2col_nchw(const niti_geom* g, const int8_t* x_nchw, int kp, int8_t* xcol, void* stream);
int niti_maxpool(const int8_t* x, int n, int h, int w, int cp, int k, int s, int p, int8_t* y, int oh, int ow,
                 void* stream);
int niti_maxpool_grad(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h, int w, int cp, int k,
                      int s, int p, int oh, int ow, int relu, int8_t* dx, void* stream);
/* the same gradient in two passes over a caller workspace of n*oh*ow*cp bytes (each window's
 * first-max position, then a gather per input pixel); equal results, for overlapping windows */
int niti_maxpool_grad_ws(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h, int w, int cp, int k,
                         int s, int p, int oh, int ow, int relu, int8_t* workspace, int8_t* dx, void* stream);
int niti_relu_grad(const int8_t* x, const int8_t* dy, int64_t n, int8_t* out, void* stream);
int niti_loss_grad(const int8_t* logits, int batch, int classes, int ld, const int8_t* ascale,
                   const int32_t* labels, int8_t* out, void* stream);

/* NITIInt8Train's input quantiser (execution-engine/tools/train/source/demo/MnistUtils.cpp:83-93):
 * mean / std / range of the uint8 batch, x = round((p - mean) / std / range * 127), ascale =
 * int8(ceilf(logf(range)) - 7) in float.  The variance divisor is the reference's literal
 * batchSize * 28 * 28 (:86), batchSize = count / (c * hw) images, for every image size.  Split so data-parallel ranks can all-reduce the statistics:
 * stats (4 x uint64, device) = {sum p, sum p^2 (SUM over ranks), max p, 255 - min p (MAX)};
 * count = pixels the statistics cover (all ranks').  The float contract (exact integer
 * statistics, the per-pixel formula in the reference's operation order) is stated in
 * csrc/niti_quant.hip.  out_nchw int8 [n][c][hw]; ascale int8 device scalar (may be NULL). */
int niti_image_stats(const uint8_t* images_nchw, int64_t n, uint64_t* stats, void* stream);
int niti_image_quantize(const uint8_t* images_nchw, int n, int c, int hw, const uint64_t* stats, int64_t count,
                        int8_t* out_nchw, int8_t* ascale, void* stream);
/* the same, x written as NHWC16 [n][hw][cp] (cp % 16 == 0, pad channels 0): a conv's input layout */
int niti_image_quantize_nhwc16(const uint8_t* images_nchw, int n, int c, int hw, int cp, const uint64_t* stats,
                               int64_t count, int8_t* out_nhwc16, int8_t* ascale, void* stream);

/* ============================ 3. device-resident training step ========================= */
/* LeNet on MNIST 1x28x28 (cfg 1/2); VGG-11 on CIFAR 3x32x32 (cfg 3); VGG-16 on ImageNet 3x224x224
 * with the 4096-4096-1000 head (cfg 4; niti_model_create2 takes another input size, a multiple
 * of 32, e.g. 32 for the oracle-checked tests); ResNet-18 on ImageNet 3x224x224 (cfg 5: 21
 * parameter layers in the order conv1, per basic block conv a / conv b / [1x1 projection], fc; the
 * residual and global-pool rules are this library's -- the reference's NITI_Eltwise_Int8 is a stub,
 * NITI_Eltwise_Int8.cpp:20-28 -- stated in csrc/niti_resnet.hip and oracle/niti_resnet_ref.py). */
enum niti_arch { NITI_ARCH_LENET = 1, NITI_ARCH_VGG11 = 2, NITI_ARCH_VGG16 = 3, NITI_ARCH_RESNET18 = 4 };
typedef struct niti_model* niti_model_t;

/* batch = this rank's images per step.  Weights start zero; load them with
 * niti_model_set_weight (OIHW int8, host memory) -- the reference initialises them with a
 * time-seeded RNG (nn/Distributions.cpp:26-51), so callers supply their own. */
int niti_model_create(int arch, int batch, niti_model_t* out);
/* The same with the input resolution (in_hw x in_hw; 0 = the architecture's default). */
int niti_model_create2(int arch, int batch, int in_hw, niti_model_t* out);
/* ... and the class count of the head (0 = the architecture's: 10 LeNet / VGG-11, 1000 VGG-16 /
 * ResNet-18; only ResNet-18 takes another, <= 2048) */
int niti_model_create3(int arch, int batch, int in_hw, int classes, niti_model_t* out);
void niti_model_destroy(niti_model_t m);
int niti_model_num_layers(niti_model_t m);
/* per layer: {c_in, c_out, kh, kw, h_in, w_in, oh, ow, pad, stride, relu, pool} */
int niti_model_layer_info(niti_model_t m, int layer, int info[12]);
int niti_model_set_weight(niti_model_t m, int layer, const int8_t* w_oihw_host, int wscale);
int niti_model_get_weight(niti_model_t m, int layer, int8_t* w_oihw_host);
/* One NITI_SGD step: forward, NITI_LOSS_Grad, backward, w <- clip(w - g).
 * x: NCHW int8 device [batch][C][H][W]; labels: int32 device [batch]; exp_in: input ascale.
 * Asynchronous on `stream`. */
int niti_model_train_step(niti_model_t m, const int8_t* x_nchw, int exp_in, const int32_t* labels, void* stream);
/* The same step from uint8 images [batch][C][H][W] (device): the input quantiser
 * (niti_image_stats / niti_image_quantize, statistics all-reduced in exact data-parallel mode)
 * runs on device first and supplies x and exp_in -- NITIInt8Train's whole per-batch work. */
int niti_model_train_step_images(niti_model_t m, const uint8_t* images_nchw, const int32_t* labels, void* stream);
/* Read back (synchronising): the step's quantised input x (NCHW int8) and its exponent. */
int niti_model_get_input(niti_model_t m, int8_t* x_nchw_host, int* ascale, void* stream);
/* Read back (synchronising `stream`): logits [batch][classes] int8 and their exponent. */
int niti_model_get_logits(niti_model_t m, int8_t* logits_host, int* exp_out, void* stream);
/* Per-layer debug taps (synchronising): which = 0 fwd output (post relu, pre pool, NCHW),
 * 1 int8 weight gradient (OIHW), 2 dy of the layer (NCHW, post relu/pool grad). */
int niti_model_get_tap(niti_model_t m, int layer, int which, int8_t* host, size_t bytes, void* stream);
/* Algorithmic int8 MACs per step (unpadded channels; no zero-dilation taps). */
int64_t niti_model_step_macs(niti_model_t m);

/* Keep each step's int8 weight gradient for niti_model_get_tap(which = 1) (default 1).  With 0 the
 * SGD kernel updates the weights from the int32 gradient without storing the int8 copy, and the
 * tap returns NITI_INVALID_VALUE; likewise ResNet-18's stem, whose requantise pass max-pools in
 * the same pass, then writes no pre-pool output (its which = 0 tap returns NITI_INVALID_VALUE). */
int niti_model_keep_grads(niti_model_t m, int enable);
/* Forward convs and input gradients of the stride-1 pad-1 3x3 layers on the register-fed kernel
 * with the rescale fused (niti_rowconv.hip; default 1), or on the LDS-staged GEMM + requantisation
 * passes (0).  Results are identical.  niti_model_rowconv_error: 1 if an in-kernel grid barrier
 * ever timed out (synchronises). */
int niti_model_set_rowconv(niti_model_t m, int enable);
int niti_model_rowconv_error(niti_model_t m);
/* the speculative row-kernel pairs' counters per layer (max_layers x 6 u32): forward hint (bit
 * width + 1), forward launches redone, forward pairs in store mode, then the same for the input
 * gradient (niti_rows_spec_slot; synchronises) */
int niti_model_spec_stats(niti_model_t m, uint32_t* out, int max_layers);
/* diagnostics: the 32 words of one row-kernel layer's speculative slot (niti_rows_spec_slot), with
 * the last 6 pairs' record (bw, input scale, guess) in words 26.. (synchronises) */
int niti_model_spec_slot(niti_model_t m, int layer, int dgrad, uint32_t* out32);
/* Replay the step as a hipGraph (single device only -- with a communicator attached the step
 * always runs as direct launches).  Default 0 (direct launches: measured faster on ROCm 7.2). */
int niti_model_set_graph(niti_model_t m, int enable);
/* Run the weight gradients on a second HIP stream, overlapping the input-gradient chain
 * (default 1; the update waits for both).  With a communicator every collective is still
 * issued on the step stream, in program order, through one communicator. */
int niti_model_set_overlap(niti_model_t m, int enable);
/* Per-shape GEMM plan autotuning (no counterpart in the reference, whose CPU kernels have a
 * fixed blocking, NITI_Conv_Int8.cpp:159-253): times every layer phase under candidate plans
 * (tile shape, store / recompute / split-K count) on `stream` and keeps the fastest for this
 * process.  Plans never change results.  Call after one train_step (it reuses that step's
 * buffers); weights are not touched.  reps <= 0 uses 5.  Synchronises `stream`. */
int niti_model_autotune(niti_model_t m, int reps, void* stream);
/* The plan a layer phase (0 forward, 1 input gradient, 2 weight gradient) runs with:
 * {bm, bn, splits, strategy 0 store / 1 recompute / 2 split-K / 3 the speculative pair (forward and
 * input gradient, unsplit: launch A requantises with the layer's previous bit width and publishes the
 * range, launch B redoes the GEMM only when the range's bit width differs) / 4 fused (forward and
 * stride-1 input gradient, unsplit: one launch whose blocks keep their accumulators in registers
 * across an in-kernel grid barrier carrying the tensor's bit width, then requantise -- where every
 * tile is resident at once and no collective sits between range and requantisation; elsewhere it
 * runs as 1)}. */
int niti_model_plan_info(niti_model_t m, int layer, int phase, int info[4]);
/* Force a plan for a layer phase ({bm 64|128, bn 64|128, splits >= 1, strategy}; split counts
 * beyond the K steps or the workspace are clamped; recompute on the weight gradient means
 * store); plan = NULL restores the default.  Overrides are per process, keyed by GEMM shape. */
int niti_model_plan_set(niti_model_t m, int layer, int phase, const int plan[4]);
/* Drop every plan override of the process (autotuned or forced). */
void niti_plan_reset(void);
/* Kernel probe: HIP events on the step's stream around one GEMM launch (layer, phase
 * 0 = forward, 1 = input gradient, 2 = weight gradient) for up to max_launches steps;
 * layer < 0 disables.  probe_read synchronises those events and returns the summed
 * duration and the number of launches timed, then resets the count. */
int niti_model_set_probe(niti_model_t m, int layer, int phase, int max_launches);
int niti_model_probe_read(niti_model_t m, double* total_ms, int* count);
/* paused != 0: the armed probe skips the next launches (no events, no span slot) until resumed;
 * a host flag, so a timed loop can time the probed launch in some of its steps only */
int niti_model_probe_pause(niti_model_t m, int paused);
/* Weight-gradient probes (phase 2) also time the launch from inside: the kernel min-es its
 * blocks' start and max-es their end on the device wall clock (s_memrealtime); this returns the
 * summed first-block-start -> last-block-end spans and their count, then re-arms. */
int niti_model_probe_read_span(niti_model_t m, double* total_ms, int* count);
/* Runs one layer phase of the last step again on `stream` (phase 0 forward, 1 input gradient,
 * 2 weight gradient; buffers as the step left them, weights untouched), single-device and
 * without the side stream: the isolated measurement next to the in-step probe. */
int niti_model_run_phase(niti_model_t m, int layer, int phase, void* stream);

/* ---- data parallel over RCCL (xGMI) ---------------------------------------------------- */
#define NITI_UNIQUE_ID_BYTES 128
/* rank 0 creates the id; every rank receives it out of band (torch.distributed store). */
int niti_dp_get_unique_id(char id[NITI_UNIQUE_ID_BYTES]);
/* Attach an RCCL communicator (one per model; all its collectives go on the step stream in
 * program order): exact mode all-reduces the input quantiser's statistics (SUM / MAX), every
 * forward and input-gradient range (MAX) and every int32 weight-gradient accumulator (SUM), so
 * N ranks of batch b are bit-identical to one device of batch N*b.  exact=0 keeps the
 * statistics and ranges shard-local (not parity; the gradient SUM stays). */
int niti_model_attach_comm(niti_model_t m, const char id[NITI_UNIQUE_ID_BYTES], int rank, int world, int exact);

/* In-process rank group on ONE device (tests and single-GPU rehearsal of the protocol): each
 * of `world` host threads drives one model attached with its rank; every collective
 * synchronises the caller's stream and the last rank to arrive reduces all ranks' buffers on
 * the device.  Same calls, order and streams as the RCCL path; no second GPU needed. */
typedef struct niti_local_group* niti_local_group_t;
int niti_local_group_create(int world, niti_local_group_t* out);
void niti_local_group_destroy(niti_local_group_t g);
int niti_model_attach_local(niti_model_t m, niti_local_group_t g, int rank, int exact);

/* library build info */
const char* niti_version(void);

#ifdef __cplusplus
}
#endif
#endif /* NITI_HIP_H */
