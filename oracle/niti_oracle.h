/*
 * niti_oracle.h -- CPU restatement of the reference NITI int8 training path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the HIP library under
 * mandheling-dsp-training_amd/) links, loads or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker.
 *
 * PARITY STATUS: parity unpinned.  The reference holds no test, golden vector or
 * fixture for any NITI op, and running the reference was denied
 * (SURVEY.md §8(c)).  This restatement is anchored by (1) the hand-derived
 * known-answer tests of SURVEY.md Appendix A, and (2) agreement between two
 * independent restatements: a naive NCHW exact-integer path and a path that
 * follows the reference's own data flow (MNN C4 layout, per-call weight reorder,
 * 4-pixel im2col tiles, 16x4 GEMM unit, the grad graph's transposes, pads,
 * stride-2 dilation and rot180).
 *
 * Arithmetic contract: the reference GEMM accumulates int8
 * products in float32 (execution-engine/source/backend/cpu/compute/
 * Int8FunctionsOpt.cpp:201-232) under -ffast-math, so its only well-defined
 * meaning is the exact integer sum, which it reproduces bit for bit whenever
 * sum|x_i*w_i| < 2^24 for an output.  The oracle accumulates exactly (int64) and
 * counts outputs past that bound ("guard") and outputs outside int32 ("overflow").
 *
 * Undefined shifts: the reference computes (1 << shift) with shift < 0 for the
 * weight-gradient rule when the range estimate is 1 (NITI_GradientConv_Int8.cpp:288)
 * and for the matmul rule when it is 1 or 2 (NITI_Matmul_Int8.cpp:222).  The oracle
 * pins those cases to what x86-64 executes for a variable shift (count & 31, int32
 * wrap-around) -- see niti_ref_pow2().
 */
#ifndef NITI_ORACLE_H
#define NITI_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- scalar helpers: CommonOptFunction.cpp:1548-1627 ---------------- */
int32_t niti_ref_int8_clip(int32_t a);                     /* :1548-1555, clips to [-127,127] */
int32_t niti_ref_sign(int32_t a);                          /* :1556-1563 */
int32_t niti_ref_pow2(int32_t s);                          /* (1 << s) as x86-64 executes it */
int32_t niti_ref_range_estimate(const int32_t* a, int64_t n);      /* :1565-1576, integer form */
int32_t niti_ref_range_estimate_libm(const int32_t* a, int64_t n); /* :1565-1576, literal ceil(log2()) */
int32_t niti_ref_psto1(int32_t a, int32_t shift);                  /* one element of :1595-1627 */
void niti_ref_psto_shift(const int32_t* in, int32_t shift, int32_t* out, int64_t n); /* :1595-1627 */

/* ---------------- requantisation rules ---------------- */
/* NITI_Conv_Int8.cpp:255-307 / NITI_DeConv_Int8.cpp:292-329.  Returns the exponent
 * increment (shift, 2 or 0) that NITI_Conv_Int8 adds to exp_in + wscale. */
int32_t niti_ref_requant_fwd(const int32_t* acc, int64_t n, int8_t* out);
/* NITI_GradientConv_Int8.cpp:272-296: bw==0 -> zeros, else PSTO(bw-2). Returns bw. */
int32_t niti_ref_requant_wgrad(const int32_t* acc, int64_t n, int8_t* out);
/* NITI_Matmul_Int8.cpp:214-228: bw==0 -> zeros, else PSTO(bw-3). Returns bw. */
int32_t niti_ref_requant_matmul(const int32_t* acc, int64_t n, int8_t* out);

/* ---------------- convolution geometry ---------------- */
typedef struct niti_ref_geom {
    int n, c_in, h, w;          /* input  NCHW */
    int c_out, kh, kw;          /* weight OIHW */
    int stride_h, stride_w;
    int pad_t, pad_l, pad_b, pad_r;
    int dilate_h, dilate_w;
    int oh, ow;                 /* filled by niti_ref_geom_finalize */
} niti_ref_geom;

/* output size: ShapeNITI_Conv_Int8.cpp:58-76 (Caffe pads) */
int niti_ref_geom_finalize(niti_ref_geom* g);

typedef struct niti_ref_stats {
    int64_t guard;      /* outputs with sum|x*w| >= 2^24 (reference float accumulation not exact) */
    int64_t overflow;   /* outputs whose exact sum leaves int32 */
} niti_ref_stats;

/* ---------------- naive exact-integer restatement (NCHW / OIHW) ---------------- */
/* acc[n][co][oy][ox] = sum_{ci,ky,kx} x[n][ci][iy][ix] * w[co][ci][ky][kx]   (NITI_Conv_Int8.cpp:162-249) */
/* threads used by the naive restatement (results do not depend on it; default 1) */
void niti_ref_set_threads(int threads);
void niti_ref_conv_fwd_acc(const niti_ref_geom* g, const int8_t* x, const int8_t* w, int32_t* acc,
                           niti_ref_stats* st);
/* acc[co][ci][ky][kx] = sum_{n,oy,ox} x[n][ci][iy][ix] * dy[n][co][oy][ox]
 * (NITI_GradientConv_Int8.cpp:165-270 on the graph of grad/NITI_Conv_Int8_Grad.cpp:124-191) */
void niti_ref_conv_wgrad_acc(const niti_ref_geom* g, const int8_t* x, const int8_t* dy, int32_t* acc,
                             niti_ref_stats* st);
/* acc[n][ci][iy][ix] = sum_{co,ky,kx} dy[n][co][oy][ox] * w[co][ci][ky][kx], iy = oy*s - pad + ky*d
 * (NITI_DeConv_Int8.cpp:187-290 on the graph of grad/NITI_Conv_Int8_Grad.cpp:29-122) */
void niti_ref_conv_dgrad_acc(const niti_ref_geom* g, const int8_t* dy, const int8_t* w, int32_t* acc,
                             niti_ref_stats* st);
/* C[m][o] = sum_k B[m][k] * A[o][k]   (NITI_Matmul_Int8.cpp:140-212) */
void niti_ref_matmul_acc(int m, int o, int k, const int8_t* B, const int8_t* A, int32_t* acc,
                         niti_ref_stats* st);

/* ---------------- reference-structured restatement (MNN C4 data flow) ---------------- */
/* C4 = MNN NC4HW4 with batch inside the channel block: [ceil(C/4)][N][H][W][4] (NITI_Conv_Int8.cpp:111). */
void niti_ref_nchw_to_c4(const int8_t* src, int n, int c, int h, int w, int8_t* dst);
void niti_ref_c4_to_nchw(const int8_t* src, int n, int c, int h, int w, int8_t* dst);
void niti_ref_c4_to_nchw_i32(const int32_t* src, int n, int c, int h, int w, int32_t* dst);

enum { NITI_REF_ACC_EXACT = 0, NITI_REF_ACC_F32_SEQ = 1 };

/* The core of NITI_Conv_Int8::onExecute (:162-249): per-call weight reorder (:19-64),
 * im2col per DST_XUNIT=4 pixel tile (Int8FunctionsOpt.cpp:296-392) and the 16x4 GEMM
 * unit (Int8FunctionsOpt.cpp:201-232).  x_c4 is C4, w is OIHW, acc_c4 is C4
 * [ceil(c_out/4)][N][OH][OW][4].  acc_mode: exact int64, or sequential float32 as the
 * portable x86 build writes it.  threads>1 splits the batch like the reference. */
void niti_ref_mnn_conv_core(const niti_ref_geom* g, const int8_t* x_c4, const int8_t* w_oihw,
                            int32_t* acc_c4, int acc_mode, int threads);

/* NITI_Conv_Int8 end to end on C4 tensors: returns exp_out. */
int32_t niti_ref_mnn_conv_fwd(const niti_ref_geom* g, const int8_t* x_c4, const int8_t* w_oihw,
                              int32_t exp_in, int32_t wscale, int8_t* y_c4, int acc_mode, int threads);
/* Weight gradient through the reference's graph: C4(x^T) conv dy^T (kernel OH x OW), with the
 * stride-2 LeftPoolGrad dilation, then PSTO(bw-2) and transpose back to OIHW.
 * x, dy are NCHW; dw is OIHW int8.  Returns bw.  Optional acc_oihw receives the int32 acc. */
int32_t niti_ref_mnn_conv_wgrad(const niti_ref_geom* g, const int8_t* x, const int8_t* dy, int8_t* dw,
                                int32_t* acc_oihw, int acc_mode, int threads);
/* Input gradient through the reference's graph: pad(dilate(dy)) conv rot180(w^T), forward
 * shift rule, no exponent.  dy NCHW, w OIHW, dx NCHW int8.  Returns the exponent increment. */
int32_t niti_ref_mnn_conv_dgrad(const niti_ref_geom* g, const int8_t* dy, const int8_t* w, int8_t* dx,
                                int32_t* acc_nchw, int acc_mode, int threads);

/* ---------------- the rest of the NITI step ---------------- */
/* NITI_CPURelu_Int8.cpp:41-50 */
void niti_ref_relu(const int8_t* x, int64_t n, int8_t* y);
/* NITI_CPUReluGrad_Int8.cpp:42-51: out = x > 0 ? dy : 0 */
void niti_ref_relu_grad(const int8_t* x, const int8_t* dy, int64_t n, int8_t* out);
/* NITI_Maxpool_Int8.cpp:24-72 on NCHW (stride, kernel, pad; kernel clipped to the input) */
void niti_ref_maxpool(const int8_t* x, int n, int c, int h, int w, int k, int s, int p, int8_t* y,
                      int oh, int ow);
/* NITI_CPUPoolGrad_Int8.cpp:21-77: first max (>=) in (ky,kx) order takes the gradient */
void niti_ref_maxpool_grad(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int c, int h,
                           int w, int k, int s, int p, int oh, int ow, int8_t* dx);
/* NITI_CPULossGrad_Int8.cpp:81-200: integer softmax-cross-entropy gradient, PSTO(4) */
void niti_ref_loss_grad(const int8_t* logits, int batch, int classes, int32_t ascale,
                        const int32_t* onehot, int target_classes, int8_t* out);
/* NITI_SGD.hpp:49-52 + niti_execute BinaryUtils.hpp:278-299: w <- clip(w - g, +-127) */
void niti_ref_sgd_update(int8_t* w, const int8_t* g, int64_t n);
/* MnistUtils.cpp:83-93: float batch -> int8, returns ascale */
/* the input quantiser over exact integer statistics (the device contract, niti_quant.hip) */
void niti_ref_image_stats(const uint8_t* img, int64_t n, uint64_t stats[4]);
int32_t niti_ref_image_quantize(const uint8_t* img, int64_t n, const uint64_t stats[4], int64_t count,
                                int64_t var_count, int8_t* out);
int32_t niti_ref_quantize_input(const float* x, int64_t n, int64_t var_n, int8_t* out);
/* sampled accumulation statistics: kind 0 forward (a = x, b = w, idx into [n][co][oy][ox]), 1 weight
 * gradient (a = x, b = dy, idx into [co][ci][ky][kx]), 2 stride-1 input gradient (a = dy, b = w, idx
 * into [n][ci][y][x]): exact sum, sum|p| and the reference-order float32 sum cast to int32 */
void niti_ref_sample_stats(const niti_ref_geom* g, int kind, const int8_t* a, const int8_t* b, const int64_t* idx,
                           int64_t ns, int64_t* exact, uint64_t* sabs, int32_t* f32);
int32_t niti_ref_quantize_input_lanes(const float* x, int64_t n, int64_t var_n, int lanes, int8_t* out);

/* ---------------- CPU baseline ---------------- */
/* One NITI_Conv_Int8 + NITI_GradientConv_Int8 + NITI_DeConv_Int8 pass in the reference's
 * structure with T threads (float32 accumulation as the x86 build).  Returns 0. */
int niti_ref_layer_step(const niti_ref_geom* g, const int8_t* x_nchw, const int8_t* w_oihw,
                        const int8_t* dy_nchw, int8_t* y_c4, int8_t* dw, int8_t* dx, int threads,
                        int with_dgrad);

#ifdef __cplusplus
}
#endif
#endif
