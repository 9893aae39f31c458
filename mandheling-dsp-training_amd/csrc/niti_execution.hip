// niti_execution.hip -- MNN Execution-shaped drop-in for the NITI int8 GEMM-class ops.
//
// Each class mirrors one reference Execution: the same OpType key, the same inputs and
// outputs in the same layouts (MNN C4 activations, OIHW / transposed weights, int8
// exponent scalars), the same onResize/onExecute split and the same ErrorCode values.
// Inside, the tensors are converted to the native layouts (niti_kernels.hpp) and the work
// runs on the gfx950 kernels; nothing here computes on the host.
//
//   NITI_Conv_Int8            execution-engine/source/backend/cpu/NITI_Conv_Int8.cpp:78-322
//   NITI_DeConv_Int8          execution-engine/source/backend/cpu/NITI_DeConv_Int8.cpp:80-345
//   NITI_GradientConv_Int8    execution-engine/source/backend/cpu/NITI_GradientConv_Int8.cpp:81-310
//   NITI_Matmul_Int8          execution-engine/source/backend/cpu/NITI_Matmul_Int8.cpp:63-243
//   NITI_DSPMatmulGradientConv_Int8
//                             execution-engine/source/backend/cpu/NITI_DSPMatmulGradientConv_Int8.cpp:105-553
//                             (op slot: NHWC/HWIO tensors, CPU weight-gradient numerics)
#include <math.h>

#include <memory>
#include <vector>

#include "../../include/niti_hip.h"
#include "niti_internal.hpp"
#include "niti_kernels.hpp"
#include "niti_map.hpp"

namespace niti {

// ------------------------------------------------------------------ boundary converters
namespace {

// C4(x^T): dims [Ci(batch), N(channel), H, W] -> x NHWC16 [N][HW][Cip]
struct C4TransposedToNhwc16 {
    const int8_t* x;
    int n, ci, hw, cip;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [n][hw][cip]
        const int c = (int)(i % cip);
        const int64_t r = i / cip;
        const int64_t p = r % hw;
        const int b = (int)(r / hw);
        out[i] = c < ci ? x[(((int64_t)(b >> 2) * ci + c) * hw + p) * 4 + (b & 3)] : (int8_t)0;
    }
};

// dy^T NCHW [Co][N][OHW] -> dy NHWC16 [N][OHW][Cop]
struct NchwTransposedToNhwc16 {
    const int8_t* d;
    int n, co, hw, cop;
    int8_t* out;
    __device__ void operator()(int64_t i) const {
        const int c = (int)(i % cop);
        const int64_t r = i / cop;
        const int64_t p = r % hw;
        const int b = (int)(r / hw);
        out[i] = c < co ? d[((int64_t)c * n + b) * hw + p] : (int8_t)0;
    }
};

// NHWC [N][HW][C] -> NHWC16 [N][HW][Cp]
struct NhwcToNhwc16 {
    const int8_t* x;
    int c, cp;
    int8_t* out;
    __device__ void operator()(int64_t i) const {
        const int ch = (int)(i % cp);
        const int64_t r = i / cp;
        out[i] = ch < c ? x[r * c + ch] : (int8_t)0;
    }
};

// NHWC16 [n][hw][cp] -> C4 [ceil(c/4)][n][hw][4] (the pad lanes of the last quad zero); one
// channel quad (4 bytes) per thread
struct Nhwc16ToC4 {
    const int8_t* in;
    int n, c, hw, cp;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [cq][n][hw]
        const int p = (int)(i % hw);
        const int64_t r = i / hw;
        const int b = (int)(r % n);
        const int cq = (int)(r / n);
        uint32_t v = *(const uint32_t*)(in + ((int64_t)b * hw + p) * cp + 4 * cq);
        const int live = c - 4 * cq;  // channels of this quad that exist
        if (live < 4) v &= (1u << (8 * live)) - 1u;
        *(uint32_t*)(out + i * 4) = v;
    }
};

// The register-fed row kernel with the rescale fused (niti_rowconv.hip) behind the conv and
// deconv Executions, where the geometry allows (stride-1 pad-1 3x3, square 2/4/8/16 maps,
// c_out padded to a multiple of 32, the grid resident): x -> C32, OHWI16 -> fragment-major WF,
// one fused launch into NHWC16, then C4.  Same results as the GEMM + requantisation path.
struct RowPath {
    Workspace ws;
    int8_t *xc32 = nullptr, *wf = nullptr, *y16 = nullptr;
    uint32_t *bar = nullptr, *err = nullptr;
    uint32_t epoch = 0;
    bool on = false;
    int resize(const ConvGeom& g) {
        ws.release();
        on = rowconv_ok(g) && rowconv_fused_ok(g);
        if (!on) return NITI_NO_ERROR;
        const int cb = (g.c_in + 31) / 32;
        xc32 = (int8_t*)ws.alloc((size_t)g.n * cb * g.h * g.w * 32);
        wf = (int8_t*)ws.alloc(rowconv_wf_bytes(g.c_out, g.c_in));
        y16 = (int8_t*)ws.alloc((size_t)g.n * g.oh * g.ow * g.cop);
        bar = (uint32_t*)ws.alloc((ROWCONV_BAR_WORDS + 1) * sizeof(uint32_t));
        if (!xc32 || !wf || !y16 || !bar) return NITI_OUT_OF_MEMORY;
        err = bar + ROWCONV_BAR_WORDS;
        if (hipMemset(bar, 0, (ROWCONV_BAR_WORDS + 1) * sizeof(uint32_t)) != hipSuccess) return NITI_NO_EXECUTION;
        epoch = 0;
        return NITI_NO_ERROR;
    }
    // x16 / w16: the Execution's NHWC16 input and OHWI16 weights (already converted); amax zeroed.
    // Under stream capture the fused launch's barrier parity (epoch, a kernel argument) would be
    // replayed unchanged with counts nobody resets, so a captured call takes the two-launch form
    // (range launch, then recompute + requantise with the published max): same results.
    hipError_t run(const ConvGeom& g, const int8_t* x16, const int8_t* w16, uint32_t* amax, const int8_t* exp_in,
                   const int8_t* wscale, int8_t* exp_out, int8_t* out_c4, hipStream_t st) {
        hipError_t e = nhwc16_to_c32(x16, g.n, g.h * g.w, g.cip, g.c_in, xc32, st);
        if (e == hipSuccess) e = weights_to_wf(w16, g.c_out, g.c_in, g.cip, false, wf, st);
        if (e != hipSuccess) return e;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess) return hipErrorInvalidValue;
        RowConvOut o;
        o.out = y16;
        o.exp_in = exp_in;
        o.wscale = wscale;
        o.exp_out = exp_out;
        if (cs == hipStreamCaptureStatusNone) {
            e = rowconv_fwd(g, xc32, wf, o, 0, amax, bar, ++epoch, err, st);
        } else {
            e = rowconv_fwd(g, xc32, wf, o, 1, amax, nullptr, 0, nullptr, st);
            if (e == hipSuccess) e = rowconv_fwd(g, xc32, wf, o, 2, amax, nullptr, 0, nullptr, st);
        }
        if (e != hipSuccess) return e;
        const int cq = (g.c_out + 3) / 4;
        return launch_map((int64_t)cq * g.n * g.oh * g.ow, Nhwc16ToC4{y16, g.n, g.c_out, g.oh * g.ow, g.cop, out_c4}, st);
    }
};

// g OHWI16 [Co][KK][Cip] -> C4 [ceil(Co/4)][Ci][KK][4] (the GradientConv output tensor,
// batch = Ci, channel = Co)
struct Ohwi16ToC4Grad {
    const int8_t* g;
    int co, ci, kk, cip;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [ceil(co/4)][ci][kk][4]
        const int j = (int)(i & 3);
        const int64_t r = i >> 2;
        const int k = (int)(r % kk);
        const int64_t r2 = r / kk;
        const int c = (int)(r2 % ci);
        const int oq = (int)(r2 / ci);
        const int o = oq * 4 + j;
        out[i] = o < co ? g[((int64_t)o * kk + k) * cip + c] : (int8_t)0;
    }
};

// g OHWI16 [Co][KK][Cip] -> HWIO [KK][Ci][Co]
struct Ohwi16ToHwio {
    const int8_t* g;
    int co, ci, kk, cip;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [kk][ci][co]
        const int o = (int)(i % co);
        const int64_t r = i / co;
        const int c = (int)(r % ci);
        const int k = (int)(r / ci);
        out[i] = g[((int64_t)o * kk + k) * cip + c];
    }
};

// w HWIO [KK][Ci][Co] -> OHWI16 [Co][KK][Cip] (the DSP ops' weights, NN.cpp:1155-1156)
struct HwioToOhwi16 {
    const int8_t* w;
    int co, ci, kk, cip;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [co][kk][cip]
        const int c = (int)(i % cip);
        const int64_t r = i / cip;
        const int k = (int)(r % kk);
        const int o = (int)(r / kk);
        out[i] = c < ci ? w[((int64_t)k * ci + c) * co + o] : (int8_t)0;
    }
};

// x^T [Ci][H][W][N] (NHWC dims batch = Ci, channel = N) -> x NHWC16 [N][HW][Cip]
struct CiHwnToNhwc16 {
    const int8_t* x;
    int n, ci, hw, cip;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [n][hw][cip]
        const int c = (int)(i % cip);
        const int64_t r = i / cip;
        const int64_t p = r % hw;
        const int b = (int)(r / hw);
        out[i] = c < ci ? x[((int64_t)c * hw + p) * n + b] : (int8_t)0;
    }
};

// g OHWI16 [Co][KK][Cip] -> [Ci][KK][Co] (the transposed-gradient op's NHWC output: batch = Ci)
struct Ohwi16ToIhwo {
    const int8_t* g;
    int co, ci, kk, cip;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [ci][kk][co]
        const int o = (int)(i % co);
        const int64_t r = i / co;
        const int k = (int)(r % kk);
        const int c = (int)(r / kk);
        out[i] = g[((int64_t)o * kk + k) * cip + c];
    }
};

// [rows][ld] int8 -> [rows][cols]
struct UnpadRows {
    const int8_t* in;
    int cols, ld;
    int8_t* out;
    __device__ void operator()(int64_t i) const {
        const int64_t r = i / cols;
        const int c = (int)(i - r * cols);
        out[i] = in[r * ld + c];
    }
};

int to_code(hipError_t e) {
    if (e == hipSuccess) return NITI_NO_ERROR;
    if (e == hipErrorOutOfMemory) return NITI_OUT_OF_MEMORY;
    if (e == hipErrorInvalidValue) return NITI_INVALID_VALUE;
    return NITI_NO_EXECUTION;
}

#define NITI_TRY(expr)                         \
    do {                                       \
        const int _c = to_code(expr);          \
        if (_c != NITI_NO_ERROR) return _c;    \
    } while (0)

inline int64_t count4(const niti_tensor& t) { return (int64_t)t.dims[0] * t.dims[1] * t.dims[2] * t.dims[3]; }

}  // namespace

// ------------------------------------------------------------------ device workspace
void* Workspace::alloc(size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    total += bytes;
    return p;
}
void* Workspace::replace(void* old, size_t bytes) {
    if (old != nullptr) {
        for (size_t i = 0; i < ptrs.size(); ++i)
            if (ptrs[i] == old) {
                (void)hipFree(old);
                ptrs.erase(ptrs.begin() + i);
                break;
            }
    }
    return alloc(bytes);
}
void Workspace::release() {
    for (void* p : ptrs) (void)hipFree(p);
    ptrs.clear();
    total = 0;
}

// Convolution2DCommon -> geometry (ConvolutionCommon::convolutionPad,
// source/core/ConvolutionCommon.cpp:550-569; output size ShapeNITI_Conv_Int8.cpp:41-76).
bool geom_from_common(const niti_conv2d_common& c, int n, int ci, int h, int w, int co, int kh, int kw,
                      ConvGeom* g) {
    ConvGeom r{};
    r.n = n;
    r.c_in = ci;
    r.h = h;
    r.w = w;
    r.c_out = co;
    r.kh = kh;
    r.kw = kw;
    r.sh = c.stride_y > 0 ? c.stride_y : 1;
    r.sw = c.stride_x > 0 ? c.stride_x : 1;
    r.dh = c.dilate_y > 0 ? c.dilate_y : 1;
    r.dw = c.dilate_x > 0 ? c.dilate_x : 1;
    const int keh = r.dh * (kh - 1) + 1, kew = r.dw * (kw - 1) + 1;
    int oh, ow;
    if (c.pad_mode == NITI_PAD_SAME) {
        oh = (h + r.sh - 1) / r.sh;
        ow = (w + r.sw - 1) / r.sw;
        const int pnh = (oh - 1) * r.sh + keh - h, pnw = (ow - 1) * r.sw + kew - w;
        r.pt = pnh / 2;
        r.pl = pnw / 2;
    } else if (c.pad_mode == NITI_PAD_VALID) {
        oh = (int)ceilf((float)(h - keh + 1) / (float)r.sh);
        ow = (int)ceilf((float)(w - kew + 1) / (float)r.sw);
        r.pt = c.has_pads ? c.pads[0] : c.pad_y;
        r.pl = c.has_pads ? c.pads[1] : c.pad_x;
    } else if (c.has_pads) {
        oh = (h + c.pads[0] + c.pads[2] - keh) / r.sh + 1;
        ow = (w + c.pads[1] + c.pads[3] - kew) / r.sw + 1;
        r.pt = c.pads[0];
        r.pl = c.pads[1];
    } else {
        oh = (h + 2 * c.pad_y - keh) / r.sh + 1;
        ow = (w + 2 * c.pad_x - kew) / r.sw + 1;
        r.pt = c.pad_y;
        r.pl = c.pad_x;
    }
    r.pb = (oh - 1) * r.sh + keh - h - r.pt;
    r.pr = (ow - 1) * r.sw + kew - w - r.pl;
    if (!r.finalize()) return false;
    r.oh = oh;
    r.ow = ow;
    *g = r;
    return oh > 0 && ow > 0;
}

// ------------------------------------------------------------------ NITI_Conv_Int8 (700)
class ConvInt8Execution : public Execution {
   public:
    explicit ConvInt8Execution(const niti_conv2d_common& c) : common_(c) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 4 || nout < 2) return NITI_INVALID_VALUE;
        const niti_tensor &x = in[0], &w = in[1], &y = out[0];
        if (x.format != NITI_FORMAT_NC4HW4 || y.format != NITI_FORMAT_NC4HW4) return NITI_NOT_SUPPORT;
        if (common_.group > 1) return NITI_NOT_SUPPORT;
        if (w.dims[1] != x.dims[1]) return NITI_COMPUTE_SIZE_ERROR;
        if (!geom_from_common(common_, x.dims[0], x.dims[1], x.dims[2], x.dims[3], w.dims[0], w.dims[2], w.dims[3], &g_))
            return NITI_COMPUTE_SIZE_ERROR;
        if (y.dims[0] != g_.n || y.dims[1] != g_.c_out || y.dims[2] != g_.oh || y.dims[3] != g_.ow)
            return NITI_COMPUTE_SIZE_ERROR;
        if (g_.c_out % 4) return NITI_NOT_SUPPORT;  // NITI_Conv_Int8.cpp:130 sizes acc N*C*H*W
        ws_.release();
        x16_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.h * g_.w * g_.cip);
        w16_ = (int8_t*)ws_.alloc((size_t)g_.c_out * g_.kh * g_.kw * g_.cip);
        acc_ = (int32_t*)ws_.alloc((size_t)g_.n * g_.oh * g_.ow * g_.cop * 4);
        amax_ = (uint32_t*)ws_.alloc(MAX_BYTES);
        slab_bytes_ = conv_fwd_workspace(g_);
        slab_ = slab_bytes_ ? ws_.alloc(slab_bytes_) : nullptr;
        if (slab_bytes_ && !slab_) return NITI_OUT_OF_MEMORY;
        if (!(x16_ && w16_ && acc_ && amax_)) return NITI_OUT_OF_MEMORY;
        return rows_.resize(g_);
    }
    uint32_t* errorFlag() override { return rows_.on ? rows_.err : nullptr; }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!acc_) return NITI_NO_EXECUTION;
        NITI_TRY(c4_to_nhwc16((const int8_t*)in[0].data, g_.n, g_.c_in, g_.h * g_.w, g_.cip, x16_, st));
        // reorderWeight every call: weights change each step (NITI_Conv_Int8.cpp:177)
        NITI_TRY(oihw_to_ohwi16((const int8_t*)in[1].data, g_.c_out, g_.c_in, g_.kh * g_.kw, g_.cip, w16_, st));
        NITI_TRY(hipMemsetAsync(amax_, 0, MAX_BYTES, st));
        if (rows_.on) {
            NITI_TRY(rows_.run(g_, x16_, w16_, amax_, (const int8_t*)in[2].data, (const int8_t*)in[3].data,
                               nout > 1 ? (int8_t*)out[1].data : nullptr, (int8_t*)out[0].data, st));
            return NITI_NO_ERROR;
        }
        NITI_TRY(conv_fwd_acc(g_, x16_, w16_, acc_, amax_, slab_, slab_bytes_, st));
        ActRequant r;
        r.acc = acc_;
        r.rows = (int64_t)g_.n * g_.oh * g_.ow;
        r.ldc = g_.cop;
        r.amax = amax_;
        r.exp_in = (const int8_t*)in[2].data;
        r.wscale = (const int8_t*)in[3].data;
        r.exp_out = nout > 1 ? (int8_t*)out[1].data : nullptr;
        r.out_c4 = (int8_t*)out[0].data;
        r.c_real = g_.c_out;
        r.n = g_.n;
        r.hw = g_.oh * g_.ow;
        NITI_TRY(requant_act(r, st));
        return NITI_NO_ERROR;
    }

   private:
    niti_conv2d_common common_;
    ConvGeom g_{};
    int8_t *x16_ = nullptr, *w16_ = nullptr;
    int32_t* acc_ = nullptr;
    uint32_t* amax_ = nullptr;
    void* slab_ = nullptr;
    size_t slab_bytes_ = 0;
    RowPath rows_;
};

// ------------------------------------------------------------------ NITI_DeConv_Int8 (701)
// Receives dy already padded / dilated by the graph (NITI_Conv_Int8_Grad.cpp:86-120) and w^T;
// rotates w^T by 180 degrees and runs a stride-1 conv with the forward shift rule (no exponent).
class DeconvInt8Execution : public Execution {
   public:
    explicit DeconvInt8Execution(const niti_conv2d_common& c) : common_(c) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 2 || nout < 1) return NITI_INVALID_VALUE;
        const niti_tensor &d = in[0], &wt = in[1], &y = out[0];
        if (d.format != NITI_FORMAT_NC4HW4 || y.format != NITI_FORMAT_NC4HW4) return NITI_NOT_SUPPORT;
        if (common_.group > 1) return NITI_NOT_SUPPORT;
        if (wt.dims[1] != d.dims[1]) return NITI_COMPUTE_SIZE_ERROR;
        if (!geom_from_common(common_, d.dims[0], d.dims[1], d.dims[2], d.dims[3], wt.dims[0], wt.dims[2], wt.dims[3],
                              &g_))
            return NITI_COMPUTE_SIZE_ERROR;
        if (y.dims[0] != g_.n || y.dims[1] != g_.c_out || y.dims[2] != g_.oh || y.dims[3] != g_.ow)
            return NITI_COMPUTE_SIZE_ERROR;
        if (g_.c_out % 4) return NITI_NOT_SUPPORT;
        ws_.release();
        x16_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.h * g_.w * g_.cip);
        w16_ = (int8_t*)ws_.alloc((size_t)g_.c_out * g_.kh * g_.kw * g_.cip);
        acc_ = (int32_t*)ws_.alloc((size_t)g_.n * g_.oh * g_.ow * g_.cop * 4);
        amax_ = (uint32_t*)ws_.alloc(MAX_BYTES);
        slab_bytes_ = conv_fwd_workspace(g_);
        slab_ = slab_bytes_ ? ws_.alloc(slab_bytes_) : nullptr;
        if (slab_bytes_ && !slab_) return NITI_OUT_OF_MEMORY;
        if (!(x16_ && w16_ && acc_ && amax_)) return NITI_OUT_OF_MEMORY;
        return rows_.resize(g_);
    }
    uint32_t* errorFlag() override { return rows_.on ? rows_.err : nullptr; }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!acc_) return NITI_NO_EXECUTION;
        NITI_TRY(c4_to_nhwc16((const int8_t*)in[0].data, g_.n, g_.c_in, g_.h * g_.w, g_.cip, x16_, st));
        NITI_TRY(oihw_to_ohwi16((const int8_t*)in[1].data, g_.c_out, g_.c_in, g_.kh * g_.kw, g_.cip, w16_, st, true));
        NITI_TRY(hipMemsetAsync(amax_, 0, MAX_BYTES, st));
        if (rows_.on) {  // the forward rule without an exponent output (rotated w^T: a plain conv)
            NITI_TRY(rows_.run(g_, x16_, w16_, amax_, nullptr, nullptr, nullptr, (int8_t*)out[0].data, st));
            return NITI_NO_ERROR;
        }
        NITI_TRY(conv_fwd_acc(g_, x16_, w16_, acc_, amax_, slab_, slab_bytes_, st));
        ActRequant r;
        r.acc = acc_;
        r.rows = (int64_t)g_.n * g_.oh * g_.ow;
        r.ldc = g_.cop;
        r.amax = amax_;
        r.out_c4 = (int8_t*)out[0].data;
        r.c_real = g_.c_out;
        r.n = g_.n;
        r.hw = g_.oh * g_.ow;
        NITI_TRY(requant_act(r, st));
        return NITI_NO_ERROR;
    }

   private:
    niti_conv2d_common common_;
    ConvGeom g_{};
    int8_t *x16_ = nullptr, *w16_ = nullptr;
    int32_t* acc_ = nullptr;
    uint32_t* amax_ = nullptr;
    void* slab_ = nullptr;
    size_t slab_bytes_ = 0;
    RowPath rows_;
};

// ------------------------------------------------------------------ NITI_GradientConv_Int8 (715)
// A conv of C4(x^T) [Ci, N, H, W] with dy^T [Co, N, OH', OW'] as its kernel; computed as the
// native weight-gradient GEMM (K = N*OH'*OW' pixels) followed by PSTO(bw-2).
class GradientConvInt8Execution : public Execution {
   public:
    explicit GradientConvInt8Execution(const niti_conv2d_common& c) : common_(c) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 2 || nout < 1) return NITI_INVALID_VALUE;
        const niti_tensor &xt = in[0], &dyt = in[1], &o = out[0];
        if (xt.format != NITI_FORMAT_NC4HW4 || o.format != NITI_FORMAT_NC4HW4) return NITI_NOT_SUPPORT;
        if (common_.group > 1 || common_.dilate_x > 1 || common_.dilate_y > 1) return NITI_NOT_SUPPORT;
        if (dyt.dims[1] != xt.dims[1]) return NITI_COMPUTE_SIZE_ERROR;
        // the op's own view: batch Ci, channel N, kernel OH' x OW'
        ConvGeom op{};
        if (!geom_from_common(common_, xt.dims[0], xt.dims[1], xt.dims[2], xt.dims[3], dyt.dims[0], dyt.dims[2],
                              dyt.dims[3], &op))
            return NITI_COMPUTE_SIZE_ERROR;
        if (op.sh != 1 || op.sw != 1) return NITI_NOT_SUPPORT;  // the grad graph always passes stride 1
        if (o.dims[0] != op.n || o.dims[1] != op.c_out || o.dims[2] != op.oh || o.dims[3] != op.ow)
            return NITI_COMPUTE_SIZE_ERROR;
        if (op.c_out % 4) return NITI_NOT_SUPPORT;
        // the native weight-gradient geometry: images N, channels Ci, kernel (op.oh, op.ow)
        ConvGeom g{};
        g.n = xt.dims[1];
        g.c_in = xt.dims[0];
        g.h = xt.dims[2];
        g.w = xt.dims[3];
        g.c_out = dyt.dims[0];
        g.kh = op.oh;
        g.kw = op.ow;
        g.sh = g.sw = g.dh = g.dw = 1;
        g.pt = op.pt;
        g.pl = op.pl;
        g.pb = op.pb;
        g.pr = op.pr;
        if (!g.finalize() || g.oh != dyt.dims[2] || g.ow != dyt.dims[3]) return NITI_COMPUTE_SIZE_ERROR;
        g_ = g;
        ws_.release();
        xT_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.h * g_.w * g_.cip);
        dyT_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.oh * g_.ow * g_.cop);
        acc_ = (int32_t*)ws_.alloc((size_t)g_.c_out * g_.kh * g_.kw * g_.cip * 4);
        g8_ = (int8_t*)ws_.alloc((size_t)g_.c_out * g_.kh * g_.kw * g_.cip);
        amax_ = (uint32_t*)ws_.alloc(MAX_BYTES);
        slab_bytes_ = conv_wgrad_workspace(g_);
        slab_ = slab_bytes_ ? ws_.alloc(slab_bytes_) : nullptr;
        if (slab_bytes_ && !slab_) return NITI_OUT_OF_MEMORY;
        return (xT_ && dyT_ && acc_ && g8_ && amax_) ? NITI_NO_ERROR : NITI_OUT_OF_MEMORY;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!acc_) return NITI_NO_EXECUTION;
        const int hw = g_.h * g_.w, ohw = g_.oh * g_.ow, kk = g_.kh * g_.kw;
        NITI_TRY(launch_map((int64_t)g_.n * hw * g_.cip,
                            C4TransposedToNhwc16{(const int8_t*)in[0].data, g_.n, g_.c_in, hw, g_.cip, xT_}, st));
        NITI_TRY(launch_map((int64_t)g_.n * ohw * g_.cop,
                            NchwTransposedToNhwc16{(const int8_t*)in[1].data, g_.n, g_.c_out, ohw, g_.cop, dyT_}, st));
        const int64_t nacc = (int64_t)g_.c_out * kk * g_.cip;
        NITI_TRY(hipMemsetAsync(amax_, 0, MAX_BYTES, st));
        NITI_TRY(conv_wgrad_acc(g_, xT_, dyT_, acc_, amax_, slab_, slab_bytes_, st));
        NITI_TRY(requant_grad(acc_, nacc, amax_, RULE_WGRAD_BW2, g8_, nullptr, st));
        NITI_TRY(launch_map((int64_t)((g_.c_out + 3) / 4) * g_.c_in * kk * 4,
                            Ohwi16ToC4Grad{g8_, g_.c_out, g_.c_in, kk, g_.cip, (int8_t*)out[0].data}, st));
        return NITI_NO_ERROR;
    }

   private:
    niti_conv2d_common common_;
    ConvGeom g_{};
    int8_t *xT_ = nullptr, *dyT_ = nullptr, *g8_ = nullptr;
    int32_t* acc_ = nullptr;
    uint32_t* amax_ = nullptr;
    void* slab_ = nullptr;
    size_t slab_bytes_ = 0;
};

// ------------------------------------------------------------------ NITI_Matmul_Int8 (713)
// C[m][o] = PSTO(sum_k B[m][k] A[o][k], bw-3).  Output tensor C [M, Co] row major: the
// values the reference computes (its output region then transposes C to [Co][M],
// NITI_GeometryConv2DBackPropFilter_Int8.cpp:105-121).
class MatmulInt8Execution : public Execution {
   public:
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 2 || nout < 1) return NITI_INVALID_VALUE;
        m_ = in[0].dims[0];
        k_ = in[0].dims[1];
        o_ = in[1].dims[0];
        if (in[1].dims[1] != k_ || out[0].dims[0] != m_ || out[0].dims[1] != o_) return NITI_COMPUTE_SIZE_ERROR;
        if (m_ <= 0 || k_ <= 0 || o_ <= 0) return NITI_COMPUTE_SIZE_ERROR;
        k16_ = round_up(k_, 16);
        ldc_ = round_up(o_, 16);
        ws_.release();
        b16_ = (int8_t*)ws_.alloc((size_t)m_ * k16_);
        a16_ = (int8_t*)ws_.alloc((size_t)o_ * k16_);
        acc_ = (int32_t*)ws_.alloc((size_t)m_ * ldc_ * 4);
        g8_ = (int8_t*)ws_.alloc((size_t)m_ * ldc_);
        amax_ = (uint32_t*)ws_.alloc(MAX_BYTES);
        slab_bytes_ = matmul_workspace(m_, ldc_, k16_);
        slab_ = slab_bytes_ ? ws_.alloc(slab_bytes_) : nullptr;
        if (slab_bytes_ && !slab_) return NITI_OUT_OF_MEMORY;
        return (b16_ && a16_ && acc_ && g8_ && amax_) ? NITI_NO_ERROR : NITI_OUT_OF_MEMORY;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!acc_) return NITI_NO_EXECUTION;
        NITI_TRY(pad_rows((const int8_t*)in[0].data, m_, k_, k16_, b16_, st));
        NITI_TRY(pad_rows((const int8_t*)in[1].data, o_, k_, k16_, a16_, st));
        NITI_TRY(hipMemsetAsync(amax_, 0, MAX_BYTES, st));
        NITI_TRY(matmul_acc(m_, o_, k16_, b16_, k16_, a16_, k16_, acc_, ldc_, amax_, slab_, slab_bytes_, st));
        NITI_TRY(requant_grad(acc_, (int64_t)m_ * ldc_, amax_, RULE_MATMUL_BW3, g8_, nullptr, st));
        NITI_TRY(launch_map((int64_t)m_ * o_, UnpadRows{g8_, o_, ldc_, (int8_t*)out[0].data}, st));
        return NITI_NO_ERROR;
    }

   private:
    int m_ = 0, k_ = 0, o_ = 0, k16_ = 0, ldc_ = 0;
    int8_t *b16_ = nullptr, *a16_ = nullptr, *g8_ = nullptr;
    int32_t* acc_ = nullptr;
    uint32_t* amax_ = nullptr;
    void* slab_ = nullptr;
    size_t slab_bytes_ = 0;
};

// ------------------------------------------------------------------ NITI_DSP_MATMUL_GRADIENT_Int8 (818)
// Op slot of the DSP weight-gradient (NHWC x, NHWC dy -> HWIO dw).  The DSP build
// requantises on the Hexagon (round-to-nearest, then /16 on the CPU,
// NITI_DSPMatmulGradientConv_Int8.cpp:543-550); this backend gives the op the CPU path's
// numerics (NITI_GradientConv_Int8: PSTO(bw-2)), SURVEY.md §8(a) A5.
// NITI_DSP_GRADIENTCONV_Int8 (810), NITI_DSP_MATMUL_Int8 (819) and
// NITI_DSP_PARALLEL_GRADIENTCONV_Int8 (820) have the same tensors; the graph rule sets the common's
// kernel to dy's OH x OW (grad/NITI_DSPConv_Int8_Grad.cpp:151-153, shape rule
// ShapeNITI_Conv_Int8.cpp:146-233), so its filter size comes from the output tensor.
class DspMatmulGradientExecution : public Execution {
   public:
    explicit DspMatmulGradientExecution(const niti_conv2d_common& c, bool kernel_from_output = false)
        : common_(c), kernel_from_output_(kernel_from_output) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 2 || nout < 1) return NITI_INVALID_VALUE;
        const niti_tensor &x = in[0], &dy = in[1], &o = out[0];
        if (x.format != NITI_FORMAT_NHWC || dy.format != NITI_FORMAT_NHWC) return NITI_NOT_SUPPORT;
        if (common_.group > 1 || common_.dilate_x > 1 || common_.dilate_y > 1) return NITI_NOT_SUPPORT;
        const int kh = kernel_from_output_ ? o.dims[0] : common_.kernel_y;
        const int kw = kernel_from_output_ ? o.dims[1] : common_.kernel_x;
        if (!geom_from_common(common_, x.dims[0], x.dims[1], x.dims[2], x.dims[3], dy.dims[1], kh, kw, &g_))
            return NITI_COMPUTE_SIZE_ERROR;
        if (dy.dims[0] != g_.n || dy.dims[2] != g_.oh || dy.dims[3] != g_.ow) return NITI_COMPUTE_SIZE_ERROR;
        if (o.dims[0] != kh || o.dims[1] != kw || o.dims[2] != g_.c_in || o.dims[3] != g_.c_out)
            return NITI_COMPUTE_SIZE_ERROR;
        ws_.release();
        xT_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.h * g_.w * g_.cip);
        dyT_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.oh * g_.ow * g_.cop);
        acc_ = (int32_t*)ws_.alloc((size_t)g_.c_out * kh * kw * g_.cip * 4);
        g8_ = (int8_t*)ws_.alloc((size_t)g_.c_out * kh * kw * g_.cip);
        amax_ = (uint32_t*)ws_.alloc(MAX_BYTES);
        slab_bytes_ = conv_wgrad_workspace(g_);
        slab_ = slab_bytes_ ? ws_.alloc(slab_bytes_) : nullptr;
        if (slab_bytes_ && !slab_) return NITI_OUT_OF_MEMORY;
        return (xT_ && dyT_ && acc_ && g8_ && amax_) ? NITI_NO_ERROR : NITI_OUT_OF_MEMORY;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!acc_) return NITI_NO_EXECUTION;
        const int hw = g_.h * g_.w, ohw = g_.oh * g_.ow, kk = g_.kh * g_.kw;
        NITI_TRY(launch_map((int64_t)g_.n * hw * g_.cip, NhwcToNhwc16{(const int8_t*)in[0].data, g_.c_in, g_.cip, xT_}, st));
        NITI_TRY(launch_map((int64_t)g_.n * ohw * g_.cop, NhwcToNhwc16{(const int8_t*)in[1].data, g_.c_out, g_.cop, dyT_}, st));
        const int64_t nacc = (int64_t)g_.c_out * kk * g_.cip;
        NITI_TRY(hipMemsetAsync(amax_, 0, MAX_BYTES, st));
        NITI_TRY(conv_wgrad_acc(g_, xT_, dyT_, acc_, amax_, slab_, slab_bytes_, st));
        NITI_TRY(requant_grad(acc_, nacc, amax_, RULE_WGRAD_BW2, g8_, nullptr, st));
        NITI_TRY(launch_map((int64_t)kk * g_.c_in * g_.c_out, Ohwi16ToHwio{g8_, g_.c_out, g_.c_in, kk, g_.cip, (int8_t*)out[0].data}, st));
        return NITI_NO_ERROR;
    }

   private:
    niti_conv2d_common common_;
    bool kernel_from_output_;
    ConvGeom g_{};
    int8_t *xT_ = nullptr, *dyT_ = nullptr, *g8_ = nullptr;
    int32_t* acc_ = nullptr;
    uint32_t* amax_ = nullptr;
    void* slab_ = nullptr;
    size_t slab_bytes_ = 0;
};

// ------------------------------------------------------------------ NITI_DSP_CONV_Int8 (800) / NITI_DSP_DECONV_Int8 (811)
// Op slots of the DSP forward conv and input-gradient conv: x (or dy) NHWC, weights HWIO
// [KH][KW][Ci][Co], exp_in, wscale -> y NHWC, exp_out (NITI_DSPConv_Int8.cpp:160-455,
// NITI_DSPDeConv_Int8.cpp: pad + supernode conv, exp_out = exp_in + wscale + shift :399-400).
// The deconv's graph rule (grad/NITI_DSPConv_Int8_Grad.cpp:35-130) hands it dy (dilated by
// LeftPoolGrad for stride 2) and the rotated, transposed weights with the extra pad, so both
// ops are one stride-s conv.  The DSP requantises round-to-nearest on the Hexagon; this
// backend gives both the CPU path's numerics (NITI_Conv_Int8.cpp:255-307: shift = bw - 7,
// PSTO; exp_out = exp_in + wscale + the applied increment), SURVEY.md §8(f)-2.
class DspConvExecution : public Execution {
   public:
    explicit DspConvExecution(const niti_conv2d_common& c) : common_(c) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 4 || nout < 2) return NITI_INVALID_VALUE;
        const niti_tensor &x = in[0], &w = in[1], &y = out[0];
        if (x.format != NITI_FORMAT_NHWC || y.format != NITI_FORMAT_NHWC) return NITI_NOT_SUPPORT;
        if (common_.group > 1) return NITI_NOT_SUPPORT;
        // x, y NHWC with logical dims {N, C, H, W}; w HWIO as dims {KH, KW, Ci, Co}
        if (w.dims[2] != x.dims[1]) return NITI_COMPUTE_SIZE_ERROR;
        if (!geom_from_common(common_, x.dims[0], x.dims[1], x.dims[2], x.dims[3], w.dims[3], w.dims[0], w.dims[1], &g_))
            return NITI_COMPUTE_SIZE_ERROR;
        if (y.dims[0] != g_.n || y.dims[1] != g_.c_out || y.dims[2] != g_.oh || y.dims[3] != g_.ow)
            return NITI_COMPUTE_SIZE_ERROR;
        ws_.release();
        x16_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.h * g_.w * g_.cip);
        w16_ = (int8_t*)ws_.alloc((size_t)g_.c_out * g_.kh * g_.kw * g_.cip);
        acc_ = (int32_t*)ws_.alloc((size_t)g_.n * g_.oh * g_.ow * g_.cop * 4);
        y16_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.oh * g_.ow * g_.cop);
        amax_ = (uint32_t*)ws_.alloc(MAX_BYTES);
        slab_bytes_ = conv_fwd_workspace(g_);
        slab_ = slab_bytes_ ? ws_.alloc(slab_bytes_) : nullptr;
        if (slab_bytes_ && !slab_) return NITI_OUT_OF_MEMORY;
        return (x16_ && w16_ && acc_ && y16_ && amax_) ? NITI_NO_ERROR : NITI_OUT_OF_MEMORY;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!acc_) return NITI_NO_EXECUTION;
        const int kk = g_.kh * g_.kw;
        NITI_TRY(launch_map((int64_t)g_.n * g_.h * g_.w * g_.cip, NhwcToNhwc16{(const int8_t*)in[0].data, g_.c_in, g_.cip, x16_}, st));
        NITI_TRY(launch_map((int64_t)g_.c_out * kk * g_.cip,
                            HwioToOhwi16{(const int8_t*)in[1].data, g_.c_out, g_.c_in, kk, g_.cip, w16_}, st));
        NITI_TRY(hipMemsetAsync(amax_, 0, MAX_BYTES, st));
        NITI_TRY(conv_fwd_acc(g_, x16_, w16_, acc_, amax_, slab_, slab_bytes_, st));
        ActRequant r;
        r.acc = acc_;
        r.rows = (int64_t)g_.n * g_.oh * g_.ow;
        r.ldc = g_.cop;
        r.amax = amax_;
        r.exp_in = (const int8_t*)in[2].data;
        r.wscale = (const int8_t*)in[3].data;
        r.exp_out = nout > 1 ? (int8_t*)out[1].data : nullptr;
        r.out_nhwc16 = y16_;
        NITI_TRY(requant_act(r, st));
        const int64_t rows = (int64_t)g_.n * g_.oh * g_.ow;
        NITI_TRY(launch_map(rows * g_.c_out, UnpadRows{y16_, g_.c_out, g_.cop, (int8_t*)out[0].data}, st));
        return NITI_NO_ERROR;
    }

   private:
    niti_conv2d_common common_;
    ConvGeom g_{};
    int8_t *x16_ = nullptr, *w16_ = nullptr, *y16_ = nullptr;
    int32_t* acc_ = nullptr;
    uint32_t* amax_ = nullptr;
    void* slab_ = nullptr;
    size_t slab_bytes_ = 0;
};

// ------------------------------------------------------------------ NITI_DSP_TRANSPOSEGRADIENT_CONV_Int8 (822)
// Op slot of the DSP weight gradient the graph emits with parallel.txt = 0
// (grad/NITI_DSPConv_Int8_Grad.cpp:216-219): x^T [Ci][H][W][N] (transpose {3,1,2,0} of the NHWC
// input), dy NHWC [N][OH][OW][Co], two zero scalars -> dw [Ci][KH][KW][Co] (shape rule
// ShapeNITI_Conv_Int8.cpp:239-320 with the kernel = dy's OH x OW) and an exponent
// (NITI_DSPTransposeGradientConv_Int8.cpp:137-440).  The DSP requantises round-to-nearest
// and divides by 32 (:426-432); this backend gives the CPU weight-gradient numerics
// (NITI_GradientConv_Int8.cpp:272-296: PSTO(bw - 2)) and exp_out = the applied shift.
// Stride 1 only: for stride 2 the graph dilates dy with LeftPoolGrad and sets stride 1 (:160-190).
// NITI_DSP_GRADIENT_SPLITBatchCONV_Int8 (821), the stride-2 variant for 8 < OW <= 16, has the
// same tensors and shape rule (ShapeNITI_Conv_Int8.cpp:529-531).
class DspTransposeGradientExecution : public Execution {
   public:
    explicit DspTransposeGradientExecution(const niti_conv2d_common& c) : common_(c) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 2 || nout < 1) return NITI_INVALID_VALUE;
        const niti_tensor &xt = in[0], &dy = in[1], &o = out[0];
        if (xt.format != NITI_FORMAT_NHWC || dy.format != NITI_FORMAT_NHWC) return NITI_NOT_SUPPORT;
        if (common_.group > 1 || common_.dilate_x > 1 || common_.dilate_y > 1 || common_.stride_x > 1 ||
            common_.stride_y > 1)
            return NITI_NOT_SUPPORT;
        // NHWC logical dims {N, C, H, W}: x^T {Ci, N, H, W}, dy {N, Co, OH, OW}, dw {Ci, Co, KH, KW}
        const int ci = xt.dims[0], n = xt.dims[1], h = xt.dims[2], w = xt.dims[3];
        if (dy.dims[0] != n) return NITI_COMPUTE_SIZE_ERROR;
        const int co = dy.dims[1];
        const int pt = common_.has_pads ? common_.pads[0] : common_.pad_y;
        const int pl = common_.has_pads ? common_.pads[1] : common_.pad_x;
        const int pb = common_.has_pads ? common_.pads[2] : common_.pad_y;
        const int pr = common_.has_pads ? common_.pads[3] : common_.pad_x;
        const int kh = h + pt + pb - dy.dims[2] + 1, kw = w + pl + pr - dy.dims[3] + 1;
        if (kh <= 0 || kw <= 0) return NITI_COMPUTE_SIZE_ERROR;
        ConvGeom r{};
        r.n = n;
        r.c_in = ci;
        r.h = h;
        r.w = w;
        r.c_out = co;
        r.kh = kh;
        r.kw = kw;
        r.sh = r.sw = r.dh = r.dw = 1;
        r.pt = pt;
        r.pl = pl;
        r.pb = pb;
        r.pr = pr;
        if (!r.finalize() || r.oh != dy.dims[2] || r.ow != dy.dims[3]) return NITI_COMPUTE_SIZE_ERROR;
        g_ = r;
        if (o.dims[0] != ci || o.dims[1] != co || o.dims[2] != kh || o.dims[3] != kw) return NITI_COMPUTE_SIZE_ERROR;
        ws_.release();
        x16_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.h * g_.w * g_.cip);
        dy16_ = (int8_t*)ws_.alloc((size_t)g_.n * g_.oh * g_.ow * g_.cop);
        acc_ = (int32_t*)ws_.alloc((size_t)g_.c_out * kh * kw * g_.cip * 4);
        g8_ = (int8_t*)ws_.alloc((size_t)g_.c_out * kh * kw * g_.cip);
        amax_ = (uint32_t*)ws_.alloc(MAX_BYTES);
        slab_bytes_ = conv_wgrad_workspace(g_);
        slab_ = slab_bytes_ ? ws_.alloc(slab_bytes_) : nullptr;
        if (slab_bytes_ && !slab_) return NITI_OUT_OF_MEMORY;
        return (x16_ && dy16_ && acc_ && g8_ && amax_) ? NITI_NO_ERROR : NITI_OUT_OF_MEMORY;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!acc_) return NITI_NO_EXECUTION;
        const int hw = g_.h * g_.w, ohw = g_.oh * g_.ow, kk = g_.kh * g_.kw;
        NITI_TRY(launch_map((int64_t)g_.n * hw * g_.cip,
                            CiHwnToNhwc16{(const int8_t*)in[0].data, g_.n, g_.c_in, hw, g_.cip, x16_}, st));
        NITI_TRY(launch_map((int64_t)g_.n * ohw * g_.cop, NhwcToNhwc16{(const int8_t*)in[1].data, g_.c_out, g_.cop, dy16_}, st));
        const int64_t nacc = (int64_t)g_.c_out * kk * g_.cip;
        NITI_TRY(hipMemsetAsync(amax_, 0, MAX_BYTES, st));
        NITI_TRY(conv_wgrad_acc(g_, x16_, dy16_, acc_, amax_, slab_, slab_bytes_, st));
        NITI_TRY(requant_grad(acc_, nacc, amax_, RULE_WGRAD_BW2, g8_, nullptr, st));
        NITI_TRY(launch_map((int64_t)g_.c_in * kk * g_.c_out,
                            Ohwi16ToIhwo{g8_, g_.c_out, g_.c_in, kk, g_.cip, (int8_t*)out[0].data}, st));
        if (nout > 1 && out[1].data != nullptr) NITI_TRY(grad_exponent(amax_, RULE_WGRAD_BW2, (int8_t*)out[1].data, st));
        return NITI_NO_ERROR;
    }

   private:
    niti_conv2d_common common_;
    ConvGeom g_{};
    int8_t *x16_ = nullptr, *dy16_ = nullptr, *g8_ = nullptr;
    int32_t* acc_ = nullptr;
    uint32_t* amax_ = nullptr;
    void* slab_ = nullptr;
    size_t slab_bytes_ = 0;
};

// ------------------------------------------------------------------ element-wise slots (CPU graph and DSP graph)
// The CPU graph's NITI_Relu_Int8 (703), NITI_ReluGrad_Int8 (704), NITI_Maxpool_Int8 (705,
// {x, ascale} -> {y, ascale}, NITI_Maxpool_Int8.cpp:128-175) and NITI_PoolGrad_Int8 (706) take
// the same execution on NC4HW4 (or, element-wise, NCHW) tensors.
// NITI_DSP_RELU_Int8 (801) {x} -> {max(x, 0)}; NITI_DSP_RELUGRAD_Int8 (805) {x, dy} -> {x > 0 ? dy : 0}
// (grad/NITI_ReluGrad_Int8.cpp:29-47); NITI_DSP_NOP_Int8 (817) {x} -> {x} (the DSP binary add's
// gradient, grad/NITI_DSPBinaryGrad.cpp:14-42); NITI_DSP_MAXPOOL_Int8 (802) {x, ascale} ->
// {y, ascale} (NITI_DSPMaxpool_Int8.cpp:183 passes the scale through) and
// NITI_DSP_MAXPOOLGRAD_Int8 (807) {x, y, dy} -> {dx} (grad/NITI_Pool_Int8_Grad.cpp:40-64), on
// NHWC tensors with the CPU path's numerics (NITI_CPURelu_Int8.cpp:28-61,
// NITI_CPUReluGrad_Int8.cpp:28-62, NITI_Maxpool_Int8.cpp:24-72, NITI_CPUPoolGrad_Int8.cpp:21-77:
// first maximum wins).  The pool's NITI_Pool_Int8 {kernelX/Y, strideX/Y, padX/Y} arrive in the
// common's kernel / stride / pad fields (square windows).
struct ReluMap {
    const int8_t* x;
    int8_t* y;
    __device__ void operator()(int64_t i) const { y[i] = x[i] > 0 ? x[i] : (int8_t)0; }
};
struct ReluGradMap {
    const int8_t* x;
    const int8_t* dy;
    int8_t* y;
    __device__ void operator()(int64_t i) const { y[i] = x[i] > 0 ? dy[i] : (int8_t)0; }
};
struct CopyMap {
    const int8_t* x;
    int8_t* y;
    __device__ void operator()(int64_t i) const { y[i] = x[i]; }
};

class DspElementwiseExecution : public Execution {
   public:
    enum Kind { RELU, RELUGRAD, NOP, POOL, POOLGRAD };
    DspElementwiseExecution(int op, const niti_conv2d_common& c) : common_(c) {
        cpu_ = op >= NITI_OP_RELU_INT8 && op <= NITI_OP_POOLGRAD_INT8;
        switch (op) {
            case NITI_OP_RELU_INT8:
            case NITI_OP_DSP_RELU_INT8: kind_ = RELU; break;
            case NITI_OP_RELUGRAD_INT8:
            case NITI_OP_DSP_RELUGRAD_INT8: kind_ = RELUGRAD; break;
            case NITI_OP_MAXPOOL_INT8:
            case NITI_OP_DSP_MAXPOOL_INT8: kind_ = POOL; break;
            case NITI_OP_POOLGRAD_INT8:
            case NITI_OP_DSP_MAXPOOLGRAD_INT8: kind_ = POOLGRAD; break;
            default: kind_ = NOP; break;
        }
    }
    // NHWC-equivalent dims {n, c, h, w} of t: NHWC as is; for the CPU slots NC4HW4
    // [C/4][N][H][W][4] is NHWC with n * ceil(c / 4) images of 4 channels (the CPU ops work per
    // 4-channel plane, NITI_CPUPoolGrad_Int8.cpp:28-40), and element-wise ops also take NCHW
    bool view(const niti_tensor& t, int d[4]) const {
        if (t.format == NITI_FORMAT_NHWC || (cpu_ && kind_ != POOL && kind_ != POOLGRAD && t.format == NITI_FORMAT_NCHW)) {
            for (int k = 0; k < 4; ++k) d[k] = t.dims[k];
            return true;
        }
        if (cpu_ && t.format == NITI_FORMAT_NC4HW4) {
            d[0] = t.dims[0] * ((t.dims[1] + 3) / 4), d[1] = 4, d[2] = t.dims[2], d[3] = t.dims[3];
            return true;
        }
        return false;
    }
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        const int need = kind_ == RELUGRAD ? 2 : kind_ == POOLGRAD ? 3 : 1;
        if (nin < need || nout < 1) return NITI_INVALID_VALUE;
        int xd[4], od[4], d1[4] = {0, 0, 0, 0}, d2[4] = {0, 0, 0, 0};
        if (!view(in[0], xd) || !view(out[0], od)) return NITI_NOT_SUPPORT;
        if (need >= 2 && !view(in[1], d1)) return NITI_NOT_SUPPORT;
        if (need >= 3 && !view(in[2], d2)) return NITI_NOT_SUPPORT;
        for (int i = 1; i < need; ++i)
            if (in[i].format != in[0].format) return NITI_NOT_SUPPORT;
        if (out[0].format != in[0].format) return NITI_NOT_SUPPORT;
        n_ = xd[0], c_ = xd[1], h_ = xd[2], w_ = xd[3];
        elems_ = (int64_t)n_ * c_ * h_ * w_;
        ready_ = false;
        if (kind_ == POOL || kind_ == POOLGRAD) {
            k_ = common_.kernel_x, s_ = common_.stride_x, p_ = common_.pad_x;
            if (common_.kernel_y != k_ || common_.stride_y != s_ || common_.pad_y != p_ || k_ < 1 || s_ < 1 || p_ < 0)
                return NITI_NOT_SUPPORT;
            oh_ = (h_ + 2 * p_ - std::min(k_, h_)) / s_ + 1;
            ow_ = (w_ + 2 * p_ - std::min(k_, w_)) / s_ + 1;
            const int* yd = kind_ == POOL ? od : d1;
            if (yd[0] != n_ || yd[1] != c_ || yd[2] != oh_ || yd[3] != ow_) return NITI_COMPUTE_SIZE_ERROR;
            if (kind_ == POOLGRAD) {
                for (int k = 0; k < 4; ++k)
                    if (d2[k] != yd[k] || od[k] != xd[k]) return NITI_COMPUTE_SIZE_ERROR;
            }
            cp_ = (c_ + 15) / 16 * 16;
            ws_.release();
            const size_t big = (size_t)n_ * h_ * w_ * cp_, small = (size_t)n_ * oh_ * ow_ * cp_;
            x16_ = (int8_t*)ws_.alloc(big);
            y16_ = (int8_t*)ws_.alloc(small);
            if (kind_ == POOLGRAD) {
                dy16_ = (int8_t*)ws_.alloc(small);
                dx16_ = (int8_t*)ws_.alloc(big);
                if (!dy16_ || !dx16_) return NITI_OUT_OF_MEMORY;
            }
            if (!x16_ || !y16_) return NITI_OUT_OF_MEMORY;
        } else {
            for (int k = 0; k < 4; ++k)
                if (od[k] != xd[k] || (need == 2 && d1[k] != xd[k])) return NITI_COMPUTE_SIZE_ERROR;
        }
        ready_ = true;
        return NITI_NO_ERROR;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!ready_) return NITI_NO_EXECUTION;
        const int8_t* x = (const int8_t*)in[0].data;
        int8_t* o = (int8_t*)out[0].data;
        switch (kind_) {
            case RELU: NITI_TRY(launch_map(elems_, ReluMap{x, o}, st)); break;
            case NOP: NITI_TRY(launch_map(elems_, CopyMap{x, o}, st)); break;
            case RELUGRAD: NITI_TRY(launch_map(elems_, ReluGradMap{x, (const int8_t*)in[1].data, o}, st)); break;
            case POOL: {
                const int64_t rows = (int64_t)n_ * oh_ * ow_;
                NITI_TRY(launch_map((int64_t)n_ * h_ * w_ * cp_, NhwcToNhwc16{x, c_, cp_, x16_}, st));
                NITI_TRY(maxpool_nhwc16(x16_, n_, h_, w_, cp_, k_, s_, p_, y16_, oh_, ow_, st));
                NITI_TRY(launch_map(rows * c_, UnpadRows{y16_, c_, cp_, o}, st));
                if (nin > 1 && nout > 1 && in[1].data && out[1].data)
                    NITI_TRY(hipMemcpyAsync(out[1].data, in[1].data, 1, hipMemcpyDeviceToDevice, st));
                break;
            }
            default: {  // POOLGRAD
                const int64_t small = (int64_t)n_ * oh_ * ow_ * cp_, rows = (int64_t)n_ * h_ * w_;
                NITI_TRY(launch_map(rows * cp_, NhwcToNhwc16{x, c_, cp_, x16_}, st));
                NITI_TRY(launch_map(small, NhwcToNhwc16{(const int8_t*)in[1].data, c_, cp_, y16_}, st));
                NITI_TRY(launch_map(small, NhwcToNhwc16{(const int8_t*)in[2].data, c_, cp_, dy16_}, st));
                NITI_TRY(maxpool_relu_grad_nhwc16(x16_, y16_, dy16_, n_, h_, w_, cp_, k_, s_, p_, oh_, ow_, 0, dx16_, st));
                NITI_TRY(launch_map(rows * c_, UnpadRows{dx16_, c_, cp_, o}, st));
                break;
            }
        }
        return NITI_NO_ERROR;
    }

   private:
    Kind kind_ = NOP;
    bool cpu_ = false;
    niti_conv2d_common common_;
    bool ready_ = false;
    int n_ = 0, c_ = 0, h_ = 0, w_ = 0, k_ = 0, s_ = 0, p_ = 0, oh_ = 0, ow_ = 0, cp_ = 0;
    int64_t elems_ = 0;
    int8_t *x16_ = nullptr, *y16_ = nullptr, *dy16_ = nullptr, *dx16_ = nullptr;
};

// ------------------------------------------------------------------ 806: reference max-pool grad
// NITI_DSP_MAXPOOLGRAD_REF_Int8 (NITI_DSPMaxPoolGradRef_Int8.cpp:17-80), restated literally.  The
// op reads its NHWC tensors as [ih = batch][iw = height][ib = width][ic = channel] (:23-28) and
// walks windows (i, j) with i += strideX over ih, j += strideY over iw (:36-37); per window and
// per 128-byte chunk of the bc = ib * ic plane (:41-43; a tail of bc % 128 bytes is never
// visited) it routes dy to the first (ky outer, kx inner) position whose x equals the pooled y and
// writes 0 to the window's other positions (:59-88).  y and dy are read at
// (offset * bc) / kernelX / kernelY, offset = i * iw + j (:54-55), integer division in that order.
// Output bytes no window visits keep their value.  Overlapping windows (stride < kernel) make the
// reference's result depend on its sequential order and windows reaching past the tensor read out
// of bounds there: both are NOT_SUPPORT.
struct PoolGradRefMap {
    const int8_t* x;   // origin
    const int8_t* y;   // outputOrigin (pooled)
    const int8_t* dy;  // outputDiff
    int8_t* out;
    int64_t bc, chunk;  // plane bytes, visited bytes per window (bc / 128 * 128)
    int iw, sx, sy, kx, ky, nwj;
    __device__ void operator()(int64_t t) const {
        const int64_t w = t / chunk, e = t - w * chunk;
        const int wi = (int)(w / nwj), wj = (int)(w - (int64_t)wi * nwj);
        const int64_t offset = (int64_t)(wi * sx) * iw + wj * sy;
        const int64_t yo = offset * bc / kx / ky + e;
        const int8_t m = y[yo], g = dy[yo];
        bool done = false;
        for (int a = 0; a < ky; ++a)
            for (int b = 0; b < kx; ++b) {
                const int64_t o = (offset + (int64_t)a * iw + b) * bc + e;
                const bool take = !done && x[o] == m;
                out[o] = take ? g : (int8_t)0;
                done = done || take;
            }
    }
};

class DspMaxPoolGradRefExecution : public Execution {
   public:
    explicit DspMaxPoolGradRefExecution(const niti_conv2d_common& c) : c_(c) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        ready_ = false;
        if (nin < 3 || nout < 1) return NITI_INVALID_VALUE;
        for (int i = 0; i < 3; ++i)
            if (in[i].format != NITI_FORMAT_NHWC) return NITI_NOT_SUPPORT;
        if (out[0].format != NITI_FORMAT_NHWC) return NITI_NOT_SUPPORT;
        // logical {N, C, H, W} of NHWC storage: ih = N, iw = H, ib = W, ic = C
        ih_ = in[0].dims[0], iw_ = in[0].dims[2];
        bc_ = (int64_t)in[0].dims[3] * in[0].dims[1];
        sx_ = c_.stride_x, sy_ = c_.stride_y, kx_ = c_.kernel_x, ky_ = c_.kernel_y;
        if (sx_ < 1 || sy_ < 1 || kx_ < 1 || ky_ < 1 || ih_ < 1 || iw_ < 1 || bc_ < 1) return NITI_INVALID_VALUE;
        if (sx_ < ky_ || sy_ < kx_) return NITI_NOT_SUPPORT;  // overlapping windows
        for (int k = 0; k < 4; ++k)
            if (out[0].dims[k] != in[0].dims[k]) return NITI_COMPUTE_SIZE_ERROR;
        nwi_ = (ih_ + sx_ - 1) / sx_, nwj_ = (iw_ + sy_ - 1) / sy_;
        if ((nwi_ - 1) * sx_ + ky_ > ih_ || (nwj_ - 1) * sy_ + kx_ > iw_) return NITI_NOT_SUPPORT;  // past the tensor
        chunk_ = bc_ / 128 * 128;
        const int64_t offset_last = (int64_t)((nwi_ - 1) * sx_) * iw_ + (nwj_ - 1) * sy_;
        const int64_t ylen = (int64_t)in[1].dims[0] * in[1].dims[1] * in[1].dims[2] * in[1].dims[3];
        const int64_t dlen = (int64_t)in[2].dims[0] * in[2].dims[1] * in[2].dims[2] * in[2].dims[3];
        if (chunk_ > 0 && (offset_last * bc_ / kx_ / ky_ + chunk_ > ylen || offset_last * bc_ / kx_ / ky_ + chunk_ > dlen))
            return NITI_COMPUTE_SIZE_ERROR;
        ready_ = true;
        return NITI_NO_ERROR;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!ready_) return NITI_NO_EXECUTION;
        if (chunk_ == 0) return NITI_NO_ERROR;
        NITI_TRY(launch_map((int64_t)nwi_ * nwj_ * chunk_,
                            PoolGradRefMap{(const int8_t*)in[0].data, (const int8_t*)in[1].data, (const int8_t*)in[2].data,
                                           (int8_t*)out[0].data, bc_, chunk_, iw_, sx_, sy_, kx_, ky_, nwj_},
                            st));
        return NITI_NO_ERROR;
    }

   private:
    niti_conv2d_common c_;
    bool ready_ = false;
    int ih_ = 0, iw_ = 0, sx_ = 0, sy_ = 0, kx_ = 0, ky_ = 0, nwi_ = 0, nwj_ = 0;
    int64_t bc_ = 0, chunk_ = 0;
};

// ------------------------------------------------------------------ loss gradient slots
// NITI_LOSS_Grad_Int8 (711, NITI_CPULossGrad_Int8.cpp:81-200) and NITI_DSP_LOSSGRAD_Int8 (804,
// grad/NITI_SoftmaxGrad.cpp:41-66 builds either from the same inputs): {logits int8 [batch][classes],
// ascale int8[1], target int32 one-hot [batch][tc], dy (unused)} -> {grad int8 [batch][classes]}.
// The target row's first 1 is the class (:169-178); a row without one counts as class 0.
struct OnehotToIndex {
    const int32_t* t;
    int tc;
    int32_t* label;
    __device__ void operator()(int64_t i) const {
        int32_t k = 0;
        for (int j = tc - 1; j >= 0; --j)
            if (t[i * tc + j] == 1) k = j;
        label[i] = k;
    }
};

class LossGradExecution : public Execution {
   public:
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < 3 || nout < 1) return NITI_INVALID_VALUE;
        const niti_tensor &x = in[0], &t = in[2], &o = out[0];
        if (x.format == NITI_FORMAT_NC4HW4 || o.format == NITI_FORMAT_NC4HW4) return NITI_NOT_SUPPORT;
        batch_ = x.dims[0];
        classes_ = x.dims[1] * x.dims[2] * x.dims[3];
        tc_ = t.dims[1] * t.dims[2] * t.dims[3];
        if (batch_ <= 0 || classes_ <= 0 || classes_ > 2048 || t.dims[0] != batch_ || tc_ <= 0)
            return classes_ > 2048 ? NITI_NOT_SUPPORT : NITI_COMPUTE_SIZE_ERROR;
        if (o.dims[0] != batch_ || o.dims[1] * o.dims[2] * o.dims[3] != classes_) return NITI_COMPUTE_SIZE_ERROR;
        ws_.release();
        label_ = (int32_t*)ws_.alloc((size_t)batch_ * 4);
        return label_ ? NITI_NO_ERROR : NITI_OUT_OF_MEMORY;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!label_) return NITI_NO_EXECUTION;
        NITI_TRY(launch_map(batch_, OnehotToIndex{(const int32_t*)in[2].data, tc_, label_}, st));
        NITI_TRY(loss_grad((const int8_t*)in[0].data, batch_, classes_, classes_, (const int8_t*)in[1].data, label_,
                           (int8_t*)out[0].data, st));
        return NITI_NO_ERROR;
    }

   private:
    int batch_ = 0, classes_ = 0, tc_ = 0;
    int32_t* label_ = nullptr;
};

// ------------------------------------------------------------------ NITI_DSP layout slots
// The DSP graph's data-movement ops, on the tensors' stored (raw) axis order -- [N][H][W][C] for
// NHWC, [N][C][H][W] for NCHW -- as MNN's NHWC kernels index them:
//   NITI_DSP_TRANSPOSE_Int8 (808)   {x, perm int32[4]} -> x permuted (NeuralNetWorkOp.cpp:2170-2182)
//   NITI_DSP_WEIGHTROTATE180_REF_Int8 (809) {w} -> w with raw axes 2 and 3 reversed (the graph
//                                    applies it to transpose(w, {2,3,0,1}): the kernel window)
//   NITI_DSP_LEFTPOOLGRAD_DECONV / _GRADIENT_Int8 (814 / 815) {dy NHWC} -> NHWC of the output's
//                                    size with dy[i][j] at (s*i, s*j) and zeros elsewhere
//                                    (NeuralNetWorkOp.cpp:2202-2230; stride in the common)
//   NITI_DSP_RESHAPE_Int8 / RESHAPEGrad (803 / 813) {x} -> the same bytes under the output's dims
//   NITI_DSP_PAD_Int8 (812)          {x NHWC} -> NHWC with a zero border of NITI_PAD_Int8.pad pixels
//                                    (ShapeNITI_Pad_Int8.cpp:42-68; the pad in the common's pad_x)
struct Raw4 {
    int d[4];
};
static Raw4 raw_dims(const niti_tensor& t) {
    if (t.format == NITI_FORMAT_NHWC) return Raw4{{t.dims[0], t.dims[2], t.dims[3], t.dims[1]}};
    return Raw4{{t.dims[0], t.dims[1], t.dims[2], t.dims[3]}};
}
struct PermuteMap {
    const int8_t* x;
    int8_t* y;
    int od[4];
    int64_t is[4];  // input stride of output axis k
    __device__ void operator()(int64_t i) const {
        int64_t off = 0, r = i;
#pragma unroll
        for (int k = 3; k >= 0; --k) {
            off += (r % od[k]) * is[k];
            r /= od[k];
        }
        y[i] = x[off];
    }
};
struct Rotate180Map {
    const int8_t* x;
    int8_t* y;
    int H, W;
    __device__ void operator()(int64_t i) const {
        const int j = (int)(i % W), r = (int)((i / W) % H);
        const int64_t base = i - (int64_t)r * W - j;
        y[i] = x[base + (int64_t)(H - 1 - r) * W + (W - 1 - j)];
    }
};
struct LeftPoolGradMap {
    const int8_t* dy;
    int8_t* y;
    int C, OW2, OH2, IH, IW, sy, sx;  // output OH2 x OW2, input IH x IW
    __device__ void operator()(int64_t i) const {
        const int c = (int)(i % C);
        int64_t r = i / C;
        const int ox = (int)(r % OW2);
        r /= OW2;
        const int oy = (int)(r % OH2);
        const int64_t n = r / OH2;
        int8_t v = 0;
        if (oy % sy == 0 && ox % sx == 0 && oy / sy < IH && ox / sx < IW)
            v = dy[((n * IH + oy / sy) * IW + ox / sx) * C + c];
        y[i] = v;
    }
};

struct PadMap {  // NHWC zero border of p pixels
    const int8_t* x;
    int8_t* y;
    int C, OW, OH, H, W, p;
    __device__ void operator()(int64_t i) const {
        const int c = (int)(i % C);
        int64_t r = i / C;
        const int ox = (int)(r % OW);
        r /= OW;
        const int oy = (int)(r % OH);
        const int64_t n = r / OH;
        const int iy = oy - p, ix = ox - p;
        y[i] = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W ? x[((n * H + iy) * W + ix) * C + c] : (int8_t)0;
    }
};

class DspLayoutExecution : public Execution {
   public:
    DspLayoutExecution(int op, const niti_conv2d_common& c) : op_(op), common_(c) {}
    int onResize(const niti_tensor* in, int nin, const niti_tensor* out, int nout) override {
        if (nin < (op_ == NITI_OP_DSP_TRANSPOSE_INT8 ? 2 : 1) || nout < 1) return NITI_INVALID_VALUE;
        ready_ = false;
        // the CPU graph's NITI_PAD_Int8 (714) pads NCHW planes (NITI_Pad_Int8.cpp:24-62) and its
        // NITI_LeftPoolGrad_Int8 (718) dilates NC4HW4 4-channel planes (NITI_CPULeftPoolGrad_Int8.cpp:
        // 18-47): both are the NHWC maps below on [N*C][H][W][1] / [N*C4][H][W][4] views
        Raw4 xi = raw_dims(in[0]), yo = raw_dims(out[0]);
        if (op_ == NITI_OP_PAD_INT8 || op_ == NITI_OP_LEFTPOOLGRAD_INT8) {
            const int f = op_ == NITI_OP_PAD_INT8 ? NITI_FORMAT_NCHW : NITI_FORMAT_NC4HW4;
            if (in[0].format != f || out[0].format != f) return NITI_NOT_SUPPORT;
            if (in[0].dims[0] != out[0].dims[0] || in[0].dims[1] != out[0].dims[1]) return NITI_COMPUTE_SIZE_ERROR;
            auto v = [&](const niti_tensor& t) {
                return f == NITI_FORMAT_NCHW ? Raw4{{t.dims[0] * t.dims[1], t.dims[2], t.dims[3], 1}}
                                             : Raw4{{t.dims[0] * ((t.dims[1] + 3) / 4), t.dims[2], t.dims[3], 4}};
            };
            xi = v(in[0]), yo = v(out[0]);
        }
        n_ = 1;
        for (int k = 0; k < 4; ++k) n_ *= yo.d[k];
        int64_t nx = 1;
        for (int k = 0; k < 4; ++k) nx *= xi.d[k];
        switch (op_) {
            case NITI_OP_DSP_TRANSPOSE_INT8: {
                int perm[4];
                if (hipMemcpy(perm, in[1].data, sizeof(perm), hipMemcpyDefault) != hipSuccess) return NITI_INVALID_VALUE;
                int64_t st[4];
                st[3] = 1;
                for (int k = 2; k >= 0; --k) st[k] = st[k + 1] * xi.d[k + 1];
                int seen = 0;
                for (int k = 0; k < 4; ++k) {
                    if (perm[k] < 0 || perm[k] > 3 || (seen >> perm[k]) & 1) return NITI_INVALID_VALUE;
                    seen |= 1 << perm[k];
                    if (yo.d[k] != xi.d[perm[k]]) return NITI_COMPUTE_SIZE_ERROR;
                    pm_.od[k] = yo.d[k];
                    pm_.is[k] = st[perm[k]];
                }
                break;
            }
            case NITI_OP_DSP_WEIGHTROTATE180_INT8:
                for (int k = 0; k < 4; ++k)
                    if (xi.d[k] != yo.d[k]) return NITI_COMPUTE_SIZE_ERROR;
                rh_ = xi.d[2], rw_ = xi.d[3];
                break;
            case NITI_OP_LEFTPOOLGRAD_INT8:
            case NITI_OP_DSP_LEFTPOOLGRAD_DECONV_INT8:
            case NITI_OP_DSP_LEFTPOOLGRAD_GRADIENT_INT8:
                if (op_ != NITI_OP_LEFTPOOLGRAD_INT8 && (in[0].format != NITI_FORMAT_NHWC || out[0].format != NITI_FORMAT_NHWC))
                    return NITI_NOT_SUPPORT;
                if (common_.stride_x < 1 || common_.stride_y < 1) return NITI_INVALID_VALUE;
                if (xi.d[0] != yo.d[0] || xi.d[3] != yo.d[3]) return NITI_COMPUTE_SIZE_ERROR;
                lp_ = LeftPoolGradMap{nullptr, nullptr, xi.d[3], yo.d[2], yo.d[1], xi.d[1], xi.d[2], common_.stride_y,
                                      common_.stride_x};
                break;
            case NITI_OP_PAD_INT8:
            case NITI_OP_DSP_PAD_INT8: {
                const int p = common_.pad_x;
                if (p < 0 || (op_ == NITI_OP_DSP_PAD_INT8 &&
                              (in[0].format != NITI_FORMAT_NHWC || out[0].format != NITI_FORMAT_NHWC)))
                    return NITI_NOT_SUPPORT;
                if (yo.d[0] != xi.d[0] || yo.d[3] != xi.d[3] || yo.d[1] != xi.d[1] + 2 * p || yo.d[2] != xi.d[2] + 2 * p)
                    return NITI_COMPUTE_SIZE_ERROR;
                pad_ = PadMap{nullptr, nullptr, xi.d[3], yo.d[2], yo.d[1], xi.d[1], xi.d[2], p};
                break;
            }
            default:  // reshape: same bytes
                if (nx != n_) return NITI_COMPUTE_SIZE_ERROR;
                break;
        }
        ready_ = true;
        return NITI_NO_ERROR;
    }
    int onExecute(const niti_tensor* in, int nin, const niti_tensor* out, int nout, hipStream_t st) override {
        if (!ready_) return NITI_NO_EXECUTION;
        const int8_t* x = (const int8_t*)in[0].data;
        int8_t* y = (int8_t*)out[0].data;
        switch (op_) {
            case NITI_OP_DSP_TRANSPOSE_INT8: {
                PermuteMap m = pm_;
                m.x = x, m.y = y;
                NITI_TRY(launch_map(n_, m, st));
                break;
            }
            case NITI_OP_DSP_WEIGHTROTATE180_INT8: NITI_TRY(launch_map(n_, Rotate180Map{x, y, rh_, rw_}, st)); break;
            case NITI_OP_LEFTPOOLGRAD_INT8:
            case NITI_OP_DSP_LEFTPOOLGRAD_DECONV_INT8:
            case NITI_OP_DSP_LEFTPOOLGRAD_GRADIENT_INT8: {
                LeftPoolGradMap m = lp_;
                m.dy = x, m.y = y;
                NITI_TRY(launch_map(n_, m, st));
                break;
            }
            case NITI_OP_PAD_INT8:
            case NITI_OP_DSP_PAD_INT8: {
                PadMap m = pad_;
                m.x = x, m.y = y;
                NITI_TRY(launch_map(n_, m, st));
                break;
            }
            default: NITI_TRY(launch_map(n_, CopyMap{x, y}, st)); break;
        }
        return NITI_NO_ERROR;
    }

   private:
    int op_;
    niti_conv2d_common common_;
    bool ready_ = false;
    int64_t n_ = 0;
    int rh_ = 0, rw_ = 0;
    PadMap pad_{};
    PermuteMap pm_{};
    LeftPoolGradMap lp_{};
};

// ------------------------------------------------------------------ tensor format conversion
// CPUTensorConverter::convert (CPUTensorConvert.cpp:98-210) for int8 tensors between NCHW,
// NHWC and MNN's CPU NC4HW4 ([ceil(C/4)][N][H][W][4], pad lanes zero), SURVEY.md §8(f)-3.
// One pass over the destination: element i decodes to (n, c, h, w) in the destination format
// and reads the source element in its own format.
struct FormatIndex {
    int N, C, H, W;
    __device__ int64_t index(int f, int n, int c, int h, int w) const {
        if (f == NITI_FORMAT_NCHW) return (((int64_t)n * C + c) * H + h) * W + w;
        if (f == NITI_FORMAT_NHWC) return (((int64_t)n * H + h) * W + w) * C + c;
        return ((((int64_t)(c >> 2) * N + n) * H + h) * W + w) * 4 + (c & 3);
    }
    __device__ void decode(int f, int64_t i, int* n, int* c, int* h, int* w) const {
        if (f == NITI_FORMAT_NCHW) {
            *w = (int)(i % W), i /= W;
            *h = (int)(i % H), i /= H;
            *c = (int)(i % C), *n = (int)(i / C);
        } else if (f == NITI_FORMAT_NHWC) {
            *c = (int)(i % C), i /= C;
            *w = (int)(i % W), i /= W;
            *h = (int)(i % H), *n = (int)(i / H);
        } else {
            const int lane = (int)(i & 3);
            i >>= 2;
            *w = (int)(i % W), i /= W;
            *h = (int)(i % H), i /= H;
            *n = (int)(i % N);
            *c = (int)(i / N) * 4 + lane;
        }
    }
};
struct ConvertFormat {
    const int8_t* src;
    int8_t* dst;
    FormatIndex ix;
    int sf, df;
    __device__ void operator()(int64_t i) const {
        int n, c, h, w;
        ix.decode(df, i, &n, &c, &h, &w);
        dst[i] = c < ix.C ? src[ix.index(sf, n, c, h, w)] : (int8_t)0;
    }
};

int convert_tensor(const niti_tensor& s, const niti_tensor& d, hipStream_t st) {
    for (int k = 0; k < 4; ++k)
        if (s.dims[k] != d.dims[k] || s.dims[k] <= 0) return NITI_COMPUTE_SIZE_ERROR;
    auto ok = [](int f) { return f == NITI_FORMAT_NCHW || f == NITI_FORMAT_NHWC || f == NITI_FORMAT_NC4HW4; };
    if (!ok(s.format) || !ok(d.format)) return NITI_NOT_SUPPORT;
    if (s.data == nullptr || d.data == nullptr || s.data == d.data) return NITI_INVALID_VALUE;
    const FormatIndex ix{s.dims[0], s.dims[1], s.dims[2], s.dims[3]};
    const int64_t cs = d.format == NITI_FORMAT_NC4HW4 ? (int64_t)(ix.C + 3) / 4 * 4 : ix.C;
    const int64_t total = (int64_t)ix.N * cs * ix.H * ix.W;
    const hipError_t e =
        launch_map(total, ConvertFormat{(const int8_t*)s.data, (int8_t*)d.data, ix, s.format, d.format}, st);
    return e == hipSuccess ? NITI_NO_ERROR : NITI_INVALID_VALUE;
}

Execution* create_execution(int op_type, const niti_conv2d_common* c, int* err) {
    *err = NITI_NO_ERROR;
    niti_conv2d_common dflt{};
    dflt.kernel_x = dflt.kernel_y = dflt.stride_x = dflt.stride_y = dflt.dilate_x = dflt.dilate_y = 1;
    dflt.group = 1;
    const niti_conv2d_common& cc = c ? *c : dflt;
    const bool no_params = op_type == NITI_OP_MATMUL_INT8 || op_type == NITI_OP_DSP_RELU_INT8 ||
                           op_type == NITI_OP_RELU_INT8 || op_type == NITI_OP_RELUGRAD_INT8 ||
                           op_type == NITI_OP_DSP_RELUGRAD_INT8 || op_type == NITI_OP_DSP_NOP_INT8 ||
                           op_type == NITI_OP_LOSS_GRAD_INT8 || op_type == NITI_OP_DSP_LOSSGRAD_INT8 ||
                           op_type == NITI_OP_DSP_TRANSPOSE_INT8 || op_type == NITI_OP_DSP_WEIGHTROTATE180_INT8 ||
                           op_type == NITI_OP_DSP_RESHAPE_INT8 || op_type == NITI_OP_DSP_RESHAPEGRAD_INT8;
    if (!no_params && c == nullptr) {
        *err = NITI_INVALID_VALUE;
        return nullptr;
    }
    if (cc.group > 1) {
        *err = NITI_NOT_SUPPORT;
        return nullptr;
    }
    switch (op_type) {
        case NITI_OP_CONV_INT8: return new ConvInt8Execution(cc);
        case NITI_OP_DECONV_INT8: return new DeconvInt8Execution(cc);
        case NITI_OP_GRADIENT_CONV_INT8: return new GradientConvInt8Execution(cc);
        case NITI_OP_MATMUL_INT8: return new MatmulInt8Execution();
        case NITI_OP_DSP_MATMUL_GRADIENT_INT8: return new DspMatmulGradientExecution(cc);
        case NITI_OP_DSP_CONV_INT8:
        case NITI_OP_DSP_DECONV_INT8: return new DspConvExecution(cc);
        case NITI_OP_DSP_GRADIENTCONV_INT8:
        case NITI_OP_DSP_MATMUL_INT8:
        case NITI_OP_DSP_PARALLEL_GRADIENTCONV_INT8: return new DspMatmulGradientExecution(cc, true);
        case NITI_OP_LOSS_GRAD_INT8:
        case NITI_OP_DSP_LOSSGRAD_INT8: return new LossGradExecution();
        case NITI_OP_DSP_TRANSPOSE_INT8:
        case NITI_OP_DSP_WEIGHTROTATE180_INT8:
        case NITI_OP_DSP_LEFTPOOLGRAD_DECONV_INT8:
        case NITI_OP_DSP_LEFTPOOLGRAD_GRADIENT_INT8:
        case NITI_OP_PAD_INT8:
        case NITI_OP_LEFTPOOLGRAD_INT8:
        case NITI_OP_DSP_PAD_INT8:
        case NITI_OP_DSP_RESHAPE_INT8:
        case NITI_OP_DSP_RESHAPEGRAD_INT8: return new DspLayoutExecution(op_type, cc);
        case NITI_OP_RELU_INT8:
        case NITI_OP_RELUGRAD_INT8:
        case NITI_OP_MAXPOOL_INT8:
        case NITI_OP_POOLGRAD_INT8:
        case NITI_OP_DSP_RELU_INT8:
        case NITI_OP_DSP_RELUGRAD_INT8:
        case NITI_OP_DSP_NOP_INT8:
        case NITI_OP_DSP_MAXPOOL_INT8:
        case NITI_OP_DSP_MAXPOOLGRAD_INT8: return new DspElementwiseExecution(op_type, cc);
        case NITI_OP_DSP_MAXPOOLGRAD_REF_INT8: return new DspMaxPoolGradRefExecution(cc);
        case NITI_OP_DSP_GRADIENT_SPLITBATCHCONV_INT8:
        case NITI_OP_DSP_TRANSPOSEGRADIENT_CONV_INT8: return new DspTransposeGradientExecution(cc);
        default: *err = NITI_NOT_SUPPORT; return nullptr;
    }
}

}  // namespace niti
