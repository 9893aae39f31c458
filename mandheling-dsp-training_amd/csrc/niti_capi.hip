// niti_capi.hip -- extern "C" entry points of sections 1 and 2 of include/niti_hip.h.
#include "../../include/niti_hip.h"
#include <vector>

#include "niti_internal.hpp"
#include "niti_kernels.hpp"

// Host tensors: MNN's CPU backend hands Executions Tensor::host<T>() pointers
// (source/core/Execution.hpp:24-82, express/Executor.cpp:559-569).  Any tensor whose pointer is
// not device memory (hipPointerGetAttributes) is staged through a device buffer the handle keeps:
// inputs and outputs copied in before onExecute, outputs copied back after, and the call returns
// once the host outputs are written (the CPU backend's onExecute is synchronous).
struct niti_execution {
    niti::Execution* impl = nullptr;
    int op = 0;
    std::vector<void*> stage;
    std::vector<size_t> stage_bytes;
    uint32_t* err_host = nullptr;  // pinned copy of the Execution's error word (synchronous calls)
    ~niti_execution() {
        delete impl;
        for (void* p : stage)
            if (p) (void)hipFree(p);
        if (err_host) (void)hipHostFree(err_host);
    }
};

namespace {
int code(hipError_t e) {
    if (e == hipSuccess) return NITI_NO_ERROR;
    if (e == hipErrorOutOfMemory) return NITI_OUT_OF_MEMORY;
    if (e == hipErrorInvalidValue) return NITI_INVALID_VALUE;
    return NITI_NO_EXECUTION;
}
// false when ConvGeom::finalize rejects the geometry (callers return COMPUTE_SIZE_ERROR)
bool to_geom(const niti_geom* g, niti::ConvGeom* out) {
    niti::ConvGeom& r = *out;
    r = niti::ConvGeom{};
    r.n = g->n;
    r.c_in = g->c_in;
    r.h = g->h;
    r.w = g->w;
    r.c_out = g->c_out;
    r.kh = g->kh;
    r.kw = g->kw;
    r.sh = g->stride_h;
    r.sw = g->stride_w;
    r.pt = g->pad_t;
    r.pl = g->pad_l;
    r.pb = g->pad_b;
    r.pr = g->pad_r;
    r.dh = g->dilate_h;
    r.dw = g->dilate_w;
    return r.finalize();
}
inline hipStream_t S(void* s) { return (hipStream_t)s; }
// true for pageable or pinned host memory (anything hipPointerGetAttributes does not report as
// device or managed memory)
bool is_host_pointer(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return true;
    }
    return a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged;
}

// bytes of one Execution tensor: int8 elements, NC4HW4 with the channel count rounded up to 4
// (MNN's CPU layout [ceil(C/4)][N][H][W][4]); the loss gradient's one-hot target and the
// transpose's permutation are int32
size_t tensor_bytes(int op, bool is_out, int idx, const niti_tensor& t) {
    int64_t d[4];
    for (int k = 0; k < 4; ++k) {
        if (t.dims[k] < 0) return 0;
        d[k] = t.dims[k];
    }
    if (!is_out && idx == 2 && (op == NITI_OP_LOSS_GRAD_INT8 || op == NITI_OP_DSP_LOSSGRAD_INT8))
        return (size_t)(d[0] * d[1] * d[2] * d[3] * 4);
    if (!is_out && idx == 1 && op == NITI_OP_DSP_TRANSPOSE_INT8) return 4 * sizeof(int32_t);
    if (t.format == NITI_FORMAT_NC4HW4) return (size_t)(d[0] * ((d[1] + 3) / 4) * 4 * d[2] * d[3]);
    return (size_t)(d[0] * d[1] * d[2] * d[3]);
}

// The Execution's error word after `st` completes: NITI_NO_EXECUTION (and the word cleared) if a
// launch flagged invalid results, else NITI_NO_ERROR.  copied: the word was already copied into
// err_host on `st` (the staged path enqueues that copy before its synchronize).
int take_error(niti_execution* e, hipStream_t st, bool copied) {
    uint32_t* dev = e->impl->errorFlag();
    if (dev == nullptr) return NITI_NO_ERROR;
    uint32_t v = 0;
    if (copied) {
        v = *e->err_host;
    } else if (hipStreamSynchronize(st) != hipSuccess || hipMemcpy(&v, dev, 4, hipMemcpyDeviceToHost) != hipSuccess) {
        return NITI_NO_EXECUTION;
    }
    if (v == 0) return NITI_NO_ERROR;
    (void)hipMemsetAsync(dev, 0, 4, st);
    (void)hipStreamSynchronize(st);
    return NITI_NO_EXECUTION;
}
}  // namespace

extern "C" {

const char* niti_version(void) { return "niti-mi355x 0.1 (gfx950, int8 MFMA v_mfma_i32_32x32x32_i8)"; }

// ------------------------------------------------------------------ section 1
int niti_create_execution(int op_type, const niti_conv2d_common* common, niti_execution_t* out) {
    if (!out) return NITI_INVALID_VALUE;
    int err = NITI_NO_ERROR;
    niti::Execution* e = niti::create_execution(op_type, common, &err);
    if (!e) return err;
    auto* h = new niti_execution();
    h->impl = e;
    h->op = op_type;
    *out = h;
    return NITI_NO_ERROR;
}

int niti_execution_resize(niti_execution_t e, const niti_tensor* in, int nin, const niti_tensor* out, int nout) {
    if (!e || !in || !out) return NITI_INVALID_VALUE;
    return e->impl->onResize(in, nin, out, nout);
}

int niti_execution_execute(niti_execution_t e, const niti_tensor* in, int nin, const niti_tensor* out, int nout,
                           void* stream) {
    if (!e || !in || !out || nin < 0 || nout < 0) return NITI_INVALID_VALUE;
    const hipStream_t st = S(stream);
    bool any_host = false;
    for (int i = 0; i < nin + nout && !any_host; ++i) {
        const niti_tensor& t = i < nin ? in[i] : out[i - nin];
        any_host = t.data != nullptr && is_host_pointer(t.data);
    }
    if (!any_host) return e->impl->onExecute(in, nin, out, nout, st);
    // stage every host tensor through the handle's device buffers
    std::vector<niti_tensor> di(in, in + nin), dout(out, out + nout);
    if (e->stage.size() < (size_t)(nin + nout)) {
        e->stage.resize(nin + nout, nullptr);
        e->stage_bytes.resize(nin + nout, 0);
    }
    for (int i = 0; i < nin + nout; ++i) {
        const bool is_out = i >= nin;
        niti_tensor& t = is_out ? dout[i - nin] : di[i];
        if (t.data == nullptr || !is_host_pointer(t.data)) continue;
        const size_t bytes = tensor_bytes(e->op, is_out, is_out ? i - nin : i, t);
        if (bytes == 0) return NITI_INVALID_VALUE;
        if (e->stage_bytes[i] < bytes) {
            if (e->stage[i]) (void)hipFree(e->stage[i]);
            e->stage[i] = nullptr;
            e->stage_bytes[i] = 0;
            if (hipMalloc(&e->stage[i], bytes) != hipSuccess) return NITI_OUT_OF_MEMORY;
            e->stage_bytes[i] = bytes;
        }
        // outputs too: an Execution may leave parts of its output untouched (pad lanes, scalars)
        if (hipMemcpyAsync(e->stage[i], t.data, bytes, hipMemcpyHostToDevice, st) != hipSuccess)
            return NITI_NO_EXECUTION;
        t.data = e->stage[i];
    }
    const int rc = e->impl->onExecute(di.data(), nin, dout.data(), nout, st);
    if (rc != NITI_NO_ERROR) return rc;
    for (int k = 0; k < nout; ++k)
        if (dout[k].data != out[k].data &&
            hipMemcpyAsync(out[k].data, dout[k].data, tensor_bytes(e->op, true, k, out[k]), hipMemcpyDeviceToHost,
                           st) != hipSuccess)
            return NITI_NO_EXECUTION;
    // a synchronous call returns its ErrorCode (ErrorCode.hpp:17-30): a launch that flagged its
    // results invalid (the fused barrier's timeout) is NO_EXECUTION, not NO_ERROR
    uint32_t* flag = e->impl->errorFlag();
    if (flag != nullptr) {
        if (e->err_host == nullptr && hipHostMalloc((void**)&e->err_host, sizeof(uint32_t)) != hipSuccess) {
            e->err_host = nullptr;
            return NITI_OUT_OF_MEMORY;
        }
        if (hipMemcpyAsync(e->err_host, flag, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return NITI_NO_EXECUTION;
    }
    if (hipStreamSynchronize(st) != hipSuccess) return NITI_NO_EXECUTION;
    return take_error(e, st, flag != nullptr);
}

int niti_execution_status(niti_execution_t e, void* stream) {
    if (!e) return NITI_INVALID_VALUE;
    return take_error(e, S(stream), false);
}

void niti_destroy_execution(niti_execution_t e) { delete e; }

size_t niti_execution_workspace_bytes(niti_execution_t e) { return e ? e->impl->workspaceBytes() : 0; }

int niti_tensor_convert(const niti_tensor* src, const niti_tensor* dst, void* stream) {
    if (!src || !dst) return NITI_INVALID_VALUE;
    return niti::convert_tensor(*src, *dst, S(stream));
}

// ------------------------------------------------------------------ section 2
int niti_geom_finalize(niti_geom* g) {
    if (!g) return NITI_INVALID_VALUE;
    niti::ConvGeom r{};
    r.n = g->n;
    r.c_in = g->c_in;
    r.h = g->h;
    r.w = g->w;
    r.c_out = g->c_out;
    r.kh = g->kh;
    r.kw = g->kw;
    r.sh = g->stride_h;
    r.sw = g->stride_w;
    r.pt = g->pad_t;
    r.pl = g->pad_l;
    r.pb = g->pad_b;
    r.pr = g->pad_r;
    r.dh = g->dilate_h;
    r.dw = g->dilate_w;
    if (!r.finalize()) return NITI_COMPUTE_SIZE_ERROR;
    g->oh = r.oh;
    g->ow = r.ow;
    g->cip = r.cip;
    g->cop = r.cop;
    g->np = r.np;
    return NITI_NO_ERROR;
}

int niti_conv_workspace_bytes(const niti_geom* g, int op, size_t* bytes) {
    if (!g || !bytes) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    if (op == 0)
        *bytes = niti::conv_fwd_workspace(r);
    else if (op == 1)
        *bytes = niti::conv_dgrad_workspace(r);
    else if (op == 2)
        *bytes = niti::conv_wgrad_workspace(r);
    else
        return NITI_INVALID_VALUE;
    return NITI_NO_ERROR;
}

int niti_conv_plan_set(const niti_geom* g, int op, const int plan[4]) {
    if (!g || op < 0 || op > 2) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    const int pop = op == 0 ? niti::PLAN_FWD : op == 1 ? niti::PLAN_DGRAD : niti::PLAN_WGRAD;
    const niti::PlanKey k = niti::conv_plan_key(pop, r);
    if (plan == nullptr) {
        niti::plan_override_clear(k);
        return NITI_NO_ERROR;
    }
    auto tile_ok = [](int t) { return t == 64 || t == 128 || t == 256; };
    const bool taps = plan[0] == niti::PLAN_TAPS_TILE && plan[1] == niti::PLAN_TAPS_TILE && pop == niti::PLAN_WGRAD &&
                      niti::conv_wgrad_taps_ok(r);
    if ((!taps && (!tile_ok(plan[0]) || !tile_ok(plan[1]))) || plan[2] < 1 || plan[2] > 4096 || plan[3] < 0 ||
        plan[3] > 4 || (taps && plan[3] == 1) || (plan[3] >= 3 && (pop == niti::PLAN_WGRAD || plan[2] != 1)))
        return NITI_INVALID_VALUE;
    niti::PlanChoice c;
    c.bm = plan[0];
    c.bn = plan[1];
    c.splits = plan[2];
    c.strat = plan[3];
    niti::plan_override_set(k, c);
    return NITI_NO_ERROR;
}

int niti_conv_plan_info(const niti_geom* g, int op, size_t ws_bytes, int info[4]) {
    if (!g || !info || op < 0 || op > 2) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_INVALID_VALUE;
    const int pop = op == 0 ? niti::PLAN_FWD : op == 1 ? niti::PLAN_DGRAD : niti::PLAN_WGRAD;
    const niti::PlanChoice c = niti::conv_plan_query(pop, r, op != 2, ws_bytes);
    info[0] = c.bm;
    info[1] = c.bn;
    info[2] = c.splits;
    info[3] = c.strat;
    return NITI_NO_ERROR;
}

int niti_matmul_workspace_bytes(int m, int ldc, int k16, size_t* bytes) {
    if (!bytes || ldc % 16 || k16 % 16) return NITI_INVALID_VALUE;
    *bytes = niti::matmul_workspace(m, ldc, k16);
    return NITI_NO_ERROR;
}

int niti_conv_fwd_acc(const niti_geom* g, const int8_t* x, const int8_t* w, int32_t* acc, uint32_t* amax, void* ws,
                      size_t ws_bytes, void* stream) {
    if (!g) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    return code(niti::conv_fwd_acc(r, x, w, acc, amax, ws, ws_bytes, S(stream)));
}

int niti_conv_dgrad_acc(const niti_geom* g, const int8_t* dy, const int8_t* wt, int32_t* acc, uint32_t* amax,
                        void* ws, size_t ws_bytes, void* stream) {
    if (!g) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    return code(niti::conv_dgrad_acc(r, dy, wt, acc, amax, ws, ws_bytes, S(stream)));
}

static niti::ActOut act_out(const int8_t* exp_in, const int8_t* wscale, int8_t* exp_out, int relu,
                            const int8_t* relu_mask, int8_t* out) {
    niti::ActOut o;
    o.out = out;
    o.relu = relu;
    o.relu_mask = relu_mask;
    o.exp_in = exp_in;
    o.wscale = wscale;
    o.exp_out = exp_out;
    return o;
}

int niti_conv_rows_ok(const niti_geom* g) {
    niti::ConvGeom r;
    return g && to_geom(g, &r) && niti::rowconv_ok(r) ? 1 : 0;
}

int niti_nhwc16_to_c32(const int8_t* in, int n, int hw, int cp, int c, int8_t* out, void* stream) {
    if (!in || !out || n <= 0 || hw <= 0 || c <= 0 || cp < c || cp % 16) return NITI_INVALID_VALUE;
    return code(niti::nhwc16_to_c32(in, n, hw, cp, c, out, S(stream)));
}

int niti_weights_to_wf(const int8_t* w, int co, int ci, int cip, int transpose, int8_t* out, void* stream) {
    if (!w || !out || co <= 0 || ci <= 0 || cip < ci || cip % 16) return NITI_INVALID_VALUE;
    return code(niti::weights_to_wf(w, co, ci, cip, transpose != 0, out, S(stream)));
}

int niti_conv_rows_nhwc_ok(const niti_geom* g, int dgrad) {
    if (!g) return 0;
    niti::ConvGeom r, d;
    if (!to_geom(g, &r)) return 0;
    const bool pd = dgrad & 2;  // bit 1: whether the model prefers it (not just whether it can)
    if (!(dgrad & 1)) return (pd ? niti::rowconv_nhwc_pref(r) : niti::rowconv_nhwc_ok(r)) ? 1 : 0;
    if (!niti::rowconv_dgrad_geom(r, &d)) return 0;
    return (pd ? niti::rowconv_nhwc_pref(d) : niti::rowconv_nhwc_ok(d)) ? 1 : 0;
}

int niti_conv_fwd_rows(const niti_geom* g, const int8_t* x_c32, const int8_t* wf, const int8_t* exp_in,
                       const int8_t* wscale, int8_t* exp_out, int relu, int8_t* out, int8_t* pool_out,
                       int8_t* next_c32, int mode, uint32_t* amax, uint32_t* state, uint32_t epoch, uint32_t* err,
                       void* stream) {
    const int x_nhwc = (mode & NITI_ROWS_X_NHWC16) ? 1 : 0;
    mode &= ~NITI_ROWS_X_NHWC16;
    if (!g || !x_c32 || !wf || !amax || mode < 0 || mode > 4) return NITI_INVALID_VALUE;
    if (mode >= 3 && state == nullptr) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    if (!niti::rowconv_ok(r)) return NITI_NOT_SUPPORT;
    if (x_nhwc && !niti::rowconv_nhwc_ok(r)) return NITI_NOT_SUPPORT;
    if (mode == 0 && !niti::rowconv_fused_ok(r)) return NITI_NOT_SUPPORT;
    niti::RowConvOut o;
    o.x_nhwc = x_nhwc;
    o.out = out;
    o.pool_out = pool_out;
    o.next = next_c32;
    o.exp_in = exp_in;
    o.wscale = wscale;
    o.exp_out = exp_out;
    o.relu = relu;
    return code(niti::rowconv_fwd(r, x_c32, wf, o, mode, amax, state, epoch, err, S(stream)));
}

int niti_conv_dgrad_rows(const niti_geom* g, const int8_t* dy_c32, const int8_t* wft, const int8_t* relu_mask,
                         const int8_t* pool_x, const int8_t* pool_y, int pool_relu, int8_t* dx, int8_t* dx_c32,
                         int8_t* dx_p16, const int8_t* exp_in, const int8_t* wscale, int8_t* exp_out, int mode,
                         uint32_t* amax, uint32_t* state, uint32_t epoch, uint32_t* err, void* stream) {
    const int x_nhwc = (mode & NITI_ROWS_X_NHWC16) ? 1 : 0;
    mode &= ~NITI_ROWS_X_NHWC16;
    if (!g || !dy_c32 || !wft || !amax || mode < 0 || mode > 4) return NITI_INVALID_VALUE;
    if (mode >= 3 && state == nullptr) return NITI_INVALID_VALUE;
    if ((pool_x == nullptr) != (pool_y == nullptr) || (pool_x && relu_mask)) return NITI_INVALID_VALUE;
    if (mode != 1 && dx == nullptr) return NITI_INVALID_VALUE;
    niti::ConvGeom r, d;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    if (!niti::rowconv_dgrad_geom(r, &d)) return NITI_NOT_SUPPORT;
    if (mode == 0 && !niti::rowconv_fused_ok(d, true)) return NITI_NOT_SUPPORT;
    if (dx_p16 != nullptr && !niti::rowconv_p16_ok(d, pool_x != nullptr)) return NITI_NOT_SUPPORT;
    if (x_nhwc && !niti::rowconv_nhwc_ok(d)) return NITI_NOT_SUPPORT;
    niti::RowConvOut o;
    o.x_nhwc = x_nhwc;
    o.p16 = dx_p16;
    o.exp_in = exp_in;
    o.wscale = wscale;
    o.exp_out = exp_out;
    o.dgrad_slot = 1;
    if (pool_x != nullptr) {
        o.pool_x = pool_x;
        o.pool_y = pool_y;
        o.pool_dx = dx;
        o.pool_dx_next = dx_c32;
        o.pool_relu = pool_relu;
    } else {
        o.out = dx;
        o.next = dx_c32;
        o.relu_mask = relu_mask;
    }
    return code(niti::rowconv_fwd(d, dy_c32, wft, o, mode, amax, state, epoch, err, S(stream)));
}

int niti_im2col(const niti_geom* g, const int8_t* x, int kp, int8_t* xcol, void* stream) {
    if (!g || !x || !xcol) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    if (r.cip > 16 || r.c_in > 4 || kp % 16 != 0 || kp > 4096 || kp < r.kh * r.kw * r.c_in) return NITI_NOT_SUPPORT;
    return code(niti::im2col_small(r, x, kp, xcol, S(stream)));
}
int niti_im2col_nchw(const niti_geom* g, const int8_t* x_nchw, int kp, int8_t* xcol, void* stream) {
    if (!g || !x_nchw || !xcol) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    if (r.c_in > 4 || kp % 16 != 0 || kp > 4096 || kp < r.kh * r.kw * r.c_in) return NITI_NOT_SUPPORT;
    return code(niti::im2col_small(r, x_nchw, kp, xcol, S(stream), true));
}

int niti_conv_fwd_phase1(const niti_geom* g, const int8_t* x, const int8_t* w, int32_t* acc, uint32_t* amax,
                         void* ws, size_t ws_bytes, void* stream) {
    if (!g || !x || !w || !acc || !amax) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    return code(niti::conv_fwd_phase1(r, x, w, acc, amax, ws, ws ? ws_bytes : 0, S(stream)));
}

int niti_conv_fwd_phase2(const niti_geom* g, const int8_t* x, const int8_t* w, const int32_t* acc,
                         const uint32_t* amax, const int8_t* exp_in, const int8_t* wscale, int8_t* exp_out, int relu,
                         const int8_t* relu_mask, int8_t* out, size_t ws_bytes, void* stream) {
    if (!g || !x || !w || !acc || !amax || !out) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    return code(niti::conv_fwd_phase2(r, x, w, acc, amax, act_out(exp_in, wscale, exp_out, relu, relu_mask, out),
                                      ws_bytes, S(stream)));
}

int niti_conv_dgrad_phase1(const niti_geom* g, const int8_t* dy, const int8_t* wt, int32_t* acc, uint32_t* amax,
                           void* ws, size_t ws_bytes, void* stream) {
    if (!g || !dy || !wt || !acc || !amax) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    return code(niti::conv_dgrad_phase1(r, dy, wt, acc, amax, ws, ws ? ws_bytes : 0, S(stream)));
}

int niti_conv_dgrad_phase2(const niti_geom* g, const int8_t* dy, const int8_t* wt, const int32_t* acc,
                           const uint32_t* amax, const int8_t* exp_in, const int8_t* wscale, int8_t* exp_out, int relu,
                           const int8_t* relu_mask, int8_t* out, size_t ws_bytes, void* stream) {
    if (!g || !dy || !wt || !acc || !amax || !out) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    return code(niti::conv_dgrad_phase2(r, dy, wt, acc, amax, act_out(exp_in, wscale, exp_out, relu, relu_mask, out),
                                        ws_bytes, S(stream)));
}

int niti_conv_wgrad_acc(const niti_geom* g, const int8_t* x, const int8_t* dy, int32_t* acc, uint32_t* amax,
                        void* ws, size_t ws_bytes, void* stream) {
    if (!g) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    return code(niti::conv_wgrad_acc(r, x, dy, acc, amax, ws, ws_bytes, S(stream)));
}

int niti_nhwc16_to_p16(const int8_t* in, int64_t pixels, int cp, int8_t* out, void* stream) {
    if (!in || !out || pixels <= 0 || pixels % 16 || cp <= 0 || cp % 16) return NITI_INVALID_VALUE;
    return code(niti::nhwc16_to_p16(in, pixels, cp, out, S(stream)));
}

void niti_diag_wgrad_stamps(void* buf) { niti::wgrad_stamps_arm((unsigned long long*)buf); }
void niti_diag_rowconv_stamps(void* buf) { niti::rowconv_stamps_arm((unsigned long long*)buf); }
uint32_t* niti_rows_spec_slot(uint32_t* state, int dgrad) {
    return state ? niti::rowconv_spec_slot(state, dgrad != 0) : nullptr;
}

void niti_diag_rowconv_barrier(uint32_t spin_limit, uint32_t expect_extra) {
    niti::rowconv_barrier_diag(spin_limit, expect_extra);
}
void niti_diag_rowconv_speculate(int mode) { niti::rowconv_speculate(mode); }
void niti_diag_gemm_speculate(int bias) { niti::gemm_speculate_bias(bias); }
unsigned long long niti_diag_gemm_fused_launches(void) { return niti::gemm_fused_launches(); }
unsigned long long niti_diag_head_chain_launches(void) { return niti::head_chain_launches(); }
void niti_diag_head_chain(int on) { niti::head_chain_enable(on); }
void niti_diag_p16_jobs_cap(int cap) { niti::model_p16_jobs_cap(cap); }

int niti_conv_wgrad_p16_workspace(const niti_geom* g, int splits, size_t* bytes) {
    if (!g || !bytes) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    if (!niti::conv_wgrad_p16_ok(r)) return NITI_NOT_SUPPORT;
    *bytes = niti::conv_wgrad_p16_workspace(r, splits);
    return NITI_NO_ERROR;
}

int niti_conv_wgrad_p16_acc(const niti_geom* g, const int8_t* x, const int8_t* dy, int32_t* acc, uint32_t* amax,
                            void* ws, size_t ws_bytes, int splits, void* stream) {
    if (!g || !x || !dy || !acc) return NITI_INVALID_VALUE;
    niti::ConvGeom r;
    if (!to_geom(g, &r)) return NITI_COMPUTE_SIZE_ERROR;
    if (!niti::conv_wgrad_p16_ok(r)) return NITI_NOT_SUPPORT;
    if (splits <= 0) splits = niti::conv_wgrad_p16_splits(r);
    if (ws_bytes < niti::conv_wgrad_p16_workspace(r, splits) || (ws_bytes > 0 && !ws)) return NITI_INVALID_VALUE;
    return code(niti::conv_wgrad_p16(r, x, dy, acc, amax, ws, ws_bytes, splits, S(stream)));
}

int niti_matmul_acc(int m, int o, int k16, const int8_t* B, int64_t ldb, const int8_t* A, int64_t lda, int32_t* acc,
                    int64_t ldc, uint32_t* amax, void* ws, size_t ws_bytes, void* stream) {
    if (k16 % 16 || ldb % 16 || lda % 16 || ldc % 16 || ldc < o) return NITI_INVALID_VALUE;
    return code(niti::matmul_acc(m, o, k16, B, ldb, A, lda, acc, ldc, amax, ws, ws_bytes, S(stream)));
}

int niti_absmax_i32(const int32_t* acc, int64_t n, uint32_t* amax, void* stream) {
    return code(niti::absmax_i32(acc, n, amax, S(stream)));
}

int niti_requant_act(const int32_t* acc, int64_t rows, int ldc, const uint32_t* amax, const int8_t* exp_in,
                     const int8_t* wscale, int8_t* exp_out, int relu, const int8_t* relu_mask, int8_t* out,
                     void* stream) {
    niti::ActRequant r;
    r.acc = acc;
    r.rows = rows;
    r.ldc = ldc;
    r.amax = amax;
    r.exp_in = exp_in;
    r.wscale = wscale;
    r.exp_out = exp_out;
    r.relu = relu;
    r.relu_mask = relu_mask;
    r.out_nhwc16 = out;
    return code(niti::requant_act(r, S(stream)));
}

int niti_requant_grad(const int32_t* acc, int64_t n, const uint32_t* amax, int rule, int8_t* g_out, int8_t* w,
                      void* stream) {
    if (rule != 2 && rule != 3) return NITI_INVALID_VALUE;
    return code(niti::requant_grad(acc, n, amax, rule, g_out, w, S(stream)));
}

int niti_sgd_update(const int32_t* acc, const uint32_t* amax, int rule, int co, int ci, int kk, int cip, int cop,
                    int8_t* w, int8_t* wt, int8_t* g_out, void* stream) {
    if (rule != 2 && rule != 3) return NITI_INVALID_VALUE;
    return code(niti::sgd_update(acc, amax, rule, co, ci, kk, cip, cop, w, wt, g_out, S(stream)));
}
int niti_sgd_update_wf(const int32_t* acc, const uint32_t* amax, int rule, int co, int ci, int kk, int cip, int cop,
                       int8_t* w, int8_t* wt, int8_t* g_out, int8_t* wf, int8_t* wft, void* stream) {
    if (rule != 2 && rule != 3) return NITI_INVALID_VALUE;
    if ((wf || wft) && (kk != 9 || ci % 32 != 0 || co % 32 != 0)) return NITI_NOT_SUPPORT;
    niti::SgdJob j{acc, amax, rule, co, ci, kk, cip, cop, w, wt, g_out};
    j.wf = wf;
    j.wft = wft;
    return code(niti::sgd_update_many(&j, 1, S(stream)));
}

int niti_nhwc16_to_chwn16(const int8_t* in, int n, int hw, int cp, int np, int8_t* out, void* stream) {
    return code(niti::nhwc16_to_chwn16(in, n, hw, cp, np, out, S(stream)));
}
int niti_ohwi16_to_ihwo16(const int8_t* w, int co, int ci, int kk, int cip, int cop, int8_t* wt, void* stream) {
    return code(niti::ohwi16_to_ihwo16(w, co, ci, kk, cip, cop, wt, S(stream)));
}
int niti_nchw_to_nhwc16(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, void* stream) {
    return code(niti::nchw_to_nhwc16(x, n, c, hw, cp, out, S(stream)));
}
int niti_nchw_to_chwn16(const int8_t* x, int n, int c, int hw, int cp, int np, int8_t* out, void* stream) {
    return code(niti::nchw_to_chwn16(x, n, c, hw, cp, np, out, S(stream)));
}
int niti_nhwc16_to_nchw(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, void* stream) {
    return code(niti::nhwc16_to_nchw(x, n, c, hw, cp, out, S(stream)));
}
int niti_oihw_to_ohwi16(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, void* stream) {
    return code(niti::oihw_to_ohwi16(w, co, ci, kk, cip, out, S(stream)));
}
int niti_ohwi16_to_oihw(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, void* stream) {
    return code(niti::ohwi16_to_oihw(w, co, ci, kk, cip, out, S(stream)));
}
int niti_residual_add(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n, int32_t* z,
                      int8_t* ez, uint32_t* amax, void* stream) {
    return code(niti::residual_add(a, ea, b, eb, n, z, ez, amax, S(stream)));
}
int niti_residual_requant(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                          const uint32_t* amax, int8_t* ez, int8_t* exp_out, int relu, int8_t* out, void* stream) {
    return code(niti::residual_requant(a, ea, b, eb, n, amax, ez, exp_out, relu, out, S(stream)));
}
int niti_residual_requant_relu_grad(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                                    const uint32_t* amax, int8_t* ez, int8_t* exp_out, const int8_t* relu_mask,
                                    int8_t* out, void* stream) {
    if (!relu_mask) return NITI_INVALID_VALUE;
    return code(niti::residual_requant(a, ea, b, eb, n, amax, ez, exp_out, 0, out, S(stream), relu_mask));
}
int niti_sum_pool(const int8_t* x, int n, int hw, int cp, int32_t* acc, uint32_t* amax, void* stream) {
    return code(niti::sum_pool(x, n, hw, cp, acc, amax, S(stream)));
}
int niti_sum_pool_grad(const int8_t* dy, int n, int hw, int cp, int8_t* dx, void* stream) {
    return code(niti::sum_pool_grad(dy, n, hw, cp, dx, S(stream)));
}
int niti_maxpool(const int8_t* x, int n, int h, int w, int cp, int k, int s, int p, int8_t* y, int oh, int ow,
                 void* stream) {
    return code(niti::maxpool_nhwc16(x, n, h, w, cp, k, s, p, y, oh, ow, S(stream)));
}
int niti_maxpool_grad(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h, int w, int cp, int k, int s,
                      int p, int oh, int ow, int relu, int8_t* dx, void* stream) {
    return code(niti::maxpool_relu_grad_nhwc16(x, y, dy, n, h, w, cp, k, s, p, oh, ow, relu, dx, S(stream)));
}
int niti_maxpool_grad_ws(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h, int w, int cp, int k,
                         int s, int p, int oh, int ow, int relu, int8_t* ws, int8_t* dx, void* stream) {
    if (!x || !y || !dy || !ws || !dx || n <= 0 || h <= 0 || w <= 0 || oh <= 0 || ow <= 0) return NITI_INVALID_VALUE;
    return code(niti::maxpool_relu_grad_ws(x, y, dy, n, h, w, cp, k, s, p, oh, ow, relu, ws, dx, S(stream)));
}
int niti_relu_grad(const int8_t* x, const int8_t* dy, int64_t n, int8_t* out, void* stream) {
    if (n % 16) return NITI_INVALID_VALUE;
    return code(niti::relu_grad_nhwc16(x, dy, n, out, S(stream)));
}
int niti_image_stats(const uint8_t* images, int64_t n, uint64_t* stats, void* stream) {
    if (!images || !stats || n <= 0) return NITI_INVALID_VALUE;
    return code(niti::image_stats(images, n, reinterpret_cast<unsigned long long*>(stats), S(stream)));
}
int niti_image_quantize(const uint8_t* images, int n, int c, int hw, const uint64_t* stats, int64_t count,
                        int8_t* out_nchw, int8_t* ascale, void* stream) {
    if (!images || !stats || !out_nchw || n <= 0 || c <= 0 || hw <= 0 || count < (int64_t)n * c * hw)
        return NITI_INVALID_VALUE;
    return code(niti::image_quantize(images, n, c, hw, c, reinterpret_cast<const unsigned long long*>(stats), count,
                                     out_nchw, ascale, false, S(stream)));
}
int niti_image_quantize_nhwc16(const uint8_t* images, int n, int c, int hw, int cp, const uint64_t* stats,
                               int64_t count, int8_t* out_nhwc16, int8_t* ascale, void* stream) {
    if (!images || !stats || !out_nhwc16 || n <= 0 || c <= 0 || hw <= 0 || cp < c || cp % 16 ||
        count < (int64_t)n * c * hw)
        return NITI_INVALID_VALUE;
    return code(niti::image_quantize(images, n, c, hw, cp, reinterpret_cast<const unsigned long long*>(stats), count,
                                     out_nhwc16, ascale, true, S(stream)));
}
int niti_loss_grad(const int8_t* logits, int batch, int classes, int ld, const int8_t* ascale, const int32_t* labels,
                   int8_t* out, void* stream) {
    return code(niti::loss_grad(logits, batch, classes, ld, ascale, labels, out, S(stream)));
}

}  // extern "C"
