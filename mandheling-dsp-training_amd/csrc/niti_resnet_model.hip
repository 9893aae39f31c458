// niti_resnet_model.hip -- ResNet-18 NITI int8 training step on the device, driven from C++
// (BASELINE config 5; declarations and the rules' provenance in niti_resnet_model.hpp).
//
// One step (uint8 images or int8 x in, NITI_SGD out), every op on the step stream:
//   input      image statistics -> [SUM / MAX over ranks] -> quantise (NCHW) -> the stem's im2col
//   stem       conv1 7x7 / 2 as a 1x1 conv over its im2col (+relu), 3x3 / 2 max pool
//   blocks     conv a (+relu), conv b, [1x1 / 2 projection], the residual sum: range pass ->
//              [MAX] -> requantise + relu with the sum recomputed from the int8 operands
//   head       global sum pool -> requantise -> fc (1x1 conv) -> NITI_LOSS_Grad
//   backward   per conv the weight gradient (descending layer order, so gradient buckets close in
//              memory order) and the input gradient with the previous relu gradient fused; the
//              residual gradient sums with the next block-output relu gradient fused; the stem's
//              overlapping max-pool gradient (first max wins) with its relu gradient
//   update     one NITI_SGD launch over all 21 layers (+ the row kernels' weight copies)
// Every forward / input-gradient conv is one of the two forms the VGG driver uses: the register-fed
// row kernels with the rescale fused (stride-1 3x3 layers, niti_rowconv.hip) or the implicit-GEMM
// range + requantise phases (strided / 1x1 / deep layers, niti_kernels.hip).  Data parallel: the
// exact protocol of niti_model.hip (ranges MAX-reduced on the step stream between the two launches
// of each requantisation, int32 weight-gradient buckets SUM-reduced on the comm stream while the
// backward pass goes on), so N ranks equal one device running the global batch bit for bit.
#include <string.h>

#include <algorithm>
#include <set>

#include "../../include/niti_hip.h"
#include "niti_resnet_model.hpp"

namespace niti {

#define RTRY(expr)                                          \
    do {                                                    \
        if ((expr) != hipSuccess) return NITI_NO_EXECUTION; \
    } while (0)

static ConvGeom make_geom(int n, int ci, int h, int co, int k, int s, int p) {
    ConvGeom g{};
    g.n = n;
    g.c_in = ci;
    g.h = g.w = h;
    g.c_out = co;
    g.kh = g.kw = k;
    g.sh = g.sw = s;
    g.pt = g.pl = g.pb = g.pr = p;
    g.dh = g.dw = 1;
    g.finalize();
    return g;
}

int ResNetModel::build(int batch_, int in_hw_, int classes_) {
    batch = batch_;
    in_hw = in_hw_ > 0 ? in_hw_ : 224;
    classes = classes_ > 0 ? classes_ : 1000;
    // every stage halves the map (stride-2 convs and the 1x1 projections agree on odd sizes too)
    if (in_hw % 16 != 0 || classes > 2048) return NITI_INVALID_VALUE;
    const int n = batch;
    // the 21 parameter layers in parameter order (oracle/niti_resnet_ref.py resnet18_convs)
    auto add = [&](int ci, int co, int k, int s, int p, int h, int relu) {
        RConv c;
        c.og = c.g = make_geom(n, ci, h, co, k, s, p);
        c.relu = relu;
        C.push_back(c);
        return (int)C.size() - 1;
    };
    stem = make_geom(n, 3, in_hw, 64, 7, 2, 3);
    add(3, 64, 7, 2, 3, in_hw, 1);
    C[0].g = make_geom(n, STEM_KP, stem.oh, 64, 1, 1, 0);
    const int ph = (stem.oh + 2 - 3) / 2 + 1;
    int h = ph, ci = 64;
    for (int stage = 0; stage < 4; ++stage) {
        const int co = 64 << stage;
        for (int blk = 0; blk < 2; ++blk) {
            const int s = stage > 0 && blk == 0 ? 2 : 1;
            RBlock b;
            b.a = add(ci, co, 3, s, 1, h, 1);
            const int ho = (h + 2 - 3) / s + 1;
            b.b = add(co, co, 3, 1, 1, ho, 0);
            if (s != 1 || ci != co) b.p = add(ci, co, 1, s, 0, h, 0);
            B.push_back(b);
            ci = co;
            h = ho;
        }
    }
    const int fc = add(512, classes, 1, 1, 0, 1, 0);
    const int nl = (int)C.size();
    // device exponents: 2 per conv, 4 per block, pool, loss gradient, input
    n_exps = 2 * nl + 4 * (int)B.size() + 3;
    exps = (int8_t*)ws.alloc(n_exps);
    if (!exps || hipMemset(exps, 0, n_exps) != hipSuccess) return NITI_OUT_OF_MEMORY;
    int ei = 0;
    auto exp_slot = [&]() { return exps + ei++; };
    exp0 = exp_slot();
    eg = exp_slot();
    ed = exp_slot();  // the loss gradient's exponent: 0, never written
    auto A8 = [&](size_t bytes) { return (int8_t*)ws.alloc(bytes); };
    // the input and the stem
    x0n = A8((size_t)n * 3 * in_hw * in_hw);
    xcol = A8((size_t)n * stem.oh * stem.ow * STEM_KP);
    p0 = A8((size_t)n * ph * ph * 64);
    pool_ws = A8((size_t)n * ph * ph * 64);
    d0 = A8((size_t)n * stem.oh * stem.ow * 64);
    if (!x0n || !xcol || !p0 || !pool_ws || !d0) return NITI_OUT_OF_MEMORY;
    size_t acc_elems = 0, grad_elems = 0;
    rc_err = (uint32_t*)ws.alloc(64);
    if (!rc_err || hipMemset(rc_err, 0, 64) != hipSuccess) return NITI_OUT_OF_MEMORY;
    res_bar = (uint32_t*)ws.alloc(ROWCONV_BAR_WORDS * 4);
    if (!res_bar || hipMemset(res_bar, 0, ROWCONV_BAR_WORDS * 4) != hipSuccess) return NITI_OUT_OF_MEMORY;
    res_slot = (uint32_t*)ws.alloc(2 * B.size() * RES_SPEC_SLOT_WORDS * 4);
    if (!res_slot || hipMemset(res_slot, 0, 2 * B.size() * RES_SPEC_SLOT_WORDS * 4) != hipSuccess)
        return NITI_OUT_OF_MEMORY;
    for (int i = 0; i < nl; ++i) {
        RConv& c = C[i];
        const ConvGeom& g = c.g;
        c.w = A8(c.w_elems());
        c.ws_dev = A8(16);
        c.g8 = A8(c.w_elems());
        c.y = A8((size_t)n * g.oh * g.ow * g.cop);
        c.y_exp = exp_slot();
        c.dx_exp = exp_slot();
        c.gspec = (uint32_t*)ws.alloc(2 * GEMM_SPEC_SLOT_WORDS * 4);
        if (!c.w || !c.ws_dev || !c.g8 || !c.y || !c.gspec) return NITI_OUT_OF_MEMORY;
        if (hipMemset(c.gspec, 0, 2 * GEMM_SPEC_SLOT_WORDS * 4) != hipSuccess) return NITI_NO_EXECUTION;
        if (hipMemset(c.w, 0, c.w_elems()) != hipSuccess || hipMemset(c.ws_dev, 0, 16) != hipSuccess)
            return NITI_NO_EXECUTION;
        if (i > 0) {
            c.wT = A8((size_t)g.c_in * g.kh * g.kw * g.cop);
            if (!c.wT) return NITI_OUT_OF_MEMORY;
            if (conv_dgrad_subpix_ok(g)) {  // the stride-2 input gradient's class weights
                c.subw = A8(conv_dgrad_subpix_bytes(g));
                if (!c.subw) return NITI_OUT_OF_MEMORY;
            }
        }
        grad_elems += (size_t)c.w_elems();
        acc_elems = std::max(acc_elems, (size_t)n * g.oh * g.ow * g.cop);
        acc_elems = std::max(acc_elems, (size_t)n * g.h * g.w * g.cip);
        slab_bytes = std::max(slab_bytes, conv_fwd_workspace(g));
        slab_bytes = std::max(slab_bytes, conv_dgrad_workspace(g));
        slab_w_bytes = std::max(slab_w_bytes, conv_wgrad_workspace(g));
        // grid-barrier state: the row kernels' fused launches and speculation slots, or the GEMM
        // path's fused-rescale launches (STRAT_FUSED)
        c.bar = (uint32_t*)ws.alloc(ROWCONV_BAR_WORDS * 4);
        if (!c.bar || hipMemset(c.bar, 0, ROWCONV_BAR_WORDS * 4) != hipSuccess) return NITI_OUT_OF_MEMORY;
        if (i > 0 && rowconv_ok(g)) {
            c.rows = 1;
            c.wf = A8(rowconv_wf_bytes(g.c_out, g.c_in));
            if (!c.wf) return NITI_OUT_OF_MEMORY;
            if (!rowconv_nhwc_pref(g) && !(c.xc32 = A8((size_t)n * round_up(g.c_in, 32) * g.h * g.w)))
                return NITI_OUT_OF_MEMORY;
            rc_acc_size = std::max(rc_acc_size, rowconv_acc_bytes(g, false));
            if (rowconv_dgrad_geom(g, &c.dg)) {
                c.rows_dg = 1;
                c.wft = A8(rowconv_wf_bytes(g.c_in, g.c_out));
                if (!c.wft) return NITI_OUT_OF_MEMORY;
                if (!rowconv_nhwc_pref(c.dg) && !(c.dyc32 = A8((size_t)n * g.oh * g.ow * round_up(g.c_out, 32))))
                    return NITI_OUT_OF_MEMORY;
                rc_acc_size = std::max(rc_acc_size, rowconv_acc_bytes(c.dg, true));
            }
        }
    }
    grad_bucket = (int32_t*)ws.alloc(grad_elems * 4);
    if (!grad_bucket) return NITI_OUT_OF_MEMORY;
    size_t off = 0;
    for (RConv& c : C) {
        c.dwacc = grad_bucket + off;
        off += (size_t)c.w_elems();
    }
    // wiring: inputs, outputs, gradients and their exponents
    C[0].in = xcol;
    C[0].in_exp = exp0;
    C[0].dy = d0;
    C[0].dy_exp = ed;  // (the stem's weight gradient reads no exponent)
    const int8_t* u = p0;
    const int8_t* u_exp = C[0].y_exp;  // max pooling keeps the exponent
    for (size_t k = 0; k < B.size(); ++k) {
        RBlock& b = B[k];
        RConv& ca = C[b.a];
        RConv& cb = C[b.b];
        b.u = u;
        b.u_exp = u_exp;
        b.out_elems = (int64_t)n * cb.g.oh * cb.g.ow * cb.g.cop;
        b.in_elems = (int64_t)n * ca.g.h * ca.g.w * ca.g.cip;
        b.out = A8(b.out_elems);
        b.dh = A8((size_t)n * ca.g.oh * ca.g.ow * ca.g.cop);
        b.dua = A8(b.in_elems);
        b.du = A8(b.in_elems);
        if (!b.out || !b.dh || !b.dua || !b.du) return NITI_OUT_OF_MEMORY;
        if (b.p >= 0 && !(b.dus = A8(b.in_elems))) return NITI_OUT_OF_MEMORY;
        b.out_exp = exp_slot();
        b.ez = exp_slot();
        b.ezb = exp_slot();
        b.du_exp = exp_slot();
        ca.in = u;
        ca.in_exp = u_exp;
        ca.dy = b.dh;
        ca.dy_exp = cb.dx_exp;
        ca.dx = b.dua;
        cb.in = ca.y;
        cb.in_exp = ca.y_exp;
        cb.dx = b.dh;
        cb.dx_mask = ca.y;  // conv a's relu gradient rides along conv b's input gradient
        if (b.p >= 0) {
            C[b.p].in = u;
            C[b.p].in_exp = u_exp;
            C[b.p].dx = b.dus;
        }
        u = b.out;
        u_exp = b.out_exp;
    }
    // dz of block k is block k + 1's residual gradient (the block-output relu gradient fused in);
    // the last block's comes from the sum pool's gradient
    const int last = (int)B.size() - 1;
    B[last].dz = A8(B[last].out_elems);
    if (!B[last].dz) return NITI_OUT_OF_MEMORY;
    B[last].dz_exp = C[fc].dx_exp;
    for (int k = last - 1; k >= 0; --k) {
        B[k].dz = B[k + 1].du;
        B[k].dz_exp = B[k + 1].du_exp;
    }
    for (RBlock& b : B) {
        C[b.b].dy = b.dz;
        C[b.b].dy_exp = b.dz_exp;
        if (b.p >= 0) {
            C[b.p].dy = b.dz;
            C[b.p].dy_exp = b.dz_exp;
        }
    }
    gsum = (int32_t*)ws.alloc((size_t)n * 512 * 4);
    g8pool = A8((size_t)n * 512);
    dg = A8((size_t)n * 512);
    RConv& f = C[fc];
    f.in = g8pool;
    f.in_exp = eg;
    f.dy = A8((size_t)n * f.g.cop);
    f.dy_exp = ed;
    f.dx = dg;
    if (!gsum || !g8pool || !dg || !f.dy) return NITI_OUT_OF_MEMORY;
    if (ei > n_exps) return NITI_NO_EXECUTION;
    acc_bytes = acc_elems * 4;
    acc = (int32_t*)ws.alloc(acc_bytes);
    qstats = (unsigned long long*)ws.alloc(64);
    qslots = (unsigned long long*)ws.alloc((size_t)IMAGE_STATS_SLOTS * 4 * sizeof(unsigned long long));
    if (!acc || !qstats || !qslots) return NITI_OUT_OF_MEMORY;
    if (slab_bytes && !(slab = ws.alloc(slab_bytes))) return NITI_OUT_OF_MEMORY;
    if (slab_w_bytes && !(slab_w = ws.alloc(slab_w_bytes))) return NITI_OUT_OF_MEMORY;
    if (rc_acc_size && !(rc_acc = (int32_t*)ws.alloc(rc_acc_size))) return NITI_OUT_OF_MEMORY;
    for (int i = 0; i < nl; ++i) {  // the GEMM-path phases that may run the speculative pair
        if (!C[i].rows) gspec_alt_bytes = std::max(gspec_alt_bytes, conv_fwd_spec_alt_bytes(C[i].g));
        if (C[i].dx != nullptr && !C[i].rows_dg) gspec_alt_bytes = std::max(gspec_alt_bytes, conv_dgrad_spec_alt_bytes(C[i].g));
    }
    if (gspec_alt_bytes && !(gspec_alt = (int8_t*)ws.alloc(gspec_alt_bytes))) return NITI_OUT_OF_MEMORY;
    amax_bytes = (3 * C.size() + 2 * B.size() + 1) * MAX_BYTES;
    amax = (uint32_t*)ws.alloc(amax_bytes);
    if (!amax) return NITI_OUT_OF_MEMORY;
    return hipDeviceSynchronize() == hipSuccess ? NITI_NO_ERROR : NITI_NO_EXECUTION;
}

ResNetModel::~ResNetModel() {
    clear_probe();
    drop_graph();
    if (cst) (void)hipStreamSynchronize(cst);
    for (auto e : ev_bucket) (void)hipEventDestroy(e);
    if (ev_grads) (void)hipEventDestroy(ev_grads);
    if (gin) (void)hipEventDestroy(gin);
    if (gout) (void)hipEventDestroy(gout);
    if (gstream) (void)hipStreamDestroy(gstream);
    coll_grad.reset();
    coll.reset();
    if (cst) (void)hipStreamDestroy(cst);
}

bool ResNetModel::ensure_slab(size_t bytes, bool wgrad) {
    void*& p = wgrad ? slab_w : slab;
    size_t& have = wgrad ? slab_w_bytes : slab_bytes;
    if (have >= bytes) return true;
    if (hipDeviceSynchronize() != hipSuccess) return false;
    void* s2 = ws.alloc(bytes);
    if (!s2) return false;
    p = s2;
    have = bytes;
    return true;
}

void ResNetModel::clear_probe() {
    for (auto e : ev0) (void)hipEventDestroy(e);
    for (auto e : ev1) (void)hipEventDestroy(e);
    ev0.clear();
    ev1.clear();
    probe_count = 0;
    probe_layer = probe_phase = -1;
}

void ResNetModel::probe(int layer, int phase, bool begin, hipStream_t st) {
    if (layer != probe_layer || phase != probe_phase || probe_paused || tuning || capturing || probe_count >= (int)ev0.size()) return;
    if (begin) {
        (void)hipEventRecord(ev0[probe_count], st);
    } else {
        (void)hipEventRecord(ev1[probe_count], st);
        ++probe_count;
    }
}

void ResNetModel::drop_graph() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    gexec = nullptr;
}

// ------------------------------------------------------------------------------ one conv phase
// Forward of conv i: the row kernel (fused single launch where the grid is resident and nothing
// sits between range and requantisation; else the speculative pair with the MAX between its
// launches), or the GEMM's range phase, [MAX], requantise phase.
int ResNetModel::fwd_conv(int i, hipStream_t st) {
    RConv& c = C[i];
    const ConvGeom& g = c.g;
    const bool dp = this->dp();
    probe(i, 0, true, st);
    if (rows_on(i)) {
        const bool xn = rowconv_nhwc_pref(g);
        if (!xn) RTRY(nhwc16_to_c32(c.in, g.n, g.h * g.w, g.cip, g.c_in, c.xc32, st));
        const int8_t* xin = xn ? c.in : c.xc32;
        RowConvOut o;
        o.x_nhwc = xn ? 1 : 0;
        o.out = c.y;
        o.exp_in = c.in_exp;
        o.wscale = c.ws_dev;
        o.exp_out = c.y_exp;
        o.relu = c.relu;
        if (!dp && !capturing && rowconv_fused_ok(g)) {
            RTRY(rowconv_fwd(g, xin, c.wf, o, 0, rng(i, 0), c.bar, ++c.epoch, rc_err, st));
        } else if (rowconv_spec2_on()) {
            o.acc_store = rowconv_acc_bytes(g, false) ? rc_acc : nullptr;
            RTRY(rowconv_fwd(g, xin, c.wf, o, RC_SPEC_A, rng(i, 0), c.bar, 0, nullptr, st));
            if (dp && exact) RTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
            RTRY(rowconv_fwd(g, xin, c.wf, o, RC_SPEC_B, rng(i, 0), c.bar, 0, nullptr, st));
        } else {
            o.acc_store = rowconv_acc_bytes(g, false) ? rc_acc : nullptr;
            RTRY(rowconv_fwd(g, xin, c.wf, o, 1, rng(i, 0), nullptr, 0, nullptr, st));
            if (dp && exact) RTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
            RTRY(rowconv_fwd(g, xin, c.wf, o, 2, rng(i, 0), nullptr, 0, nullptr, st));
        }
        probe(i, 0, false, st);
        return NITI_NO_ERROR;
    }
    ActOut o;
    o.out = c.y;
    o.relu = c.relu;
    o.exp_in = c.in_exp;
    o.wscale = c.ws_dev;
    o.exp_out = c.y_exp;
    if (i == 0) {  // the stem: its 3x3 / 2 max pool in the requantise pass when there is one
        stem_pooled = !conv_fwd_spec_ok(g) && conv_fwd_phase2_separate(g, slab_bytes);
        if (stem_pooled) {
            const int ph = C[B[0].a].g.h;
            o.pool3.out = p0;
            o.pool3.arg = pool_ws;
            o.pool3.H = g.oh;
            o.pool3.W = g.ow;
            o.pool3.OH = o.pool3.OW = ph;
            if (!keep_grads) o.out = nullptr;  // (the pre-pool output: only its tap reads it)
        }
        stem_y_written = o.out != nullptr;
    }
    if (!dp && !capturing) {  // one launch with the rescale fused (plan strategy 4, every tile resident)
        const hipError_t e = conv_fwd_fused(g, c.in, c.w, o, FusedBar{c.bar, c.epoch + 1, rc_err}, st);
        if (e != hipErrorNotSupported) {
            ++c.epoch;
            RTRY(e);
            probe(i, 0, false, st);
            return NITI_NO_ERROR;
        }
    }
    if (conv_fwd_spec_ok(g)) {  // the GEMM's speculative pair (plan strategy 3)
        int8_t* alt = conv_fwd_spec_alt_bytes(g) <= gspec_alt_bytes ? gspec_alt : nullptr;
        RTRY(conv_fwd_spec(g, c.in, c.w, rng(i, 0), o, c.gspec, 0, st, alt));
        if (dp && exact) RTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
        RTRY(conv_fwd_spec(g, c.in, c.w, rng(i, 0), o, c.gspec, 1, st, alt));
    } else {
        RTRY(conv_fwd_phase1(g, c.in, c.w, acc, rng(i, 0), slab, slab_bytes, st));
        if (dp && exact) RTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
        RTRY(conv_fwd_phase2(g, c.in, c.w, acc, rng(i, 0), o, slab_bytes, st));
    }
    probe(i, 0, false, st);
    return NITI_NO_ERROR;
}

// Input gradient of conv i into c.dx (exponent dy_exp + wscale + inc), the previous op's relu
// gradient (dx_mask) fused into its requantisation.
int ResNetModel::dgrad_conv(int i, hipStream_t st) {
    RConv& c = C[i];
    const ConvGeom& g = c.g;
    const bool dp = this->dp();
    if (c.dx == nullptr) return NITI_NO_ERROR;
    probe(i, 1, true, st);
    if (rows_dg_on(i)) {
        const ConvGeom& d = c.dg;
        const bool xn = rowconv_nhwc_pref(d);
        if (!xn) RTRY(nhwc16_to_c32(c.dy, g.n, g.oh * g.ow, g.cop, g.c_out, c.dyc32, st));
        const int8_t* dyin = xn ? c.dy : c.dyc32;
        RowConvOut o;
        o.x_nhwc = xn ? 1 : 0;
        o.out = c.dx;
        o.relu_mask = c.dx_mask;
        o.exp_in = c.dy_exp;
        o.wscale = c.ws_dev;
        o.exp_out = c.dx_exp;
        o.dgrad_slot = 1;
        if (!dp && !capturing && rowconv_fused_ok(d, true)) {
            RTRY(rowconv_fwd(d, dyin, c.wft, o, 0, rng(i, 1), c.bar, ++c.epoch, rc_err, st));
        } else if (rowconv_spec2_on()) {
            o.acc_store = rowconv_acc_bytes(d, true) ? rc_acc : nullptr;
            RTRY(rowconv_fwd(d, dyin, c.wft, o, RC_SPEC_A, rng(i, 1), c.bar, 0, nullptr, st));
            if (dp && exact) RTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
            RTRY(rowconv_fwd(d, dyin, c.wft, o, RC_SPEC_B, rng(i, 1), c.bar, 0, nullptr, st));
        } else {
            o.acc_store = rowconv_acc_bytes(d, true) ? rc_acc : nullptr;
            RTRY(rowconv_fwd(d, dyin, c.wft, o, 1, rng(i, 1), nullptr, 0, nullptr, st));
            if (dp && exact) RTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
            RTRY(rowconv_fwd(d, dyin, c.wft, o, 2, rng(i, 1), nullptr, 0, nullptr, st));
        }
        probe(i, 1, false, st);
        return NITI_NO_ERROR;
    }
    ActOut o;
    o.out = c.dx;
    o.relu_mask = c.dx_mask;
    o.exp_in = c.dy_exp;
    o.wscale = c.ws_dev;
    o.exp_out = c.dx_exp;
    uint32_t* slot = c.gspec + GEMM_SPEC_SLOT_WORDS;
    if (!dp && !capturing) {  // one launch with the rescale fused (plan strategy 4; stride 1)
        const hipError_t e = conv_dgrad_fused(g, c.dy, c.wT, o, FusedBar{c.bar, c.epoch + 1, rc_err}, st);
        if (e != hipErrorNotSupported) {
            ++c.epoch;
            RTRY(e);
            probe(i, 1, false, st);
            return NITI_NO_ERROR;
        }
    }
    if (conv_dgrad_spec_ok(g)) {
        int8_t* alt = conv_dgrad_spec_alt_bytes(g) <= gspec_alt_bytes ? gspec_alt : nullptr;
        RTRY(conv_dgrad_spec(g, c.dy, c.wT, rng(i, 1), o, slot, 0, st, alt));
        if (dp && exact) RTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
        RTRY(conv_dgrad_spec(g, c.dy, c.wT, rng(i, 1), o, slot, 1, st, alt));
    } else {
        const int8_t* subw = subpix_on() ? c.subw : nullptr;  // stride 2: four sub-pixel class GEMMs
        RTRY(conv_dgrad_phase1(g, c.dy, c.wT, acc, rng(i, 1), slab, slab_bytes, st, subw));
        if (dp && exact) RTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
        RTRY(conv_dgrad_phase2(g, c.dy, c.wT, acc, rng(i, 1), o, slab_bytes, st, subw));
    }
    probe(i, 1, false, st);
    return NITI_NO_ERROR;
}

// Weight gradient of conv i (int32, and on one device its range; data parallel, the bucket SUM and
// the range follow on the comm stream)
int ResNetModel::wgrad_conv(int i, hipStream_t st) {
    RConv& c = C[i];
    probe(i, 2, true, st);
    // single device, in the step: a split-K plan leaves its (own) slabs to the update's combine
    const bool defer = in_step && !dp() && !capturing && !tuning && ensure_wslab(i);
    c.defer = SgdJob{};
    RTRY(conv_wgrad_acc(c.g, c.in, c.dy, c.dwacc, dp() ? nullptr : rng(i, 2), defer ? c.wslab : slab_w,
                        defer ? c.wslab_bytes : slab_w_bytes, st, nullptr, defer ? &c.defer : nullptr));
    probe(i, 2, false, st);
    return NITI_NO_ERROR;
}

// conv i's own slab buffer for a deferred weight-gradient combine is big enough for the plan it
// runs with (false: the plan does not split K into C-shaped slabs, or the buffer was not sized)
bool ResNetModel::ensure_wslab(int i) {
    const RConv& c = C[i];
    const PlanChoice p = conv_plan_query(PLAN_WGRAD, c.g, false, slab_w_bytes);
    if (p.strat != 2 || p.splits < 2 || p.bm == PLAN_P16_TILE) return false;
    return c.wslab_bytes >= conv_wgrad_slab_bytes(c.g, p);  // (GEMM or tap-sharing slabs)
}

// Size every conv's deferred-combine slab for the current plans: at the head of run(), before
// anything is enqueued, whenever a plan override changed since the last sizing (one device sync,
// the old buffer freed).  Inside the step ensure_wslab only checks.
int ResNetModel::size_wslabs() {
    if (wslab_epoch == plan_override_epoch()) return NITI_NO_ERROR;
    bool synced = false;
    for (RConv& c : C) {
        const PlanChoice p = conv_plan_query(PLAN_WGRAD, c.g, false, slab_w_bytes);
        if (p.strat != 2 || p.splits < 2 || p.bm == PLAN_P16_TILE) continue;
        const size_t need = conv_wgrad_slab_bytes(c.g, p);
        if (c.wslab_bytes >= need) continue;
        if (!synced && hipDeviceSynchronize() != hipSuccess) return NITI_NO_EXECUTION;
        synced = true;
        void* q = ws.replace(c.wslab, need);
        c.wslab = (int32_t*)q;
        c.wslab_bytes = q ? need : 0;
        if (!q) return NITI_OUT_OF_MEMORY;
    }
    wslab_epoch = plan_override_epoch();
    return NITI_NO_ERROR;
}

// Block k's output: relu(requant(aligned y_b + shortcut)) -- range pass (the sum not stored),
// [MAX], the sum recomputed and requantised (niti_resnet.hip)
int ResNetModel::residual_fwd(int k, hipStream_t st) {
    RBlock& b = B[k];
    const RConv& cb = C[b.b];
    const int8_t* sc = b.p >= 0 ? C[b.p].y : b.u;
    const int8_t* es = b.p >= 0 ? C[b.p].y_exp : b.u_exp;
    if (res_fused_on()) {  // one launch: the range through the in-kernel grid barrier
        const hipError_t e = residual_fused(cb.y, cb.y_exp, sc, es, b.out_elems, b.ez, b.out_exp, 1, b.out, res_bar,
                                            ++res_epoch, rc_err, st);
        if (e != hipErrorNotSupported) {
            RTRY(e);
            return NITI_NO_ERROR;
        }
        --res_epoch;
    }
    if (res_spec_on()) {  // the speculative pair: one pass of the sum while its bit width holds
        uint32_t* slot = res_slot + (2 * k) * RES_SPEC_SLOT_WORDS;
        RTRY(residual_requant(cb.y, cb.y_exp, sc, es, b.out_elems, rng_blk(k, 0), b.ez, b.out_exp, 1, b.out, st,
                              nullptr, 1, slot));
        if (dp() && exact) RTRY(coll->allreduce(rng_blk(k, 0), MAX_WORDS, COLL_MAX_U32, st));
        RTRY(residual_requant(cb.y, cb.y_exp, sc, es, b.out_elems, rng_blk(k, 0), b.ez, b.out_exp, 1, b.out, st,
                              nullptr, 2, slot));
        return NITI_NO_ERROR;
    }
    RTRY(residual_add(cb.y, cb.y_exp, sc, es, b.out_elems, nullptr, nullptr, rng_blk(k, 0), st));
    if (dp() && exact) RTRY(coll->allreduce(rng_blk(k, 0), MAX_WORDS, COLL_MAX_U32, st));
    RTRY(residual_requant(cb.y, cb.y_exp, sc, es, b.out_elems, rng_blk(k, 0), b.ez, b.out_exp, 1, b.out, st));
    return NITI_NO_ERROR;
}

// The gradient at block k's input: requant(aligned dx_a + shortcut gradient), the previous block
// output's relu gradient fused (block 0: the stem's max-pool gradient takes it)
int ResNetModel::residual_bwd(int k, hipStream_t st) {
    RBlock& b = B[k];
    const RConv& ca = C[b.a];
    const int8_t* s = b.p >= 0 ? b.dus : b.dz;
    const int8_t* es = b.p >= 0 ? C[b.p].dx_exp : b.dz_exp;
    if (res_fused_on()) {
        const hipError_t e = residual_fused(b.dua, ca.dx_exp, s, es, b.in_elems, b.ezb, b.du_exp, 0, b.du, res_bar,
                                            ++res_epoch, rc_err, st, k > 0 ? B[k - 1].out : nullptr);
        if (e != hipErrorNotSupported) {
            RTRY(e);
            return NITI_NO_ERROR;
        }
        --res_epoch;
    }
    const int8_t* mask = k > 0 ? B[k - 1].out : nullptr;
    if (res_spec_on()) {  // the speculative pair (residual_fwd)
        uint32_t* slot = res_slot + (2 * k + 1) * RES_SPEC_SLOT_WORDS;
        RTRY(residual_requant(b.dua, ca.dx_exp, s, es, b.in_elems, rng_blk(k, 1), b.ezb, b.du_exp, 0, b.du, st, mask,
                              1, slot));
        if (dp() && exact) RTRY(coll->allreduce(rng_blk(k, 1), MAX_WORDS, COLL_MAX_U32, st));
        RTRY(residual_requant(b.dua, ca.dx_exp, s, es, b.in_elems, rng_blk(k, 1), b.ezb, b.du_exp, 0, b.du, st, mask,
                              2, slot));
        return NITI_NO_ERROR;
    }
    RTRY(residual_add(b.dua, ca.dx_exp, s, es, b.in_elems, nullptr, nullptr, rng_blk(k, 1), st));
    if (dp() && exact) RTRY(coll->allreduce(rng_blk(k, 1), MAX_WORDS, COLL_MAX_U32, st));
    RTRY(residual_requant(b.dua, ca.dx_exp, s, es, b.in_elems, rng_blk(k, 1), b.ezb, b.du_exp, 0, b.du, st, mask));
    return NITI_NO_ERROR;
}

// ------------------------------------------------------------------------------ data parallel
void ResNetModel::plan_buckets() {
    const int nl = (int)C.size();
    bucket_lo.assign(nl, 0);
    closes_bucket.assign(nl, 0);
    size_t a = 0;
    int hi = nl - 1;
    for (int i = nl - 1; i >= 0; --i) {
        a += (size_t)C[i].w_elems() * 4;
        if (a >= bucket_min_bytes || i == 0) {
            closes_bucket[i] = 1;
            for (int j = i; j <= hi; ++j) bucket_lo[j] = i;
            a = 0;
            hi = i - 1;
        }
    }
}

int ResNetModel::ensure_comm_stream() {
    if (cst) return NITI_NO_ERROR;
    if (hipStreamCreateWithFlags(&cst, hipStreamNonBlocking) != hipSuccess) return NITI_NO_EXECUTION;
    constexpr unsigned kFlags = hipEventDisableTiming | hipEventReleaseToDevice;
    ev_bucket.assign(C.size(), nullptr);
    for (auto& e : ev_bucket)
        if (hipEventCreateWithFlags(&e, kFlags) != hipSuccess) return NITI_NO_EXECUTION;
    if (hipEventCreateWithFlags(&ev_grads, kFlags) != hipSuccess) return NITI_NO_EXECUTION;
    plan_buckets();
    return NITI_NO_ERROR;
}

// the bucket of convs [lo, hi] (contiguous in grad_bucket; the weight gradients run in descending
// layer order, so it is complete once conv lo's is in): SUM over the ranks, then every layer's range
// of the summed gradient (NITI_GradientConv_Int8.cpp:274-296 over the global batch)
int ResNetModel::sum_bucket(int lo, hipStream_t st) {
    int hi = lo;
    while (hi + 1 < (int)C.size() && bucket_lo[hi + 1] == lo) ++hi;
    if (hi - lo + 1 > ABSMAX_MAX_JOBS) return NITI_NOT_SUPPORT;
    size_t elems = 0;
    for (int j = lo; j <= hi; ++j) elems += (size_t)C[j].w_elems();
    AbsmaxJob jobs[ABSMAX_MAX_JOBS];
    for (int j = lo; j <= hi; ++j) jobs[j - lo] = AbsmaxJob{C[j].dwacc, C[j].w_elems(), rng(j, 2), 0};
    hipStream_t s = st;
    if (!shared_comm) {  // own communicator: its own stream, overlapping the rest of the backward pass
        RTRY(hipEventRecord(ev_bucket[lo], st));
        RTRY(hipStreamWaitEvent(cst, ev_bucket[lo], 0));
        s = cst;
    }
    RTRY(coll_grad->allreduce(C[lo].dwacc, elems, COLL_SUM_I32, s));
    RTRY(absmax_many(jobs, hi - lo + 1, s));
    return NITI_NO_ERROR;
}

// ------------------------------------------------------------------------------ the step
int ResNetModel::run(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st) {
    const int n = batch;
    const int nl = (int)C.size();
    const int fc = nl - 1;
    const bool dp = this->dp();
    if (dp) {
        const int rc = ensure_comm_stream();
        if (rc != NITI_NO_ERROR) return rc;
    }
    struct InStep {  // weight gradients inside this step may defer their combine
        bool& f;
        explicit InStep(bool& x) : f(x) { f = true; }
        ~InStep() { f = false; }
    } in_step_guard(in_step);
    for (RConv& c : C) c.defer = SgdJob{};
    if (!dp && !capturing && !tuning) {
        const int rc = size_wslabs();  // (plan changes: no allocation or sync inside the step)
        if (rc != NITI_NO_ERROR) return rc;
    }
    // the range words start each step at zero: zeroed by the input statistics launch (uint8
    // images), else here
    if (images == nullptr || amax_bytes % 16 != 0) RTRY(hipMemsetAsync(amax, 0, amax_bytes, st));
    // input: NITIInt8Train's quantiser (MnistUtils.cpp:83-93) on uint8 images, or int8 x as given
    const int64_t px = (int64_t)n * 3 * in_hw * in_hw;
    const int8_t* xq = x_nchw;
    if (images != nullptr) {
        int ns = 0;
        RTRY(image_stats_slots(images, px, qslots, &ns, st, amax_bytes % 16 == 0 ? amax : nullptr,
                               amax_bytes % 16 == 0 ? amax_bytes : 0));
        RTRY(stats_finalize(qslots, ns, qstats, st));
        if (dp && exact) {
            RTRY(coll->allreduce(qstats, 2, COLL_SUM_U64, st));
            RTRY(coll->allreduce(qstats + 2, 2, COLL_MAX_U64, st));
        }
        RTRY(image_quantize(images, n, 3, in_hw * in_hw, 3, qstats, dp && exact ? px * world : px, x0n, exp0, false, st));
        xq = x0n;
    } else {
        RTRY(hipMemsetAsync(exp0, exp_in, 1, st));
        RTRY(hipMemcpyAsync(x0n, x_nchw, (size_t)px, hipMemcpyDeviceToDevice, st));
    }
    RTRY(im2col_small(stem, xq, STEM_KP, xcol, st, true));
    // forward
    int rc = fwd_conv(0, st);
    if (rc != NITI_NO_ERROR) return rc;
    const int ph = C[B[0].a].g.h;  // the stem's pooled size
    if (!stem_pooled)  // (else fused into the stem's requantise pass)
        RTRY(maxpool_nhwc16(C[0].y, n, stem.oh, stem.ow, 64, 3, 2, 1, p0, ph, ph, st, pool_ws));  // + first-max positions
    for (int k = 0; k < (int)B.size(); ++k) {
        const RBlock& b = B[k];
        if ((rc = fwd_conv(b.a, st)) != NITI_NO_ERROR) return rc;
        if ((rc = fwd_conv(b.b, st)) != NITI_NO_ERROR) return rc;
        if (b.p >= 0 && (rc = fwd_conv(b.p, st)) != NITI_NO_ERROR) return rc;
        if ((rc = residual_fwd(k, st)) != NITI_NO_ERROR) return rc;
    }
    // global sum pool + requantisation, the fc head, the loss gradient
    const RBlock& bl = B.back();
    const ConvGeom& gl = C[bl.b].g;
    RTRY(sum_pool(bl.out, n, gl.oh * gl.ow, gl.cop, gsum, rng_pool(), st));
    if (dp && exact) RTRY(coll->allreduce(rng_pool(), MAX_WORDS, COLL_MAX_U32, st));
    {
        ActRequant r;
        r.acc = gsum;
        r.rows = n;
        r.ldc = 512;
        r.amax = rng_pool();
        r.exp_in = bl.out_exp;
        r.exp_out = eg;
        r.out_nhwc16 = g8pool;
        RTRY(requant_act(r, st));
    }
    if ((rc = fwd_conv(fc, st)) != NITI_NO_ERROR) return rc;
    RConv& f = C[fc];
    RTRY(loss_grad(f.y, n, classes, f.g.cop, f.y_exp, labels, f.dy, st));
    // backward: weight gradients in descending layer order (gradient buckets close in memory order)
    auto wg = [&](int i) {
        int r = wgrad_conv(i, st);
        if (r == NITI_NO_ERROR && dp && closes_bucket[i]) r = sum_bucket(i, st);
        return r;
    };
    if ((rc = dgrad_conv(fc, st)) != NITI_NO_ERROR || (rc = wg(fc)) != NITI_NO_ERROR) return rc;
    RTRY(sum_pool_grad(dg, n, gl.oh * gl.ow, 512, bl.dz, st, bl.out));  // + the last block's relu gradient
    for (int k = (int)B.size() - 1; k >= 0; --k) {
        const RBlock& b = B[k];
        if (b.p >= 0 && (rc = wg(b.p)) != NITI_NO_ERROR) return rc;
        if ((rc = dgrad_conv(b.b, st)) != NITI_NO_ERROR || (rc = wg(b.b)) != NITI_NO_ERROR) return rc;
        if ((rc = dgrad_conv(b.a, st)) != NITI_NO_ERROR || (rc = wg(b.a)) != NITI_NO_ERROR) return rc;
        if (b.p >= 0 && (rc = dgrad_conv(b.p, st)) != NITI_NO_ERROR) return rc;
        if ((rc = residual_bwd(k, st)) != NITI_NO_ERROR) return rc;
    }
    // the stem: overlapping 3x3 / 2 max-pool gradient (first max wins) with the relu gradient, then
    // its weight gradient over the im2col
    // (the relu mask from the pooled output: the pre-pool output may not exist)
    RTRY(maxpool_relu_grad_arg(nullptr, pool_ws, B[0].du, n, stem.oh, stem.ow, 64, 3, 2, 1, ph, ph, 1, d0, st, p0));
    if ((rc = wg(0)) != NITI_NO_ERROR) return rc;
    if (dp) {  // every bucket summed and ranged before the update
        if (!shared_comm) {
            RTRY(hipEventRecord(ev_grads, cst));
            RTRY(hipStreamWaitEvent(st, ev_grads, 0));
        }
    }
    // NITI_SGD (NITI_SGD.hpp:20-54) for every layer in one launch, after every input gradient read the
    // old weights; it also rewrites the row kernels' fragment-major copies and the GEMM input
    // gradient's transposed copy
    SgdJob jobs[SGD_MAX_JOBS];
    if (nl > SGD_MAX_JOBS) return NITI_NOT_SUPPORT;
    for (int i = 0; i < nl; ++i) {
        RConv& c = C[i];
        const ConvGeom& g = c.g;
        jobs[i] = SgdJob{c.dwacc, rng(i, 2), RULE_WGRAD_BW2, g.c_out, g.c_in, g.kh * g.kw, g.cip, g.cop, c.w,
                         i > 0 && !rows_dg_on(i) ? c.wT : nullptr, keep_grads ? c.g8 : nullptr};
        jobs[i].wf = c.rows ? c.wf : nullptr;
        jobs[i].wft = c.rows_dg ? c.wft : nullptr;
        if (c.subw != nullptr) {  // the stride-2 input gradient's sub-pixel class weights
            jobs[i].subw = c.subw;
            jobs[i].sub_kh = g.kh;
            jobs[i].sub_kw = g.kw;
            jobs[i].sub_pt = g.pt;
            jobs[i].sub_pl = g.pl;
        }
        if (c.defer.slab != nullptr) {  // this conv's split-K slabs, combined in the update launch
            jobs[i].slab = c.defer.slab;
            jobs[i].splits = c.defer.splits;
            jobs[i].slab_stride = c.defer.slab_stride;
            jobs[i].slab_n = c.defer.slab_n;
            jobs[i].slab_map = c.defer.slab_map;  // (the tap-sharing kernel's tile-blocked slabs)
            jobs[i].tb_tiles_ci = c.defer.tb_tiles_ci;
            jobs[i].tb_cip4 = c.defer.tb_cip4;
            jobs[i].tb_ld4 = c.defer.tb_ld4;
            jobs[i].tb_m = c.defer.tb_m;
            jobs[i].tb_s = c.defer.tb_s;
        }
    }
    RTRY(sgd_update_many(jobs, nl, st));
    g8_written = keep_grads;
    return NITI_NO_ERROR;
}

int ResNetModel::step(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) return NITI_NO_EXECUTION;
    if (cs == hipStreamCaptureStatusActive) {  // the caller captures the step: no fused grid barrier in it
        if (coll != nullptr) return NITI_NOT_SUPPORT;
        capturing = true;
        const int rc = run(x_nchw, exp_in, images, labels, st);
        capturing = false;
        return rc;
    }
    if (!use_graph || coll != nullptr) return run(x_nchw, exp_in, images, labels, st);
    const void* kx = x_nchw ? (const void*)x_nchw : (const void*)images;
    if (gexec == nullptr || kx != gkey_x || labels != gkey_l || exp_in != gkey_e) {
        drop_graph();
        if (!gstream) {
            RTRY(hipStreamCreateWithFlags(&gstream, hipStreamNonBlocking));
            RTRY(hipEventCreateWithFlags(&gin, hipEventDisableTiming));
            RTRY(hipEventCreateWithFlags(&gout, hipEventDisableTiming));
        }
        RTRY(hipStreamBeginCapture(gstream, hipStreamCaptureModeThreadLocal));
        capturing = true;
        const int rc = run(x_nchw, exp_in, images, labels, gstream);
        capturing = false;
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(gstream, &g);
        if (e == hipSuccess && rc == NITI_NO_ERROR) e = hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0);
        if (g) (void)hipGraphDestroy(g);
        if (rc != NITI_NO_ERROR || e != hipSuccess) {
            drop_graph();
            use_graph = false;  // direct launches for this model
            (void)hipGetLastError();
            return run(x_nchw, exp_in, images, labels, st);
        }
        gkey_x = kx;
        gkey_l = labels;
        gkey_e = exp_in;
    }
    RTRY(hipEventRecord(gin, st));
    RTRY(hipStreamWaitEvent(gstream, gin, 0));
    RTRY(hipGraphLaunch(gexec, gstream));
    RTRY(hipEventRecord(gout, gstream));
    RTRY(hipStreamWaitEvent(st, gout, 0));
    return NITI_NO_ERROR;
}

// Per-shape GEMM plan autotuning of the GEMM-path phases (as Model::autotune): every candidate
// tile / strategy / K split of each forward, input-gradient and weight-gradient GEMM, timed as the
// whole conv phase on the last step's buffers; the fastest kept as a plan override (keyed by GEMM
// shape, so convs of one shape share it).  Plans never change results.
int ResNetModel::autotune(hipStream_t st, int reps) {
    if (reps < 1) reps = 5;
    if (!ensure_slab(size_t(96) << 20, false) || !ensure_slab(size_t(96) << 20, true)) return NITI_OUT_OF_MEMORY;
    drop_graph();
    hipEvent_t ev[2];
    for (auto& e : ev)
        if (hipEventCreate(&e) != hipSuccess) return NITI_NO_EXECUTION;
    tuning = true;
    int rc = NITI_NO_ERROR;
    auto run_op = [&](int i, int op) {
        if (op == PLAN_FWD && i == 0) {  // the stem with its max pool (fused into a separate requantise pass)
            int r = fwd_conv(0, st);
            if (r == NITI_NO_ERROR && !stem_pooled &&
                maxpool_nhwc16(C[0].y, batch, stem.oh, stem.ow, 64, 3, 2, 1, p0, C[B[0].a].g.h, C[B[0].a].g.w, st,
                               pool_ws) != hipSuccess)
                r = NITI_NO_EXECUTION;
            return r;
        }
        return op == PLAN_FWD ? fwd_conv(i, st) : op == PLAN_WGRAD ? wgrad_conv(i, st) : dgrad_conv(i, st);
    };
    auto time_op = [&](int i, int op, float* us) -> int {
        int r = run_op(i, op);
        float best = 1e30f;
        for (int t = 0; t < 3 && r == NITI_NO_ERROR; ++t) {
            if (hipEventRecord(ev[0], st) != hipSuccess) return NITI_NO_EXECUTION;
            for (int k = 0; k < reps && r == NITI_NO_ERROR; ++k) r = run_op(i, op);
            if (hipEventRecord(ev[1], st) != hipSuccess || hipEventSynchronize(ev[1]) != hipSuccess)
                return NITI_NO_EXECUTION;
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, ev[0], ev[1]) != hipSuccess) return NITI_NO_EXECUTION;
            best = std::min(best, ms * 1000.f / reps);
        }
        *us = best;
        return r;
    };
    const bool log = getenv("NITI_DIAG_TUNE_LOG") != nullptr;
    static const int tiles[7][2] = {{PLAN_TAPS_TILE, PLAN_TAPS_TILE}, {128, 128}, {128, 64}, {64, 128}, {64, 64},
                                    {256, 128}, {128, 256}};
    static const int split_opts[] = {2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64};
    std::set<PlanKey> done;
    for (int i = 0; i < (int)C.size() && rc == NITI_NO_ERROR; ++i) {
        for (int op : {PLAN_FWD, PLAN_WGRAD, PLAN_DGRAD}) {
            if (op == PLAN_FWD && rows_on(i)) continue;
            if (op == PLAN_DGRAD && (C[i].dx == nullptr || rows_dg_on(i))) continue;
            const ConvGeom& g = C[i].g;
            const PlanKey key = conv_plan_key(op, g);
            if (!done.insert(key).second) continue;
            const int k_step = conv_plan_k_step(op, g);
            const int steps = (key.K + k_step - 1) / k_step;
            const bool act = op != PLAN_WGRAD;
            plan_override_clear(key);
            const size_t wsb = op == PLAN_WGRAD ? slab_w_bytes : slab_bytes;
            PlanChoice best = conv_plan_query(op, g, act, wsb);
            float best_us = 0.f;
            rc = time_op(i, op, &best_us);
            const bool taps = op == PLAN_WGRAD && conv_wgrad_taps_ok(g);
            for (const auto& t : tiles) {
                if (rc != NITI_NO_ERROR) break;
                if (t[0] == PLAN_TAPS_TILE && !taps) continue;
                std::vector<PlanChoice> cands;
                PlanChoice c;
                c.bm = t[0];
                c.bn = t[1];
                cands.push_back(c);
                if (act) {
                    c.strat = 1;
                    cands.push_back(c);
                    // the speculative pair only on request (NITI_TUNE_SPEC=1): timed here on one
                    // batch its guess always holds, but over a run of batches 60-80 % of the deep
                    // layers' pairs miss (profiles/r05_gemm_spec.txt) and then cost more than STORE
                    if (tune_spec()) {
                        c.strat = 3;
                        cands.push_back(c);
                    }
                    c.strat = 4;  // one launch, the rescale fused (where every tile is resident)
                    cands.push_back(c);
                }
                for (int s : split_opts) {
                    if (s > steps / 2 || plan_slab_bytes(key.M, key.N, s) > wsb) break;
                    c.strat = 2;
                    c.splits = s;
                    cands.push_back(c);
                }
                for (const PlanChoice& cand : cands) {
                    plan_override_set(key, cand);
                    float us = 0.f;
                    rc = time_op(i, op, &us);
                    if (log)
                        fprintf(stderr, "tune conv %d op %d plan (%d,%d,%d,%d) %.2f us\n", i, op, cand.bm, cand.bn,
                                cand.splits, cand.strat, us);
                    if (rc != NITI_NO_ERROR) break;
                    if (us < best_us) {
                        best_us = us;
                        best = cand;
                    }
                }
            }
            plan_override_set(key, best);
        }
    }
    tuning = false;
    for (auto e : ev) (void)hipEventDestroy(e);
    if (hipStreamSynchronize(st) != hipSuccess) rc = NITI_NO_EXECUTION;
    return rc;
}

int ResNetModel::run_phase(int layer, int phase, hipStream_t st) {
    if (layer < 0 || layer >= (int)C.size() || phase < 0 || phase > 2) return NITI_INVALID_VALUE;
    if (phase == 1 && C[layer].dx == nullptr) return NITI_INVALID_VALUE;
    std::unique_ptr<Collective> c = std::move(coll), cg = std::move(coll_grad);
    const int rc = phase == 0 ? fwd_conv(layer, st) : phase == 1 ? dgrad_conv(layer, st) : wgrad_conv(layer, st);
    coll = std::move(c);
    coll_grad = std::move(cg);
    return rc;
}

// ------------------------------------------------------------------------------ host access
// the stem's weights as the im2col GEMM holds them: [co][STEM_KP], column (ky * 7 + kx) * 3 + c
static void stem_cols_from_oihw(const ConvGeom& o, const int8_t* w, int8_t* wc, int kp) {
    memset(wc, 0, (size_t)o.c_out * kp);
    for (int co = 0; co < o.c_out; ++co)
        for (int c = 0; c < o.c_in; ++c)
            for (int t = 0; t < o.kh * o.kw; ++t)
                wc[(size_t)co * kp + t * o.c_in + c] = w[((size_t)co * o.c_in + c) * o.kh * o.kw + t];
}
static void oihw_from_stem_cols(const ConvGeom& o, const int8_t* wc, int8_t* w, int kp) {
    for (int co = 0; co < o.c_out; ++co)
        for (int c = 0; c < o.c_in; ++c)
            for (int t = 0; t < o.kh * o.kw; ++t)
                w[((size_t)co * o.c_in + c) * o.kh * o.kw + t] = wc[(size_t)co * kp + t * o.c_in + c];
}

int ResNetModel::refresh_copies(int i, hipStream_t st) {
    RConv& c = C[i];
    const ConvGeom& g = c.g;
    if (c.wT && ohwi16_to_ihwo16(c.w, g.c_out, g.c_in, g.kh * g.kw, g.cip, g.cop, c.wT, st) != hipSuccess)
        return NITI_NO_EXECUTION;
    if (c.rows && weights_to_wf(c.w, g.c_out, g.c_in, g.cip, false, c.wf, st) != hipSuccess) return NITI_NO_EXECUTION;
    if (c.rows_dg && weights_to_wf(c.w, g.c_out, g.c_in, g.cip, true, c.wft, st) != hipSuccess) return NITI_NO_EXECUTION;
    if (c.subw && conv_dgrad_subpix_weights(g, c.wT, c.subw, st) != hipSuccess) return NITI_NO_EXECUTION;
    return NITI_NO_ERROR;
}

int ResNetModel::set_weight(int i, const int8_t* w_host, int wscale) {
    if (i < 0 || i >= (int)C.size() || !w_host) return NITI_INVALID_VALUE;
    RConv& c = C[i];
    const ConvGeom& g = c.g;
    std::vector<int8_t> colw;
    if (i == 0) {
        colw.resize((size_t)g.c_out * STEM_KP);
        stem_cols_from_oihw(c.og, w_host, colw.data(), STEM_KP);
        w_host = colw.data();
    }
    const size_t nb = (size_t)g.c_out * g.c_in * g.kh * g.kw;
    int8_t* tmp = nullptr;
    if (hipMalloc(&tmp, nb) != hipSuccess) return NITI_OUT_OF_MEMORY;
    int rc = NITI_NO_ERROR;
    if (hipMemcpy(tmp, w_host, nb, hipMemcpyHostToDevice) != hipSuccess ||
        oihw_to_ohwi16(tmp, g.c_out, g.c_in, g.kh * g.kw, g.cip, c.w, nullptr) != hipSuccess ||
        hipMemset(c.ws_dev, (int)(int8_t)wscale, 1) != hipSuccess)
        rc = NITI_NO_EXECUTION;
    if (rc == NITI_NO_ERROR) rc = refresh_copies(i, nullptr);
    if (rc == NITI_NO_ERROR && hipDeviceSynchronize() != hipSuccess) rc = NITI_NO_EXECUTION;
    c.wscale = (int8_t)wscale;
    (void)hipFree(tmp);
    drop_graph();
    return rc;
}

int ResNetModel::get_weight(int i, int8_t* w_host) {
    if (i < 0 || i >= (int)C.size() || !w_host) return NITI_INVALID_VALUE;
    const RConv& c = C[i];
    const ConvGeom& g = c.g;
    const size_t nb = (size_t)g.c_out * g.c_in * g.kh * g.kw;
    int8_t* tmp = nullptr;
    if (hipDeviceSynchronize() != hipSuccess || hipMalloc(&tmp, nb) != hipSuccess) return NITI_OUT_OF_MEMORY;
    std::vector<int8_t> colw(i == 0 ? nb : 0);
    int rc = NITI_NO_ERROR;
    if (ohwi16_to_oihw(c.w, g.c_out, g.c_in, g.kh * g.kw, g.cip, tmp, nullptr) != hipSuccess ||
        hipMemcpy(i == 0 ? colw.data() : w_host, tmp, nb, hipMemcpyDeviceToHost) != hipSuccess)
        rc = NITI_NO_EXECUTION;
    if (rc == NITI_NO_ERROR && i == 0) oihw_from_stem_cols(c.og, colw.data(), w_host, STEM_KP);
    (void)hipFree(tmp);
    return rc;
}

int ResNetModel::get_tap(int layer, int which, int8_t* host, size_t bytes, hipStream_t st) {
    if (layer < 0 || layer >= (int)C.size()) return NITI_INVALID_VALUE;
    const RConv& c = C[layer];
    const ConvGeom& g = c.g;
    const int n = batch;
    if (hipStreamSynchronize(st) != hipSuccess) return NITI_NO_EXECUTION;
    size_t need = 0;
    if (which == 0 && layer == 0 && !stem_y_written) return NITI_INVALID_VALUE;  // (not written by the last step)
    if (which == 0 || which == 2)
        need = (size_t)n * g.c_out * g.oh * g.ow;
    else if (which == 1 && g8_written)
        need = (size_t)g.c_out * g.c_in * g.kh * g.kw;
    else
        return NITI_INVALID_VALUE;
    const size_t out_need = which == 1 ? (size_t)c.og.c_out * c.og.c_in * c.og.kh * c.og.kw : need;
    if (bytes < out_need) return NITI_INVALID_VALUE;
    int8_t* tmp = nullptr;
    if (hipMalloc(&tmp, need) != hipSuccess) return NITI_OUT_OF_MEMORY;
    hipError_t e;
    if (which == 0)
        e = nhwc16_to_nchw(c.y, n, g.c_out, g.oh * g.ow, g.cop, tmp, nullptr);
    else if (which == 2)
        e = nhwc16_to_nchw(c.dy, n, g.c_out, g.oh * g.ow, g.cop, tmp, nullptr);
    else
        e = ohwi16_to_oihw(c.g8, g.c_out, g.c_in, g.kh * g.kw, g.cip, tmp, nullptr);
    if (which == 1 && layer == 0) {
        std::vector<int8_t> colw(need);
        if (e == hipSuccess) e = hipMemcpy(colw.data(), tmp, need, hipMemcpyDeviceToHost);
        if (e == hipSuccess) oihw_from_stem_cols(c.og, colw.data(), host, STEM_KP);
    } else if (e == hipSuccess) {
        e = hipMemcpy(host, tmp, need, hipMemcpyDeviceToHost);
    }
    (void)hipFree(tmp);
    return e == hipSuccess ? NITI_NO_ERROR : NITI_NO_EXECUTION;
}

int ResNetModel::get_logits(int8_t* host, int* exp_out, hipStream_t st) {
    const RConv& f = C.back();
    const int n = batch;
    if (hipStreamSynchronize(st) != hipSuccess) return NITI_NO_EXECUTION;
    std::vector<int8_t> buf((size_t)n * f.g.cop);
    int8_t e = 0;
    if (hipMemcpy(buf.data(), f.y, buf.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&e, f.y_exp, 1, hipMemcpyDeviceToHost) != hipSuccess)
        return NITI_NO_EXECUTION;
    for (int i = 0; i < n; ++i) memcpy(host + (size_t)i * f.g.c_out, buf.data() + (size_t)i * f.g.cop, f.g.c_out);
    if (exp_out) *exp_out = e;
    return NITI_NO_ERROR;
}

int ResNetModel::get_input(int8_t* host, int* ascale, hipStream_t st) {
    if (hipStreamSynchronize(st) != hipSuccess) return NITI_NO_EXECUTION;
    int8_t e = 0;
    if (hipMemcpy(host, x0n, (size_t)batch * 3 * in_hw * in_hw, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&e, exp0, 1, hipMemcpyDeviceToHost) != hipSuccess)
        return NITI_NO_EXECUTION;
    if (ascale) *ascale = e;
    return NITI_NO_ERROR;
}

int64_t ResNetModel::step_macs() const {
    // every layer's forward and weight gradient, every input gradient but the stem's (never run)
    int64_t s = 0;
    for (size_t i = 0; i < C.size(); ++i) s += C[i].macs() * (i > 0 ? 3 : 2);
    return s;
}

int ResNetModel::spec_stats(uint32_t* out, int max_layers) {
    const int nl = std::min(max_layers, (int)C.size());
    std::fill(out, out + (size_t)nl * 6, 0u);
    for (int i = 0; i < nl; ++i) {
        for (int d = 0; d < 2; ++d) {  // the row kernels' pair and the GEMM's (its own slot, no store mode)
            uint32_t w[5] = {0, 0, 0, 0, 0}, gw[4] = {0, 0, 0, 0};
            if (C[i].bar != nullptr &&
                hipMemcpy(w, rowconv_spec_slot(C[i].bar, d != 0), sizeof(w), hipMemcpyDeviceToHost) != hipSuccess)
                return NITI_INVALID_VALUE;
            if (hipMemcpy(gw, C[i].gspec + d * GEMM_SPEC_SLOT_WORDS, sizeof(gw), hipMemcpyDeviceToHost) != hipSuccess)
                return NITI_INVALID_VALUE;
            out[i * 6 + d * 3] = std::max(w[0], gw[0]);
            out[i * 6 + d * 3 + 1] = w[2] + gw[2];
            out[i * 6 + d * 3 + 2] = w[4] + gw[3];  // the GEMM pair: misses settled from an alternate
        }
    }
    return NITI_NO_ERROR;
}

int ResNetModel::rowconv_error() {
    uint32_t e = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&e, rc_err, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return NITI_NO_EXECUTION;
    return (int)e;
}

}  // namespace niti
