// niti_model.hip -- device-resident NITI int8 training step (+ RCCL data parallelism).
//
// One NITI_SGD step of the reference's NITIInt8Train (execution-engine/tools/train/source/
// demo/MnistUtils.cpp:68-147, optimizer/NITI_SGD.hpp:20-54) executed entirely on the GPU:
//   forward   : per layer NITI_Conv_Int8 (+ NITI_Relu_Int8, NITI_Maxpool_Int8)
//   loss      : NITI_LOSS_Grad_Int8 (NITI_CPULossGrad_Int8.cpp:81-200)
//   backward  : grad/NITI_Conv_Int8_Grad.cpp -- NITI_GradientCONV_Int8 (weight gradient) and
//               NITI_DeCONV_Int8 (input gradient, skipped for the first layer exactly as the
//               lazy reference graph skips it), pool / relu gradients
//   update    : w <- clip(w - g, +-127)  (NITI_SGD.hpp:49-52)
// With a communicator (exact mode) the input quantiser's statistics are all-reduced (SUM,
// MAX), every forward / input-gradient range with MAX and every int32 weight-gradient
// accumulator with SUM before it is requantised, so N ranks of batch b reproduce one device of
// batch N*b bit for bit.
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/niti_hip.h"
#include "niti_internal.hpp"
#include "niti_kernels.hpp"
#include "niti_coll.hpp"
#include "niti_map.hpp"
#include "niti_resnet_model.hpp"

namespace niti {

namespace {
extern int g_p16_jobs_cap;
}
void model_p16_jobs_cap(int cap) { g_p16_jobs_cap = cap <= 0 ? P16_MAX_JOBS : cap; }

namespace {

// im2col of the first layer: xcol[p][(ky * KW + kx) * C + c] = x[n][oy * sh + ky - pt][ox * sw + kx - pl][c]
// (NHWC16 input, zero outside the image and for k >= C * KH * KW), one output pixel (32 bytes) per
// thread; C / KH / KW as template arguments keep the byte positions compile-time (VGG 3/3/3,
// LeNet 1/5/5), 0 selects the runtime fallback.
template <int C, int KH, int KW>
struct Im2Col32 {
    const int8_t* x;
    int cip, h, w, oh, ow, c, kh, kw, sh, sw, pt, pl;
    int8_t* out;
    __device__ void operator()(int64_t p) const {
        typedef signed char v16c_t __attribute__((ext_vector_type(16)));
        const int64_t img = p / ((int64_t)oh * ow);
        const int r = (int)(p - img * oh * ow);
        const int oy = r / ow, ox = r - (r / ow) * ow;
        const int8_t* base = x + img * h * w * cip;
        if constexpr (C > 0) {
            v16c_t v[2] = {v16c_t{}, v16c_t{}};
#pragma unroll
            for (int ky = 0; ky < KH; ++ky)
#pragma unroll
                for (int kx = 0; kx < KW; ++kx) {
                    const int iy = oy * sh + ky - pt, ix = ox * sw + kx - pl;
                    const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
                    // the pixel's first 16 channels in one 16-byte load (zeros outside the image)
                    const v16c_t px = ok ? *(const v16c_t*)(base + ((int64_t)iy * w + ix) * cip) : v16c_t{};
#pragma unroll
                    for (int ch = 0; ch < C; ++ch) {
                        const int k = (ky * KW + kx) * C + ch;
                        v[k >> 4][k & 15] = px[ch];
                    }
                }
            *(v16c_t*)(out + p * 32) = v[0];
            *(v16c_t*)(out + p * 32 + 16) = v[1];
        } else {
            int k = 0;
            for (int ky = 0; ky < kh; ++ky)
                for (int kx = 0; kx < kw; ++kx) {
                    const int iy = oy * sh + ky - pt, ix = ox * sw + kx - pl;
                    const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
                    for (int ch = 0; ch < c; ++ch, ++k)
                        out[p * 32 + k] = ok ? base[((int64_t)iy * w + ix) * cip + ch] : (int8_t)0;
                }
            for (; k < 32; ++k) out[p * 32 + k] = 0;
        }
    }
};

// diagnostic: jobs per P16 conversion launch (niti_diag_p16_jobs_cap)
int g_p16_jobs_cap = P16_MAX_JOBS;

static hipError_t im2col32(const ConvGeom& o, const int8_t* x16, int8_t* out, hipStream_t st) {
    const int64_t px = (int64_t)o.n * o.oh * o.ow;
    const int cip = round_up(o.c_in, 16);
    if (o.c_in == 3 && o.kh == 3 && o.kw == 3)
        return launch_map(px, Im2Col32<3, 3, 3>{x16, cip, o.h, o.w, o.oh, o.ow, 3, 3, 3, o.sh, o.sw, o.pt, o.pl, out}, st);
    if (o.c_in == 1 && o.kh == 5 && o.kw == 5)
        return launch_map(px, Im2Col32<1, 5, 5>{x16, cip, o.h, o.w, o.oh, o.ow, 1, 5, 5, o.sh, o.sw, o.pt, o.pl, out}, st);
    return launch_map(px, Im2Col32<0, 0, 0>{x16, cip, o.h, o.w, o.oh, o.ow, o.c_in, o.kh, o.kw, o.sh, o.sw, o.pt, o.pl,
                                            out},
                      st);
}

// NCHW flatten of a pooled NHWC16 map: out[n][c*HW + p] = in[n][p][c] (c < C); LeNet's
// _Reshape(x, {0, -1, 1, 1}) after _Convert(x, NCHW) (mnistTrain.cpp:175-176).
struct FlattenFwd {
    const int8_t* in;
    int hw, c, cp, ldo;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [n][ldo]
        const int64_t b = i / ldo;
        const int j = (int)(i - b * ldo);
        const int ch = j / hw, p = j - ch * hw;
        out[i] = ch < c ? in[(b * hw + p) * cp + ch] : (int8_t)0;
    }
};
struct FlattenBwd {
    const int8_t* dout;
    int hw, c, cp, ldo;
    int8_t* din;
    __device__ void operator()(int64_t i) const {  // i over [n][hw][cp]
        const int ch = (int)(i % cp);
        const int64_t r = i / cp;
        const int p = (int)(r % hw);
        const int64_t b = r / hw;
        din[i] = ch < c ? dout[b * ldo + ch * hw + p] : (int8_t)0;
    }
};

}  // namespace

struct Layer {
    ConvGeom g{};
    int relu = 0, pool = 0, flatten = 0;
    int ph = 0, pw = 0;      // pooled size
    int8_t wscale = 0;
    // persistent
    int8_t* w = nullptr;     // OHWI16
    int8_t* ws_dev = nullptr;  // wscale scalar
    // per step
    int8_t* wT = nullptr;    // IHWO16, kept in step with w by sgd_update
    int8_t* r = nullptr;     // conv (+relu) output NHWC16 [n][oh][ow][cop]
    int8_t* p = nullptr;     // pooled NHWC16
    // the 2x2 pool's gradient route recorded by the forward (pool_code4, [n][ph][pw][cop] bytes; the
    // pooled layers whose forward and next input gradient run on the kernels that know it)
    int8_t* pc = nullptr;
    bool r_written = false;  // this step wrote r (a pooled layer with a recorded route skips it
                             // under keep_grads(0): nothing else reads it; its tap is then invalid)
    int8_t* flat = nullptr;  // flattened NHWC16 [n][1][1][c*ph*pw]
    int8_t* dy = nullptr;    // output gradient NHWC16 [n][oh][ow][cop]
    int8_t* dtmp = nullptr;  // gradient wrt the pooled / flattened output
    int8_t* dflat = nullptr;
    int32_t* dwacc = nullptr;  // [co][kk][cip]
    // the P16 weight gradient's own split-K slabs when its combine is deferred to the NITI_SGD
    // launch (sgd_update_many), and this step's deferred combine (slab == null: none)
    int32_t* slab16 = nullptr;
    size_t slab16_bytes = 0;
    // the GEMM-path weight gradient's own split-K slabs when its combine is deferred the same way
    // (sized for the current plans at the head of run(), size_wslabs)
    int32_t* wslab = nullptr;
    size_t wslab_bytes = 0;
    SgdJob defer{};
    bool fc_sgd = false;  // this step's weight gradient took the fused NITI_SGD form (pass 1 in run())
    int8_t* g8 = nullptr;    // int8 weight gradient OHWI16
    int8_t* exp = nullptr;   // exponent of this layer's output
    const int8_t* in = nullptr;  // NHWC16 input (previous output or x0)
    // First layer with C_in * KH * KW <= 32 (VGG: 3 x 3 x 3, LeNet: 1 x 5 x 5): the conv runs as a
    // 1x1 conv over an im2col copy of its input (xcol [pixels][32], k = (ky * KW + kx) * C_in + c,
    // zero padded), so its GEMMs take K = 32 instead of 16 channels x 9 taps and the padded taps
    // cost nothing.  g is that 1x1 geometry; og the layer as the network defines it (reported,
    // weights and taps converted to / from it on the host).
    int col = 0;
    ConvGeom og{};
    int8_t* xcol = nullptr;
    // stride-1 pad-1 3x3 layers on the register-fed forward with the fused rescale
    // (niti_rowconv.hip): its C32 input copy, fragment-major weights, grid-barrier state
    int rc = 0;
    int8_t* xc32 = nullptr;
    int8_t* wf = nullptr;
    uint32_t* bar = nullptr;
    uint32_t epoch = 0;
    // its input gradient on the same kernel (rotated transposed weights in WF, dy in C32, the
    // previous layer's relu / pool gradient in the epilogue); dg = that conv's geometry
    int rcd = 0;
    ConvGeom dg{};
    // the GEMM path's speculative pair (plan strategy 3): hint slots, forward and input gradient
    uint32_t* gspec = nullptr;  // 2 x GEMM_SPEC_SLOT_WORDS
    int8_t* wft = nullptr;
    int8_t* dyc32 = nullptr;
    int64_t w_elems() const { return (int64_t)g.c_out * g.kh * g.kw * g.cip; }
    int64_t macs() const { return (int64_t)og.n * og.oh * og.ow * og.c_out * og.c_in * og.kh * og.kw; }
};

struct Model {
    int arch = 0, batch = 0, in_c = 0, in_h = 0, in_w = 0, classes = 10;
    std::vector<Layer> L;
    Workspace ws;
    int8_t* x0 = nullptr;   // NHWC16 input
    int8_t* exp0 = nullptr; // input exponent
    int32_t* acc = nullptr; // shared fwd / dgrad accumulator
    void* slab = nullptr;   // split-K slabs of the forward / input-gradient GEMMs (step stream)
    size_t slab_bytes = 0;
    void* slab_w = nullptr; // split-K slabs of the weight-gradient GEMMs (their own stream)
    size_t slab_w_bytes = 0;
    // P16 copies of the weight-gradient operands (niti_wgrad.hip): one input copy per layer (all
    // converted together when the backward pass starts, off the step stream) and one
    // output-gradient copy per layer, written by the input-gradient requantisation that produces
    // dy (requant_act's out_p16) where that pass can, else converted before the weight gradient
    int32_t* grad_bucket = nullptr;  // every layer's dwacc, contiguous
    size_t grad_bucket_elems = 0;
    std::vector<int8_t*> xp16, dp16;
    std::vector<char> dp16_valid;  // dp16[i] holds L[i].dy as it is now
    std::vector<char> xp16_valid;  // xp16[i] holds L[i].in as it is now (cleared when a step starts)
    void invalidate_xp16() { std::fill(xp16_valid.begin(), xp16_valid.end(), 0); }
    bool fuse_dp16 = true;    // dy's P16 copy written by the requantisation that produces dy
    // register-fed forward (niti_rowconv.hip) for the layers it takes; xc32_valid[i]: L[i].xc32
    // holds L[i].in as it is now (written by the previous layer's epilogue, else converted)
    bool use_rowconv = true;
    std::vector<char> xc32_valid;
    uint32_t* rc_err = nullptr;
    bool in_step = false;  // run(): weight gradients may defer their combine to the update launch
    // a fully connected layer's weight gradient as a range pass plus a recompute that applies
    // NITI_SGD in its epilogue (conv_wgrad_fc_sgd): single device, inside run() (NITI_FC_SGD=0: off)
    bool fc_sgd_layer(int i) const {
        static const bool off = getenv("NITI_FC_SGD") && atoi(getenv("NITI_FC_SGD")) == 0;
        const ConvGeom& g = L[i].g;
        return in_step && !off && !dp() && !tuning && conv_wgrad_fc_sgd_ok(g) &&
               !(head_layer(i) && g.c_out <= 32 && g.cip % 32 == 0) && wgrad_p16_splits(i) == 0;
    }
    bool defer_combine() const {
        static const bool off = getenv("NITI_DIAG_SGD_COMBINE") && atoi(getenv("NITI_DIAG_SGD_COMBINE")) == 0;
        return in_step && !off && !dp() && !capturing && !tuning;
    }
    // the row kernels' accumulator store for their two-launch form (data parallel, graph capture):
    // the range launch keeps its int32 accumulators here, the requantise launch reads them back
    int32_t* rc_acc = nullptr;
    size_t rc_acc_size = 0;
    // the GEMM speculative pairs' alternates (one bit width below / above A's guess), shared by every
    // layer phase: a pair's B consumes them before the next pair's A writes them
    int8_t* gspec_alt = nullptr;
    size_t gspec_alt_bytes = 0;
    // the first layer's range came with its im2col copy (input_im2col's Conv0Range) this step
    bool conv0_ranged = false;
    bool rowconv_layer(int i) const { return use_rowconv && L[i].rc; }
    // dyc32_valid[i]: L[i].dyc32 holds L[i].dy as it is now (written by the next layer's input
    // gradient epilogue, else converted)
    std::vector<char> dyc32_valid;
    // dy16_valid[i]: L[i].dy (NHWC16) was written this step; a row-kernel input gradient leaves it
    // out when the layer's own consumers read its C32 (input gradient) and P16 (weight gradient)
    // copies (niti_model_get_tap rebuilds it from the C32 copy)
    std::vector<char> dy16_valid;
    bool rowconv_dgrad_layer(int i) const { return use_rowconv && L[i].rcd; }
    // layer i's 2x2 pool route travels as codes (Layer::pc): its forward (the first layer's conv0
    // kernel or a row kernel) records it and layer i + 1's input gradient (a row kernel, or the
    // head's) reads it instead of the pre-pool output and the pooled one
    bool pool_code_layer(int i) const {
        const Layer& l = L[i];
        if (!l.pool || l.flatten || l.pc == nullptr || i + 1 >= (int)L.size()) return false;
        const bool fwd = (l.col && conv0_ok(l.g)) || rowconv_layer(i);
        const bool bwd = rowconv_dgrad_layer(i + 1) || head_dgrad_ok(i + 1);
        return fwd && bwd;
    }
    // the classifier head (a 1x1 conv over 1x1 maps, at most 64 outputs) on the row kernel's
    // W = 1 path: forward, and its input gradient into the previous layer's relu / 2x2 pool
    bool head_layer(int i) const {
        const Layer& l = L[i];
        const ConvGeom& g = l.g;
        return use_rowconv && !l.col && l.bar != nullptr && g.kh == 1 && g.kw == 1 && g.h == 1 && g.w == 1 &&
               g.c_out <= 64 && !l.pool && !l.flatten;
    }
    bool head_dgrad_ok(int i) const {
        if (i == 0 || !head_layer(i)) return false;
        const Layer& pv = L[i - 1];
        if (pv.flatten || pv.col || pv.g.cop != L[i].g.cip) return false;
        return pv.pool ? (pv.ph == 1 && pv.pw == 1 && pv.g.oh == 2 && pv.g.ow == 2) : (pv.g.oh == 1 && pv.g.ow == 1);
    }
    // the int8 weight gradient of the last step kept for niti_model_get (which = 1)
    bool keep_grads = true;
    bool g8_written = false;  // the last step stored the int8 weight gradients (tap(layer, 1))
    // IHWO16 weights of the layers whose input gradient ran on the row kernel (the SGD kernel
    // skips them there) -- rebuilt when the GEMM input gradient takes over again
    int refresh_wt(hipStream_t st) {
        for (Layer& l : L)
            if (l.rcd && ohwi16_to_ihwo16(l.w, l.g.c_out, l.g.c_in, l.g.kh * l.g.kw, l.g.cip, l.g.cop, l.wT, st) !=
                             hipSuccess)
                return NITI_NO_EXECUTION;
        return NITI_NO_ERROR;
    }
    // refresh every rowconv layer's fragment-major weights from w (after set_weight / NITI_SGD)
    int refresh_wf(hipStream_t st) {
        for (Layer& l : L) {
            if (l.rc && weights_to_wf(l.w, l.g.c_out, l.g.c_in, l.g.cip, false, l.wf, st) != hipSuccess)
                return NITI_NO_EXECUTION;
            if (l.rcd && weights_to_wf(l.w, l.g.c_out, l.g.c_in, l.g.cip, true, l.wft, st) != hipSuccess)
                return NITI_NO_EXECUTION;
        }
        return NITI_NO_ERROR;
    }
    // jobs per P16 conversion launch: P16_MAX_JOBS, lowered only by niti_diag_p16_jobs_cap (tests
    // reach the more-than-one-launch branches with a small net)
    static int p16_jobs_cap() { return std::min(std::max(g_p16_jobs_cap, 1), P16_MAX_JOBS); }
    // every P16 input copy of the backward pass as one job list (false: more than one launch holds)
    bool p16_input_jobs(P16Conv* jobs, int* n) {
        *n = 0;
        for (int j = 0; j < (int)L.size(); ++j)
            if (wgrad_p16_splits(j)) {
                if (*n == p16_jobs_cap()) return false;
                const ConvGeom& g = L[j].g;
                jobs[(*n)++] = P16Conv{L[j].in, (int64_t)g.n * g.h * g.w, g.cip, xp16[j]};
            }
        return true;
    }
    int convert_p16_inputs(hipStream_t st) {
        P16Conv jobs[P16_MAX_JOBS];
        int n = 0;
        for (int j = 0; j < (int)L.size(); ++j)
            if (wgrad_p16_splits(j)) {
                const ConvGeom& g = L[j].g;
                jobs[n++] = P16Conv{L[j].in, (int64_t)g.n * g.h * g.w, g.cip, xp16[j]};
                xp16_valid[j] = 1;
                if (n == p16_jobs_cap() || j + 1 == (int)L.size()) {
                    if (nhwc16_to_p16_many(jobs, n, st) != hipSuccess) return NITI_NO_EXECUTION;
                    n = 0;
                }
            }
        if (n > 0 && nhwc16_to_p16_many(jobs, n, st) != hipSuccess) return NITI_NO_EXECUTION;
        return NITI_NO_ERROR;
    }
    // the K split the P16 weight gradient of layer i runs with, 0 when layer i runs on the NHWC16
    // kernels (a plan override of another tile, or a geometry the P16 kernel does not take)
    int wgrad_p16_splits(int i) const {
        const ConvGeom& g = L[i].g;
        if (!conv_wgrad_p16_ok(g)) return 0;
        PlanChoice c;
        if (plan_override_lookup(conv_plan_key(PLAN_WGRAD, g), &c)) return c.bm == PLAN_P16_TILE ? c.splits : 0;
        return conv_wgrad_p16_splits(g);
    }
    // the probed launch's own begin / end events and span slot (P16 weight gradient)
    void probe_launch(int layer, int phase, hipEvent_t* b, hipEvent_t* e, unsigned long long** sp) {
        *b = *e = nullptr;
        *sp = nullptr;
        if (layer != probe_layer || phase != probe_phase || probe_paused || tuning || capturing) return;
        if (probe_count < (int)ev0.size()) {
            *b = ev0[probe_count];
            *e = ev1[probe_count];
            ++probe_count;
        }
        if (span != nullptr && span_count < span_cap) *sp = span + 2 * SPAN_MAX_BLOCKS * span_count++;
    }
    // The weight gradient of layer i and the input gradient of layer i both read dy_i and
    // nothing else the other writes, so the weight gradients run on a second stream, each
    // released by an event after its dy is produced, and overlap the input-gradient chain
    // (the launches are small enough that one alone leaves most of the chip idle).  The SGD
    // launch joins the two streams.
    bool overlap = true;
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> ev_dy;
    hipEvent_t ev_side = nullptr;
    uint32_t* amax = nullptr;  // 3 ranges per layer (forward, input gradient, weight gradient)
    size_t amax_bytes = 0;
    uint32_t* rng(int layer, int which) { return amax + (size_t)(3 * layer + which) * MAX_WORDS; }
    // data parallel (see "collectives" above): ranges on the step stream through `coll`,
    // gradient-bucket SUMs on the comm stream `cst` through `coll_grad`.  Attached at any world
    // size (a world of 1 runs every collective call site on one GPU).
    std::unique_ptr<Collective> coll, coll_grad;
    int world = 1, rank = 0, exact = 1;
    bool dp() const { return coll != nullptr && coll_grad != nullptr && !tuning; }
    hipStream_t cst = nullptr;
    // the gradient SUMs share the range communicator (ncclCommSplit unavailable): they then run on
    // the weight-gradient stream itself, keeping that one communicator in program order
    bool shared_comm = false;
    std::vector<hipEvent_t> ev_bucket;  // per layer: the bucket closed after this layer's weight gradient
    hipEvent_t ev_grads = nullptr;      // every bucket summed and ranged (the NITI_SGD join)
    size_t bucket_min_bytes = grad_bucket_bytes();
    // the bucket a layer's gradient SUM rides in: layers (backward order) accumulate until the
    // bucket holds bucket_min_bytes; closes_bucket[i] marks the layer whose weight gradient
    // completes one (its first layer in memory order is bucket_lo[i])
    std::vector<int> bucket_lo;
    std::vector<char> closes_bucket;
    void plan_buckets() {
        const int nl = (int)L.size();
        bucket_lo.assign(nl, 0);
        closes_bucket.assign(nl, 0);
        size_t acc = 0;
        int hi = nl - 1;
        for (int i = nl - 1; i >= 0; --i) {
            acc += (size_t)L[i].w_elems() * 4;
            if (acc >= bucket_min_bytes || i == 0) {
                closes_bucket[i] = 1;
                for (int j = i; j <= hi; ++j) bucket_lo[j] = i;
                acc = 0;
                hi = i - 1;
            }
        }
    }
    int ensure_comm_stream() {
        if (cst) return NITI_NO_ERROR;
        if (hipStreamCreateWithFlags(&cst, hipStreamNonBlocking) != hipSuccess) return NITI_NO_EXECUTION;
        constexpr unsigned kFlags = hipEventDisableTiming | hipEventReleaseToDevice;
        ev_bucket.assign(L.size(), nullptr);
        for (auto& e : ev_bucket)
            if (hipEventCreateWithFlags(&e, kFlags) != hipSuccess) return NITI_NO_EXECUTION;
        if (hipEventCreateWithFlags(&ev_grads, kFlags) != hipSuccess) return NITI_NO_EXECUTION;
        plan_buckets();
        return NITI_NO_ERROR;
    }
    int sum_bucket(int hi_layer, hipStream_t wst);
    // input quantiser statistics {S1, S2, xmax, 255 - xmin} (niti_quant.hip)
    unsigned long long* qstats = nullptr;
    unsigned long long* qslots = nullptr;  // per-block partial statistics (IMAGE_STATS_SLOTS x 4)
    int8_t* x0n = nullptr;                 // the int8 input NCHW (written by the fused input pass)
    bool x0_nchw_valid = false;
    // Optional hipGraph replay of the single-device step: ~95 launches become one graph launch
    // (or three when a probe splits it around the probed GEMM).  Captured on an internal
    // stream, fenced against the caller's stream with events; re-captured when the captured
    // inputs (input / label pointers, input exponent, probe target) change.  Off by default:
    // on ROCm 7.2 the replayed step measured 0.97 ms against 0.84 ms for direct launches (each
    // graph kernel node ran slower, e.g. the probed GEMM + reduce 43 us vs 33 us).
    bool use_graph = false;
    hipStream_t gstream = nullptr;
    hipEvent_t gin = nullptr, gout = nullptr;
    std::vector<hipGraphExec_t> segs;
    struct Key {
        const void* x = nullptr;
        const void* labels = nullptr;
        int exp_in = 0, pl = -1, pp = -1;
        bool operator==(const Key& o) const {
            return x == o.x && labels == o.labels && exp_in == o.exp_in && pl == o.pl && pp == o.pp;
        }
    } key;
    bool capturing = false;
    hipError_t cap_err = hipSuccess;
    void drop_graph() {
        for (auto e : segs) (void)hipGraphExecDestroy(e);
        segs.clear();
    }
    // close the current capture into a segment and open the next one
    void seg_cut(hipStream_t st) {
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(st, &g);
        hipGraphExec_t ex = nullptr;
        if (e == hipSuccess) e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        if (g) (void)hipGraphDestroy(g);
        if (e == hipSuccess) segs.push_back(ex);
        if (cap_err == hipSuccess) cap_err = e;
        e = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
        if (cap_err == hipSuccess) cap_err = e;
    }
    // kernel probe: HIP events around one GEMM (layer, phase 0 fwd / 1 dgrad / 2 wgrad); in a
    // graph the probe points are segment boundaries and the events go between the launches
    int probe_layer = -1, probe_phase = -1, probe_count = 0;
    std::vector<hipEvent_t> ev0, ev1;
    // kernel-span probe (weight gradient): per launch {min block start, max block end} on the
    // device wall clock, written by the kernel itself (niti_kernels.hpp probe_span_arm)
    unsigned long long* span = nullptr;
    int span_cap = 0, span_count = 0;
    void arm_kernel_events(int layer, int phase) {
        if (layer != probe_layer || phase != probe_phase || probe_paused || tuning || capturing || probe_count >= (int)ev0.size())
            return;
        probe_events_arm(ev0[probe_count], ev1[probe_count]);
        ++probe_count;
    }
    void arm_span(int layer, int phase) {
        if (layer != probe_layer || phase != probe_phase || probe_paused || tuning || capturing || span == nullptr ||
            span_count >= span_cap)
            return;
        probe_span_arm(span + 2 * SPAN_MAX_BLOCKS * span_count++);
    }
    void probe(int layer, int phase, bool begin, hipStream_t st) {
        if (layer != probe_layer || phase != probe_phase || tuning) return;
        if (capturing) {
            seg_cut(st);
            return;
        }
        if (probe_paused) return;
        if (probe_count >= (int)ev0.size()) return;
        if (begin) {
            (void)hipEventRecord(ev0[probe_count], st);
        } else {
            (void)hipEventRecord(ev1[probe_count], st);
            ++probe_count;
        }
    }
    // the end event of a probe that the callee records itself (right after the GEMM launch)
    hipEvent_t probe_end_event(int layer, int phase) {
        if (layer != probe_layer || phase != probe_phase || probe_paused || capturing || tuning || probe_count >= (int)ev0.size())
            return nullptr;
        return ev1[probe_count++];
    }
    void clear_probe() {
        for (auto e : ev0) (void)hipEventDestroy(e);
        for (auto e : ev1) (void)hipEventDestroy(e);
        ev0.clear();
        ev1.clear();
        probe_count = 0;
        probe_layer = probe_phase = -1;
        if (span) (void)hipFree(span);
        span = nullptr;
        span_cap = span_count = 0;
    }

    int build(int arch_, int batch_, int in_hw = 0);
    bool tuning = false;  // autotune in progress: no collectives, no probe
    bool probe_paused = false;  // niti_model_probe_pause: the armed probe skips these launches
    int fwd_layer(int i, hipStream_t st);
    int wgrad_layer(int i, hipStream_t st);
    int dgrad_layer(int i, hipStream_t st);
    // the input gradient of layer i need not write L[i - 1].dy in NHWC16: its weight gradient reads
    // the P16 copy (p16) and its input gradient the C32 copy (next) this same launch writes (layer 0's
    // GEMM weight gradient reads NHWC16).  NITI_DY16=1 keeps the copy (A/B diagnostics).
    // the classifier head's whole chain (forward, loss gradient, weight and input gradient into the
    // previous layer's pool routes) as one launch (niti_head.hip): single device, the head on the
    // row kernel's W = 1 path after a pooled layer whose routes travel as codes (VGG-11)
    bool head_chain_on() const {
        const int h = (int)L.size() - 1;
        if (!head_chain_enabled() || h < 1 || dp() || tuning || probe_layer == h) return false;
        const Layer& l = L[h];
        return head_layer(h) && head_dgrad_ok(h) && L[h - 1].pool && pool_code_layer(h - 1) &&
               head_chain_ok(batch, l.g.cip, l.g.c_out, l.g.cop) && L[h - 1].g.cop == l.g.cip && l.g.kh * l.g.kw == 1;
    }
    bool skip_dy16(int i, const int8_t* next, const int8_t* p16) const {
        static const bool keep = getenv("NITI_DY16") != nullptr && getenv("NITI_DY16")[0] == '1';
        return !keep && i - 1 >= 1 && next != nullptr && p16 != nullptr && wgrad_p16_splits(i - 1) > 0;
    }
    int autotune(hipStream_t st, int reps);
    // grow a split-K workspace (the old one stays owned by ws until the model is destroyed)
    bool ensure_slab(size_t bytes, bool wgrad) {
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
    size_t ws_bytes_for(int op) const { return op == PLAN_WGRAD ? slab_w_bytes : slab_bytes; }
    // layer i's own slab buffer for a deferred GEMM weight-gradient combine is big enough for the
    // plan it runs with (false: its plan does not split K into C-shaped slabs, or not sized)
    bool ensure_wslab(int i) const {
        const Layer& l = L[i];
        const PlanChoice c = conv_plan_query(PLAN_WGRAD, l.g, false, slab_w_bytes);
        if (c.strat != 2 || c.splits < 2 || c.bm == PLAN_P16_TILE) return false;
        return l.wslab_bytes >= conv_wgrad_slab_bytes(l.g, c);  // (GEMM or tap-sharing slabs)
    }
    // size every layer's deferred-combine slab for the current plans, at the head of run() whenever a
    // plan override changed since the last sizing (one device sync, the old buffer freed): no
    // allocation or sync inside the step
    unsigned wslab_epoch = 0;
    int size_wslabs() {
        if (wslab_epoch == plan_override_epoch()) return NITI_NO_ERROR;
        bool synced = false;
        for (Layer& l : L) {
            const PlanChoice c = conv_plan_query(PLAN_WGRAD, l.g, false, slab_w_bytes);
            if (c.strat != 2 || c.splits < 2 || c.bm == PLAN_P16_TILE) continue;
            const size_t need = conv_wgrad_slab_bytes(l.g, c);
            if (l.wslab_bytes >= need) continue;
            if (!synced && hipDeviceSynchronize() != hipSuccess) return NITI_NO_EXECUTION;
            synced = true;
            void* p = ws.replace(l.wslab, need);
            l.wslab = (int32_t*)p;
            l.wslab_bytes = p ? need : 0;
            if (!p) return NITI_OUT_OF_MEMORY;
        }
        wslab_epoch = plan_override_epoch();
        return NITI_NO_ERROR;
    }
    int ensure_streams() {
        if (side) return NITI_NO_ERROR;
        if (hipStreamCreateWithFlags(&side, hipStreamNonBlocking) != hipSuccess) return NITI_NO_EXECUTION;
        // cross-stream hand-offs on one device need a device-scope release only (the default
        // system-scope fence writes back and invalidates the caches: ~7 us per record, measured)
        constexpr unsigned kFlags = hipEventDisableTiming | hipEventReleaseToDevice;
        if (hipEventCreateWithFlags(&ev_side, kFlags) != hipSuccess) return NITI_NO_EXECUTION;
        ev_dy.resize(L.size());
        for (auto& e : ev_dy)
            if (hipEventCreateWithFlags(&e, kFlags) != hipSuccess) return NITI_NO_EXECUTION;
        return NITI_NO_ERROR;
    }
    // x_nchw int8 with exponent exp_in, or (x_nchw == null) uint8 images through the on-device
    // input quantiser (MnistUtils.cpp:83-93)
    int run(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st);
    int step(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st);
    ~Model() {
        clear_probe();
        drop_graph();
        if (cst) (void)hipStreamSynchronize(cst);
        for (auto e : ev_bucket) (void)hipEventDestroy(e);
        if (ev_grads) (void)hipEventDestroy(ev_grads);
        if (gin) (void)hipEventDestroy(gin);
        if (gout) (void)hipEventDestroy(gout);
        if (gstream) (void)hipStreamDestroy(gstream);
        for (auto e : ev_dy) (void)hipEventDestroy(e);
        if (ev_side) (void)hipEventDestroy(ev_side);
        if (side) (void)hipStreamDestroy(side);
        coll_grad.reset();
        coll.reset();
        if (cst) (void)hipStreamDestroy(cst);
    }
};

static void add_conv(Model& m, int ci, int co, int k, int pad, int h, int relu, int pool, int flatten = 0) {
    Layer l;
    l.g.n = m.batch;
    l.g.c_in = ci;
    l.g.h = l.g.w = h;
    l.g.c_out = co;
    l.g.kh = l.g.kw = k;
    l.g.sh = l.g.sw = 1;
    l.g.pt = l.g.pl = l.g.pb = l.g.pr = pad;
    l.g.dh = l.g.dw = 1;
    l.g.finalize();
    l.og = l.g;
    l.relu = relu;
    l.pool = pool;
    l.flatten = flatten;
    if (pool) {
        l.ph = (l.g.oh - 2) / 2 + 1;
        l.pw = (l.g.ow - 2) / 2 + 1;
    }
    m.L.push_back(l);
}

int Model::build(int arch_, int batch_, int in_hw) {
    arch = arch_;
    batch = batch_;
    if (arch == NITI_ARCH_LENET) {  // mnistTrain.cpp:131-181
        in_c = 1;
        in_h = in_w = 28;
        add_conv(*this, 1, 20, 5, 0, 28, 1, 1);
        add_conv(*this, 20, 52, 5, 0, 12, 1, 1, /*flatten=*/1);
        add_conv(*this, 832, 500, 1, 0, 1, 1, 0);
        add_conv(*this, 500, 12, 1, 0, 1, 0, 0);
    } else if (arch == NITI_ARCH_VGG11) {  // VGG-11 for 32x32 inputs, NITI layers (BASELINE cfg 3)
        in_c = 3;
        in_h = in_w = 32;
        add_conv(*this, 3, 64, 3, 1, 32, 1, 1);
        add_conv(*this, 64, 128, 3, 1, 16, 1, 1);
        add_conv(*this, 128, 256, 3, 1, 8, 1, 0);
        add_conv(*this, 256, 256, 3, 1, 8, 1, 1);
        add_conv(*this, 256, 512, 3, 1, 4, 1, 0);
        add_conv(*this, 512, 512, 3, 1, 4, 1, 1);
        add_conv(*this, 512, 512, 3, 1, 2, 1, 0);
        add_conv(*this, 512, 512, 3, 1, 2, 1, 1);
        add_conv(*this, 512, 12, 1, 0, 1, 0, 0);
    } else if (arch == NITI_ARCH_VGG16) {  // VGG-16 (configuration D), NITI layers (BASELINE cfg 4)
        const int r = in_hw > 0 ? in_hw : 224;
        if (r % 32 != 0) return NITI_INVALID_VALUE;
        in_c = 3;
        in_h = in_w = r;
        classes = 1000;
        static const int cfg[13][3] = {{3, 64, 0},    {64, 64, 1},   {64, 128, 0},  {128, 128, 1}, {128, 256, 0},
                                       {256, 256, 0}, {256, 256, 1}, {256, 512, 0}, {512, 512, 0}, {512, 512, 1},
                                       {512, 512, 0}, {512, 512, 0}, {512, 512, 1}};
        int h = r;
        for (int i = 0; i < 13; ++i) {
            add_conv(*this, cfg[i][0], cfg[i][1], 3, 1, h, 1, cfg[i][2], /*flatten=*/i == 12);
            if (cfg[i][2]) h /= 2;
        }
        add_conv(*this, 512 * h * h, 4096, 1, 0, 1, 1, 0);
        add_conv(*this, 4096, 4096, 1, 0, 1, 1, 0);
        add_conv(*this, 4096, 1000, 1, 0, 1, 0, 0);
    } else {
        return NITI_NOT_SUPPORT;
    }
    const int n = batch;
    {
        Layer& f = L[0];
        const ConvGeom o = f.og;
        if (o.c_in * o.kh * o.kw <= 32 && o.dh == 1 && o.dw == 1) {
            f.col = 1;
            ConvGeom c{};
            c.n = o.n;
            c.c_in = 32;
            c.h = o.oh;
            c.w = o.ow;
            c.c_out = o.c_out;
            c.kh = c.kw = 1;
            c.sh = c.sw = 1;
            c.dh = c.dw = 1;
            c.finalize();
            f.g = c;
            f.xcol = (int8_t*)ws.alloc((size_t)n * o.oh * o.ow * 32);
            if (!f.xcol) return NITI_OUT_OF_MEMORY;
        }
    }
    x0 = (int8_t*)ws.alloc((size_t)n * in_h * in_w * round_up(in_c, 16));
    exp0 = (int8_t*)ws.alloc(16);
    size_t acc_elems = 0;
    const int nl = (int)L.size();
    // every layer's int32 weight gradient in one contiguous bucket: data parallel, one SUM
    // all-reduce covers the whole step's gradients
    size_t grad_elems = 0;
    for (const Layer& l : L) grad_elems += (size_t)l.w_elems();
    grad_bucket = (int32_t*)ws.alloc(grad_elems * 4);
    if (!grad_bucket) return NITI_OUT_OF_MEMORY;
    grad_bucket_elems = grad_elems;
    size_t grad_off = 0;
    xp16.assign(nl, nullptr);
    xp16_valid.assign(nl, 0);
    dp16.assign(nl, nullptr);
    dp16_valid.assign(nl, 0);
    xc32_valid.assign(nl, 0);
    dyc32_valid.assign(nl, 0);
    dy16_valid.assign(nl, 1);
    rc_err = (uint32_t*)ws.alloc(64);
    if (!rc_err || hipMemset(rc_err, 0, 64) != hipSuccess) return NITI_OUT_OF_MEMORY;
    for (int i = 0; i < nl; ++i) {
        Layer& l = L[i];
        const ConvGeom& g = l.g;
        const size_t out_px = (size_t)n * g.oh * g.ow;
        l.w = (int8_t*)ws.alloc(l.w_elems());
        l.ws_dev = (int8_t*)ws.alloc(16);
        l.wT = (int8_t*)ws.alloc((size_t)g.c_in * g.kh * g.kw * g.cop);
        l.r = (int8_t*)ws.alloc(out_px * g.cop);
        if (l.pool) {
            l.p = (int8_t*)ws.alloc((size_t)n * l.ph * l.pw * g.cop);
            l.dtmp = (int8_t*)ws.alloc((size_t)n * l.ph * l.pw * g.cop);
            if (!l.flatten && l.ph * 2 == g.oh && l.pw * 2 == g.ow) {
                l.pc = (int8_t*)ws.alloc((size_t)n * l.ph * l.pw * g.cop);
                if (!l.pc) return NITI_OUT_OF_MEMORY;
            }
        }
        if (l.flatten) {
            const int fc = g.c_out * l.ph * l.pw;
            l.flat = (int8_t*)ws.alloc((size_t)n * round_up(fc, 16));
            l.dflat = (int8_t*)ws.alloc((size_t)n * round_up(fc, 16));
        }
        l.dy = (int8_t*)ws.alloc(out_px * g.cop);
        l.dwacc = grad_bucket + grad_off;
        grad_off += (size_t)l.w_elems();
        l.g8 = (int8_t*)ws.alloc(l.w_elems());
        l.exp = (int8_t*)ws.alloc(16);
        l.gspec = (uint32_t*)ws.alloc(2 * GEMM_SPEC_SLOT_WORDS * 4);
        if (!l.w || !l.ws_dev || !l.wT || !l.r || !l.dy || !l.dwacc || !l.g8 || !l.exp || !l.gspec)
            return NITI_OUT_OF_MEMORY;
        if (hipMemset(l.gspec, 0, 2 * GEMM_SPEC_SLOT_WORDS * 4) != hipSuccess) return NITI_NO_EXECUTION;
        if (hipMemset(l.w, 0, l.w_elems()) != hipSuccess) return NITI_NO_EXECUTION;
        if (hipMemset(l.ws_dev, 0, 16) != hipSuccess) return NITI_NO_EXECUTION;
        acc_elems = std::max(acc_elems, out_px * g.cop);
        acc_elems = std::max(acc_elems, (size_t)n * g.h * g.w * g.cip);
        slab_bytes = std::max(slab_bytes, conv_fwd_workspace(g));
        slab_bytes = std::max(slab_bytes, conv_dgrad_workspace(g));
        slab_w_bytes = std::max(slab_w_bytes, conv_wgrad_workspace(g));
        // grid-barrier state of every layer: the row kernels' fused launches and speculation slots,
        // the head's, or the GEMM path's fused-rescale launches (STRAT_FUSED)
        l.bar = (uint32_t*)ws.alloc(ROWCONV_BAR_WORDS * 4);
        if (!l.bar || hipMemset(l.bar, 0, ROWCONV_BAR_WORDS * 4) != hipSuccess) return NITI_OUT_OF_MEMORY;
        if (!l.col && rowconv_ok(g)) {
            l.rc = 1;
            l.wf = (int8_t*)ws.alloc(rowconv_wf_bytes(g.c_out, g.c_in));
            l.xc32 = (int8_t*)ws.alloc((size_t)n * round_up(g.c_in, 32) * g.h * g.w);
            if (!l.wf || !l.xc32) return NITI_OUT_OF_MEMORY;
            if (hipMemset(l.wf, 0, rowconv_wf_bytes(g.c_out, g.c_in)) != hipSuccess)
                return NITI_NO_EXECUTION;
            rc_acc_size = std::max(rc_acc_size, rowconv_acc_bytes(g, false));
            // the input gradient too, where the previous layer's output (pooled 2x2 or not) is
            // this layer's input as is
            const Layer* pv = i > 0 ? &L[i - 1] : nullptr;
            const bool pv_ok = pv != nullptr && !pv->flatten && pv->g.cop == g.cip &&
                               (pv->pool ? (pv->ph == g.h && pv->pw == g.w && pv->g.oh == 2 * g.h && pv->g.ow == 2 * g.w)
                                         : (pv->g.oh == g.h && pv->g.ow == g.w));
            if (pv_ok && rowconv_dgrad_geom(g, &l.dg)) {
                l.rcd = 1;
                rc_acc_size = std::max(rc_acc_size, rowconv_acc_bytes(l.dg, true));
                l.wft = (int8_t*)ws.alloc(rowconv_wf_bytes(g.c_in, g.c_out));
                l.dyc32 = (int8_t*)ws.alloc(out_px * round_up(g.c_out, 32));
                if (!l.wft || !l.dyc32) return NITI_OUT_OF_MEMORY;
                if (hipMemset(l.wft, 0, rowconv_wf_bytes(g.c_in, g.c_out)) != hipSuccess) return NITI_NO_EXECUTION;
            }
        }
        if (conv_wgrad_p16_ok(g)) {
            slab_w_bytes = std::max(slab_w_bytes, conv_wgrad_p16_workspace(g, 8));
            xp16[i] = (int8_t*)ws.alloc((size_t)n * g.h * g.w * g.cip);
            l.slab16_bytes = conv_wgrad_p16_workspace(g, 8);
            l.slab16 = l.slab16_bytes ? (int32_t*)ws.alloc(l.slab16_bytes) : nullptr;
            if (l.slab16_bytes && !l.slab16) return NITI_OUT_OF_MEMORY;
            dp16[i] = (int8_t*)ws.alloc(out_px * g.cop);
            if (!xp16[i] || !dp16[i]) return NITI_OUT_OF_MEMORY;
        }
        // layer input / its C alignment with the previous output
        if (i == 0) {
            l.in = l.col ? l.xcol : x0;
        } else {
            const Layer& pr = L[i - 1];
            l.in = pr.flatten ? pr.flat : (pr.pool ? pr.p : pr.r);
        }
    }
    acc = (int32_t*)ws.alloc(acc_elems * 4);
    qstats = (unsigned long long*)ws.alloc(64);
    qslots = (unsigned long long*)ws.alloc((size_t)IMAGE_STATS_SLOTS * 4 * sizeof(unsigned long long));
    x0n = (int8_t*)ws.alloc((size_t)n * in_c * in_h * in_w);
    if (!qstats || !qslots || !x0n) return NITI_OUT_OF_MEMORY;
    if (slab_bytes) {
        slab = ws.alloc(slab_bytes);
        if (!slab) return NITI_OUT_OF_MEMORY;
    }
    if (slab_w_bytes) {
        slab_w = ws.alloc(slab_w_bytes);
        if (!slab_w) return NITI_OUT_OF_MEMORY;
    }
    if (rc_acc_size) {
        rc_acc = (int32_t*)ws.alloc(rc_acc_size);
        if (!rc_acc) return NITI_OUT_OF_MEMORY;
    }
    for (int i = 0; i < nl; ++i) {  // the GEMM-path phases that may run the speculative pair
        const Layer& l = L[i];
        if (!(l.col && conv0_ok(l.g)) && !l.rc) gspec_alt_bytes = std::max(gspec_alt_bytes, conv_fwd_spec_alt_bytes(l.g));
        if (i > 0 && !l.rcd) gspec_alt_bytes = std::max(gspec_alt_bytes, conv_dgrad_spec_alt_bytes(l.g));
    }
    if (gspec_alt_bytes && !(gspec_alt = (int8_t*)ws.alloc(gspec_alt_bytes))) return NITI_OUT_OF_MEMORY;
    amax_bytes = (size_t)3 * nl * MAX_BYTES;
    amax = (uint32_t*)ws.alloc(amax_bytes);
    if (!x0 || !exp0 || !acc || !amax) return NITI_OUT_OF_MEMORY;
    if (hipMemset(x0, 0, (size_t)n * in_h * in_w * round_up(in_c, 16)) != hipSuccess) return NITI_NO_EXECUTION;
    return hipDeviceSynchronize() == hipSuccess ? NITI_NO_ERROR : NITI_NO_EXECUTION;
}

#define MTRY(expr)                                             \
    do {                                                       \
        if ((expr) != hipSuccess) return NITI_NO_EXECUTION;    \
    } while (0)
#define CTRY(expr)                                             \
    do {                                                       \
        if ((expr) != hipSuccess) return NITI_NO_EXECUTION;    \
    } while (0)

int Model::step(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st) {
    if (!use_graph || coll != nullptr) return run(x_nchw, exp_in, images, labels, st);
    Key k;
    k.x = x_nchw ? (const void*)x_nchw : (const void*)images;
    k.labels = labels;
    k.exp_in = exp_in;
    k.pl = probe_layer;
    k.pp = probe_phase;
    if (segs.empty() || !(k == key)) {
        drop_graph();
        if (!gstream) {
            MTRY(hipStreamCreateWithFlags(&gstream, hipStreamNonBlocking));
            MTRY(hipEventCreateWithFlags(&gin, hipEventDisableTiming));
            MTRY(hipEventCreateWithFlags(&gout, hipEventDisableTiming));
        }
        MTRY(hipStreamBeginCapture(gstream, hipStreamCaptureModeThreadLocal));
        capturing = true;
        cap_err = hipSuccess;
        const int rc = run(x_nchw, exp_in, images, labels, gstream);
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(gstream, &g);
        capturing = false;
        hipGraphExec_t ex = nullptr;
        if (e == hipSuccess && rc == NITI_NO_ERROR) e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        if (g) (void)hipGraphDestroy(g);
        if (e == hipSuccess && rc == NITI_NO_ERROR) segs.push_back(ex);
        if (rc != NITI_NO_ERROR || e != hipSuccess || cap_err != hipSuccess || (segs.size() != 1 && segs.size() != 3)) {
            drop_graph();
            use_graph = false;  // fall back to direct launches for this model
            (void)hipGetLastError();
            return run(x_nchw, exp_in, images, labels, st);
        }
        key = k;
    }
    MTRY(hipEventRecord(gin, st));
    MTRY(hipStreamWaitEvent(gstream, gin, 0));
    const bool probing = segs.size() == 3 && !probe_paused && probe_count < (int)ev0.size();
    for (size_t j = 0; j < segs.size(); ++j) {
        if (probing && j == 1) MTRY(hipEventRecord(ev0[probe_count], gstream));
        if (probing && j == 2) MTRY(hipEventRecord(ev1[probe_count++], gstream));
        MTRY(hipGraphLaunch(segs[j], gstream));
    }
    MTRY(hipEventRecord(gout, gstream));
    MTRY(hipStreamWaitEvent(st, gout, 0));
    return NITI_NO_ERROR;
}

// One layer's forward: GEMM range pass -> [all-reduce MAX] -> requantise (+relu, fused pool
// when the requant is a separate pass) -> pool / flatten.
int Model::fwd_layer(int i, hipStream_t st) {
    const int n = batch;
    const bool dp = this->dp();
    Layer& l = L[i];
    const ConvGeom& g = l.g;
    probe(i, 0, true, st);
    l.r_written = true;
    if (l.col && conv0_ok(g) && !l.flatten) {
        // first layer on its im2col copy: range pass, [all-reduce MAX], requant + relu + pool pass
        ActOut o;
        const bool code = pool_code_layer(i);
        l.r_written = keep_grads || !code;
        o.out = l.r_written ? l.r : nullptr;
        o.relu = l.relu;
        o.exp_in = exp0;
        o.wscale = l.ws_dev;
        o.exp_out = l.exp;
        o.pool.pool_out = l.pool ? l.p : nullptr;
        // the (pooled) output also as the next layer's C32 input when it runs on the row kernel
        const bool next_c32 = i + 1 < (int)L.size() && rowconv_layer(i + 1) && !rowconv_nhwc_pref(L[i + 1].g);
        if (!conv0_ranged) MTRY(conv0_fwd(g, l.in, l.w, rng(i, 0), o, 0, st));
        conv0_ranged = false;
        if (dp && exact) CTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
        MTRY(conv0_fwd(g, l.in, l.w, rng(i, 0), o, 1, st, next_c32 && l.pool ? L[i + 1].xc32 : nullptr,
                       next_c32 && !l.pool ? L[i + 1].xc32 : nullptr, code ? l.pc : nullptr));
        if (next_c32) xc32_valid[i + 1] = 1;
        probe(i, 0, false, st);
        return NITI_NO_ERROR;
    }
    if (head_layer(i)) {
        // the classifier head on the row kernel (W = 1): one fused launch, or range + requantise
        RowConvOut o;
        o.out = l.r;
        o.exp_in = i == 0 ? exp0 : L[i - 1].exp;
        o.wscale = l.ws_dev;
        o.exp_out = l.exp;
        o.relu = l.relu;
        const int K = g.c_in, rows = g.c_out;
        if (!dp && !capturing && rowconv_fc_ok(n, K, rows, true)) {
            MTRY(rowconv_fc(n, K, rows, l.in, g.cip, l.w, g.cip, o, 0, rng(i, 0), l.bar, ++l.epoch, rc_err, st));
        } else if (rowconv_spec2_on()) {  // the speculative pair: one GEMM pass while the bit width holds
            MTRY(rowconv_fc(n, K, rows, l.in, g.cip, l.w, g.cip, o, RC_SPEC_A, rng(i, 0), l.bar, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fc(n, K, rows, l.in, g.cip, l.w, g.cip, o, RC_SPEC_B, rng(i, 0), l.bar, 0, nullptr, st));
        } else {
            MTRY(rowconv_fc(n, K, rows, l.in, g.cip, l.w, g.cip, o, 1, rng(i, 0), nullptr, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fc(n, K, rows, l.in, g.cip, l.w, g.cip, o, 2, rng(i, 0), nullptr, 0, nullptr, st));
        }
        probe(i, 0, false, st);
        return NITI_NO_ERROR;
    }
    if (rowconv_layer(i)) {
        // register-fed forward, rescale fused: one launch with an in-kernel grid barrier (single
        // device, every workgroup resident, not inside a graph capture), else a range launch,
        // [all-reduce MAX], and a recompute-and-requantise launch
        // a row-segment layer reads its NHWC16 input in place; the others their C32 copy
        const bool xn = rowconv_nhwc_pref(g);
        if (!xn && !xc32_valid[i]) {
            MTRY(nhwc16_to_c32(l.in, n, g.h * g.w, g.cip, g.c_in, l.xc32, st));
            xc32_valid[i] = 1;
        }
        const int8_t* xin = xn ? l.in : l.xc32;
        RowConvOut o;
        o.x_nhwc = xn ? 1 : 0;
        const bool code = pool_code_layer(i);
        l.r_written = keep_grads || !code;
        o.out = l.r_written ? l.r : nullptr;
        o.pool_out = l.pool ? l.p : nullptr;
        o.pool_code_out = code ? l.pc : nullptr;
        const bool feeds_next = i + 1 < (int)L.size() && rowconv_layer(i + 1) && !l.flatten &&
                                !rowconv_nhwc_pref(L[i + 1].g);
        o.next = feeds_next ? L[i + 1].xc32 : nullptr;
        o.exp_in = i == 0 ? exp0 : L[i - 1].exp;
        o.wscale = l.ws_dev;
        o.exp_out = l.exp;
        o.relu = l.relu;
        if (!dp && !capturing && rowconv_fused_ok(g)) {
            MTRY(rowconv_fwd(g, xin, l.wf, o, 0, rng(i, 0), l.bar, ++l.epoch, rc_err, st));
        } else if (rowconv_spec2_on()) {  // the speculative pair: one GEMM pass while the bit width holds
            o.acc_store = rowconv_acc_bytes(g, false) ? rc_acc : nullptr;  // its store mode after a change
            MTRY(rowconv_fwd(g, xin, l.wf, o, RC_SPEC_A, rng(i, 0), l.bar, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fwd(g, xin, l.wf, o, RC_SPEC_B, rng(i, 0), l.bar, 0, nullptr, st));
        } else {
            o.acc_store = rowconv_acc_bytes(g, false) ? rc_acc : nullptr;  // else the requantise launch recomputes
            MTRY(rowconv_fwd(g, xin, l.wf, o, 1, rng(i, 0), nullptr, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fwd(g, xin, l.wf, o, 2, rng(i, 0), nullptr, 0, nullptr, st));
        }
        if (feeds_next) xc32_valid[i + 1] = 1;
        probe(i, 0, false, st);
        if (l.flatten) {
            const int fc = g.c_out * l.ph * l.pw, ld = round_up(fc, 16);
            MTRY(launch_map((int64_t)n * ld, FlattenFwd{l.p, l.ph * l.pw, g.c_out, g.cop, ld, l.flat}, st));
        }
        return NITI_NO_ERROR;
    }
    ActOut o;
    o.out = l.r;
    o.relu = l.relu;
    o.exp_in = i == 0 ? exp0 : L[i - 1].exp;
    o.wscale = l.ws_dev;
    o.exp_out = l.exp;
    const bool spec = conv_fwd_spec_ok(g);
    // the 2x2 pool rides along the separate requant pass when there is one
    const bool fuse_pool = !spec && l.pool && g.oh % 2 == 0 && g.ow % 2 == 0 && conv_fwd_phase2_separate(g, slab_bytes);
    if (fuse_pool) {
        o.pool.pool_out = l.p;
        o.pool.H = g.oh;
        o.pool.W = g.ow;
    }
    hipError_t fe = hipErrorNotSupported;
    if (!dp && !capturing && !fuse_pool) {  // one launch with the rescale fused (plan strategy 4)
        fe = conv_fwd_fused(g, l.in, l.w, o, FusedBar{l.bar, l.epoch + 1, rc_err}, st);
        if (fe != hipErrorNotSupported) {
            ++l.epoch;
            MTRY(fe);
        }
    }
    if (fe != hipErrorNotSupported) {
    } else if (spec) {  // the speculative pair: one GEMM pass while the bit width holds, no int32 tensor
        int8_t* alt = conv_fwd_spec_alt_bytes(g) <= gspec_alt_bytes ? gspec_alt : nullptr;
        MTRY(conv_fwd_spec(g, l.in, l.w, rng(i, 0), o, l.gspec, 0, st, alt));
        if (dp && exact) CTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
        MTRY(conv_fwd_spec(g, l.in, l.w, rng(i, 0), o, l.gspec, 1, st, alt));
    } else {
        MTRY(conv_fwd_phase1(g, l.in, l.w, acc, rng(i, 0), slab, slab_bytes, st));
        if (dp && exact) CTRY(coll->allreduce(rng(i, 0), MAX_WORDS, COLL_MAX_U32, st));
        MTRY(conv_fwd_phase2(g, l.in, l.w, acc, rng(i, 0), o, slab_bytes, st));
    }
    probe(i, 0, false, st);
    if (l.pool && !fuse_pool) MTRY(maxpool_nhwc16(l.r, n, g.oh, g.ow, g.cop, 2, 2, 0, l.p, l.ph, l.pw, st));
    if (l.flatten) {
        const int fc = g.c_out * l.ph * l.pw, ld = round_up(fc, 16);
        MTRY(launch_map((int64_t)n * ld, FlattenFwd{l.p, l.ph * l.pw, g.c_out, g.cop, ld, l.flat}, st));
    }
    return NITI_NO_ERROR;
}

// One layer's weight gradient (the int32 gradient and, single device, its range; data
// parallel, the SUM and the range follow on the comm stream in sum_bucket).
int Model::wgrad_layer(int i, hipStream_t st) {
    const bool dp = this->dp();
    Layer& l = L[i];
    const ConvGeom& g = l.g;
    if (head_layer(i) && g.c_out <= 32 && g.cip % 32 == 0) {
        // the classifier head: one small launch, its range published (single device)
        probe(i, 2, true, st);
        MTRY(head_wgrad(g.n, g.c_out, g.cip, l.in, g.cip, l.dy, g.cop, l.dwacc, dp ? nullptr : rng(i, 2), st));
        probe(i, 2, false, st);
        return NITI_NO_ERROR;
    }
    l.fc_sgd = fc_sgd_layer(i);
    if (l.fc_sgd) {  // its range now; the recompute with the update after the backward pass
        l.defer = SgdJob{};
        MTRY(conv_wgrad_fc_sgd(g, l.in, l.dy, rng(i, 2), SgdJob{}, 0, st));
        return NITI_NO_ERROR;
    }
    if (const int s = wgrad_p16_splits(i)) {
        // P16 weight gradient: x (unless run() converted every input already) and dy to pixel
        // blocks, then the register-fed kernel (+ its split-K reduce); the probe times the kernel
        // launch itself
        if (!xp16_valid[i]) {
            MTRY(nhwc16_to_p16(l.in, (int64_t)g.n * g.h * g.w, g.cip, xp16[i], st));
            xp16_valid[i] = 1;
        }
        if (!dp16_valid[i]) {
            MTRY(nhwc16_to_p16(l.dy, (int64_t)g.n * g.oh * g.ow, g.cop, dp16[i], st));
            dp16_valid[i] = 1;
        }
        hipEvent_t eb, ee;
        unsigned long long* sp;
        probe_launch(i, 2, &eb, &ee, &sp);
        // single device: the split-K combine (+ range) runs with every other layer's in one launch
        // ahead of NITI_SGD, over this layer's own slabs (the shared workspace is reused by the
        // next layer)
        const bool defer = defer_combine() && s > 1 && l.slab16 != nullptr &&
                           conv_wgrad_p16_workspace(g, s) <= l.slab16_bytes;
        l.defer = SgdJob{};
        MTRY(conv_wgrad_p16(g, xp16[i], dp16[i], l.dwacc, dp ? nullptr : rng(i, 2), defer ? l.slab16 : slab_w,
                            defer ? l.slab16_bytes : slab_w_bytes, s, st, eb, ee, sp, defer ? &l.defer : nullptr));
        return NITI_NO_ERROR;
    }
    // the weight-gradient probe is the GEMM launch's own begin / end (its split-K reduce excluded)
    if (capturing)
        probe(i, 2, true, st);
    else
        arm_kernel_events(i, 2);
    arm_span(i, 2);
    // single device: a split-K plan leaves its slabs (this layer's own) to the NITI_SGD launch's
    // combine, which sums them and takes the range (no reduce launch, no int32 round trip)
    const bool defer = defer_combine() && ensure_wslab(i);
    l.defer = SgdJob{};
    MTRY(conv_wgrad_acc(g, l.in, l.dy, l.dwacc, dp ? nullptr : rng(i, 2), defer ? l.wslab : slab_w,
                        defer ? l.wslab_bytes : slab_w_bytes, st, capturing ? probe_end_event(i, 2) : nullptr,
                        defer ? &l.defer : nullptr));
    return NITI_NO_ERROR;
}

// Data parallel: the bucket of layers [bucket_lo[hi], hi] (contiguous in grad_bucket) is complete
// once layer bucket_lo[hi]'s weight gradient is in on `wst`: the comm stream waits for it, SUMs
// the bucket's int32 gradients over the ranks and takes every layer's range of the summed
// gradient (NITI_RangeEstimate over the global batch, NITI_GradientConv_Int8.cpp:274-296), while
// the step stream goes on with the input-gradient chain.
int Model::sum_bucket(int lo, hipStream_t wst) {
    int hi = lo;
    while (hi + 1 < (int)L.size() && bucket_lo[hi + 1] == lo) ++hi;
    MTRY(hipEventRecord(ev_bucket[lo], wst));
    if (shared_comm) {  // one communicator: the SUMs stay in the step's program order
        size_t elems = 0;
        for (int j = lo; j <= hi; ++j) elems += (size_t)L[j].w_elems();
        CTRY(coll_grad->allreduce(L[lo].dwacc, elems, COLL_SUM_I32, wst));
        AbsmaxJob jobs[ABSMAX_MAX_JOBS];
        if (hi - lo + 1 > ABSMAX_MAX_JOBS) return NITI_NOT_SUPPORT;
        for (int j = lo; j <= hi; ++j) jobs[j - lo] = AbsmaxJob{L[j].dwacc, L[j].w_elems(), rng(j, 2), 0};
        MTRY(absmax_many(jobs, hi - lo + 1, wst));
        return NITI_NO_ERROR;
    }
    MTRY(hipStreamWaitEvent(cst, ev_bucket[lo], 0));
    size_t elems = 0;
    for (int j = lo; j <= hi; ++j) elems += (size_t)L[j].w_elems();
    CTRY(coll_grad->allreduce(L[lo].dwacc, elems, COLL_SUM_I32, cst));
    AbsmaxJob jobs[ABSMAX_MAX_JOBS];
    if (hi - lo + 1 > ABSMAX_MAX_JOBS) return NITI_NOT_SUPPORT;
    for (int j = lo; j <= hi; ++j) jobs[j - lo] = AbsmaxJob{L[j].dwacc, L[j].w_elems(), rng(j, 2), 0};
    MTRY(absmax_many(jobs, hi - lo + 1, cst));
    return NITI_NO_ERROR;
}

// Input gradient of layer i (i > 0) into the previous layer's output gradient, with the
// previous layer's pool / flatten / relu gradients.
int Model::dgrad_layer(int i, hipStream_t st) {
    const int n = batch;
    const bool dp = this->dp();
    Layer& l = L[i];
    const ConvGeom& g = l.g;
    Layer& pv = L[i - 1];
    probe(i, 1, true, st);
    if (head_dgrad_ok(i)) {
        // the head's input gradient on the row kernel (W = 1), into the previous layer's relu or
        // 2x2-pool gradient (+ its C32 / P16 copies)
        RowConvOut o;
        o.dgrad_slot = 1;  // (every input-gradient launch: its own speculation hint slot)
        int8_t* next = rowconv_dgrad_layer(i - 1) && !rowconv_nhwc_pref(pv.dg) ? pv.dyc32 : nullptr;
        if (pv.pool) {
            if (pool_code_layer(i - 1)) {
                o.pool_code = pv.pc;
            } else {
                o.pool_x = pv.r;
                o.pool_y = pv.p;
            }
            o.pool_dx = pv.dy;
            o.pool_dx_next = next;
            o.pool_relu = pv.relu;
            o.p16 = fuse_dp16 && wgrad_p16_splits(i - 1) > 0 && (4 * n) % 16 == 0 ? dp16[i - 1] : nullptr;
            o.pool_dx_nhwc = skip_dy16(i, next, o.p16) ? 0 : 1;
        } else {
            o.out = pv.dy;
            o.relu_mask = pv.relu ? pv.r : nullptr;
            next = nullptr;  // a 1x1 previous layer has no row-kernel input gradient
        }
        dy16_valid[i - 1] = !(pv.pool && o.pool_dx_nhwc == 0);
        const int K = g.c_out, rows = g.c_in;
        if (!dp && !capturing && rowconv_fc_ok(n, K, rows, true)) {
            MTRY(rowconv_fc(n, K, rows, l.dy, g.cop, l.wT, g.cop, o, 0, rng(i, 1), l.bar, ++l.epoch, rc_err, st));
        } else if (rowconv_spec2_on()) {
            MTRY(rowconv_fc(n, K, rows, l.dy, g.cop, l.wT, g.cop, o, RC_SPEC_A, rng(i, 1), l.bar, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fc(n, K, rows, l.dy, g.cop, l.wT, g.cop, o, RC_SPEC_B, rng(i, 1), l.bar, 0, nullptr, st));
        } else {
            MTRY(rowconv_fc(n, K, rows, l.dy, g.cop, l.wT, g.cop, o, 1, rng(i, 1), nullptr, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fc(n, K, rows, l.dy, g.cop, l.wT, g.cop, o, 2, rng(i, 1), nullptr, 0, nullptr, st));
        }
        probe(i, 1, false, st);
        dp16_valid[i - 1] = o.p16 != nullptr ? 1 : 0;
        dyc32_valid[i - 1] = next != nullptr ? 1 : 0;
        return NITI_NO_ERROR;
    }
    if (rowconv_dgrad_layer(i)) {
        // register-fed input gradient, its requantisation and the previous layer's relu / pool
        // gradient fused; the previous layer's dy also in C32 when its own input gradient runs here
        const ConvGeom& d = l.dg;
        // a row-segment input gradient reads dy (NHWC16) in place; the others its C32 copy
        const bool xn = rowconv_nhwc_pref(d);
        if (xn && !dy16_valid[i]) MTRY(c32_to_nhwc16(l.dyc32, n, g.oh * g.ow, g.cop, g.c_out, l.dy, st));
        if (!xn && !dyc32_valid[i]) {
            MTRY(nhwc16_to_c32(l.dy, n, g.oh * g.ow, g.cop, g.c_out, l.dyc32, st));
            dyc32_valid[i] = 1;
        }
        const int8_t* dyin = xn ? l.dy : l.dyc32;
        RowConvOut o;
        o.dgrad_slot = 1;  // (every input-gradient launch: its own speculation hint slot)
        o.x_nhwc = xn ? 1 : 0;
        int8_t* next = rowconv_dgrad_layer(i - 1) && !rowconv_nhwc_pref(pv.dg) ? pv.dyc32 : nullptr;
        // the previous layer's P16 dy for its weight gradient, when the launch's pixels make whole
        // 16-pixel blocks; else wgrad_layer converts
        o.p16 = fuse_dp16 && wgrad_p16_splits(i - 1) > 0 && rowconv_p16_ok(l.dg, pv.pool) ? dp16[i - 1] : nullptr;
        const bool skip16 = skip_dy16(i, next, o.p16);
        if (pv.pool) {
            if (pool_code_layer(i - 1)) {
                o.pool_code = pv.pc;
            } else {
                o.pool_x = pv.r;
                o.pool_y = pv.p;
            }
            o.pool_dx = pv.dy;
            o.pool_dx_next = next;
            o.pool_relu = pv.relu;
            o.pool_dx_nhwc = skip16 ? 0 : 1;
        } else {
            o.out = skip16 ? nullptr : pv.dy;
            o.next = next;
            o.relu_mask = pv.relu ? pv.r : nullptr;
        }
        dy16_valid[i - 1] = !skip16;
        if (!dp && !capturing && rowconv_fused_ok(d, true)) {
            MTRY(rowconv_fwd(d, dyin, l.wft, o, 0, rng(i, 1), l.bar, ++l.epoch, rc_err, st));
        } else if (rowconv_spec2_on()) {
            o.acc_store = rowconv_acc_bytes(d, true) ? rc_acc : nullptr;
            MTRY(rowconv_fwd(d, dyin, l.wft, o, RC_SPEC_A, rng(i, 1), l.bar, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fwd(d, dyin, l.wft, o, RC_SPEC_B, rng(i, 1), l.bar, 0, nullptr, st));
        } else {
            o.acc_store = rowconv_acc_bytes(d, true) ? rc_acc : nullptr;
            MTRY(rowconv_fwd(d, dyin, l.wft, o, 1, rng(i, 1), nullptr, 0, nullptr, st));
            if (dp && exact) CTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
            MTRY(rowconv_fwd(d, dyin, l.wft, o, 2, rng(i, 1), nullptr, 0, nullptr, st));
        }
        probe(i, 1, false, st);
        dp16_valid[i - 1] = o.p16 != nullptr ? 1 : 0;
        dyc32_valid[i - 1] = next != nullptr ? 1 : 0;
        return NITI_NO_ERROR;
    }
    dy16_valid[i - 1] = 1;
    const ConvGeom& pg = pv.g;
    const bool spec = conv_dgrad_spec_ok(g);
    // dy of layer i - 1 is rewritten here; its P16 copy comes along where the requant pass can
    // write it (the plain and the fused pool-gradient passes), else wgrad_layer converts it
    int8_t* p16_out = !spec && fuse_dp16 && wgrad_p16_splits(i - 1) > 0 ? dp16[i - 1] : nullptr;
    dp16_valid[i - 1] = 0;
    ActOut o;
    bool fuse = false;
    if (pv.flatten) {
        o.out = pv.dflat;
    } else if (pv.pool) {
        fuse = !spec && pg.oh % 2 == 0 && pg.ow % 2 == 0 && conv_dgrad_phase2_separate(g, slab_bytes);
        if (fuse) {  // pool gradient + relu gradient ride along the requant pass
            o.out = nullptr;
            o.pool.x = pv.r;
            o.pool.y = pv.p;
            o.pool.dx = pv.dy;
            o.pool.relu = pv.relu;
            o.pool.H = pg.oh;
            o.pool.W = pg.ow;
            o.out_p16 = p16_out;
            // the previous layer's row-kernel input gradient reads dy as C32: the same pass writes it
            // (VGG-16 conv2_2 at 112 px: no 205 MB layout launch)
            if (p16_out == nullptr && rowconv_dgrad_layer(i - 1) && !rowconv_nhwc_pref(pv.dg) && pg.cop % 32 == 0)
                o.pool.dx_c32 = pv.dyc32;
        } else {
            o.out = pv.dtmp;
        }
    } else {
        o.relu_mask = pv.relu ? pv.r : nullptr;
        o.out = pv.dy;
        if (conv_dgrad_phase2_separate(g, slab_bytes)) o.out_p16 = p16_out;
    }
    hipError_t fe = hipErrorNotSupported;
    if (!dp && !capturing && !fuse && o.out_p16 == nullptr && o.out != nullptr) {  // one launch, the rescale fused
        fe = conv_dgrad_fused(g, l.dy, l.wT, o, FusedBar{l.bar, l.epoch + 1, rc_err}, st);
        if (fe != hipErrorNotSupported) {
            ++l.epoch;
            MTRY(fe);
        }
    }
    if (fe != hipErrorNotSupported) {
    } else if (spec) {  // the speculative pair (no int32 tensor while the bit width holds)
        int8_t* alt = conv_dgrad_spec_alt_bytes(g) <= gspec_alt_bytes ? gspec_alt : nullptr;
        MTRY(conv_dgrad_spec(g, l.dy, l.wT, rng(i, 1), o, l.gspec + GEMM_SPEC_SLOT_WORDS, 0, st, alt));
        if (dp && exact) CTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
        MTRY(conv_dgrad_spec(g, l.dy, l.wT, rng(i, 1), o, l.gspec + GEMM_SPEC_SLOT_WORDS, 1, st, alt));
    } else {
        MTRY(conv_dgrad_phase1(g, l.dy, l.wT, acc, rng(i, 1), slab, slab_bytes, st));
        if (dp && exact) CTRY(coll->allreduce(rng(i, 1), MAX_WORDS, COLL_MAX_U32, st));
        MTRY(conv_dgrad_phase2(g, l.dy, l.wT, acc, rng(i, 1), o, slab_bytes, st));
    }
    probe(i, 1, false, st);
    if (pv.flatten) {
        const int fc = pg.c_out * pv.ph * pv.pw, ld = round_up(fc, 16);
        MTRY(launch_map((int64_t)n * pv.ph * pv.pw * pg.cop,
                        FlattenBwd{pv.dflat, pv.ph * pv.pw, pg.c_out, pg.cop, ld, pv.dtmp}, st));
        MTRY(maxpool_relu_grad_nhwc16(pv.r, pv.p, pv.dtmp, n, pg.oh, pg.ow, pg.cop, 2, 2, 0, pv.ph, pv.pw, pv.relu,
                                      pv.dy, st));
    } else if (pv.pool && !fuse) {
        MTRY(maxpool_relu_grad_nhwc16(pv.r, pv.p, pv.dtmp, n, pg.oh, pg.ow, pg.cop, 2, 2, 0, pv.ph, pv.pw, pv.relu,
                                      pv.dy, st));
    }
    if (o.out_p16 != nullptr) dp16_valid[i - 1] = 1;
    dyc32_valid[i - 1] = fuse && o.pool.dx_c32 != nullptr ? 1 : 0;
    return NITI_NO_ERROR;
}

// Per-shape plan autotuning.  For every GEMM of the step (layer x {forward, weight gradient,
// input gradient}) time the layer's whole phase -- GEMM(s), split-K reduce, requantisation,
// fused / separate pool -- under each candidate plan on the caller's stream and keep the
// fastest as a plan override (niti_kernels.hpp).  Candidates: the tap-sharing weight-gradient
// kernel where it applies and 6 GEMM tile shapes, each x {store acc,
// recompute (activation GEMMs), split-K 2..64 within the tuning workspace}.  The layer phases
// are idempotent on the buffers left by the previous step, so tuning leaves the weights
// untouched; a fixed default plan (plan_gemm) is the starting point and is kept unless beaten.
int Model::autotune(hipStream_t st, int reps) {
    if (reps < 1) reps = 5;
    const int nl = (int)L.size();
    // split-K room for the candidates
    if (!ensure_slab(size_t(96) << 20, false) || !ensure_slab(size_t(96) << 20, true)) return NITI_OUT_OF_MEMORY;
    drop_graph();
    hipEvent_t ev[4];
    for (auto& e : ev)
        if (hipEventCreate(&e) != hipSuccess) return NITI_NO_EXECUTION;
    tuning = true;
    int rc = NITI_NO_ERROR;
    auto run_op = [&](int i, int op) {
        return op == PLAN_FWD ? fwd_layer(i, st) : op == PLAN_WGRAD ? wgrad_layer(i, st) : dgrad_layer(i, st);
    };
    // min over three event-bracketed batches of `reps` back-to-back runs (no host sync inside)
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
    if (hipMemsetAsync(amax, 0, amax_bytes, st) != hipSuccess) rc = NITI_NO_EXECUTION;
    // NITI_DIAG_TUNE_LOG=1 (diagnostics): every candidate's time on stderr
    const bool log = getenv("NITI_DIAG_TUNE_LOG") != nullptr;
    auto note = [&](int i, int op, const PlanChoice& c, float us) {
        if (log) fprintf(stderr, "tune layer %d op %d plan (%d,%d,%d,%d) %.2f us\n", i, op, c.bm, c.bn, c.splits, c.strat, us);
    };
    static const int tiles[7][2] = {{PLAN_TAPS_TILE, PLAN_TAPS_TILE}, {128, 128}, {128, 64}, {64, 128}, {64, 64},
                                    {256, 128}, {128, 256}};
    static const int split_opts[] = {2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64};
    for (int i = 0; i < nl && rc == NITI_NO_ERROR; ++i) {
        for (int op : {PLAN_FWD, PLAN_WGRAD, PLAN_DGRAD}) {
            if (op == PLAN_DGRAD && i == 0) continue;
            if (op == PLAN_FWD && rowconv_layer(i)) continue;  // no GEMM plan: the register-fed forward
            if (op == PLAN_DGRAD && rowconv_dgrad_layer(i)) continue;
            if ((op == PLAN_FWD && head_layer(i)) || (op == PLAN_DGRAD && head_dgrad_ok(i))) continue;
            if (op == PLAN_WGRAD && head_layer(i) && L[i].g.c_out <= 32 && L[i].g.cip % 32 == 0) continue;
            const ConvGeom& g = L[i].g;
            const PlanKey key = conv_plan_key(op, g);
            const int k_step = conv_plan_k_step(op, g);
            const int steps = (key.K + k_step - 1) / k_step;
            const bool act = op != PLAN_WGRAD;
            plan_override_clear(key);
            const size_t wsb = ws_bytes_for(op);
            PlanChoice best = conv_plan_query(op, g, act, wsb);
            if (op == PLAN_WGRAD && wgrad_p16_splits(i) > 0) {
                best.bm = best.bn = PLAN_P16_TILE;
                best.splits = wgrad_p16_splits(i);
                best.strat = best.splits > 1 ? 2 : 0;
            }
            // P16 candidates are timed without their input conversion: run() converts every
            // layer's input in one launch off the step stream when the backward pass starts
            invalidate_xp16();
            if (op == PLAN_WGRAD && conv_wgrad_p16_ok(g)) {
                if (nhwc16_to_p16(L[i].in, (int64_t)g.n * g.h * g.w, g.cip, xp16[i], st) != hipSuccess) {
                    rc = NITI_NO_EXECUTION;
                    break;
                }
                xp16_valid[i] = 1;
            }
            float best_us = 0.f;
            rc = time_op(i, op, &best_us);
            note(i, op, best, best_us);
            const bool taps = op == PLAN_WGRAD && conv_wgrad_taps_ok(g);
            if (op == PLAN_WGRAD && conv_wgrad_p16_ok(g)) {
                for (int sp : {1, 2, 4, 8}) {
                    if (rc != NITI_NO_ERROR) break;
                    if (conv_wgrad_p16_workspace(g, sp) > slab_w_bytes) continue;
                    PlanChoice cand;
                    cand.bm = cand.bn = PLAN_P16_TILE;
                    cand.splits = sp;
                    cand.strat = sp > 1 ? 2 : 0;
                    plan_override_set(key, cand);
                    float us = 0.f;
                    rc = time_op(i, op, &us);
                    note(i, op, cand, us);
                    if (rc == NITI_NO_ERROR && us < best_us) {
                        best_us = us;
                        best = cand;
                    }
                }
            }
            for (const auto& t : tiles) {
                if (rc != NITI_NO_ERROR) break;
                if (t[0] == PLAN_TAPS_TILE && !taps) continue;
                std::vector<PlanChoice> cands;
                PlanChoice c;
                c.bm = t[0];
                c.bn = t[1];
                c.splits = 1;
                c.strat = 0;
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
                    note(i, op, cand, us);
                    if (rc != NITI_NO_ERROR) break;
                    if (us < best_us) {
                        best_us = us;
                        best = cand;
                    }
                }
            }
            plan_override_set(key, best);
            invalidate_xp16();
            if (rc != NITI_NO_ERROR) break;
        }
    }
    invalidate_xp16();
    tuning = false;
    for (auto e : ev) (void)hipEventDestroy(e);
    if (hipStreamSynchronize(st) != hipSuccess) rc = NITI_NO_EXECUTION;
    return rc;
}

int Model::run(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st) {
    const int n = batch;
    const int nl = (int)L.size();
    const bool dp = this->dp();
    SgdJob jobs[SGD_MAX_JOBS];
    if (nl > SGD_MAX_JOBS) return NITI_NOT_SUPPORT;
    struct InStep {  // weight gradients inside this step may defer their combine (defer_combine)
        bool& f;
        explicit InStep(bool& x) : f(x) { f = true; }
        ~InStep() { f = false; }
    } in_step_guard(in_step);
    for (auto& l : L) l.defer = SgdJob{};
    if (dp) {
        const int rc = ensure_comm_stream();
        if (rc != NITI_NO_ERROR) return rc;
    }
    if (!dp && !capturing && !tuning) {
        const int rc = size_wslabs();  // (plan changes: no allocation or sync inside the step)
        if (rc != NITI_NO_ERROR) return rc;
    }
    invalidate_xp16();  // the forward pass rewrites every layer input
    std::fill(xc32_valid.begin(), xc32_valid.end(), 0);
    std::fill(dyc32_valid.begin(), dyc32_valid.end(), 0);
    // the range words start each step at zero: zeroed by the input statistics launch (uint8
    // images), else here
    if (x_nchw != nullptr || amax_bytes % 16 != 0) MTRY(hipMemsetAsync(amax, 0, amax_bytes, st));
    // the first layer's im2col copy straight from the batch where the fused pass takes the layer
    const ConvGeom& o0 = L[0].og;
    const bool fused_in = L[0].col && input_im2col_ok(o0.c_in, o0.kh, o0.kw) && o0.sh == 1 && o0.sw == 1;
    x0_nchw_valid = fused_in;
    // the first conv's range pass rides in the im2col launch (its rows are in registers there)
    Conv0Range r0;
    if (fused_in && conv0_ok(L[0].g) && !L[0].flatten && L[0].g.cop <= 64) {
        r0.w = L[0].w;
        r0.co = L[0].g.c_out;
        r0.cop = L[0].g.cop;
        r0.amax = rng(0, 0);
    }
    conv0_ranged = r0.w != nullptr;
    if (x_nchw != nullptr) {
        MTRY(hipMemsetAsync(exp0, exp_in, 1, st));
        if (fused_in)
            MTRY(input_im2col(x_nchw, false, n, in_c, in_h, in_w, o0.kh, o0.kw, o0.pt, o0.pl, nullptr, 0, 0, x0n,
                              L[0].xcol, nullptr, st, r0));
        else
            MTRY(nchw_to_nhwc16(x_nchw, n, in_c, in_h * in_w, round_up(in_c, 16), x0, st));
    } else {
        // NITIInt8Train's input quantiser (MnistUtils.cpp:83-93): batch statistics (per-block
        // partials; summed and all-reduced over the ranks in exact mode), then x and its exponent
        // ascale straight into the layer-0 input
        const int64_t px = (int64_t)n * in_c * in_h * in_w;
        int ns = 0;
        MTRY(image_stats_slots(images, px, qslots, &ns, st, amax_bytes % 16 == 0 ? amax : nullptr,
                               amax_bytes % 16 == 0 ? amax_bytes : 0));
        const unsigned long long* slots = qslots;
        if ((dp && exact) || !fused_in) {
            MTRY(stats_finalize(qslots, ns, qstats, st));
            slots = qstats;
            ns = 1;
        }
        if (dp && exact) {
            CTRY(coll->allreduce(qstats, 2, COLL_SUM_U64, st));
            CTRY(coll->allreduce(qstats + 2, 2, COLL_MAX_U64, st));
        }
        const int64_t count = dp && exact ? px * world : px;
        if (fused_in)
            MTRY(input_im2col(images, true, n, in_c, in_h, in_w, o0.kh, o0.kw, o0.pt, o0.pl, slots, ns, count, x0n,
                              L[0].xcol, exp0, st, r0));
        else
            MTRY(image_quantize(images, n, in_c, in_h * in_w, round_up(in_c, 16), qstats, count, x0, exp0, true, st));
    }
    if (L[0].col && !fused_in) MTRY(im2col32(L[0].og, x0, L[0].xcol, st));
    const bool hc = head_chain_on();  // (then the head's forward runs in the chain launch below)
    for (int i = 0; i < nl - (hc ? 1 : 0); ++i) {
        const int rc = fwd_layer(i, st);
        if (rc != NITI_NO_ERROR) return rc;
    }
    // weight gradients on the side stream (not inside a graph capture)
    const bool ov = overlap && !capturing && !(dp && shared_comm);  // one communicator: one stream
    bool p16_done = false;
    {
        Layer& t = L[nl - 1];
        P16Conv jobs[P16_MAX_JOBS];
        int nj = 0;
        if (hc) {
            // the head's forward, loss gradient, weight gradient and input gradient (through the
            // last pool's recorded routes, + its C32 / P16 copies) in one launch; then, on one
            // stream, every P16 input copy in one more
            const bool with_jobs = !ov && p16_input_jobs(jobs, &nj);
            if (!with_jobs) nj = 0;
            Layer& pv = L[nl - 2];
            HeadChain h;
            h.x = t.in;
            h.xld = t.g.cip;
            h.w = t.w;
            h.wT = t.wT;
            h.n = n;
            h.K = t.g.cip;
            h.c_out = t.g.c_out;
            h.cop = t.g.cop;
            h.relu = t.relu;
            h.exp_in = pv.exp;
            h.wscale = t.ws_dev;
            h.exp_out = t.exp;
            h.logits = t.r;
            h.labels = labels;
            h.dy = t.dy;
            h.dw = t.dwacc;
            h.dw_amax = rng(nl - 1, 2);
            h.code = pv.pc;
            int8_t* next = rowconv_dgrad_layer(nl - 2) && !rowconv_nhwc_pref(pv.dg) ? pv.dyc32 : nullptr;
            h.p16 = fuse_dp16 && wgrad_p16_splits(nl - 2) > 0 ? dp16[nl - 2] : nullptr;
            h.pool_dx = skip_dy16(nl - 1, next, h.p16) ? nullptr : pv.dy;
            h.pool_dx_c32 = next;
            MTRY(head_chain(h, st));
            if (with_jobs && nj > 0) {  // (a launch of its own: see niti_head.hip)
                MTRY(nhwc16_to_p16_many(jobs, nj, st));
                for (int j = 0; j < nl; ++j)
                    if (wgrad_p16_splits(j)) xp16_valid[j] = 1;
                p16_done = true;
            }
            t.r_written = true;
            dy16_valid[nl - 1] = 1;
            dy16_valid[nl - 2] = h.pool_dx != nullptr;
            dp16_valid[nl - 2] = h.p16 != nullptr ? 1 : 0;
            dyc32_valid[nl - 2] = next != nullptr ? 1 : 0;
        } else if (!ov && p16_input_jobs(jobs, &nj) && nj > 0) {
            // one stream: the loss gradient and every P16 input copy in one launch (the copies read
            // forward activations only); A/B on one box, 8 alternating 200-step runs: median step
            // 0.395 vs 0.400 ms (profiles/r03_lossp16_ab.txt)
            MTRY(loss_grad_p16(t.r, n, t.g.c_out, t.g.cop, t.exp, labels, t.dy, jobs, nj, st));
            for (int j = 0; j < nl; ++j)
                if (wgrad_p16_splits(j)) xp16_valid[j] = 1;
            p16_done = true;
        } else {
            MTRY(loss_grad(t.r, n, t.g.c_out, t.g.cop, t.exp, labels, t.dy, st));
        }
        dp16_valid[nl - 1] = 0;
    }
    if (ov) {
        const int rc = ensure_streams();
        if (rc != NITI_NO_ERROR) return rc;
    }
    hipStream_t wst = ov ? side : st;
    for (int i = nl - 1; i >= 0; --i) {
        // (an event record leaves a ~6.5 us bubble before the next launch on the step stream;
        // hipStreamWriteValue64 / WaitValue64 run as blit kernels here and cost more)
        if (ov) {  // dy_i is ready on the step stream
            MTRY(hipEventRecord(ev_dy[i], st));
            MTRY(hipStreamWaitEvent(side, ev_dy[i], 0));
        }
        if (i == nl - 1 && !p16_done) {  // the forward outputs are final: every P16 input copy in one go
            const int rc = convert_p16_inputs(wst);
            if (rc != NITI_NO_ERROR) return rc;
        }
        Layer& l = L[i];
        const ConvGeom& g = l.g;
        const bool in_chain = hc && i == nl - 1;  // (the head chain launch did both)
        int rc = in_chain ? NITI_NO_ERROR : wgrad_layer(i, wst);
        // data parallel: a completed gradient bucket goes to the comm stream right away
        if (rc == NITI_NO_ERROR && dp && closes_bucket[i]) rc = sum_bucket(i, wst);
        if (rc == NITI_NO_ERROR && i > 0 && !in_chain) rc = dgrad_layer(i, st);
        if (rc != NITI_NO_ERROR) return rc;
        // NITI_SGD (NITI_SGD.hpp:20-54) for this layer is deferred: every layer's update runs in one
        // launch after the backward pass (the input gradients above read the old weights); the IHWO16
        // transpose feeds only the GEMM input gradient, the int8 gradient only the
        // niti_model_get tap (keep_grads)
        jobs[i] = SgdJob{l.dwacc, rng(i, 2), RULE_WGRAD_BW2, g.c_out, g.c_in, g.kh * g.kw, g.cip, g.cop, l.w,
                         i > 0 && !rowconv_dgrad_layer(i) ? l.wT : nullptr, keep_grads ? l.g8 : nullptr};
        jobs[i].wf = l.rc ? l.wf : nullptr;
        jobs[i].wft = l.rcd ? l.wft : nullptr;
        if (l.defer.slab != nullptr) {  // the combine of this layer's split-K slabs, in the update launch
            jobs[i].slab = l.defer.slab;
            jobs[i].splits = l.defer.splits;
            jobs[i].slab_stride = l.defer.slab_stride;
            jobs[i].slab_n = l.defer.slab_n;
            jobs[i].slab_map = l.defer.slab_map;  // (the tap-sharing kernel's tile-blocked slabs)
            jobs[i].tb_tiles_ci = l.defer.tb_tiles_ci;
            jobs[i].tb_cip4 = l.defer.tb_cip4;
            jobs[i].tb_ld4 = l.defer.tb_ld4;
            jobs[i].tb_m = l.defer.tb_m;
            jobs[i].tb_s = l.defer.tb_s;
        }
    }
    if (dp) {  // every bucket summed and ranged on the comm stream before the update
        MTRY(hipEventRecord(ev_grads, cst));
        MTRY(hipStreamWaitEvent(st, ev_grads, 0));
    } else if (ov) {  // every weight gradient is in before the update
        MTRY(hipEventRecord(ev_side, side));
        MTRY(hipStreamWaitEvent(st, ev_side, 0));
    }
    // the fully connected layers that took the fused form update in their own recompute pass
    SgdJob many[SGD_MAX_JOBS];
    int n_many = 0;
    for (int i = 0; i < nl; ++i)
        if (!L[i].fc_sgd) many[n_many++] = jobs[i];
    MTRY(sgd_update_many(many, n_many, st));  // (+ the deferred combines) also rewrites the fragment-major weight copies
    for (int i = 0; i < nl; ++i)
        if (L[i].fc_sgd) MTRY(conv_wgrad_fc_sgd(L[i].g, L[i].in, L[i].dy, rng(i, 2), jobs[i], 1, st));
    g8_written = keep_grads;
    return NITI_NO_ERROR;
}

}  // namespace niti

// =========================================================================== C ABI (section 3)
struct niti_model {
    niti::Model m;                         // LeNet / VGG-11 / VGG-16
    std::unique_ptr<niti::ResNetModel> r;  // ResNet-18 (niti_resnet_model.hip); m unused then
};

extern "C" {

int niti_model_create(int arch, int batch, niti_model_t* out) { return niti_model_create2(arch, batch, 0, out); }

int niti_model_create2(int arch, int batch, int in_hw, niti_model_t* out) {
    return niti_model_create3(arch, batch, in_hw, 0, out);
}

int niti_model_create3(int arch, int batch, int in_hw, int classes, niti_model_t* out) {
    if (!out || batch <= 0 || in_hw < 0 || classes < 0) return NITI_INVALID_VALUE;
    auto* h = new niti_model();
    int rc;
    if (arch == NITI_ARCH_RESNET18) {
        h->r = std::make_unique<niti::ResNetModel>();
        rc = h->r->build(batch, in_hw, classes);
    } else {
        if (classes != 0) {  // the LeNet / VGG heads are fixed (10 or 1000 classes)
            delete h;
            return NITI_NOT_SUPPORT;
        }
        rc = h->m.build(arch, batch, in_hw);
    }
    if (rc != NITI_NO_ERROR) {
        delete h;
        return rc;
    }
    *out = h;
    return NITI_NO_ERROR;
}

void niti_model_destroy(niti_model_t m) { delete m; }

int niti_model_num_layers(niti_model_t m) { return !m ? 0 : m->r ? (int)m->r->C.size() : (int)m->m.L.size(); }

int niti_model_layer_info(niti_model_t m, int layer, int info[12]) {
    if (m && m->r) {
        if (layer < 0 || layer >= (int)m->r->C.size() || !info) return NITI_INVALID_VALUE;
        const niti::RConv& c = m->r->C[layer];
        const niti::ConvGeom& g = c.og;
        const int v[12] = {g.c_in, g.c_out, g.kh, g.kw, g.h, g.w, g.oh, g.ow, g.pt, g.sh, c.relu, 0};
        memcpy(info, v, sizeof(v));
        return NITI_NO_ERROR;
    }
    if (!m || layer < 0 || layer >= (int)m->m.L.size()) return NITI_INVALID_VALUE;
    const niti::Layer& l = m->m.L[layer];
    const niti::ConvGeom& g = l.og;  // the layer as the network defines it
    const int v[12] = {g.c_in, g.c_out, g.kh, g.kw, g.h, g.w, g.oh, g.ow, g.pt, g.sh, l.relu, l.pool};
    memcpy(info, v, sizeof(v));
    return NITI_NO_ERROR;
}

// the first layer's im2col weights [co][32] (k = (ky * KW + kx) * C_in + c) <-> OIHW
static void col_from_oihw(const niti::ConvGeom& o, const int8_t* w, int8_t* wc) {
    memset(wc, 0, (size_t)o.c_out * 32);
    for (int co = 0; co < o.c_out; ++co)
        for (int c = 0; c < o.c_in; ++c)
            for (int t = 0; t < o.kh * o.kw; ++t) wc[co * 32 + t * o.c_in + c] = w[((size_t)co * o.c_in + c) * o.kh * o.kw + t];
}
static void oihw_from_col(const niti::ConvGeom& o, const int8_t* wc, int8_t* w) {
    for (int co = 0; co < o.c_out; ++co)
        for (int c = 0; c < o.c_in; ++c)
            for (int t = 0; t < o.kh * o.kw; ++t) w[((size_t)co * o.c_in + c) * o.kh * o.kw + t] = wc[co * 32 + t * o.c_in + c];
}

int niti_model_set_weight(niti_model_t m, int layer, const int8_t* w_host, int wscale) {
    if (m && m->r) return m->r->set_weight(layer, w_host, wscale);
    if (!m || layer < 0 || layer >= (int)m->m.L.size() || !w_host) return NITI_INVALID_VALUE;
    niti::Layer& l = m->m.L[layer];
    std::vector<int8_t> colw;
    if (l.col) {  // upload the [co][32] im2col weights as the 1x1 geometry's OIHW
        colw.resize((size_t)l.g.c_out * 32);
        col_from_oihw(l.og, w_host, colw.data());
        w_host = colw.data();
    }
    const size_t n = (size_t)l.g.c_out * l.g.c_in * l.g.kh * l.g.kw;
    int8_t* tmp = nullptr;
    if (hipMalloc(&tmp, n) != hipSuccess) return NITI_OUT_OF_MEMORY;
    int rc = NITI_NO_ERROR;
    if (hipMemcpy(tmp, w_host, n, hipMemcpyHostToDevice) != hipSuccess ||
        niti::oihw_to_ohwi16(tmp, l.g.c_out, l.g.c_in, l.g.kh * l.g.kw, l.g.cip, l.w, nullptr) != hipSuccess ||
        niti::oihw_to_ihwo16(tmp, l.g.c_out, l.g.c_in, l.g.kh * l.g.kw, l.g.cop, l.wT, nullptr) != hipSuccess ||
        hipMemset(l.ws_dev, (int)(int8_t)wscale, 1) != hipSuccess ||
        (l.rc && niti::weights_to_wf(l.w, l.g.c_out, l.g.c_in, l.g.cip, false, l.wf, nullptr) != hipSuccess) ||
        (l.rcd && niti::weights_to_wf(l.w, l.g.c_out, l.g.c_in, l.g.cip, true, l.wft, nullptr) != hipSuccess) ||
        hipDeviceSynchronize() != hipSuccess)
        rc = NITI_NO_EXECUTION;
    l.wscale = (int8_t)wscale;
    (void)hipFree(tmp);
    return rc;
}

int niti_model_get_weight(niti_model_t m, int layer, int8_t* w_host) {
    if (m && m->r) return m->r->get_weight(layer, w_host);
    if (!m || layer < 0 || layer >= (int)m->m.L.size() || !w_host) return NITI_INVALID_VALUE;
    niti::Layer& l = m->m.L[layer];
    const size_t n = (size_t)l.g.c_out * l.g.c_in * l.g.kh * l.g.kw;
    int8_t* tmp = nullptr;
    if (hipDeviceSynchronize() != hipSuccess || hipMalloc(&tmp, n) != hipSuccess) return NITI_OUT_OF_MEMORY;
    int rc = NITI_NO_ERROR;
    std::vector<int8_t> colw(l.col ? n : 0);
    if (niti::ohwi16_to_oihw(l.w, l.g.c_out, l.g.c_in, l.g.kh * l.g.kw, l.g.cip, tmp, nullptr) != hipSuccess ||
        hipMemcpy(l.col ? colw.data() : w_host, tmp, n, hipMemcpyDeviceToHost) != hipSuccess)
        rc = NITI_NO_EXECUTION;
    if (rc == NITI_NO_ERROR && l.col) oihw_from_col(l.og, colw.data(), w_host);
    (void)hipFree(tmp);
    return rc;
}

int niti_model_train_step(niti_model_t m, const int8_t* x_nchw, int exp_in, const int32_t* labels, void* stream) {
    if (m && m->r) return x_nchw && labels ? m->r->step(x_nchw, exp_in, nullptr, labels, (hipStream_t)stream) : NITI_INVALID_VALUE;
    if (!m || !x_nchw || !labels) return NITI_INVALID_VALUE;
    return m->m.step(x_nchw, exp_in, nullptr, labels, (hipStream_t)stream);
}

int niti_model_train_step_images(niti_model_t m, const uint8_t* images_nchw, const int32_t* labels, void* stream) {
    if (m && m->r) return images_nchw && labels ? m->r->step(nullptr, 0, images_nchw, labels, (hipStream_t)stream) : NITI_INVALID_VALUE;
    if (!m || !images_nchw || !labels) return NITI_INVALID_VALUE;
    return m->m.step(nullptr, 0, images_nchw, labels, (hipStream_t)stream);
}

int niti_model_get_input(niti_model_t m, int8_t* x_nchw_host, int* ascale, void* stream) {
    if (m && m->r) return x_nchw_host ? m->r->get_input(x_nchw_host, ascale, (hipStream_t)stream) : NITI_INVALID_VALUE;
    if (!m || !x_nchw_host) return NITI_INVALID_VALUE;
    niti::Model& mm = m->m;
    const int n = mm.batch, hw = mm.in_h * mm.in_w;
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return NITI_NO_EXECUTION;
    const size_t need = (size_t)n * mm.in_c * hw;
    int8_t* tmp = nullptr;
    if (hipMalloc(&tmp, need) != hipSuccess) return NITI_OUT_OF_MEMORY;
    int8_t e = 0;
    hipError_t err = mm.x0_nchw_valid ? hipMemcpy(tmp, mm.x0n, need, hipMemcpyDeviceToDevice)
                                      : niti::nhwc16_to_nchw(mm.x0, n, mm.in_c, hw, niti::round_up(mm.in_c, 16), tmp, nullptr);
    if (err == hipSuccess) err = hipMemcpy(x_nchw_host, tmp, need, hipMemcpyDeviceToHost);
    if (err == hipSuccess) err = hipMemcpy(&e, mm.exp0, 1, hipMemcpyDeviceToHost);
    (void)hipFree(tmp);
    if (ascale) *ascale = e;
    return err == hipSuccess ? NITI_NO_ERROR : NITI_NO_EXECUTION;
}

int niti_model_get_logits(niti_model_t m, int8_t* logits_host, int* exp_out, void* stream) {
    if (m && m->r) return logits_host ? m->r->get_logits(logits_host, exp_out, (hipStream_t)stream) : NITI_INVALID_VALUE;
    if (!m) return NITI_INVALID_VALUE;
    niti::Layer& t = m->m.L.back();
    const int n = m->m.batch;
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return NITI_NO_EXECUTION;
    std::vector<int8_t> buf((size_t)n * t.g.cop);
    int8_t e = 0;
    if (hipMemcpy(buf.data(), t.r, buf.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&e, t.exp, 1, hipMemcpyDeviceToHost) != hipSuccess)
        return NITI_NO_EXECUTION;
    for (int i = 0; i < n; ++i) memcpy(logits_host + (size_t)i * t.g.c_out, buf.data() + (size_t)i * t.g.cop, t.g.c_out);
    if (exp_out) *exp_out = e;
    return NITI_NO_ERROR;
}

int niti_model_get_tap(niti_model_t m, int layer, int which, int8_t* host, size_t bytes, void* stream) {
    if (m && m->r) return host ? m->r->get_tap(layer, which, host, bytes, (hipStream_t)stream) : NITI_INVALID_VALUE;
    if (!m || layer < 0 || layer >= (int)m->m.L.size()) return NITI_INVALID_VALUE;
    niti::Layer& l = m->m.L[layer];
    const niti::ConvGeom& g = l.g;
    const int n = m->m.batch;
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return NITI_NO_EXECUTION;
    int8_t* tmp = nullptr;
    size_t need = 0;
    if (which == 0 || which == 2)
        need = (size_t)n * g.c_out * g.oh * g.ow;
    else if (which == 1 && m->m.g8_written)
        need = (size_t)g.c_out * g.c_in * g.kh * g.kw;
    else
        return NITI_INVALID_VALUE;
    const size_t out_need = which == 1 && l.col ? (size_t)l.og.c_out * l.og.c_in * l.og.kh * l.og.kw : need;
    if (bytes < out_need) return NITI_INVALID_VALUE;
    if (hipMalloc(&tmp, need) != hipSuccess) return NITI_OUT_OF_MEMORY;
    hipError_t e;
    if (which == 0 && !l.r_written) {  // (a pooled layer whose route went as codes under keep_grads(0))
        (void)hipFree(tmp);
        return NITI_INVALID_VALUE;
    }
    if (which == 0)
        e = niti::nhwc16_to_nchw(l.r, n, g.c_out, g.oh * g.ow, g.cop, tmp, nullptr);
    else if (which == 2 && !m->m.dy16_valid[layer]) {  // rebuilt from the C32 copy the step wrote
        int8_t* d16 = nullptr;
        e = hipMalloc(&d16, (size_t)n * g.oh * g.ow * g.cop);
        if (e == hipSuccess) e = niti::c32_to_nhwc16(l.dyc32, n, g.oh * g.ow, g.cop, g.c_out, d16, nullptr);
        if (e == hipSuccess) e = niti::nhwc16_to_nchw(d16, n, g.c_out, g.oh * g.ow, g.cop, tmp, nullptr);
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (d16) (void)hipFree(d16);
    } else if (which == 2)
        e = niti::nhwc16_to_nchw(l.dy, n, g.c_out, g.oh * g.ow, g.cop, tmp, nullptr);
    else
        e = niti::ohwi16_to_oihw(l.g8, g.c_out, g.c_in, g.kh * g.kw, g.cip, tmp, nullptr);
    if (which == 1 && l.col) {
        std::vector<int8_t> colw(need);
        if (e == hipSuccess) e = hipMemcpy(colw.data(), tmp, need, hipMemcpyDeviceToHost);
        if (e == hipSuccess) oihw_from_col(l.og, colw.data(), host);
    } else if (e == hipSuccess) {
        e = hipMemcpy(host, tmp, need, hipMemcpyDeviceToHost);
    }
    (void)hipFree(tmp);
    return e == hipSuccess ? NITI_NO_ERROR : NITI_NO_EXECUTION;
}

int64_t niti_model_step_macs(niti_model_t m) {
    if (m && m->r) return m->r->step_macs();
    if (!m) return 0;
    int64_t s = 0;
    const int world = m->m.world > 0 ? m->m.world : 1;
    for (size_t i = 0; i < m->m.L.size(); ++i) {
        const int64_t f = m->m.L[i].macs();
        s += f;            // forward
        s += f;            // weight gradient
        if (i > 0) s += f; // input gradient
    }
    (void)world;
    return s;
}

int niti_model_set_overlap(niti_model_t m, int enable) {
    if (m && m->r) return NITI_NO_ERROR;  // one stream (the weight gradients interleave with the input gradients)
    if (!m) return NITI_INVALID_VALUE;
    m->m.overlap = enable != 0;
    return NITI_NO_ERROR;
}

int niti_model_keep_grads(niti_model_t m, int enable) {
    if (m && m->r) {
        m->r->keep_grads = enable != 0;
        m->r->drop_graph();
        return NITI_NO_ERROR;
    }
    if (!m) return NITI_INVALID_VALUE;
    m->m.keep_grads = enable != 0;
    m->m.drop_graph();
    return NITI_NO_ERROR;
}

int niti_model_set_rowconv(niti_model_t m, int enable) {
    if (m && m->r) {
        niti::ResNetModel& r = *m->r;
        if (r.use_rowconv && enable == 0) {  // the GEMM input gradients read IHWO16 copies the update skipped
            for (int i = 0; i < (int)r.C.size(); ++i)
                if (r.refresh_copies(i, nullptr) != NITI_NO_ERROR) return NITI_NO_EXECUTION;
            if (hipDeviceSynchronize() != hipSuccess) return NITI_NO_EXECUTION;
        }
        r.use_rowconv = enable != 0;
        r.drop_graph();
        return NITI_NO_ERROR;
    }
    if (!m) return NITI_INVALID_VALUE;
    if (m->m.use_rowconv && enable == 0) {
        const int rc = m->m.refresh_wt(nullptr);
        if (rc != NITI_NO_ERROR || hipDeviceSynchronize() != hipSuccess) return NITI_NO_EXECUTION;
    }
    m->m.use_rowconv = enable != 0;
    m->m.drop_graph();
    return NITI_NO_ERROR;
}

int niti_model_spec_slot(niti_model_t m, int layer, int dgrad, uint32_t* out32) {
    if (!m || !out32 || layer < 0) return NITI_INVALID_VALUE;
    const uint32_t* bar = nullptr;
    if (m->r) {
        if (layer >= (int)m->r->C.size()) return NITI_INVALID_VALUE;
        bar = m->r->C[layer].bar;
    } else {
        if (layer >= (int)m->m.L.size()) return NITI_INVALID_VALUE;
        bar = m->m.L[layer].bar;
    }
    std::fill(out32, out32 + 32, 0u);
    if (bar == nullptr) return NITI_NO_ERROR;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out32, niti::rowconv_spec_slot(const_cast<uint32_t*>(bar), dgrad != 0), 32 * 4,
                  hipMemcpyDeviceToHost) != hipSuccess)
        return NITI_NO_EXECUTION;
    return NITI_NO_ERROR;
}

int niti_model_spec_stats(niti_model_t m, uint32_t* out, int max_layers) {
    if (m && m->r) return out && max_layers >= 0 ? m->r->spec_stats(out, max_layers) : NITI_INVALID_VALUE;
    if (!m || !out || max_layers < 0) return NITI_INVALID_VALUE;
    const int nl = std::min(max_layers, (int)m->m.L.size());
    std::fill(out, out + (size_t)nl * 6, 0u);
    for (int i = 0; i < nl; ++i) {
        const niti::Layer& l = m->m.L[i];
        for (int d = 0; d < 2; ++d) {  // forward / input-gradient slot: hint, redone launches, stored pairs
            uint32_t w[5] = {0, 0, 0, 0, 0}, gw[4] = {0, 0, 0, 0};
            if (l.bar != nullptr && hipMemcpy(w, niti::rowconv_spec_slot(const_cast<uint32_t*>(l.bar), d != 0), sizeof(w),
                                              hipMemcpyDeviceToHost) != hipSuccess)
                return NITI_INVALID_VALUE;
            // the GEMM path's pair (plan strategy 3): its own slot, no store mode
            if (l.gspec != nullptr && hipMemcpy(gw, l.gspec + d * niti::GEMM_SPEC_SLOT_WORDS, sizeof(gw),
                                                hipMemcpyDeviceToHost) != hipSuccess)
                return NITI_INVALID_VALUE;
            out[i * 6 + d * 3] = std::max(w[0], gw[0]);
            out[i * 6 + d * 3 + 1] = w[2] + gw[2];
            out[i * 6 + d * 3 + 2] = w[4] + gw[3];  // the GEMM pair: misses settled from an alternate
        }
    }
    return NITI_NO_ERROR;
}

int niti_model_rowconv_error(niti_model_t m) {
    if (m && m->r) return m->r->rowconv_error();
    if (!m) return NITI_INVALID_VALUE;
    uint32_t e = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&e, m->m.rc_err, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return NITI_NO_EXECUTION;
    return (int)e;
}

int niti_model_set_graph(niti_model_t m, int enable) {
    if (m && m->r) {
        m->r->drop_graph();
        m->r->use_graph = enable != 0;
        return NITI_NO_ERROR;
    }
    if (!m) return NITI_INVALID_VALUE;
    m->m.drop_graph();
    m->m.use_graph = enable != 0;
    return NITI_NO_ERROR;
}

int niti_model_autotune(niti_model_t m, int reps, void* stream) {
    if (m && m->r) return m->r->autotune((hipStream_t)stream, reps);
    if (!m) return NITI_INVALID_VALUE;
    return m->m.autotune((hipStream_t)stream, reps);
}

int niti_model_run_phase(niti_model_t m, int layer, int phase, void* stream) {
    if (m && m->r) return m->r->run_phase(layer, phase, (hipStream_t)stream);
    if (!m || layer < 0 || layer >= (int)m->m.L.size() || phase < 0 || phase > 2 || (phase == 1 && layer == 0))
        return NITI_INVALID_VALUE;
    const bool t = m->m.tuning;
    m->m.tuning = false;  // keep the probe armed; collectives stay off (single-device phase)
    std::unique_ptr<niti::Collective> c = std::move(m->m.coll), cg = std::move(m->m.coll_grad);
    hipStream_t st = (hipStream_t)stream;
    const int rc = phase == 0 ? m->m.fwd_layer(layer, st) : phase == 1 ? m->m.dgrad_layer(layer, st) : m->m.wgrad_layer(layer, st);
    m->m.coll = std::move(c);
    m->m.coll_grad = std::move(cg);
    m->m.tuning = t;
    return rc;
}

int niti_model_plan_info(niti_model_t m, int layer, int phase, int info[4]) {
    if (m && m->r) {
        if (!info || layer < 0 || layer >= (int)m->r->C.size() || phase < 0 || phase > 2) return NITI_INVALID_VALUE;
        const int op = phase == 0 ? niti::PLAN_FWD : phase == 1 ? niti::PLAN_DGRAD : niti::PLAN_WGRAD;
        const niti::PlanChoice c = niti::conv_plan_query(op, m->r->C[layer].g, phase != 2,
                                                         phase == 2 ? m->r->slab_w_bytes : m->r->slab_bytes);
        info[0] = c.bm;
        info[1] = c.bn;
        info[2] = c.splits;
        info[3] = c.strat;
        return NITI_NO_ERROR;
    }
    if (!m || !info || layer < 0 || layer >= (int)m->m.L.size() || phase < 0 || phase > 2)
        return NITI_INVALID_VALUE;
    const niti::ConvGeom& g = m->m.L[layer].g;
    const int op = phase == 0 ? niti::PLAN_FWD : phase == 1 ? niti::PLAN_DGRAD : niti::PLAN_WGRAD;
    niti::PlanChoice c = niti::conv_plan_query(op, g, phase != 2, m->m.ws_bytes_for(op));
    if (phase == 2 && m->m.wgrad_p16_splits(layer) > 0) {
        c.bm = c.bn = niti::PLAN_P16_TILE;
        c.splits = m->m.wgrad_p16_splits(layer);
        c.strat = c.splits > 1 ? 2 : 0;
    }
    info[0] = c.bm;
    info[1] = c.bn;
    info[2] = c.splits;
    info[3] = c.strat;
    return NITI_NO_ERROR;
}

int niti_model_plan_set(niti_model_t m, int layer, int phase, const int plan[4]) {
    if (m && m->r) {
        if (layer < 0 || layer >= (int)m->r->C.size() || phase < 0 || phase > 2) return NITI_INVALID_VALUE;
        const int op = phase == 0 ? niti::PLAN_FWD : phase == 1 ? niti::PLAN_DGRAD : niti::PLAN_WGRAD;
        const niti::ConvGeom& g = m->r->C[layer].g;
        const niti::PlanKey k = niti::conv_plan_key(op, g);
        m->r->drop_graph();
        if (plan == nullptr) {
            niti::plan_override_clear(k);
            return NITI_NO_ERROR;
        }
        auto tile_ok = [](int t) { return t == 64 || t == 128 || t == 256; };
        const bool taps = plan[0] == niti::PLAN_TAPS_TILE && plan[1] == niti::PLAN_TAPS_TILE && op == niti::PLAN_WGRAD &&
                          niti::conv_wgrad_taps_ok(g);
        if ((!taps && (!tile_ok(plan[0]) || !tile_ok(plan[1]))) || plan[2] < 1 || plan[2] > 4096 || plan[3] < 0 ||
            plan[3] > 4 || (taps && plan[3] == 1) || (plan[3] >= 3 && (op == niti::PLAN_WGRAD || plan[2] != 1)))
            return NITI_INVALID_VALUE;
        niti::PlanChoice c;
        c.bm = plan[0];
        c.bn = plan[1];
        c.splits = plan[2];
        c.strat = plan[3];
        if (c.strat == 2 &&
            !m->r->ensure_slab(std::min(niti::plan_slab_bytes(k.M, k.N, c.splits), size_t(1) << 30), op == niti::PLAN_WGRAD))
            return NITI_OUT_OF_MEMORY;
        niti::plan_override_set(k, c);
        return NITI_NO_ERROR;
    }
    if (!m || layer < 0 || layer >= (int)m->m.L.size() || phase < 0 || phase > 2) return NITI_INVALID_VALUE;
    const int op = phase == 0 ? niti::PLAN_FWD : phase == 1 ? niti::PLAN_DGRAD : niti::PLAN_WGRAD;
    const niti::PlanKey k = niti::conv_plan_key(op, m->m.L[layer].g);
    if (plan == nullptr) {
        niti::plan_override_clear(k);
    } else {
        auto tile_ok = [](int t) { return t == 64 || t == 128 || t == 256; };
        const niti::ConvGeom& g = m->m.L[layer].g;
        const bool taps = plan[0] == niti::PLAN_TAPS_TILE && plan[1] == niti::PLAN_TAPS_TILE &&
                          op == niti::PLAN_WGRAD && niti::conv_wgrad_taps_ok(g);
        const bool p16 = plan[0] == niti::PLAN_P16_TILE && plan[1] == niti::PLAN_P16_TILE &&
                         op == niti::PLAN_WGRAD && niti::conv_wgrad_p16_ok(g);
        if ((!taps && !p16 && (!tile_ok(plan[0]) || !tile_ok(plan[1]))) || plan[2] < 1 || plan[3] < 0 ||
            plan[3] > 4 || ((taps || p16) && plan[3] == 1) || (plan[3] >= 3 && (op == niti::PLAN_WGRAD || plan[2] != 1)))
            return NITI_INVALID_VALUE;
        if (p16) {
            if (plan[2] > 64) return NITI_INVALID_VALUE;
            if (!m->m.ensure_slab(niti::conv_wgrad_p16_workspace(g, plan[2]), true)) return NITI_OUT_OF_MEMORY;
        }
        niti::PlanChoice c;
        c.bm = plan[0];
        c.bn = plan[1];
        c.splits = plan[2];
        c.strat = plan[3];
        if (c.strat == 2 && !p16 &&
            !m->m.ensure_slab(std::min(niti::plan_slab_bytes(k.M, k.N, c.splits), size_t(1) << 30), op == niti::PLAN_WGRAD))
            return NITI_OUT_OF_MEMORY;
        niti::plan_override_set(k, c);
    }
    m->m.drop_graph();
    return NITI_NO_ERROR;
}

void niti_plan_reset(void) { niti::plan_override_clear_all(); }

int niti_model_set_probe(niti_model_t m, int layer, int phase, int max_launches) {
    if (m && m->r) {
        if (max_launches < 0) return NITI_INVALID_VALUE;
        niti::ResNetModel& r = *m->r;
        r.clear_probe();
        if (layer < 0) return NITI_NO_ERROR;
        r.probe_layer = layer;
        r.probe_phase = phase;
        r.ev0.resize(max_launches);
        r.ev1.resize(max_launches);
        for (int i = 0; i < max_launches; ++i)
            if (hipEventCreateWithFlags(&r.ev0[i], hipEventDisableSystemFence) != hipSuccess ||
                hipEventCreateWithFlags(&r.ev1[i], hipEventDisableSystemFence) != hipSuccess)
                return NITI_OUT_OF_MEMORY;
        return NITI_NO_ERROR;
    }
    if (!m || max_launches < 0) return NITI_INVALID_VALUE;
    m->m.clear_probe();
    if (layer < 0) return NITI_NO_ERROR;
    m->m.probe_layer = layer;
    m->m.probe_phase = phase;
    m->m.ev0.resize(max_launches);
    m->m.ev1.resize(max_launches);
    for (int i = 0; i < max_launches; ++i)
        // timing events without the system-scope cache writeback / invalidate (it delays the
        // launch after the begin marker and is not needed to read the timestamps)
        if (hipEventCreateWithFlags(&m->m.ev0[i], hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&m->m.ev1[i], hipEventDisableSystemFence) != hipSuccess)
            return NITI_OUT_OF_MEMORY;
    if (phase == 2 && max_launches > 0) {  // per launch, a {start, end} pair per block (zero: no block)
        const size_t bytes = (size_t)max_launches * 2 * niti::SPAN_MAX_BLOCKS * 8;
        if (hipMalloc(&m->m.span, bytes) != hipSuccess || hipMemset(m->m.span, 0, bytes) != hipSuccess)
            return NITI_OUT_OF_MEMORY;
        m->m.span_cap = max_launches;
    }
    return NITI_NO_ERROR;
}

int niti_model_probe_read_span(niti_model_t m, double* total_ms, int* count) {
    if (m && m->r) {
        if (!total_ms || !count) return NITI_INVALID_VALUE;
        *total_ms = 0;  // no in-kernel span probe on this driver
        *count = 0;
        return NITI_NO_ERROR;
    }
    if (!m || !total_ms || !count) return NITI_INVALID_VALUE;
    *total_ms = 0;
    *count = 0;
    if (m->m.span == nullptr || m->m.span_count == 0) return NITI_NO_ERROR;
    int dev = 0, khz = 0;
    if (hipDeviceSynchronize() != hipSuccess || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        return NITI_NO_EXECUTION;
    constexpr size_t per = 2 * niti::SPAN_MAX_BLOCKS;
    std::vector<unsigned long long> h(per * (size_t)m->m.span_count);
    if (hipMemcpy(h.data(), m->m.span, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return NITI_NO_EXECUTION;
    double t = 0;
    int n = 0;
    for (int i = 0; i < m->m.span_count; ++i) {  // first block start to last block end of launch i
        unsigned long long lo = ~0ull, hi = 0;
        for (size_t b = 0; b < per; b += 2) {
            const unsigned long long s0 = h[per * i + b], s1 = h[per * i + b + 1];
            if (s1 == 0) continue;
            lo = s0 < lo ? s0 : lo;
            hi = s1 > hi ? s1 : hi;
        }
        if (hi > lo) {
            t += (double)(hi - lo) / khz;  // ticks / kHz = ms
            ++n;
        }
    }
    *total_ms = t;
    *count = n;
    // re-arm the slots for the next measurement
    if (hipMemset(m->m.span, 0, h.size() * 8) != hipSuccess) return NITI_NO_EXECUTION;
    m->m.span_count = 0;
    return NITI_NO_ERROR;
}

int niti_model_probe_pause(niti_model_t m, int paused) {
    if (!m) return NITI_INVALID_VALUE;
    if (m->r)
        m->r->probe_paused = paused != 0;
    else
        m->m.probe_paused = paused != 0;
    return NITI_NO_ERROR;
}

int niti_model_probe_read(niti_model_t m, double* total_ms, int* count) {
    if (m && m->r) {
        if (!total_ms || !count) return NITI_INVALID_VALUE;
        niti::ResNetModel& r = *m->r;
        double t = 0;
        for (int i = 0; i < r.probe_count; ++i) {
            float ms = 0.f;
            if (hipEventSynchronize(r.ev1[i]) != hipSuccess || hipEventElapsedTime(&ms, r.ev0[i], r.ev1[i]) != hipSuccess)
                return NITI_NO_EXECUTION;
            t += ms;
        }
        *total_ms = t;
        *count = r.probe_count;
        r.probe_count = 0;
        return NITI_NO_ERROR;
    }
    if (!m || !total_ms || !count) return NITI_INVALID_VALUE;
    double t = 0;
    for (int i = 0; i < m->m.probe_count; ++i) {
        float ms = 0.f;
        if (hipEventSynchronize(m->m.ev1[i]) != hipSuccess ||
            hipEventElapsedTime(&ms, m->m.ev0[i], m->m.ev1[i]) != hipSuccess)
            return NITI_NO_EXECUTION;
        t += ms;
    }
    *total_ms = t;
    *count = m->m.probe_count;
    m->m.probe_count = 0;
    return NITI_NO_ERROR;
}

extern "C++" {
// hand a communicator pair to whichever step driver the handle holds
template <class M>
static void attach_to(M& d, std::unique_ptr<niti::Collective> c, std::unique_ptr<niti::Collective> cg, bool shared,
                      int world, int rank, int exact) {
    d.drop_graph();
    d.coll = std::move(c);
    d.coll_grad = std::move(cg);
    d.shared_comm = shared;
    d.world = world;
    d.rank = rank;
    d.exact = exact ? 1 : 0;
}
static void attach(niti_model_t m, std::unique_ptr<niti::Collective> c, std::unique_ptr<niti::Collective> cg,
                   bool shared, int world, int rank, int exact) {
    if (m->r)
        attach_to(*m->r, std::move(c), std::move(cg), shared, world, rank, exact);
    else
        attach_to(m->m, std::move(c), std::move(cg), shared, world, rank, exact);
}
}  // extern "C++"

int niti_dp_get_unique_id(char id[NITI_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == NITI_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return NITI_NO_EXECUTION;
    memcpy(id, &u, sizeof(u));
    return NITI_NO_ERROR;
}

int niti_model_attach_comm(niti_model_t m, const char id[NITI_UNIQUE_ID_BYTES], int rank, int world, int exact) {
    if (!m || !id || world < 1 || rank < 0 || rank >= world) return NITI_INVALID_VALUE;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    // the split-agreement flag and stream first: a local allocation failure then returns before any
    // collective call, instead of leaving the peers blocked in one this rank never enters
    int32_t* flag = nullptr;
    hipStream_t ast = nullptr;
    if (hipMalloc(&flag, sizeof(int32_t)) != hipSuccess || hipStreamCreate(&ast) != hipSuccess) {
        if (flag) (void)hipFree(flag);
        return NITI_OUT_OF_MEMORY;
    }
    auto c = std::make_unique<niti::RcclCollective>();
    if (ncclCommInitRank(&c->comm, world, u, rank) != ncclSuccess) {
        (void)hipFree(flag);
        (void)hipStreamDestroy(ast);
        return NITI_NO_EXECUTION;
    }
    c->world = world;
    // the gradient communicator: split off the first (collective over the ranks), its own
    // resources, so its SUMs and the ranges' MAXes are not serialised against each other
    auto cg = std::make_unique<niti::RcclCollective>();
    const bool split_ok = ncclCommSplit(c->comm, 0, rank, &cg->comm, nullptr) == ncclSuccess;
    // every rank must pick the same mode (the SUMs run on different communicators and streams in
    // the two modes): agree on the split's success with a MIN over the range communicator, which
    // every rank enters whatever its own split did
    int32_t ok = split_ok ? 1 : 0;
    const bool agreed = hipMemcpyAsync(flag, &ok, sizeof(ok), hipMemcpyHostToDevice, ast) == hipSuccess &&
                        ncclAllReduce(flag, flag, 1, ncclInt32, ncclMin, c->comm, ast) == ncclSuccess &&
                        hipMemcpyAsync(&ok, flag, sizeof(ok), hipMemcpyDeviceToHost, ast) == hipSuccess &&
                        hipStreamSynchronize(ast) == hipSuccess;
    (void)hipFree(flag);
    (void)hipStreamDestroy(ast);
    if (!agreed) {
        if (split_ok) (void)ncclCommDestroy(cg->comm);
        cg->comm = nullptr;
        (void)ncclCommDestroy(c->comm);
        c->comm = nullptr;
        return NITI_NO_EXECUTION;
    }
    bool shared = false;
    if (ok == 0) {
        // some rank has no split: every rank's gradient SUMs use the range communicator, in the
        // step's program order
        if (split_ok) (void)ncclCommDestroy(cg->comm);
        cg->comm = c->comm;
        cg->owns = false;
        shared = true;
    }
    cg->world = world;
    attach(m, std::move(c), std::move(cg), shared, world, rank, exact);
    return NITI_NO_ERROR;
}

struct niti_local_group {
    std::shared_ptr<niti::LocalGroup> g;
};

int niti_local_group_create(int world, niti_local_group_t* out) {
    if (!out || world < 1 || world > niti::LocalGroup::MAX_RANKS) return NITI_INVALID_VALUE;
    auto* h = new niti_local_group();
    h->g = std::make_shared<niti::LocalGroup>();
    h->g->world = world;
    if (hipStreamCreateWithFlags(&h->g->rst, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return NITI_NO_EXECUTION;
    }
    *out = h;
    return NITI_NO_ERROR;
}

void niti_local_group_destroy(niti_local_group_t g) { delete g; }

int niti_model_attach_local(niti_model_t m, niti_local_group_t g, int rank, int exact) {
    if (!m || !g || rank < 0 || rank >= g->g->world) return NITI_INVALID_VALUE;
    auto c = std::make_unique<niti::LocalCollective>();
    c->g = g->g;
    c->rank = rank;
    c->chan = 0;
    auto cg = std::make_unique<niti::LocalCollective>();
    cg->g = g->g;
    cg->rank = rank;
    // NITI_DIAG_SHARED_COMM=1 (tests): the gradient SUMs on the range channel, as attach_comm's
    // no-split fallback runs them on one RCCL communicator
    const bool shared = getenv("NITI_DIAG_SHARED_COMM") != nullptr;
    cg->chan = shared ? 0 : 1;
    attach(m, std::move(c), std::move(cg), shared, g->g->world, rank, exact);
    return NITI_NO_ERROR;
}

}  // extern "C"
