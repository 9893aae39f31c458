// niti_resnet_model.hpp -- the ResNet-18 NITI training step driven from C++ (BASELINE config 5),
// behind the same niti_model_* C ABI as the LeNet / VGG driver (niti_model.hip).
//
// The reference has no ResNet NITI model: its graph builder would chain NITI_Conv_Int8_Module
// instances (tools/train/source/nn/NN.cpp:1181-1207) and its residual op NITI_Eltwise_Int8 is an
// empty stub (execution-engine/source/backend/cpu/NITI_Eltwise_Int8.cpp:20-28).  The convs, relu,
// max pool, loss gradient and NITI_SGD follow the reference ops; the residual add, the global sum
// pool and the gradient exponents are this library's rules (csrc/niti_resnet.hip, restated in
// oracle/niti_resnet_ref.py).
#pragma once

#include <memory>
#include <vector>

#include "niti_coll.hpp"
#include "niti_internal.hpp"
#include "niti_kernels.hpp"

namespace niti {

// one parameter layer (conv1, per basic block conv a / conv b / the 1x1 projection, the fc head)
struct RConv {
    ConvGeom g{};   // as it runs (the stem: a 1x1 conv over its im2col, c_in = the im2col columns)
    ConvGeom og{};  // as the network defines it (the stem: 7x7 / 2, pad 3)
    int relu = 0;   // relu fused into the forward requantisation (conv1, conv a)
    int rows = 0;   // forward and input gradient on the register-fed row kernels (niti_rowconv.hip)
    int rows_dg = 0;
    ConvGeom dg{};  // the input gradient's geometry on the row kernel (rowconv_dgrad_geom)
    int8_t wscale = 0;
    int8_t* w = nullptr;       // OHWI16
    int8_t* wT = nullptr;      // IHWO16 (GEMM input gradient)
    int8_t* subw = nullptr;    // stride 2: the sub-pixel classes' weights (conv_dgrad_subpix_bytes)
    int8_t* wf = nullptr;      // fragment-major copies (row kernels)
    int8_t* wft = nullptr;
    int8_t* ws_dev = nullptr;  // wscale, device
    int8_t* g8 = nullptr;      // int8 weight gradient (keep_grads)
    uint32_t* bar = nullptr;   // row-kernel state: grid barrier words + speculation slots
    uint32_t* gspec = nullptr; // the GEMM path's speculative pair: forward / input-gradient hint slots
    uint32_t epoch = 0;
    int8_t* xc32 = nullptr;    // C32 copies where the row kernel reads C32 (not NHWC16 in place)
    int8_t* dyc32 = nullptr;
    const int8_t* in = nullptr;      // input NHWC16 (the stem: its im2col)
    const int8_t* in_exp = nullptr;
    int8_t* y = nullptr;             // output NHWC16 (relu'd where relu)
    int8_t* y_exp = nullptr;
    int8_t* dy = nullptr;            // output gradient NHWC16 (conv b and the projection share one)
    const int8_t* dy_exp = nullptr;
    int8_t* dx = nullptr;            // input gradient (null: none -- the stem)
    int8_t* dx_exp = nullptr;
    const int8_t* dx_mask = nullptr; // the previous op's relu gradient fused into the input gradient
    int32_t* dwacc = nullptr;        // int32 weight gradient (in the contiguous gradient bucket)
    // single device: a split-K weight gradient's own slabs, combined by the NITI_SGD launch
    int32_t* wslab = nullptr;
    size_t wslab_bytes = 0;
    SgdJob defer{};
    int64_t w_elems() const { return (int64_t)g.c_out * g.kh * g.kw * g.cip; }
    int64_t macs() const { return (int64_t)og.n * og.oh * og.ow * og.c_out * og.c_in * og.kh * og.kw; }
};

struct RBlock {
    int a = 0, b = 0, p = -1;   // conv indices (p: the projection, -1 none)
    const int8_t* u = nullptr;  // block input and its exponent
    const int8_t* u_exp = nullptr;
    int8_t* out = nullptr;      // relu(requant(aligned y_b + shortcut))
    int8_t* out_exp = nullptr;
    int8_t* ez = nullptr;       // the residual sum's exponent (forward)
    int8_t* dz = nullptr;       // gradient of the block output after its relu (conv b's and proj's dy)
    int8_t* dz_exp = nullptr;
    int8_t* dh = nullptr;       // conv a's output gradient (after its relu)
    int8_t* dua = nullptr;      // conv a's input gradient
    int8_t* dus = nullptr;      // the projection's input gradient
    int8_t* du = nullptr;       // gradient at the block input (the residual sum's requantisation)
    int8_t* du_exp = nullptr;
    int8_t* ezb = nullptr;      // the backward sum's exponent
    int64_t out_elems = 0, in_elems = 0;
};

struct ResNetModel {
    static constexpr int STEM_KP = 160;  // the stem's im2col columns: 7 * 7 * 3 = 147, padded
    int batch = 0, in_hw = 0, classes = 1000;
    std::vector<RConv> C;
    std::vector<RBlock> B;
    Workspace ws;
    ConvGeom stem{};              // conv1 as defined (the im2col's geometry)
    int8_t* x0n = nullptr;        // the quantised input, NCHW int8
    int8_t* exp0 = nullptr;
    int8_t* xcol = nullptr;       // the stem's im2col [n * oh * ow][STEM_KP]
    int8_t* p0 = nullptr;         // 3x3 / 2 max pool of the stem output
    int8_t* pool_ws = nullptr;    // each pool window's first-max position (the pool gradient's)
    // the stem's requantise pass also max-pooled (Pool3) this step; with keep_grads off its pre-pool
    // output is then never written (its forward tap is unavailable)
    bool stem_pooled = false;
    // what the last step wrote for the debug taps (get_tap reads these, not the current
    // keep_grads): the stem's pre-pool output, the int8 weight gradients
    bool stem_y_written = false;
    bool g8_written = false;
    int8_t* d0 = nullptr;         // the stem's output gradient
    int32_t* gsum = nullptr;      // global sum pool [n][512]
    int8_t* g8pool = nullptr;     // its requantisation (the fc input)
    int8_t* eg = nullptr;
    int8_t* dg = nullptr;         // the fc head's input gradient [n][512]
    int8_t* ed = nullptr;         // the loss gradient's exponent (0)
    int8_t* exps = nullptr;       // device int8 exponents, handed out in build()
    int n_exps = 0;
    int32_t* acc = nullptr;       // shared int32 accumulator of the GEMM paths
    size_t acc_bytes = 0;
    void* slab = nullptr;         // split-K slabs (forward / input gradient)
    size_t slab_bytes = 0;
    void* slab_w = nullptr;       // split-K slabs (weight gradients)
    size_t slab_w_bytes = 0;
    int32_t* rc_acc = nullptr;    // the row kernels' accumulator store (two-launch store mode)
    size_t rc_acc_size = 0;
    int8_t* gspec_alt = nullptr;  // the GEMM speculative pairs' alternates (shared)
    size_t gspec_alt_bytes = 0;
    uint32_t* rc_err = nullptr;
    // the residual sums' single-launch form (residual_fused, NITI_RES_FUSED=1: measured slower than
    // the two launches): one grid-barrier state for all of them (in order on the step stream)
    // the stride-2 input gradients as sub-pixel classes (NITI_SUBPIX=0: the generic masked loader)
    static bool subpix_on() {
        static const bool off = getenv("NITI_SUBPIX") && atoi(getenv("NITI_SUBPIX")) == 0;
        return !off;
    }
    uint32_t* res_bar = nullptr;
    uint32_t res_epoch = 0;
    // the residual sums' speculative pairs: one slot per block and direction (residual_requant)
    uint32_t* res_slot = nullptr;
    static bool res_spec_on() {
        static const bool off = getenv("NITI_RES_SPEC") && atoi(getenv("NITI_RES_SPEC")) == 0;
        return !off;
    }
    bool res_fused_on() const {
        static const bool on = getenv("NITI_RES_FUSED") && atoi(getenv("NITI_RES_FUSED")) == 1;
        return on && !dp() && !capturing && res_bar != nullptr;
    }
    unsigned long long* qstats = nullptr;
    unsigned long long* qslots = nullptr;
    int32_t* grad_bucket = nullptr;
    uint32_t* amax = nullptr;     // 3 ranges per conv, then 2 per block, then the pool's
    size_t amax_bytes = 0;
    uint32_t* rng(int conv, int which) { return amax + (size_t)(3 * conv + which) * MAX_WORDS; }
    uint32_t* rng_blk(int blk, int bwd) { return amax + (size_t)(3 * C.size() + 2 * blk + bwd) * MAX_WORDS; }
    uint32_t* rng_pool() { return amax + (size_t)(3 * C.size() + 2 * B.size()) * MAX_WORDS; }
    bool keep_grads = true;
    bool use_rowconv = true;
    bool tuning = false;
    bool probe_paused = false;  // niti_model_probe_pause
    bool capturing = false;
    // data parallel: ranges on the step stream (coll), gradient-bucket SUMs on cst (coll_grad)
    std::unique_ptr<Collective> coll, coll_grad;
    int world = 1, rank = 0, exact = 1;
    bool shared_comm = false;
    bool dp() const { return coll != nullptr && coll_grad != nullptr && !tuning; }
    hipStream_t cst = nullptr;
    std::vector<hipEvent_t> ev_bucket;
    hipEvent_t ev_grads = nullptr;
    std::vector<int> bucket_lo;
    std::vector<char> closes_bucket;
    size_t bucket_min_bytes = grad_bucket_bytes();
    // kernel probe: HIP events on the step stream around one conv phase (both launches of a
    // two-launch form), up to ev0.size() launches
    int probe_layer = -1, probe_phase = -1, probe_count = 0;
    std::vector<hipEvent_t> ev0, ev1;
    // optional hipGraph replay of the single-device step
    bool use_graph = false;
    hipStream_t gstream = nullptr;
    hipEvent_t gin = nullptr, gout = nullptr;
    hipGraphExec_t gexec = nullptr;
    const void* gkey_x = nullptr;
    const void* gkey_l = nullptr;
    int gkey_e = 0;

    int build(int batch_, int in_hw_, int classes_);
    bool rows_on(int i) const { return use_rowconv && C[i].rows; }
    bool rows_dg_on(int i) const { return use_rowconv && C[i].rows_dg; }
    int fwd_conv(int i, hipStream_t st);
    int dgrad_conv(int i, hipStream_t st);
    int wgrad_conv(int i, hipStream_t st);
    bool in_step = false;  // run(): weight gradients may leave their split-K combine to the update
    bool ensure_wslab(int i);
    int size_wslabs();
    unsigned wslab_epoch = 0;  // plan_override_epoch() the slabs were last sized for
    int residual_fwd(int k, hipStream_t st);
    int residual_bwd(int k, hipStream_t st);
    int run(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st);
    int step(const int8_t* x_nchw, int exp_in, const uint8_t* images, const int32_t* labels, hipStream_t st);
    int autotune(hipStream_t st, int reps);
    int run_phase(int layer, int phase, hipStream_t st);
    int sum_bucket(int lo, hipStream_t st);
    void plan_buckets();
    int ensure_comm_stream();
    bool ensure_slab(size_t bytes, bool wgrad);
    void probe(int layer, int phase, bool begin, hipStream_t st);
    void clear_probe();
    void drop_graph();
    int refresh_copies(int i, hipStream_t st);  // wT / wf / wft from w
    int set_weight(int i, const int8_t* w_oihw_host, int wscale);
    int get_weight(int i, int8_t* w_oihw_host);
    int get_tap(int layer, int which, int8_t* host, size_t bytes, hipStream_t st);
    int get_logits(int8_t* host, int* exp_out, hipStream_t st);
    int get_input(int8_t* host, int* ascale, hipStream_t st);
    int64_t step_macs() const;
    int spec_stats(uint32_t* out, int max_layers);
    int rowconv_error();
    ~ResNetModel();
};

}  // namespace niti
