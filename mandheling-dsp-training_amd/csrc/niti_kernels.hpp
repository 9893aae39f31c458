// niti_kernels.hpp -- internal launch API of the MI355X (gfx950) NITI int8 kernels.
//
// Native device layouts (all int8 unless noted; padded lanes are always zero):
//   NHWC16 activations  [N][H][W][Cp]      Cp = round_up(C, 16)     (fwd / dgrad operand)
//   CHWN16 activations  [Cp][H][W][Np]     Np = round_up(N, 16)     (wgrad operand: K = (oy,ox,n))
//   OHWI16 weights      [Co][KH][KW][Cip]                           (fwd B operand, wgrad output)
//   IHWO16 weights      [Ci][KH][KW][Cop]                           (dgrad B operand)
//   accumulators        int32 [rows][ld] with ld a multiple of 16
// The reference's layouts (MNN C4 [C/4][N][H][W][4], NCHW, OIHW) only appear at the
// drop-in boundary (niti_execution.hip) and are converted by the kernels declared at
// the end of this file.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/niti_hip.h"

namespace niti {

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// A range estimate (max|acc| of one tensor) is kept in MAX_SLOTS words, one per 128-byte
// line (MAX_WORDS words in all, zeroed before the producing launch); publishers atomically
// max into one slot each, readers take the max over the slots (NITI_MAX_WORDS in
// include/niti_hip.h).  Atomics serialise per cache line, so the slots must not share one.
constexpr int MAX_SLOTS = 64;
constexpr int MAX_SLOT_STRIDE = 32;  // words (128 bytes)
constexpr int MAX_WORDS = MAX_SLOTS * MAX_SLOT_STRIDE;
constexpr size_t MAX_BYTES = MAX_WORDS * sizeof(uint32_t);

struct ConvGeom {
    int n, c_in, h, w;
    int c_out, kh, kw;
    int sh, sw, pt, pl, pb, pr, dh, dw;
    int oh, ow;
    int cip, cop, np;  // padded channel / batch counts (multiples of 16)
    // fills oh/ow/cip/cop/np; returns false on an invalid geometry
    bool finalize();
};

// Exponent rules (NITI_Conv_Int8.cpp:260-307 / NITI_GradientConv_Int8.cpp:272-296 /
// NITI_Matmul_Int8.cpp:214-228).
enum GradRule { RULE_WGRAD_BW2 = 2, RULE_MATMUL_BW3 = 3 };

// ---- GEMM-class accumulation (int8 MFMA v_mfma_i32_32x32x32_i8, exact int32) ----------
// Every op materialises acc [rows][ld] int32 and, when amax != null, max-es |acc| into it
// (caller zeroes it).  Shapes with too few output tiles for 256 CUs split K over workgroups
// into int32 slabs in the caller's workspace `ws` and reduce them (exact, order independent);
// a workspace smaller than *_workspace() just means no split.
size_t conv_fwd_workspace(const ConvGeom& g);
size_t conv_dgrad_workspace(const ConvGeom& g);
size_t conv_wgrad_workspace(const ConvGeom& g);
size_t matmul_workspace(int M, int ldc, int k16);

// Per-shape plan overrides (filled by the model's autotuner).  A plan is a tile shape (bm x bn,
// 64 or 128 each), a strategy (0 store acc, 1 recompute the GEMM for the requantisation --
// forward / input gradient only, 2 split-K slabs + reduce) and a split count.  Keys: op and the
// GEMM extents (M, N, K in the planner's units).  Overrides never change results.
enum PlanOp { PLAN_FWD = 0, PLAN_DGRAD = 1, PLAN_WGRAD = 2, PLAN_MATMUL = 3 };
struct PlanKey {
    int op, M, N, K;
    bool operator<(const PlanKey& o) const {
        if (op != o.op) return op < o.op;
        if (M != o.M) return M < o.M;
        if (N != o.N) return N < o.N;
        return K < o.K;
    }
};
struct PlanChoice {
    int bm = 128, bn = 128, splits = 1, strat = 0;
};
// bm = bn = PLAN_TAPS_TILE selects the tap-sharing weight-gradient kernel (64 output channels x
// all taps x 32 input channels per block) where conv_wgrad_taps_ok(g)
constexpr int PLAN_TAPS_TILE = 32;
// bm = bn = PLAN_P16_TILE: the P16 weight gradient (niti_wgrad.hip, splits = its K split), which the
// model runs on P16 copies of x and dy; the NHWC16 entry points ignore such plans
constexpr int PLAN_P16_TILE = 16;
bool plan_override_lookup(const PlanKey& k, PlanChoice* c);
bool conv_wgrad_taps_ok(const ConvGeom& g);
PlanKey conv_plan_key(int op, const ConvGeom& g);
// the plan a conv GEMM runs with now (override or default), tap-sharing wgrad included
PlanChoice conv_plan_query(int op, const ConvGeom& g, bool recompute_ok, size_t ws_bytes);
int conv_plan_k_step(int op, const ConvGeom& g);
void plan_override_set(const PlanKey& k, const PlanChoice& c);
void plan_override_clear(const PlanKey& k);
void plan_override_clear_all();
// bumped by every override change: callers that size buffers per plan re-check when it moves
unsigned plan_override_epoch();
// the plan the GEMM of key k runs with now (override or default) under a workspace of ws_bytes
PlanChoice plan_query(const PlanKey& k, int k_step, bool recompute_ok, size_t ws_bytes);
size_t plan_slab_bytes(int M, int N, int splits);
struct PlanChoice;
size_t conv_wgrad_slab_bytes(const ConvGeom& g, const PlanChoice& c);
// acc[M = n*oh*ow][cop] = conv(x NHWC16, w OHWI16)
hipError_t conv_fwd_acc(const ConvGeom& g, const int8_t* x_nhwc16, const int8_t* w_ohwi16, int32_t* acc,
                        uint32_t* amax, void* ws, size_t ws_bytes, hipStream_t st);
// acc[M = n*h*w][cip] = transposed conv of dy (NHWC16) with w^T (IHWO16): the input gradient
hipError_t conv_dgrad_acc(const ConvGeom& g, const int8_t* dy_nhwc16, const int8_t* wt_ihwo16, int32_t* acc,
                          uint32_t* amax, void* ws, size_t ws_bytes, hipStream_t st);
// Kernel-span probe: the next weight-gradient GEMM launch (either kernel) min-es its blocks'
// start and max-es their end s_memrealtime (device wall clock) into slot[0] / slot[1]; the slot
// is consumed by that launch.  Host-side, not thread-safe (one model per thread).
void probe_span_arm(unsigned long long* slot);
// a span slot is one {start, end} pair per block (block = blockIdx.x + blockIdx.y * gridDim.x)
constexpr int SPAN_MAX_BLOCKS = 4096;
// Kernel-event probe: the next weight-gradient GEMM launch records `begin` / `end` as part of its
// own dispatch (hipExtLaunchKernel: the kernel's begin and end, as rocprofv3 times it).
void probe_events_arm(hipEvent_t begin, hipEvent_t end);
// acc[co][kh][kw][cip] = sum over (n, oy, ox) of dy * x (x, dy NHWC16): the weight gradient,
// a K-major GEMM over pixels whose operand tiles are transposed in LDS (ds_read_b64_tr_b8).
// defer (may be null): where the plan splits K into C-shaped slabs (the GEMM path; not the
// tap-sharing kernel's tile-blocked slabs), leave the slabs in ws unreduced and describe them in
// *defer (slab, splits, stride, n) for sgd_update_many's combine, which sums them into acc and
// takes the range -- one launch and an int32 round trip less per layer.  ws must then stay the
// layer's own until the update; *defer.slab stays null when the launch reduced itself.
struct SgdJob;
hipError_t conv_wgrad_acc(const ConvGeom& g, const int8_t* x_nhwc16, const int8_t* dy_nhwc16, int32_t* acc,
                          uint32_t* amax, void* ws, size_t ws_bytes, hipStream_t st, hipEvent_t after_gemm = nullptr,
                          SgdJob* defer = nullptr);
// C[i] = sum over z < splits of slab[z * stride + i] (+ max|C| into amax); n % 4 == 0
hipError_t splitk_reduce_linear(const int32_t* slab, int splits, int64_t n, int64_t stride, int32_t* C,
                                uint32_t* amax, hipStream_t st);
// ---- residual add / global sum pool (niti_resnet.hip) ------------------------------------
// residual_add (range) + residual_requant in one launch with an in-kernel grid barrier (single
// device; bar: ROWCONV_BAR_WORDS zeroed words, epoch: this state's launch count, 1 on the first;
// a barrier timeout sets *err).  hipErrorNotSupported when the grid cannot be resident at once
// (the caller then takes the two launches)
hipError_t residual_fused(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n, int8_t* ez,
                          int8_t* exp_out, int relu, int8_t* out, uint32_t* bar, uint32_t epoch, uint32_t* err,
                          hipStream_t st, const int8_t* relu_mask = nullptr);
// workgroups of 256 threads of kernel f the device holds at once (0 without a device)
int resident_wgs(const void* f, int threads = 256);
// z = aligned a + b (int32, n % 16 == 0 elements), its exponent into ez, max|z| into amax
hipError_t residual_add(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                        int32_t* z, int8_t* ez, uint32_t* amax, hipStream_t st);
// the fused form: z recomputed from a, b and requantised with the range in amax (from residual_add
// with z = null); out int8 (n elements), *ez and *exp_out = *ez + inc (either may be null).
// spec 1 / 2: the speculative pair instead of range pass + requantise pass -- launch A (1)
// requantises with the guessed bit width (spec_pick over slot, RES_SPEC_SLOT_WORDS zeroed words)
// and publishes max|z| into amax (zeroed by the caller); launch B (2; after any MAX all-reduce)
// writes the exponents and redoes the pass only when the range's bit width differs: 3 bytes per
// element on a hit instead of 5.  slot word [2] counts the redone launches.
constexpr int RES_SPEC_SLOT_WORDS = 32;
hipError_t residual_requant(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                            const uint32_t* amax, int8_t* ez, int8_t* exp_out, int relu, int8_t* out, hipStream_t st,
                            const int8_t* relu_mask = nullptr, int spec = 0, uint32_t* slot = nullptr);
// acc[n][cp] = sum over hw pixels of x NHWC16 (+ max into amax); its gradient: dy broadcast
hipError_t sum_pool(const int8_t* x, int n, int hw, int cp, int32_t* acc, uint32_t* amax, hipStream_t st);
// (relu_mask: the pooled map, NHWC16 -- its relu gradient applied too, dx = mask > 0 ? dy : 0)
hipError_t sum_pool_grad(const int8_t* dy, int n, int hw, int cp, int8_t* dx, hipStream_t st,
                         const int8_t* relu_mask = nullptr);
hipError_t im2col_small(const ConvGeom& g, const int8_t* x, int kp, int8_t* xcol, hipStream_t st, bool nchw = false);
// ---- weight gradient on P16 pixel blocks (niti_wgrad.hip) --------------------------------
// P16: [pixels/16][Cp][16] int8 (Cp % 16 == 0, pixels % 16 == 0)
hipError_t nhwc16_to_p16(const int8_t* in, int64_t pixels, int cp, int8_t* out, hipStream_t st);
// several conversions in one launch (at most P16_MAX_JOBS)
struct P16Conv {
    const int8_t* in = nullptr;
    int64_t pixels = 0;
    int cp = 0;
    int8_t* out = nullptr;
};
constexpr int P16_MAX_JOBS = 16;
hipError_t nhwc16_to_p16_many(const P16Conv* jobs, int n, hipStream_t st);
// loss_grad and nhwc16_to_p16_many(jobs, n) in one launch (two launches for wide class rows)
hipError_t loss_grad_p16(const int8_t* logits, int batch, int classes, int ld, const int8_t* ascale,
                         const int32_t* labels, int8_t* out, const P16Conv* jobs, int n, hipStream_t st);
bool conv_wgrad_p16_ok(const ConvGeom& g);
// diagnostic builds (NITI_WG_STAMPS): per-block stamps of the following launches, 8 u64 per block
void wgrad_stamps_arm(unsigned long long* buf);
int conv_wgrad_p16_splits(const ConvGeom& g);
// workspace: the split-K partial slabs (0 bytes when the plan does not split)
size_t conv_wgrad_p16_workspace(const ConvGeom& g, int splits);
struct SgdJob;
hipError_t conv_wgrad_p16(const ConvGeom& g, const int8_t* x_p16, const int8_t* dy_p16, int32_t* acc,
                          uint32_t* amax, void* ws, size_t ws_bytes, int splits, hipStream_t st,
                          hipEvent_t ev_b = nullptr, hipEvent_t ev_e = nullptr, unsigned long long* span = nullptr,
                          SgdJob* defer = nullptr);
// acc[m][o] = sum_k B[m][k] * A[o][k] (NITI_Matmul_Int8); k16 multiple of 16 (zero padded rows),
// ldb/lda bytes, ldc elements (multiple of 16; columns o..ldc come out 0)
hipError_t matmul_acc(int M, int O, int k16, const int8_t* B, int64_t ldb, const int8_t* A, int64_t lda,
                      int32_t* acc, int64_t ldc, uint32_t* amax, void* ws, size_t ws_bytes, hipStream_t st);

// Fused forward / input-gradient path used by the training step: phase 1 establishes the
// tensor-wide max|acc| (either materialising acc, or -- for small K -- computing the max
// only and recomputing the GEMM in phase 2 with the requantisation in its epilogue).
// Between the phases a data-parallel run all-reduces *amax (MAX).
// 2x2 / stride-2 max pool fused into the requantisation (NITI_Maxpool_Int8.cpp:24-72 and its
// gradient NITI_CPUPoolGrad_Int8.cpp:21-77, first max wins), for images with even H, W:
//  forward: rows are pixels of [n][H][W]; pool_out [n][H/2][W/2] gets the window max of the
//           (relu'd) output, which is also written whole to `out`
//  backward: rows are pooled pixels [n][H/2][W/2]; each requantised value goes to the first
//           maximum of its window of x (the forward's pre-pool output, max y) in dx [n][H][W],
//           zero elsewhere and where x <= 0 when relu (NITI_CPUReluGrad_Int8.cpp:28-62)
struct PoolFuse {
    int8_t* pool_out = nullptr;
    const int8_t* x = nullptr;
    const int8_t* y = nullptr;
    int8_t* dx = nullptr;
    int relu = 0;
    int H = 0, W = 0;  // pre-pool image size
    // the pool gradient dx also as the row kernels' C32 layout [n][ld/32][H][W][32] (the next input
    // gradient's operand; separate requant pass without a P16 copy, ld % 32 == 0), or null
    int8_t* dx_c32 = nullptr;
};
// The 3x3 / 2 max pool (pad 1, NITI_Maxpool_Int8.cpp:24-72) over the requantised output: rows =
// pixels [n][H][W]; out [n][OH][OW][ld] the pooled image, arg the same with each window's
// first-max position ky * 3 + kx (maxpool_nhwc16's `arg`); the pre-pool output (ActOut::out) is
// optional.  Separate plain requant pass only (ResNet-18's stem).
struct Pool3 {
    int8_t* out = nullptr;
    int8_t* arg = nullptr;
    int H = 0, W = 0, OH = 0, OW = 0;
};
struct ActOut {
    int8_t* out = nullptr;             // NHWC16 [rows][ld] (may be null with pool.dx or pool3)
    int relu = 0;                      // fused NITI_Relu_Int8
    const int8_t* relu_mask = nullptr; // fused NITI_ReluGrad_Int8 (out = mask > 0 ? q : 0)
    const int8_t* exp_in = nullptr;
    const int8_t* wscale = nullptr;
    int8_t* exp_out = nullptr;
    PoolFuse pool;                     // only where the phase runs as a separate requant pass
    int8_t* out_p16 = nullptr;         // P16 copy of the output (of pool.dx), separate pass only
    // rows = pixels [n][zc_h][zc_w]: pixels of the parity classes (y & 1, x & 1) whose bit
    // 2 (y & 1) + (x & 1) is set in zero_cls are 0 and their accumulators are never read (a stride-2
    // input gradient's tap-less sub-pixel classes; the plain requantise pass only)
    int zero_cls = 0, zc_h = 0, zc_w = 0;
    Pool3 pool3;
};
// whether phase 2 of the forward / input-gradient conv requantises in a separate pass (and so
// can take ActOut::pool); otherwise it recomputes the GEMM with a requantising epilogue
bool conv_fwd_phase2_separate(const ConvGeom& g, size_t ws_bytes);
// the first layer as a K = 32 conv over its im2col copy (1x1 geometry, OW % 32 == 0, OH even):
// range pass + requantise / relu / 2x2 pool pass on register-fed MFMAs (niti_kernels.hip)
bool conv0_ok(const ConvGeom& g);
// pass 0: range into amax; pass 1: requantise with it (a MAX all-reduce may sit between them)
hipError_t conv0_fwd(const ConvGeom& g, const int8_t* xcol, const int8_t* w, uint32_t* amax, const ActOut& o,
                     int pass, hipStream_t st,
                     int8_t* pool_c32 = nullptr, int8_t* out_c32 = nullptr, int8_t* pool_code = nullptr);
bool conv_dgrad_phase2_separate(const ConvGeom& g, size_t ws_bytes);
// The speculative pair on the implicit GEMM (plan strategy 3 = STRAT_SPEC, forward / input
// gradient, no K split; NITI_Conv_Int8.cpp:260-307, NITI_DeConv_Int8.cpp:294-329): pass 0 (launch A)
// multiplies, requantises with the bit width the layer had last time and publishes max|acc| into
// amax (zeroed by the caller); pass 1 (launch B, after any MAX all-reduce of amax) writes the
// exponent and redoes the GEMM, requantised with the max, only when its bit width differs -- on a
// hit every block of B exits at once: one GEMM pass and no int32 tensor.  slot: the layer phase's
// own GEMM_SPEC_SLOT_WORDS zeroed device words ([0] hint, [1] the bit width A used, [2] launches B
// redid, [3] misses B settled from an alternate, [4] the alternates' window: A writes them only
// within GEMM_SPEC_ALT_PAIRS pairs of a miss).  alt (may be null; the same scratch for both
// passes, *_alt_bytes): launch A also writes the output requantised one bit width below and above
// its guess, and launch B settles a +-1 change by copying one instead of redoing the GEMM.  ActOut
// without pool / P16 fusion.  Results equal phase 1 + phase 2's.
constexpr int GEMM_SPEC_SLOT_WORDS = 32;  // one 128-byte line per slot
constexpr int GEMM_SPEC_ALT_PAIRS = 8;
// whether the model autotuners time the speculative pair (NITI_TUNE_SPEC=1)
inline bool tune_spec() {
    static const bool on = getenv("NITI_TUNE_SPEC") && atoi(getenv("NITI_TUNE_SPEC")) == 1;
    return on;
}
bool conv_fwd_spec_ok(const ConvGeom& g);    // the plan (autotuned / forced) is STRAT_SPEC
bool conv_dgrad_spec_ok(const ConvGeom& g);
void gemm_speculate_bias(int bias);  // diagnostics: A guesses the hint + bias (niti_diag_gemm_speculate)
size_t conv_fwd_spec_alt_bytes(const ConvGeom& g);
size_t conv_dgrad_spec_alt_bytes(const ConvGeom& g);
hipError_t conv_fwd_spec(const ConvGeom& g, const int8_t* x, const int8_t* w, uint32_t* amax, const ActOut& o,
                         uint32_t* slot, int pass, hipStream_t st, int8_t* alt = nullptr);
hipError_t conv_dgrad_spec(const ConvGeom& g, const int8_t* dy, const int8_t* wt, uint32_t* amax, const ActOut& o,
                           uint32_t* slot, int pass, hipStream_t st, int8_t* alt = nullptr);
// The implicit GEMM with the rescale fused (plan strategy 4 = STRAT_FUSED, forward / stride-1 input
// gradient, no K split; NITI_Conv_Int8.cpp:260-307, NITI_DeConv_Int8.cpp:294-329): ONE launch whose
// blocks keep their accumulators in registers across an in-kernel grid barrier carrying the tensor's
// bit width (the row kernels' protocol, niti_gridbar.hpp), then requantise -- no int32 tensor and no
// second GEMM pass.  Needs every tile resident at once (checked with the occupancy API) and no rank
// boundary: hipErrorNotSupported (nothing launched) otherwise or when the plan is not STRAT_FUSED,
// and the caller runs phase 1 + phase 2, which take the plan as STRAT_RECOMPUTE.  bar:
// ROWCONV_BAR_WORDS zeroed words per layer phase, epoch its launch count (1 first), err set on a
// barrier timeout.  ActOut without pool / P16 fusion.  Results equal phase 1 + phase 2's.
struct FusedBar {
    uint32_t* bar = nullptr;
    uint32_t epoch = 0;
    uint32_t* err = nullptr;
    uint32_t spin_limit = 0;  // 0: the default
};
unsigned long long gemm_fused_launches();  // (diagnostics: launches that ran fused)
hipError_t conv_fwd_fused(const ConvGeom& g, const int8_t* x, const int8_t* w, const ActOut& o, const FusedBar& fb,
                          hipStream_t st);
hipError_t conv_dgrad_fused(const ConvGeom& g, const int8_t* dy, const int8_t* wt, const ActOut& o, const FusedBar& fb,
                            hipStream_t st);
hipError_t conv_fwd_phase1(const ConvGeom& g, const int8_t* x, const int8_t* w, int32_t* acc, uint32_t* amax,
                           void* ws, size_t ws_bytes, hipStream_t st);
hipError_t conv_fwd_phase2(const ConvGeom& g, const int8_t* x, const int8_t* w, const int32_t* acc,
                           const uint32_t* amax, const ActOut& o, size_t ws_bytes, hipStream_t st);
// subw (may be null): the stride-2 sub-pixel form's class weights (conv_dgrad_subpix_weights, kept
// current by NITI_SGD through SgdJob::subw) where conv_dgrad_subpix_ok: four class GEMMs over dy
hipError_t conv_dgrad_phase1(const ConvGeom& g, const int8_t* dy, const int8_t* wt, int32_t* acc, uint32_t* amax,
                             void* ws, size_t ws_bytes, hipStream_t st, const int8_t* subw = nullptr);
hipError_t conv_dgrad_phase2(const ConvGeom& g, const int8_t* dy, const int8_t* wt, const int32_t* acc,
                             const uint32_t* amax, const ActOut& o, size_t ws_bytes, hipStream_t st,
                             const int8_t* subw = nullptr);
bool conv_dgrad_subpix_ok(const ConvGeom& g);
size_t conv_dgrad_subpix_bytes(const ConvGeom& g);
// the class weights [class (py, px)][ci][taps ky = ky0 + 2 j][taps kx][cop] from IHWO16 wT
hipError_t conv_dgrad_subpix_weights(const ConvGeom& g, const int8_t* wt, int8_t* out, hipStream_t st);

// ---- forward conv of stride-1 pad-1 3x3 layers with the rescale fused (niti_rowconv.hip) -------
// Activations in C32 [n][ceil(C/32)][H][W][32], weights in WF [Co/32][Ci/32][9][2][32][16] (a 1 KiB
// MFMA fragment per (co block, ci block, tap)).  Square H = W in {2, 4, 8, 16}, Cop % 32 == 0.
struct RowConvOut {
    int8_t* out = nullptr;       // NHWC16 [n][H][W][cop] (relu'd)
    int8_t* pool_out = nullptr;  // NHWC16 [n][H/2][W/2][cop] 2x2 max pool of out
    int8_t* next = nullptr;      // C32 copy of the next layer's input (pooled when pool_out)
    const int8_t* exp_in = nullptr;
    const int8_t* wscale = nullptr;
    int8_t* exp_out = nullptr;
    int relu = 0;
    // input gradient (the conv of dy with the rotated transposed weights): the previous layer's
    // relu gradient, out = relu_mask > 0 ? q : 0 (NITI_ReluGrad_Int8) ...
    const int8_t* relu_mask = nullptr;
    // ... or its 2x2 max-pool gradient: q of pooled pixel p goes to the first element of the
    // window in pool_x (2H x 2W, NHWC16) that is >= pool_y[p] (NITI_CPUPoolGrad_Int8), zero
    // elsewhere and, with pool_relu, where pool_x <= 0; written to pool_dx (+ its C32 copy)
    const int8_t* pool_x = nullptr;
    const int8_t* pool_y = nullptr;
    int8_t* pool_dx = nullptr;
    int8_t* pool_dx_next = nullptr;
    int pool_relu = 0;
    // the route as the forward pass that pooled recorded it (pool_code4, NHWC16-shaped [n][H][W][cop]
    // bytes): read instead of pool_x / pool_y, which may then be null
    const int8_t* pool_code = nullptr;
    // forward with pool_out: record that route here (relu decides the code's relu bit)
    int8_t* pool_code_out = nullptr;
    // 0: pool_dx (NHWC16) is not written, only its C32 (pool_dx_next) / P16 copies; the pool
    // gradient's routing still needs pool_dx non-null.  Likewise out may be null in the input
    // gradient when its consumers read the C32 (next) and P16 copies.
    int pool_dx_nhwc = 1;
    // input gradient: the same gradient in the weight gradient's P16 layout (rowconv_p16_ok)
    int8_t* p16 = nullptr;
    // modes RANGE + REQUANT (data parallel: the MAX all-reduce sits between them): the range
    // launch also stores every unit's int32 accumulators here (rowconv_acc_bytes) and the
    // requantise launch reads them back instead of recomputing the GEMM
    int32_t* acc_store = nullptr;
    // the speculative pair's hint slot: 0 forward, 1 input gradient (set by input-gradient callers
    // whose call has no relu / pool / P16 operand, so the two directions never share a slot)
    int dgrad_slot = 0;
    // input layout: 0 C32 [n][C/32][H][W][32]; 1 NHWC16 [n][H][W][cip] (row-segment maps, cip % 32
    // == 0: read in place, no C32 copy)
    int x_nhwc = 0;
};
size_t rowconv_acc_bytes(const ConvGeom& g, bool dg);
bool rowconv_nhwc_ok(const ConvGeom& g);
bool rowconv_nhwc_pref(const ConvGeom& g);
constexpr int ROWCONV_BAR_WORDS = 2 * 19 * 32;  // grid-barrier state (both parities)
static_assert(ROWCONV_BAR_WORDS == NITI_ROWCONV_STATE_WORDS, "header constant");
bool rowconv_ok(const ConvGeom& g);
bool rowconv_seg(const ConvGeom& g);  // the row-segment form (W = 0) takes g
// the input-gradient conv of a stride-1 pad-1 3x3 layer as a forward conv (dy -> dx, ci <-> co);
// false if the layer's input gradient cannot run on the row kernel
bool rowconv_dgrad_geom(const ConvGeom& layer, ConvGeom* d);
// the input-gradient launch of geometry d (rowconv_dgrad_geom) can also write its output's P16
// copy: a wave's pixels make whole 16-pixel blocks (pool: through a 2x2 pool)
bool rowconv_p16_ok(const ConvGeom& d, bool pool);
// FUSED (one launch, in-kernel grid barrier) possible: one unit per wave, every workgroup resident
// dg: for the input-gradient epilogues (at most 4 rows per unit)
bool rowconv_fused_ok(const ConvGeom& g, bool dg = false);
int rowconv_units(const ConvGeom& g, bool dg = false);
size_t rowconv_wf_bytes(int co, int ci);
hipError_t nhwc16_to_c32(const int8_t* in, int n, int hw, int cp, int c, int8_t* out, hipStream_t st);
// C32 [n][cb][hw][32] -> NHWC16 [n][hw][cp] (channels >= c written as zero)
hipError_t c32_to_nhwc16(const int8_t* in, int n, int hw, int cp, int c, int8_t* out, hipStream_t st);
// OHWI16 [co][9][cip] -> WF; transpose: the input-gradient conv's WF (rotate180, ci <-> co)
hipError_t weights_to_wf(const int8_t* w_ohwi16, int co, int ci, int cip, bool transpose, int8_t* out,
                         hipStream_t st);
// mode 0 FUSED (bar, err, epoch != 0 required; epoch + 1 per launch), 1 RANGE (max|y| into amax),
// 2 REQUANT (recompute with the max in amax, requantise, store); 3 / 4 the speculative pair (bar
// required, the same outputs and amax for both): 3 multiplies, requantises with the bit width the
// layer had last time and publishes max|y| into amax; 4 (after any all-reduce of amax) writes the
// exponent and redoes the launch only where the bit width differs -- the results are mode 1 + 2's
constexpr int RC_SPEC_A = 3, RC_SPEC_B = 4;
// whether the model's two-launch row convs take the speculative pair (NITI_RC_SPEC2=0: range +
// recompute-or-stored requantise, A/B diagnostics)
bool rowconv_spec2_on();
// diagnostics: 8 u64 per wave of the following launches (niti_diag_rowconv_stamps), null disarms
void rowconv_stamps_arm(unsigned long long* buf);
// diagnostics: the fused barrier's poll limit (0 = the default) and arrivals it waits for that never
// come (> 0 forces a timeout: the launch sets its err word), for the launches that follow
void rowconv_barrier_diag(uint32_t spin_limit, uint32_t expect_extra);
// the fused mode's speculative epilogue (the previous launch's bit width applied while the barrier
// completes): 1 on (default), 0 off, 2 always guess wrong (diagnostics: every launch redoes it)
void rowconv_speculate(int mode);
// the speculative pair's miss count of a state buffer (forward / input-gradient slot), device words
uint32_t* rowconv_spec_slot(uint32_t* bar, bool dg);
void model_p16_jobs_cap(int cap);  // niti_model.hip, diagnostic
hipError_t rowconv_fwd(const ConvGeom& g, const int8_t* x_c32, const int8_t* wf, const RowConvOut& o, int mode,
                       uint32_t* amax, uint32_t* bar, uint32_t epoch, uint32_t* err, hipStream_t st);
// A 1x1 layer over 1x1 maps (the classifier head) on the same kernel: rows output channels of
// Σ_k x[n][k] w[row][k] (x [n][xld], w [rows][wld], row-major), with the same epilogues (the
// pool-gradient one routes into 2x2 windows: the head's input is a 1x1 pooled map)
// The classifier head's step chain in one launch (niti_head.hip): forward with the rescale, the loss
// gradient, the int32 weight gradient (+ range) and the input gradient routed through the previous
// layer's 2x2 max pool by its recorded codes; no grid barrier (every head workgroup recomputes the
// tiny forward and the input gradient's range).  n % 4 == 0, n <= 512,
// K % 32 == 0, c_out <= 16, cop == 16.
struct HeadChain {
    const int8_t* x = nullptr;  // [n][xld] the head's input (the previous layer's pooled output)
    int xld = 0;
    const int8_t* w = nullptr;   // [c_out][K] (OHWI16 of the 1x1 head)
    const int8_t* wT = nullptr;  // [K][cop] (IHWO16)
    int n = 0, K = 0, c_out = 0, cop = 0, relu = 0;
    const int8_t* exp_in = nullptr;
    const int8_t* wscale = nullptr;
    int8_t* exp_out = nullptr;
    int8_t* logits = nullptr;  // [n][cop]
    const int32_t* labels = nullptr;
    int8_t* dy = nullptr;  // [n][cop]
    int32_t* dw = nullptr;  // [c_out][K]
    uint32_t* dw_amax = nullptr;
    const int8_t* code = nullptr;   // [n][K] the previous layer's pool routes (pool_code4)
    int8_t* pool_dx = nullptr;      // [n][2][2][K] NHWC16, or null
    int8_t* pool_dx_c32 = nullptr;  // [n][K/32][2][2][32], or null
    int8_t* p16 = nullptr;          // [4n/16][K][16], or null
    int G = 0;                      // (set by head_chain: K / 32 head workgroups)
    int stamps = 0;                 // (diagnostics)
};
bool head_chain_ok(int n, int K, int c_out, int cop);
hipError_t head_chain(const HeadChain& h, hipStream_t st);
unsigned long long head_chain_launches();  // (diagnostics)
bool head_chain_enabled();  // NITI_HEAD_CHAIN=1 / niti_diag_head_chain(1); off by default
void head_chain_enable(int on);
bool rowconv_fc_ok(int n, int K, int rows, bool fused);
// its weight gradient: dw [c_out][cip] int32 = Σ_p dy[p][co] x[p][ci] (c_out <= 32, cip % 32 == 0),
// max|dw| published into amax (may be null)
hipError_t head_wgrad(int n, int c_out, int cip, const int8_t* x, int xld, const int8_t* dy, int dld, int32_t* dw,
                      uint32_t* amax, hipStream_t st);
hipError_t rowconv_fc(int n, int K, int rows, const int8_t* x, int xld, const int8_t* w, int wld,
                      const RowConvOut& o, int mode, uint32_t* amax, uint32_t* bar, uint32_t epoch, uint32_t* err,
                      hipStream_t st);

// ---- range estimate + requantisation ----------------------------------------------------
hipError_t absmax_i32(const int32_t* a, int64_t n, uint32_t* amax, hipStream_t st);
// max|a| of several int32 ranges in one launch (b0 is filled in by absmax_many)
struct AbsmaxJob {
    const int32_t* a;
    int64_t n;
    uint32_t* amax;
    uint32_t b0;
};
constexpr int ABSMAX_MAX_JOBS = 24;
struct AbsmaxJobs {
    AbsmaxJob j[ABSMAX_MAX_JOBS];
    int n;
};
hipError_t absmax_many(const AbsmaxJob* jobs, int n, hipStream_t st);

struct ActRequant {
    const int32_t* acc = nullptr;  // [rows][ldc]
    int64_t rows = 0;
    int ldc = 0;                   // multiple of 16 (the padded channel count)
    const uint32_t* amax = nullptr;
    // exponent bookkeeping (device int8 scalars); exp_out = exp_in + wscale + inc
    const int8_t* exp_in = nullptr;
    const int8_t* wscale = nullptr;
    int8_t* exp_out = nullptr;
    int relu = 0;                     // fused NITI_Relu_Int8 (forward)
    const int8_t* relu_mask = nullptr;  // fused NITI_ReluGrad_Int8: out = mask > 0 ? q : 0 (NHWC16)
    int8_t* out_nhwc16 = nullptr;     // [rows][ldc]
    // optional reference-layout copy: MNN C4 [ceil(C/4)][N][HW][4]; rows = N*HW
    int8_t* out_c4 = nullptr;
    int c_real = 0, n = 0, hw = 0;
    PoolFuse pool;  // fused 2x2 max pool / pool gradient (see ActOut)
    // optional P16 copy [pixels/16][ldc][16] of out_nhwc16 (of pool.dx with the pool gradient):
    // the weight-gradient operand of niti_wgrad.hip, written by the same pass
    int8_t* out_p16 = nullptr;
    int zero_cls = 0, zc_h = 0, zc_w = 0;  // as ActOut's (plain pass, no P16 copy)
    Pool3 pool3;                           // as ActOut's (out_nhwc16 optional)
};
hipError_t requant_act(const ActRequant& r, hipStream_t st);
// whether requant_act can write out_p16 for this pass: plain (rows % 16 == 0) or the 2x2 pool
// gradient of a square 2 / 4 / 8 / 16 image
bool requant_p16_ok(const ActRequant& r);

// Gradient rule: bw==0 -> 0, else PSTO(bw - rule).  Optional fused NITI_SGD update
// w <- clip(w - g, +-127) (NITI_SGD.hpp:49-52, BinaryUtils.hpp:278-299).
hipError_t requant_grad(const int32_t* acc, int64_t n, const uint32_t* amax, int rule, int8_t* g_out,
                        int8_t* w_update, hipStream_t st);

// Fused NITI_SGD on an OHWI16 layer: g = rule(acc, amax), w <- clip(w - g, +-127); the new weights
// are also written transposed to wT (IHWO16, may be null) and g to g_out (may be null).
// One layer's NITI_SGD update (rule-2/3 requant of the int32 gradient, w <- clip(w - g),
// transposed copy); sgd_update_many runs several layers' updates in one launch.
struct SgdJob {
    const int32_t* acc;
    const uint32_t* amax;
    int rule, co, ci, kk, cip, cop;
    int8_t* w;
    int8_t* wT;
    int8_t* g_out;
    // 3x3 layers on the register-fed convs (niti_rowconv.hip): the new weights also as the
    // forward's and the input gradient's fragment-major copies (may be null; kk == 9)
    int8_t* wf = nullptr;
    int8_t* wft = nullptr;
    // a stride-2 layer's sub-pixel class weights (conv_dgrad_subpix_weights' layout), or null; pads
    // of the conv (the class of tap (ky, kx) is ((ky - pt) & 1, (kx - pl) & 1)), kh / kw = kk split
    int8_t* subw = nullptr;
    int sub_kw = 0, sub_kh = 0, sub_pt = 0, sub_pl = 0;
    // a deferred split-K combine (the P16 weight gradient's slabs, conv_wgrad_p16 with defer):
    // sgd_update_many first sums `splits` C-shaped slabs `slab_stride` elements apart into acc
    // (slab_n elements) with its range into amax, for every such job in one launch
    const int32_t* slab = nullptr;
    int splits = 0;
    int64_t slab_stride = 0, slab_n = 0;
    // slab layout: 0 = C-shaped (acc index = slab index); 1 = the tap-sharing weight gradient's
    // tile-blocked slabs (wgrad_taps_kernel: 64-row tiles of 72 16-byte columns, mapped back to
    // [co][tap][ci] with these fields; tb_m / tb_s: the magic division by tb_tiles_ci)
    int slab_map = 0;
    int tb_tiles_ci = 0, tb_cip4 = 0, tb_ld4 = 0;
    uint32_t tb_m = 0, tb_s = 0;
};
constexpr int SGD_MAX_JOBS = 24;
struct SgdJobs {
    SgdJob job[SGD_MAX_JOBS];
    int start[SGD_MAX_JOBS];
    int cstart[SGD_MAX_JOBS + 1];  // combine chunks (1024 elements) per job, prefix sums
    int n;
};
hipError_t sgd_update_many(const SgdJob* jobs, int n, hipStream_t st);
// a fully connected layer (1x1 map): its weight gradient's range (pass 0), then the gradient
// recomputed with job j's NITI_SGD step in the GEMM epilogue (pass 1; j.acc, wf, wft and the
// slab fields unused) -- no int32 gradient tensor
bool conv_wgrad_fc_sgd_ok(const ConvGeom& g);
hipError_t conv_wgrad_fc_sgd(const ConvGeom& g, const int8_t* x, const int8_t* dy, uint32_t* amax, const SgdJob& j,
                             int pass, hipStream_t st);
// exponent of a requantised weight gradient: bw - rule (0 for an all-zero gradient)
hipError_t grad_exponent(const uint32_t* amax, int rule, int8_t* out, hipStream_t st);
hipError_t sgd_update(const int32_t* acc, const uint32_t* amax, int rule, int co, int ci, int kk, int cip, int cop,
                      int8_t* w, int8_t* wT, int8_t* g_out, hipStream_t st);

// ---- the rest of the NITI step -----------------------------------------
// (arg: each window's first-max position too, [n][oh][ow][cp] bytes, for maxpool_relu_grad_arg)
hipError_t maxpool_nhwc16(const int8_t* x, int n, int h, int w, int cp, int k, int s, int p, int8_t* y,
                          int oh, int ow, hipStream_t st, int8_t* arg = nullptr);
// dx = maxpool_grad(x, y, dy) then, if relu, dx = x > 0 ? dx : 0 (x is the relu output)
hipError_t maxpool_relu_grad_nhwc16(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h,
                                    int w, int cp, int k, int s, int p, int oh, int ow, int relu,
                                    int8_t* dx, hipStream_t st);
hipError_t relu_grad_nhwc16(const int8_t* x, const int8_t* dy, int64_t n, int8_t* out, hipStream_t st);
// the same gradient in two passes over a workspace of n*oh*ow*cp bytes (each window's first-max
// position, then a gather per input pixel): for overlapping windows (ResNet's 3x3 / 2 stem pool)
hipError_t maxpool_relu_grad_ws(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h, int w, int cp, int k,
                                int s, int p, int oh, int ow, int relu, int8_t* ws, int8_t* dx, hipStream_t st);
// the same from the forward's first-max positions (maxpool_nhwc16 with arg): one pass.  With
// `pooled` (the forward's pooled output y) the relu gradient's mask comes from y instead of x (x
// may be null): a pixel gets a gradient only from windows whose first max it is, where y = x
hipError_t maxpool_relu_grad_arg(const int8_t* x, const int8_t* arg, const int8_t* dy, int n, int h, int w, int cp,
                                 int k, int s, int p, int oh, int ow, int relu, int8_t* dx, hipStream_t st,
                                 const int8_t* pooled = nullptr);
// logits int8 [batch][ld] (first `classes` used), labels int32 [batch] (class index);
// out int8 [batch][ld] (padded lanes zeroed).  classes <= 2048 (one thread per sample up to 16,
// one block per sample above).  NITI_CPULossGrad_Int8.cpp:81-200.
hipError_t loss_grad(const int8_t* logits, int batch, int classes, int ld, const int8_t* ascale,
                     const int32_t* labels, int8_t* out, hipStream_t st);

// ---- input quantiser (MnistUtils.cpp:83-93; niti_quant.hip states the exact contract) -------
// stats (4 x u64, device) = {S1 = sum x, S2 = sum x^2, xmax, 255 - xmin} of n uint8 pixels
hipError_t image_stats(const uint8_t* img, int64_t n, unsigned long long* stats, hipStream_t st);
// x = round((p - mean) / std / range * 127) from stats over `count` pixels (count > n*c*hw when
// the statistics were all-reduced over data-parallel ranks); out NHWC16 [n][hw][cp] (nhwc16) or
// NCHW; *ascale = int8(ceil(ln(range)) - 7) (ascale may be null)
hipError_t image_quantize(const uint8_t* img, int n, int c, int hw, int cp, const unsigned long long* stats,
                          int64_t count, int8_t* out, int8_t* ascale, bool nhwc16, hipStream_t st);
// the training step's form: per-block partial statistics (IMAGE_STATS_SLOTS x 4 u64, no
// atomics), summed by their consumer; stats_finalize sums them into stats[4] (data parallel:
// before the all-reduce)
constexpr int IMAGE_STATS_SLOTS = 256;
// (zero / zero_bytes, multiple of 16: a buffer the same launch zeroes, e.g. the step's range words)
hipError_t image_stats_slots(const uint8_t* img, int64_t n, unsigned long long* slots, int* nslots, hipStream_t st,
                             void* zero = nullptr, size_t zero_bytes = 0);
hipError_t stats_finalize(const unsigned long long* slots, int nslots, unsigned long long* stats, hipStream_t st);
// the first layer's im2col copy (xcol [n*oh*ow][32]) straight from the NCHW batch: uint8 images
// quantised with the statistics in `slots` (nslots partials over `count` pixels), or int8 pixels
// as they are (quant = false); x_nchw (may be null) receives the int8 input; stride 1, C / KH / KW
// = 3/3/3 or 1/5/5 (input_im2col_ok)
bool input_im2col_ok(int c, int kh, int kw);
// optional: the first conv's range (NITI_RangeEstimate of its int32 output) from the im2col rows as
// they are built -- w [co][32] (the K = 32 conv0 weights), cop <= 64 -- published into amax
struct Conv0Range {
    const int8_t* w = nullptr;
    int co = 0, cop = 0;
    uint32_t* amax = nullptr;
};
hipError_t input_im2col(const void* in, bool quant, int n, int c, int h, int w, int kh, int kw, int pt, int pl,
                        const unsigned long long* slots, int nslots, int64_t count, int8_t* x_nchw, int8_t* xcol,
                        int8_t* ascale, hipStream_t st, const Conv0Range& r0 = Conv0Range{});

// ---- layout transforms --------------------------------------------------------------------
// NHWC16 [N][H][W][Cp] -> CHWN16 [Cp][H][W][Np]
hipError_t nhwc16_to_chwn16(const int8_t* in, int n, int hw, int cp, int np, int8_t* out, hipStream_t st);
// OHWI16 [Co][KK][Cip] -> IHWO16 [Ci][KK][Cop]
hipError_t ohwi16_to_ihwo16(const int8_t* w, int co, int ci, int kk, int cip, int cop, int8_t* wt,
                            hipStream_t st);
// reference-layout conversions (drop-in boundary)
hipError_t c4_to_nhwc16(const int8_t* x_c4, int n, int c, int hw, int cp, int8_t* out, hipStream_t st);
hipError_t nchw_to_nhwc16(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, hipStream_t st);
hipError_t nchw_to_chwn16(const int8_t* x, int n, int c, int hw, int cp, int np, int8_t* out,
                          hipStream_t st);
hipError_t c4_to_chwn16(const int8_t* x_c4, int n, int c, int hw, int cp, int np, int8_t* out,
                        hipStream_t st);
hipError_t nhwc16_to_nchw(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, hipStream_t st);
// reverse_taps: NITI_DeConv_Int8's rotate180 (NITI_DeConv_Int8.cpp:179-184) reverses each KH*KW plane
hipError_t oihw_to_ohwi16(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, hipStream_t st,
                          bool reverse_taps = false);
hipError_t oihw_to_ihwo16(const int8_t* w, int co, int ci, int kk, int cop, int8_t* out, hipStream_t st);
// OHWI16 int8 -> OIHW (drop the channel padding)
hipError_t ohwi16_to_oihw(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, hipStream_t st);
// row-major [rows][cols] int8 -> zero-padded [rows][ld] (ld multiple of 16)
hipError_t pad_rows(const int8_t* in, int rows, int cols, int ld, int8_t* out, hipStream_t st);
// [rows][ld] int32 -> transpose [cols][rows] int32 (cols <= ld)
hipError_t transpose_i32(const int32_t* in, int rows, int cols, int ld, int32_t* out, hipStream_t st);

}  // namespace niti
