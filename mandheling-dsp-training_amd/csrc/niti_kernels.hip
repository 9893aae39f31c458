// niti_kernels.hip -- gfx950 (MI355X / CDNA4) kernels for the NITI int8 training path.
//
// The three GEMM-class ops of the reference (NITI_Conv_Int8, NITI_GradientConv_Int8 /
// NITI_Matmul_Int8 / NITI_DSPMatmulGradientConv_Int8, NITI_DeConv_Int8) are one
// implicit-GEMM kernel template on v_mfma_i32_32x32x32_i8 with exact int32
// accumulation; the im2col gather happens in the global->LDS staging of each operand
// (an operand "loader" per op), never as a materialised column buffer.  The per-layer
// power-of-two rescale (NITI_RangeEstimate + NITI_MNNPstoShiftInt32,
// CommonOptFunction.cpp:1565-1627) is split around a grid-wide max: the GEMM epilogue
// reduces max|acc| per workgroup and atomically max-es it into one word; the requant
// kernel reads that word (after a kernel boundary -- or an RCCL all-reduce(MAX) in
// data-parallel exact mode) and applies the shift.
#include <stdlib.h>

#include <map>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <vector>
#include <algorithm>
#include <stdio.h>

#include <hip/hip_ext.h>

#include "niti_device.hpp"
#include "niti_gridbar.hpp"
#include "niti_kernels.hpp"
#include "niti_sgd.hpp"
#include "niti_map.hpp"

namespace niti {


bool ConvGeom::finalize() {
    if (n <= 0 || c_in <= 0 || h <= 0 || w <= 0 || c_out <= 0 || kh <= 0 || kw <= 0) return false;
    if (sh <= 0 || sw <= 0 || dh <= 0 || dw <= 0) return false;
    const int keh = dh * (kh - 1) + 1, kew = dw * (kw - 1) + 1;
    if (pt < 0 || pb < 0 || pl < 0 || pr < 0) return false;
    // reject before dividing: C++ division truncates toward zero, so a negative numerator
    // smaller than the stride would otherwise still give oh = 1
    if (h + pt + pb < keh || w + pl + pr < kew) return false;
    oh = (h + pt + pb - keh) / sh + 1;  // ShapeNITI_Conv_Int8.cpp:58-76
    ow = (w + pl + pr - kew) / sw + 1;
    cip = round_up(c_in, 16);
    cop = round_up(c_out, 16);
    np = round_up(n, 16);
    return oh > 0 && ow > 0;
}

__device__ __forceinline__ v4i zero4() {
    v4i z = {0, 0, 0, 0};
    return z;
}

// =====================================================================================
// Operand loaders.  Each GEMM row's K dimension is a sequence of 16-byte chunks; a loader
// turns (row, chunk) into a byte offset inside one tensor, or OOB (>= 2^31) for a zero
// chunk (padding, out-of-image taps, rows past M, chunks past the K split).  Loads are
// raw buffer loads, so an OOB offset reads zeros without a branch.  Per-thread iterators
// advance by one K step (a template chunk count) with compares instead of divisions.
// =====================================================================================

// Forward conv, A operand: row m = output pixel (n, oy, ox) of an NHWC16 input, K-chunk
// kc = (ky, kx, cc) with cc the 16-channel group (the im2col of Int8FunctionsOpt.cpp:342-392,
// channel-contiguous and never materialised).
struct LoadConvFwd {
    const int8_t* x;
    uint32_t bytes;
    int H, W, CPC, OH, OW, KW, sh, sw, pt, pl, dh, dw, M, kc_total;
    uint32_t img;  // bytes per image
    __device__ __forceinline__ const int8_t* ptr() const { return x; }
    struct It {
        uint32_t base;
        int iy0, ix0, ky, kx, cc, kc;
        bool ok;
    };
    __device__ __forceinline__ It begin(int m, int kc) const {
        It t;
        t.ok = m < M;
        const int mm = t.ok ? m : 0;
        const int ox = mm % OW, r = mm / OW, oy = r % OH, n = r / OH;
        t.base = (uint32_t)n * img;
        t.iy0 = oy * sh - pt;
        t.ix0 = ox * sw - pl;
        const int tap = kc / CPC;
        t.cc = kc - tap * CPC;
        t.ky = tap / KW;
        t.kx = tap - t.ky * KW;
        t.kc = kc;
        return t;
    }
    template <int S>
    __device__ __forceinline__ void next(It& t) const {
        t.kc += S;
        t.cc += S;
        while (t.cc >= CPC) {
            t.cc -= CPC;
            if (++t.kx == KW) {
                t.kx = 0;
                ++t.ky;
            }
        }
    }
    __device__ __forceinline__ uint32_t off(const It& t, int kc_end) const {
        const int iy = t.iy0 + t.ky * dh, ix = t.ix0 + t.kx * dw;
        const bool ok = t.ok && t.kc < kc_end && t.kc < kc_total && (unsigned)iy < (unsigned)H &&
                        (unsigned)ix < (unsigned)W;
        return ok ? t.base + ((uint32_t)(iy * W + ix) * CPC + t.cc) * 16u : OOB;
    }
};

// Input-gradient conv, A operand: row m = input pixel (n, iy, ix), K-chunk = (ky, kx, cc)
// over the NHWC16 output gradient, oy = (iy + pt - ky*dh) / sh when divisible.  This is the
// transposed convolution the reference builds from pad(dilate(dy)) and rot180(w^T)
// (grad/NITI_Conv_Int8_Grad.cpp:29-122, NITI_DeConv_Int8.cpp:179-219).
struct LoadConvDgrad {
    const int8_t* dy;
    uint32_t bytes;
    int OH, OW, CPC, H, W, KW, sh, sw, pt, pl, dh, dw, M, kc_total;
    uint32_t img;
    __device__ __forceinline__ const int8_t* ptr() const { return dy; }
    struct It {
        uint32_t base;
        int ty0, tx0, ky, kx, cc, kc;
        bool ok;
    };
    __device__ __forceinline__ It begin(int m, int kc) const {
        It t;
        t.ok = m < M;
        const int mm = t.ok ? m : 0;
        const int ix = mm % W, r = mm / W, iy = r % H, n = r / H;
        t.base = (uint32_t)n * img;
        t.ty0 = iy + pt;
        t.tx0 = ix + pl;
        const int tap = kc / CPC;
        t.cc = kc - tap * CPC;
        t.ky = tap / KW;
        t.kx = tap - t.ky * KW;
        t.kc = kc;
        return t;
    }
    template <int S>
    __device__ __forceinline__ void next(It& t) const {
        t.kc += S;
        t.cc += S;
        while (t.cc >= CPC) {
            t.cc -= CPC;
            if (++t.kx == KW) {
                t.kx = 0;
                ++t.ky;
            }
        }
    }
    __device__ __forceinline__ uint32_t off(const It& t, int kc_end) const {
        const int ty = t.ty0 - t.ky * dh, tx = t.tx0 - t.kx * dw;
        int oy = ty, ox = tx;
        bool ok = t.ok && t.kc < kc_end && t.kc < kc_total && ty >= 0 && tx >= 0;
        if (sh != 1) {
            oy = ty / sh;
            ok = ok && oy * sh == ty;
        }
        if (sw != 1) {
            ox = tx / sw;
            ok = ok && ox * sw == tx;
        }
        ok = ok && oy < OH && ox < OW;
        return ok ? t.base + ((uint32_t)(oy * OW + ox) * CPC + t.cc) * 16u : OOB;
    }
};

// =====================================================================================
// Range estimate and PSTO helpers (used by the GEMM epilogue and the requant kernels)
// =====================================================================================

// (bitwidth_of, clip127, pow2_x86, psto_fast / psto_generic / psto_any: niti_sgd.hpp)


// =====================================================================================
// The GEMM: C[m][n] = sum_k A[m][k] * B[n][k], int8 x int8 -> exact int32.
//   256 threads = 4 waves; BM x BN block tile; 4-stage LDS pipeline (gemm_kernel below).
//   Workgroups are remapped so each XCD walks a contiguous range of tiles (A-row panels
//   stay in one L2).
// Epilogues:
//   EPI_STORE    int32 C + max|C| (one word, agent-scope atomic)
//   EPI_AMAX     max|C| only                          (first pass of the recompute strategy)
//   EPI_REQUANT  reads the max word, applies the NITI forward shift rule, writes int8
//                (+ fused relu / relu-grad mask, + exponent)   (second pass)
//   EPI_SLAB     int32 partial sums of one K split -> slab[split] (reduced later)
//   EPI_SGD      reads the weight gradient's max word, applies NITI_SGD to the weights in place
//                (the second pass of a fully connected layer's weight gradient)
// =====================================================================================
// K bytes per step (KT = false) is the A loader's BK: 128 (full 128-byte lines per row and
// step) where the operand allows it, else 64.

enum EpiMode { EPI_STORE = 0, EPI_AMAX = 1, EPI_REQUANT = 2, EPI_SLAB = 3, EPI_SGD = 4 };

// Output row map of a sub-pixel class GEMM (the stride-2 input gradient, conv_dgrad_phase1): GEMM
// row m = (img, my, mx) of the class grid [n][hc][wc] is pixel (img, sy*my + py, sx*mx + px) of the
// [n][h][w] output.  off: rows are output pixels as they stand.
struct RowMap {
    int on = 0;
    int hc = 0, wc = 0, h = 0, w = 0, py = 0, px = 0, sy = 2, sx = 2;
};
__device__ __forceinline__ int64_t map_row(const RowMap& m, int row) {
    if (!m.on) return row;
    const int mx = row % m.wc, t = row / m.wc, my = t % m.hc, img = t / m.hc;
    return ((int64_t)img * m.h + m.sy * my + m.py) * m.w + m.sx * mx + m.px;
}

struct Epi {
    int32_t* C = nullptr;  // STORE: C; SLAB: slab base
    int64_t ldc = 0;
    int64_t slab_stride = 0;  // elements between K-split slabs
    int split_major = 0;      // XCD-aware order over (split, tile) instead of tiles only
    uint32_t* amax = nullptr;
    int8_t* out = nullptr;  // REQUANT output [M][ldo]
    int64_t ldo = 0;
    int relu = 0;
    const int8_t* relu_mask = nullptr;  // [M][ldo]
    const int8_t* exp_in = nullptr;
    const int8_t* wscale = nullptr;
    int8_t* exp_out = nullptr;
    unsigned long long* span = nullptr;  // kernel-span probe slot (probe_span_arm)
    // the speculative pair (plan strategy STRAT_SPEC, EPI_REQUANT only): spec 1 = launch A --
    // requantise with the bit width hint[0] gives (the layer's previous one on its input's scale,
    // spec_pick; 0 none) and publish
    // max|C| into amax; spec 2 = launch B -- every block exits at once unless the max's bit width
    // differs from the one A used (hint[1]), and otherwise requantises with it.  Slot words as the
    // row kernels' (niti_rowconv.hip spec_guess / spec_settle): [0] hint (written by B), [1] the guess
    // A used (written by A), [2] launches B redid.
    int spec = 0;
    uint32_t* hint = nullptr;
    int hint_scale = 0;  // the hint on the input's scale (forward) or bare (input gradient)
    // launch A also writes the output requantised one bit width below and above its guess into
    // alt[0 .. M*ldo) / alt[M*ldo .. 2*M*ldo) (may be null): launch B then settles a +-1 change --
    // the common miss, a max near a power of two -- by copying instead of redoing the GEMM
    int8_t* alt = nullptr;
    int spec_bias = 0;  // diagnostics (niti_diag_gemm_speculate): launch A guesses hint + bias
    // EPI_SGD (the fully connected layers' weight gradient recomputed after its range pass): the
    // update in the epilogue -- weights [M][ldo], their transpose [sgd_ci][sgd_ldt], int8 gradient
    int8_t* sgd_w = nullptr;
    int8_t* sgd_wT = nullptr;
    int8_t* sgd_g = nullptr;
    int sgd_rule = 0, sgd_ci = 0;
    int64_t sgd_ldt = 0;
    RowMap rmap;  // STORE / REQUANT: where GEMM row m lands (sub-pixel classes)
    // REQUANT with the rescale fused (plan strategy STRAT_FUSED, every tile resident): each block
    // keeps its accumulators in registers across the row kernels' in-kernel grid barrier, which
    // carries the tensor's bit width (niti_gridbar.hpp), then requantises -- no int32 tensor, no
    // second pass.  bar: ROWCONV_BAR_WORDS words, epoch: this state's launch count (1 first).
    uint32_t* bar = nullptr;
    uint32_t epoch = 0;
    uint32_t* err = nullptr;
    uint32_t spin_limit = 0;
};

// the input's scale for the pair's hint (spec_pick, niti_device.hpp): exponent in + weight scale
__device__ __forceinline__ int gemm_spec_escale(const Epi& epi) {
    if (!epi.hint_scale) return 0;
    return __builtin_amdgcn_readfirstlane((epi.exp_in ? (int)*epi.exp_in : 0) + (epi.wscale ? (int)*epi.wscale : 0));
}

// launch B of the pair: the rule's bit width of the (all-reduced) max against the one A used
// (hint[1] = bw + 1); block 0 writes the exponent and the next hint.  Returns 0 when A's output
// stands (every block of B then exits), 1 / 2 when A's alternate one bit width below / above holds
// it (B copies it over the output), -1 when the GEMM must be redone.  Called by whole waves
// (read_max: one slot per lane).
__device__ __forceinline__ int gemm_spec_settle(const Epi& epi) {
    const uint32_t g = read_max(epi.amax);
    const int bw = bitwidth_of(g);
    const uint32_t h1 = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(epi.hint + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const int used = (int)(h1 & 0x7fffffffu) - 1;
    const bool alts = (h1 >> 31) != 0u;  // A wrote the alternates
    const int esc = gemm_spec_escale(epi);  // (before the exponent write: exp_out may alias exp_in)
    const int act = bw == used ? 0 : !alts ? -1 : (bw == used - 1 && used >= 1) ? 1 : bw == used + 1 ? 2 : -1;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) spec_learn(epi.hint, bw, esc, threadIdx.x);
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        if (act >= 0 && epi.exp_out != nullptr) {  // (a redo writes it in its epilogue)
            const int shift = bw - 7;
            const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
            *epi.exp_out = (int8_t)((epi.exp_in ? (int)*epi.exp_in : 0) + (epi.wscale ? (int)*epi.wscale : 0) + inc);
        }
        if (act < 0) __hip_atomic_fetch_add(epi.hint + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (act > 0) __hip_atomic_fetch_add(epi.hint + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the alternates' window: a miss opens it for the next GEMM_SPEC_ALT_PAIRS pairs, a hit
        // narrows it (a layer whose bit width holds pays for one output only)
        const uint32_t win = __hip_atomic_load(epi.hint + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(epi.hint + 4, act != 0 ? (uint32_t)GEMM_SPEC_ALT_PAIRS : (win > 0u ? win - 1u : 0u),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return act;
}



// Shared epilogue: D[row][col] of the 32x32 MFMA tiles, row = (i&3) + 8*(i>>2) + 4*(lane>>5),
// col = lane&31.  `smem` is reused for the block max (every LDS read finished at the last barrier).
// REQUANT: the int8 values leave as dwords of 4 columns of one row, packed in registers (see
// below); the relu-grad mask is applied in the same pass.
// whether the STORE / SLAB epilogue stages the int32 tile through LDS (tiles up to 128 x 128)
constexpr bool epi_stage_c(int mode, int bm, int bn) {
    return (mode == EPI_STORE || mode == EPI_SLAB) && bm * (bn + 4) * 4 <= 72 * 1024;
}

template <int TM, int TN, int NW, int MODE, int BM, int BN>
__device__ __forceinline__ void gemm_epilogue(v16i (&acc)[TM][TN], int r0, int c0, int M, int N, const Epi& epi,
                                              int8_t* smem, int split, int m0, int n0) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    int rq_shift = 2;
    bool rq_raw = false;
    // launch A of the speculative pair: requantise with the hinted bit width, publish the max
    const bool spec_a = MODE == EPI_REQUANT && epi.spec == 1;
    const bool fused = MODE == EPI_REQUANT && epi.bar != nullptr;
    int abw = 0;             // the bit width launch A requantises with
    bool spec_alts = false;  // and whether it writes the alternates
    int fused_bw = 0;
    if (fused) {
        // NITI_RangeEstimate over the whole tensor (NITI_Conv_Int8.cpp:260) through the grid barrier:
        // this block's max|acc| over its valid outputs, its bit width ORed in, the grid's read back
        uint32_t m = 0;
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const int col = c0 + b * 32 + (lane & 31);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int row = r0 + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
                    const uint32_t u = row < M && col < N ? uabs32(acc[a][b][i]) : 0u;
                    m = m > u ? m : u;
                }
            }
        m = wave_max(m);
        uint32_t* red = (uint32_t*)smem;  // (every LDS read of the K loop / exchange is finished)
        if (lane == 0) red[wid] = m;
        __syncthreads();
        if (wid == 0) {
            uint32_t bm = red[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) bm = bm > red[i] ? bm : red[i];
            grid_bw_arrive(epi.bar, epi.epoch, bitwidth_of(bm), lane);
            const int gbw = grid_bw_wait(epi.bar, epi.epoch, epi.err, epi.spin_limit, 0u, lane);
            if (lane == 0) red[NW] = (uint32_t)gbw;
        }
        __syncthreads();
        fused_bw = __builtin_amdgcn_readfirstlane((int)red[NW]);
    }
    if (MODE == EPI_REQUANT) {
        int bw;
        if (fused) {
            bw = fused_bw;
        } else if (spec_a) {
            uint32_t f = 0;
            const uint32_t h = spec_pick_e(epi.hint, epi.exp_in, epi.wscale, epi.hint_scale != 0, &f);  // bw + 1
            bw = (int)h - 1;  // no hint yet: 0 (B redoes unless the max is 0)
            if (h != 0u) bw += epi.spec_bias;
            if (bw < 0) bw = 0;
            abw = bw;
            // the alternates only while the window a recent miss opened lasts (hint[4], written by B)
            spec_alts = epi.alt != nullptr &&
                        __builtin_amdgcn_readfirstlane((int)__hip_atomic_load(epi.hint + 4, __ATOMIC_RELAXED,
                                                                              __HIP_MEMORY_SCOPE_AGENT)) != 0;
            if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0)
                __hip_atomic_store(epi.hint + 1, ((uint32_t)bw + 1u) | (spec_alts ? 0x80000000u : 0u), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            bw = bitwidth_of(read_max(epi.amax));
        }
        const int shift = bw - 7;  // NITI_Conv_Int8.cpp:262-307
        rq_shift = shift > 1 ? shift : 2;
        rq_raw = shift <= 0;
        if (!spec_a && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0 && epi.exp_out != nullptr) {
            const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
            const int ein = epi.exp_in ? (int)*epi.exp_in : 0;
            const int ws = epi.wscale ? (int)*epi.wscale : 0;
            *epi.exp_out = (int8_t)(ein + ws + inc);
        }
    }
    int32_t* Cs = MODE == EPI_SLAB ? epi.C + (int64_t)split * epi.slab_stride : epi.C;
    constexpr bool STAGE_C = epi_stage_c(MODE, BM, BN);
    constexpr int LDT = BN + 4;  // int32 row pitch of the staged C tile (STORE / SLAB)
    int32_t* ctile = (int32_t*)smem;
    uint32_t lmax = 0;
    if (MODE != EPI_REQUANT || spec_a) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const int col = c0 + b * 32 + (lane & 31);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int row = r0 + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
                    const int v = acc[a][b][i];
                    if (STAGE_C) ctile[(row - m0) * LDT + (col - n0)] = v;
                    if (row < M && col < N) {
                        if (!STAGE_C && (MODE == EPI_STORE || MODE == EPI_SLAB)) Cs[map_row(epi.rmap, row) * epi.ldc + col] = v;
                        if (MODE == EPI_STORE || MODE == EPI_AMAX || spec_a) {
                            const uint32_t u = uabs32(v);
                            lmax = lmax > u ? lmax : u;
                        }
                    }
                }
            }
    }
    if (MODE == EPI_REQUANT) {
        // Straight from the accumulators, no LDS: a lane holds 4 consecutive rows of one column per
        // 4 accumulator registers; a 4 x 4 byte transpose inside each lane quad (two DPP swaps, two
        // byte permutes) gives it 4 consecutive columns of one row -- a dword store; the 8 quads of a
        // half-wave write 32 contiguous bytes of each of 4 rows.
        const int j = lane & 3;
        const int col4 = c0 + 4 * ((lane & 31) >> 2);  // + b * 32: the dword's first column
        auto put = [&](int sh, bool raw, int8_t* dst) {
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        uint32_t d = 0;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int v = acc[a][b][4 * gq + r];
                            int32_t q = raw ? (int32_t)(int8_t)v : psto_any(v, sh);
                            if (epi.relu && q < 0) q = 0;
                            d |= ((uint32_t)q & 0xffu) << (8 * r);
                        }
                        d = quad_transpose(d, j);  // byte r of lane k = (row r, column k) -> byte k of lane r
                        const int row = r0 + a * 32 + 8 * gq + 4 * (lane >> 5) + j;
                        const int col = col4 + b * 32;
                        if (row < M && col < N) {  // N is a multiple of 16
                            const int64_t o = map_row(epi.rmap, row) * epi.ldo + col;
                            if (epi.relu_mask != nullptr) {
                                const uint32_t mk = *(const uint32_t*)(epi.relu_mask + o);
                                uint32_t keep = 0;
#pragma unroll
                                for (int k = 0; k < 4; ++k)
                                    keep |= ((int8_t)(mk >> (8 * k)) > 0 ? 0xffu : 0u) << (8 * k);
                                d &= keep;
                            }
                            *(uint32_t*)(dst + o) = d;
                        }
                    }
        };
        put(rq_shift, rq_raw, epi.out);
        if (spec_a && spec_alts) {
            // the alternates: the same tile requantised one bit width below / above the guess
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int sh = (k == 0 ? (abw > 0 ? abw - 1 : 0) : abw + 1) - 7;
                put(sh > 1 ? sh : 2, sh <= 0, epi.alt + (int64_t)k * M * epi.ldo);
            }
        }
    }
    if (MODE == EPI_SGD) {
        // NITI_SGD on the weight-gradient tile (NITI_GradientConv_Int8.cpp:274-296, NITI_SGD.hpp:20-54):
        // g = PSTO(C, bw - rule), w <- clip(w - g, +-127) with w [M][ldo] (OHWI16, one tap), the
        // int8 gradient to sgd_g, and the new weights transposed into sgd_wT [sgd_ci][sgd_ldt] (IHWO16)
        // through an LDS tile, leaving as 16-byte row chunks.  Every weight of the tile is loaded
        // before the first store (the stores to w could alias later loads: issued in between, each
        // load would wait for a memory round trip of its own).
        const int bw = bitwidth_of(read_max(epi.amax));
        const int sh = bw - epi.sgd_rule;
        const int j = lane & 3;
        const int col4 = c0 + 4 * ((lane & 31) >> 2);
        uint32_t wv[TM][TN][4];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int row = r0 + a * 32 + 8 * gq + 4 * (lane >> 5) + j, col = col4 + b * 32;
                    wv[a][b][gq] = row < M && col < N ? *(const uint32_t*)(epi.sgd_w + (int64_t)row * epi.ldo + col) : 0u;
                }
        __syncthreads();  // (LDS: every wave is past the main loop's last reads)
        constexpr int TP = BM + 16;  // byte pitch of the transposed tile [BN][TP]
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    uint32_t gd = 0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int32_t q = bw == 0 ? 0 : psto_any(acc[a][b][4 * gq + r], sh);
                        gd |= ((uint32_t)q & 0xffu) << (8 * r);
                    }
                    gd = quad_transpose(gd, j);
                    const int row = r0 + a * 32 + 8 * gq + 4 * (lane >> 5) + j;
                    const int col = col4 + b * 32;
                    uint32_t wn = 0;
                    if (row < M && col < N) {
                        const int64_t o = (int64_t)row * epi.ldo + col;
                        const uint32_t wo = wv[a][b][gq];
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            wn |= ((uint32_t)clip127((int32_t)(int8_t)(wo >> (8 * k)) - (int32_t)(int8_t)(gd >> (8 * k))) &
                                   0xffu)
                                  << (8 * k);
                        *(uint32_t*)(epi.sgd_w + o) = wn;
                        if (epi.sgd_g != nullptr) *(uint32_t*)(epi.sgd_g + o) = gd;
                    }
                    // back to 4 rows of one column: a dword of the transposed tile
                    const uint32_t wt = quad_transpose(wn, j);
                    const int trow = a * 32 + 8 * gq + 4 * (lane >> 5) + (r0 - m0), tcol = b * 32 + (lane & 31) + (c0 - n0);
                    *(uint32_t*)(smem + tcol * TP + trow) = wt;
                }
        __syncthreads();
        if (epi.sgd_wT != nullptr) {
            constexpr int CPR = BM / 16;  // 16-byte chunks per transposed row
            for (int t = tid; t < BN * CPR; t += NW * 64) {
                const int cl = t / CPR, rl = (t - cl * CPR) * 16;
                if (n0 + cl < epi.sgd_ci && m0 + rl < epi.sgd_ldt)
                    *(v16c*)(epi.sgd_wT + (int64_t)(n0 + cl) * epi.sgd_ldt + m0 + rl) = *(const v16c*)(smem + cl * TP + rl);
            }
        }
    }
    if (STAGE_C) {
        // the int32 tile leaves as whole 16-byte row chunks (one dword per lane per MFMA row
        // would be 4x the store instructions, and store issue bounds this epilogue)
        __syncthreads();
        constexpr int CPR = BN / 4;
        for (int t = tid; t < BM * CPR; t += NW * 64) {
            const int rl = t / CPR, cl = (t - rl * CPR) * 4;
            const int row = m0 + rl, col = n0 + cl;
            if (row < M && col < N)  // N is a multiple of 16
                *(v4i*)(Cs + map_row(epi.rmap, row) * epi.ldc + col) = *(const v4i*)(ctile + rl * LDT + cl);
        }
    }
    if (MODE == EPI_STORE || MODE == EPI_AMAX || spec_a) {
        lmax = wave_max(lmax);
        __syncthreads();  // LDS reads of the staged tile / the last K step are finished
        uint32_t* red = (uint32_t*)smem;
        if (lane == 0) red[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            uint32_t m = red[0];
            for (int i = 1; i < NW; ++i) m = m > red[i] ? m : red[i];
            if (epi.amax != nullptr) publish_max(epi.amax, m);
        }
    }
}

// =====================================================================================
// K-major GEMM for the weight gradient: C[m][n] = sum_k A[k][m] * B[k][n].
// The reduction runs over pixels (n, oy, ox), which are the OUTER index of the NHWC16
// activations.  Both operand tiles are staged into LDS as they lie in HBM -- [k rows][16-byte
// column chunks], i.e. NHWC rows of dy and im2col rows of x -- and the MFMA fragments are
// read transposed with ds_read_b64_tr_b8 (gfx950): per 16-lane group, lane 2q+p names row q,
// columns 8p..8p+7 of an 8 x 16 byte block, and lane j receives column j of the 8 rows.  Two
// such reads give a lane the 16 consecutive k of its column that v_mfma_i32_32x32x32_i8
// expects.  No transposed copy of any activation is ever written to HBM.
// =====================================================================================
constexpr int KT_BK = 64;  // k rows (pixels) per step


// 16-byte chunk c of LDS row r (BM bytes per row) lives at chunk c ^ swz(r): the 32 lanes of
// a half-wave transposed read (8 consecutive rows x 4 eight-byte columns) then cover all 64
// banks once.
template <int BW>
__device__ __forceinline__ int kt_swz(int r) {
    return BW == 256 ? (r & 7) * 2 : (BW == 128 ? ((r >> 1) & 3) * 2 : (BW == 64 ? ((r >> 2) & 1) * 2 : 0));
}
template <int BW>
__device__ __forceinline__ int kt_off16(int r, int c) { return r * BW + ((c ^ kt_swz<BW>(r)) << 4); }
template <int BW>
__device__ __forceinline__ int kt_off8(int r, int c8) {
    return r * BW + (((c8 >> 1) ^ kt_swz<BW>(r)) << 4) + ((c8 & 1) << 3);
}

__device__ __forceinline__ v2i ds_tr8(const int8_t* p) {
    return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(p));
}

// B operand of the weight gradient: column n' = (ky, kx, ci) of the OHWI16 gradient, row k =
// output pixel (n, oy, ox); the value is x[n][oy*sh - pt + ky*dh][ox*sw - pl + kx*dw][ci]
// from an NHWC16 activation (zero outside the image).
struct KtIm2col {
    const int8_t* x;
    uint32_t bytes;
    int H, W, OH, OW, CIP, KW, sh, sw, pt, pl, dh, dw, ncols, K;
    FastDiv fOW, fOH;
    __device__ __forceinline__ const int8_t* ptr() const { return x; }
    struct It {
        int k, ci0, offy, offx;
        bool ok;
    };
    __device__ __forceinline__ It begin(int k, int c16) const {
        It t;
        const int nn = c16 * 16;
        t.ok = nn < ncols;
        const int tap = t.ok ? nn / CIP : 0;
        t.ci0 = nn - tap * CIP;
        const int ky = tap / KW, kx = tap - ky * KW;
        t.offy = ky * dh - pt;
        t.offx = kx * dw - pl;
        t.k = k;
        return t;
    }
    template <int S>
    __device__ __forceinline__ void next(It& t) const { t.k += S; }
    __device__ __forceinline__ uint32_t off(const It& t, int k_end) const {
        if (!t.ok || t.k >= k_end || t.k >= K) return OOB;
        const uint32_t q = fdiv(fOW, (uint32_t)t.k);
        const int ox = t.k - (int)q * OW;
        const uint32_t n = fdiv(fOH, q);
        const int oy = (int)q - (int)n * OH;
        const int iy = oy * sh + t.offy, ix = ox * sw + t.offx;
        if ((unsigned)iy >= (unsigned)H || (unsigned)ix >= (unsigned)W) return OOB;
        return (((uint32_t)n * H + iy) * W + ix) * (uint32_t)CIP + t.ci0;
    }
};

// =====================================================================================
// Staging interface of the GEMM kernel.  A loader splits each DMA slot's byte offset into a
// per-lane part (Lane, fixed when the block starts) and a wave-uniform part (Uni, advanced
// once per K step in scalar registers and passed as the buffer instruction's soffset), so the
// steady-state K loop does almost no vector address arithmetic:
//   Lane lane(a, b, k_begin)  NON-KT: a = GEMM row, b = 16-byte chunk inside the K step
//                             KT:     a = k row inside the step, b = absolute column chunk
//   Uni  uni(k_begin, k_end)  fetch<S>(Lane&, Uni) -> voffset   soff(Uni) -> soffset
//   step<S>(Uni&)             advance one K step (S chunks, or S k rows)
// A voffset of OOB reads zeros; a valid voffset + soffset stays inside the tensor.
// =====================================================================================

// Any per-lane iterator loader (LoadConvFwd / LoadConvDgrad / KtIm2col) behind the interface:
// the general case (ragged channels, strided input gradient, unaligned pixel counts).
template <class G, bool KT_>
struct PerLane {
    static constexpr int BK = 64;
    G g;
    uint32_t bytes;
    __device__ __forceinline__ const int8_t* ptr() const { return g.ptr(); }
    struct Lane {
        typename G::It it;
    };
    struct Uni {
        int k_end;
    };
    __device__ __forceinline__ Lane lane(int a, int b, int kb) const {
        return {KT_ ? g.begin(kb + a, b) : g.begin(a, kb + b)};
    }
    __device__ __forceinline__ Uni uni(int, int ke) const { return {ke}; }
    template <int S>
    __device__ __forceinline__ uint32_t fetch(Lane& l, const Uni& u) const {
        const uint32_t o = g.off(l.it, u.k_end);
        g.template next<S>(l.it);
        return o;
    }
    __device__ __forceinline__ uint32_t soff(const Uni&) const { return 0u; }
    template <int S>
    __device__ __forceinline__ void step(Uni&) const {}
};
template <class G, bool KT_>
static PerLane<G, KT_> per_lane(const G& g) {
    PerLane<G, KT_> r;
    r.g = g;
    r.bytes = g.bytes;
    return r;
}

// Row-major operand [rows][ld] with K chunks contiguous (weights, matmul operands).
struct RowsK {
    static constexpr int BK = 64;
    const int8_t* p;
    int64_t ld;
    int rows, kc_total;
    uint32_t bytes;
    __device__ __forceinline__ const int8_t* ptr() const { return p; }
    struct Lane {
        uint32_t cur;
        int c;
    };
    struct Uni {
        int kc0, kc_end;
    };
    __device__ __forceinline__ Lane lane(int row, int c, int) const {
        return {row < rows ? (uint32_t)(row * ld + c * 16) : OOB, c};
    }
    __device__ __forceinline__ Uni uni(int kb, int ke) const { return {kb, ke < kc_total ? ke : kc_total}; }
    template <int S>
    __device__ __forceinline__ uint32_t fetch(Lane& l, const Uni& u) const {
        if (u.kc0 + S <= u.kc_end) return l.cur;
        return u.kc0 + l.c < u.kc_end ? l.cur : OOB;
    }
    __device__ __forceinline__ uint32_t soff(const Uni& u) const { return (uint32_t)u.kc0 * 16u; }
    template <int S>
    __device__ __forceinline__ void step(Uni& u) const { u.kc0 += S; }
};

// Convolution operand whose K steps never straddle a tap (channels padded to a multiple of
// 64 bytes, kh*kw <= 32): row = pixel, K = (ky, kx, channel).  Each lane keeps a bit mask of
// the taps that fall inside the image for its pixel and re-derives its voffset only when the
// step enters a new tap; the channel offset inside the tap is the uniform soffset.
//   forward:         source x [N][SH][SW][C], y0 = oy*sh - pt, tap moves by +(ky*dh, kx*dw)
//   input gradient:  source dy [N][OH][OW][C] (stride 1), y0 = iy + pt, tap moves by -(ky*dh, kx*dw)
template <int BKB>
struct ConvTaps {
    static constexpr int BK = BKB;
    const int8_t* src;
    uint32_t bytes;
    int SH, SW, CPC;  // source image and channel chunks
    int PH, PW;       // pixel grid of the GEMM rows
    int sh, sw, oy_add, ox_add, dh, dw, KH, KW, M;
    int sgn;  // +1 forward, -1 input gradient
    uint32_t img;
    __device__ __forceinline__ const int8_t* ptr() const { return src; }
    struct Lane {
        int base;
        uint32_t mask, cur;
    };
    struct Uni {
        int cc, ky, kx, tapoff;
        bool fresh;
    };
    __device__ __forceinline__ Lane lane(int m, int c, int) const {
        Lane l;
        l.cur = OOB;
        l.mask = 0;
        l.base = 0;
        if (m < M) {
            const int px = m % PW, r = m / PW, py = r % PH, n = r / PH;
            const int y0 = py * sh + oy_add, x0 = px * sw + ox_add;
            l.base = (int)((uint32_t)n * img) + ((y0 * SW + x0) * CPC + c) * 16;
            for (int ky = 0, t = 0; ky < KH; ++ky)
                for (int kx = 0; kx < KW; ++kx, ++t) {
                    const int y = y0 + sgn * ky * dh, x = x0 + sgn * kx * dw;
                    if ((unsigned)y < (unsigned)SH && (unsigned)x < (unsigned)SW) l.mask |= 1u << t;
                }
        }
        return l;
    }
    __device__ __forceinline__ int tap_off(int ky, int kx) const { return sgn * ((ky * dh * SW + kx * dw) * CPC * 16); }
    __device__ __forceinline__ Uni uni(int kb, int) const {
        Uni u;
        const int tap = kb / CPC;
        u.cc = kb - tap * CPC;
        u.ky = tap / KW;
        u.kx = tap - u.ky * KW;
        u.tapoff = tap_off(u.ky, u.kx);
        u.fresh = true;
        return u;
    }
    template <int S>
    __device__ __forceinline__ uint32_t fetch(Lane& l, const Uni& u) const {
        if (u.fresh) l.cur = ((l.mask >> (u.ky * KW + u.kx)) & 1u) ? (uint32_t)(l.base + u.tapoff) : OOB;
        return l.cur;
    }
    __device__ __forceinline__ uint32_t soff(const Uni& u) const { return (uint32_t)u.cc * 16u; }
    template <int S>
    __device__ __forceinline__ void step(Uni& u) const {
        u.cc += S;
        u.fresh = u.cc >= CPC;
        if (u.fresh) {
            u.cc = 0;
            if (++u.kx == KW) {
                u.kx = 0;
                ++u.ky;
            }
            u.tapoff = tap_off(u.ky, u.kx);
        }
    }
};

// K-major rows (weight gradient A operand: dy [pixels][cop]); the k row offset is uniform.
struct KtRowsU {
    static constexpr int BK = 64;
    const int8_t* p;
    uint32_t bytes;
    int64_t ld;
    int cols, K;
    __device__ __forceinline__ const int8_t* ptr() const { return p; }
    struct Lane {
        uint32_t cur;
        int r;
    };
    struct Uni {
        int k0, k_end;
    };
    __device__ __forceinline__ Lane lane(int r, int c16, int) const {
        return {c16 * 16 < cols ? (uint32_t)(r * ld + c16 * 16) : OOB, r};
    }
    __device__ __forceinline__ Uni uni(int kb, int ke) const { return {kb, ke < K ? ke : K}; }
    template <int S>
    __device__ __forceinline__ uint32_t fetch(Lane& l, const Uni& u) const {
        if (u.k0 + S <= u.k_end) return l.cur;
        return l.r < u.k_end - u.k0 ? l.cur : OOB;
    }
    __device__ __forceinline__ uint32_t soff(const Uni& u) const { return (uint32_t)((int64_t)u.k0 * ld); }
    template <int S>
    __device__ __forceinline__ void step(Uni& u) const { u.k0 += S; }
};

// Weight-gradient B operand (im2col of x, rows = output pixels) when every 64-pixel K step is
// a whole number of output rows of one image (OW | 64, 64 | OH*OW) or of whole images
// (OH*OW | 64): a lane's position inside the step is then the same at every step, and only
// the step's image / first row (uniform) moves.
struct KtIm2colU {
    static constexpr int BK = 64;
    const int8_t* x;
    uint32_t bytes;
    int H, W, OH, OW, CIP, KW, sh, sw, pt, pl, dh, dw, ncols, K;
    bool rows_mode;  // true: a step = 64/OW output rows of one image; false: 64/(OH*OW) images
    __device__ __forceinline__ const int8_t* ptr() const { return x; }
    struct Lane {
        int rel, dy, r;
        bool ok;
    };
    struct Uni {
        int k0, k_end, n0, oy0, ubase;
    };
    __device__ __forceinline__ Lane lane(int r, int c16, int) const {
        Lane l;
        const int nn = c16 * 16;
        l.ok = nn < ncols;
        const int tap = l.ok ? nn / CIP : 0;
        const int ci0 = nn - tap * CIP;
        const int ky = tap / KW, kx = tap - ky * KW;
        int dn = 0, rem = r;
        if (!rows_mode) {
            dn = r / (OH * OW);
            rem = r - dn * OH * OW;
        }
        const int doy = rem / OW, dox = rem - doy * OW;
        const int ix = dox * sw + kx * dw - pl;
        l.dy = doy * sh + ky * dh - pt;
        l.ok = l.ok && (unsigned)ix < (unsigned)W;
        if (!rows_mode) l.ok = l.ok && (unsigned)l.dy < (unsigned)H;
        l.rel = ((dn * H + l.dy) * W + ix) * CIP + ci0;
        l.r = r;
        return l;
    }
    __device__ __forceinline__ Uni uni(int kb, int ke) const {
        Uni u;
        u.k0 = kb;
        u.k_end = ke < K ? ke : K;
        u.n0 = kb / (OH * OW);
        u.oy0 = (kb - u.n0 * OH * OW) / OW;
        u.ubase = (u.n0 * H + u.oy0 * sh) * W * CIP;
        return u;
    }
    template <int S>
    __device__ __forceinline__ uint32_t fetch(Lane& l, const Uni& u) const {
        bool v = l.ok;
        if (rows_mode) v = v && (unsigned)(u.oy0 * sh + l.dy) < (unsigned)H;
        if (u.k0 + S > u.k_end) v = v && l.r < u.k_end - u.k0;
        return v ? (uint32_t)(u.ubase + l.rel) : OOB;
    }
    __device__ __forceinline__ uint32_t soff(const Uni&) const { return 0u; }
    template <int S>
    __device__ __forceinline__ void step(Uni& u) const {
        u.k0 += S;
        if (rows_mode) {
            u.oy0 += S / OW;
            if (u.oy0 >= OH) {
                u.oy0 = 0;
                ++u.n0;
            }
        } else {
            u.n0 += S / (OH * OW);
        }
        u.ubase = (u.n0 * H + u.oy0 * sh) * W * CIP;
    }
};

// =====================================================================================
// The GEMM kernel (both operand orientations), a STAGES-deep LDS pipeline fed by LDS-DMA.
//
//   KT = false  C[m][n] = sum_k A[m][k] B[n][k]: tiles are [BM|BN rows][BK=64 bytes of K];
//               fragments by ds_read_b128 (forward conv, input-gradient conv, matmul).
//   KT = true   C[m][n] = sum_k A[k][m] B[k][n]: tiles are [KT_BK=64 k rows][BM|BN bytes];
//               fragments by ds_read_b64_tr_b8 (weight gradient; see gemm_kt notes above).
//
// Staging: every 1 KiB of a tile is one buffer_load_dwordx4 ... lds wave-instruction (the
// LDS image is lane-linear per instruction); the XOR swizzle of the image is applied by
// choosing which global 16-byte chunk each lane fetches.  Out-of-range chunks read zeros.
// Pipeline: loads for step s+STAGES-1 are issued right after the barrier of step s, into
// the stage step s-1 used; before that barrier every wave waits with a counted vmcnt for its
// own step-s loads only, so up to STAGES-2 later steps stay in flight across the barrier.
// All LDS lives in one __shared__ array and the loop issues no register loads, so hipcc has
// no reason to drain vmcnt early (cdna_hip_programming.md §5, "Pipelining across barriers").
// =====================================================================================
#ifndef NITI_LDS_BUDGET_KB
#define NITI_LDS_BUDGET_KB 96
#endif
#ifndef NITI_MAX_STAGES
#define NITI_MAX_STAGES 4
#endif
constexpr int LDS_STAGE_BUDGET = NITI_LDS_BUDGET_KB * 1024;  // pipeline depth = min(MAX_STAGES, budget / stage bytes)
constexpr int MAX_STAGES = NITI_MAX_STAGES;
#ifndef NITI_ABLATE
#define NITI_ABLATE 0  // diagnostic builds only: 1 = no global->LDS copies, 2 = no MFMA, 5 = no taps tile stores, 6 = 2 + 5, 7 = 1 + 5, 8 = empty taps kernel,
                       // 3 = no copies and no per-step barrier, 4 = no per-step barrier
#endif



// swizzled 16-byte chunk of LDS row r (row of RB bytes) for the two orientations
template <bool KT, int RB>
__device__ __forceinline__ int swz16(int r) {
    if (KT) return kt_swz<RB>(r);
    // ds_read_b128 fragment reads conflict-free: 64-byte rows (r>>2)&3, 128-byte rows (r>>1)&7
    return RB == 128 ? (r >> 1) & 7 : (r >> 2) & 3;
}

template <int BM, int BN, int WM, int WN, class LA, class LB, int MODE, bool KT, int NW>
__global__ void __launch_bounds__(NW * 64) gemm_kernel(LA la, LB lb, int M, int N, int tiles_n, int k_total,
                                                        int k_per_split, Epi epi) {
    constexpr int WP = WM * WN;  // wave positions over the output tile
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    static_assert(NW % WP == 0 && NW / WP <= 2, "one or two wave groups");
    constexpr int KG = NW / WP;  // wave groups splitting each step's K sub-steps
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    // staging geometry: rows x row-bytes per operand tile
    constexpr int BK = KT ? 64 : LA::BK;
    constexpr int A_ROWS = KT ? KT_BK : BM, A_RB = KT ? BM : BK;
    constexpr int B_ROWS = KT ? KT_BK : BN, B_RB = KT ? BN : BK;
    constexpr int A_BYTES = A_ROWS * A_RB, B_BYTES = B_ROWS * B_RB;
    constexpr int A_PW = A_BYTES / 1024 / NW, B_PW = B_BYTES / 1024 / NW;  // DMA instructions per wave
    static_assert(A_PW >= 1 && B_PW >= 1 && A_BYTES % (1024 * NW) == 0 && B_BYTES % (1024 * NW) == 0,
                  "tile too small for the wave count");
    constexpr int LOADS = A_PW + B_PW;  // per lane per step
    constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
    constexpr int STAGES_FIT = LDS_STAGE_BUDGET / STAGE_BYTES;
    constexpr int STAGES = STAGES_FIT >= MAX_STAGES ? MAX_STAGES : (STAGES_FIT >= 2 ? STAGES_FIT : 2);
    constexpr int K_STEP = KT ? KT_BK : BK / 16;  // K units (k rows or 16-byte chunks) per step
    constexpr int KSUB = (KT ? KT_BK : BK) / 32;   // 32-deep MFMA sub-steps per step
    constexpr int KW_ = KSUB / KG;                 // sub-steps per wave per step
    static_assert(KSUB % KG == 0, "sub-steps split evenly");
    constexpr int XCH_BYTES = KG > 1 ? NW * (TM / 2) * TN * 64 * 64 : 0;  // accumulator exchange
    constexpr int SMEM0 = STAGES * STAGE_BYTES > XCH_BYTES ? STAGES * STAGE_BYTES : XCH_BYTES;
    constexpr int CT_BYTES = epi_stage_c(MODE, BM, BN) ? BM * (BN + 4) * 4 : 0;  // staged C tile
    constexpr int SMEM = SMEM0 > CT_BYTES ? SMEM0 : CT_BYTES;
    static_assert(SMEM >= BM * (BN + 16), "requant epilogue staging fits in the pipeline's LDS");
    static_assert(MODE != EPI_SGD || SMEM >= BN * (BM + 16), "the NITI_SGD epilogue's transposed tile fits");
    __shared__ __attribute__((aligned(16))) int8_t smem[SMEM];

    if constexpr (MODE == EPI_REQUANT) {
        if (epi.spec == 2) {  // launch B of the pair
            const int act = gemm_spec_settle(epi);
            if (act == 0) return;  // A's output stands
            if (act > 0) {         // one bit width off: A's alternate is the output
                const int64_t n16 = (int64_t)M * epi.ldo / 16;
                const v16c* src = (const v16c*)(epi.alt + (int64_t)(act - 1) * M * epi.ldo);
                const int64_t nb = (int64_t)gridDim.x * gridDim.y;
                for (int64_t i = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; i < n16;
                     i += nb * blockDim.x)
                    ((v16c*)epi.out)[i] = src[i];
                return;
            }
        }
    }
    const unsigned long long span_t0 = span_begin(epi.span);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS bases stay scalar
    const int kg = wid / WP, wq = wid % WP;
    const int wm = wq / WN, wn = wq % WN;
    // XCD-aware tile order inside each K split.  (A split-major order over the whole grid, which
    // keeps one K range per XCD and cuts the weight gradient's HBM fetch ~8x, measured slower.)
    int split = blockIdx.y, tile = xcd_remap(blockIdx.x, gridDim.x);
    if (epi.split_major) {  // one K range per XCD: its operand panels are fetched into one L2
        const int logical = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, gridDim.x * gridDim.y);
        split = logical / gridDim.x;
        tile = logical - split * gridDim.x;
    }
    const int tm_ = tile / tiles_n, tn_ = tile % tiles_n;
    const int m0 = tm_ * BM, n0 = tn_ * BN;
    const int k_begin = split * k_per_split;
    const int k_end = min(k_total, k_begin + k_per_split);
    const int nsteps = k_end > k_begin ? (k_end - k_begin + K_STEP - 1) / K_STEP : 0;

    const __amdgpu_buffer_rsrc_t rA = make_rsrc(la.ptr(), la.bytes);
    const __amdgpu_buffer_rsrc_t rB = make_rsrc(lb.ptr(), lb.bytes);
    typename LA::Lane ia[A_PW];
    typename LB::Lane ib[B_PW];
#pragma unroll
    for (int i = 0; i < A_PW; ++i) {
        const int byte = (wid * A_PW + i) * 1024 + lane * 16;
        const int r = byte / A_RB, c = ((byte % A_RB) >> 4) ^ swz16<KT, A_RB>(r);
        ia[i] = KT ? la.lane(r, m0 / 16 + c, k_begin) : la.lane(m0 + r, c, k_begin);
    }
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
        const int byte = (wid * B_PW + i) * 1024 + lane * 16;
        const int r = byte / B_RB, c = ((byte % B_RB) >> 4) ^ swz16<KT, B_RB>(r);
        ib[i] = KT ? lb.lane(r, n0 / 16 + c, k_begin) : lb.lane(n0 + r, c, k_begin);
    }
    typename LA::Uni ua = la.uni(k_begin, k_end);
    typename LB::Uni ub = lb.uni(k_begin, k_end);
    auto issue = [&](int stage) {
        int8_t* sa = smem + stage * STAGE_BYTES;
        int8_t* sb = sa + A_BYTES;
        const uint32_t soa = la.soff(ua), sob = lb.soff(ub);
#pragma unroll
        for (int i = 0; i < A_PW; ++i) {
            const uint32_t vo = la.template fetch<K_STEP>(ia[i], ua);
            if (NITI_ABLATE != 1 && NITI_ABLATE != 3) dma16(rA, sa + (wid * A_PW + i) * 1024, vo, soa);
        }
#pragma unroll
        for (int i = 0; i < B_PW; ++i) {
            const uint32_t vo = lb.template fetch<K_STEP>(ib[i], ub);
            if (NITI_ABLATE != 1 && NITI_ABLATE != 3) dma16(rB, sb + (wid * B_PW + i) * 1024, vo, sob);
        }
        la.template step<K_STEP>(ua);
        lb.template step<K_STEP>(ub);
    };

    v16i acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[a][b][i] = 0;

    // per-lane fragment offsets inside a stage (loop invariant); wave group kg takes the
    // sub-steps kk = kg, kg + KG, ...
    const uint32_t smem_base = lds_addr(smem);
    uint32_t offA[KW_][TM], offB[KW_][TN];
#pragma unroll
    for (int j = 0; j < KW_; ++j) {
        const int kk = kg + KG * j;
        if (KT) {
            // transposed reads: lane 2q+p of each 16-lane group names row q, 8-byte column p
            const int r0 = kk * 32 + 16 * (lane >> 5) + ((lane & 15) >> 1);
            const int cofs = 16 * ((lane >> 4) & 1) + 8 * (lane & 1);
#pragma unroll
            for (int a = 0; a < TM; ++a) offA[j][a] = kt_off8<BM>(r0, (wm * (BM / WM) + a * 32 + cofs) >> 3);
#pragma unroll
            for (int b = 0; b < TN; ++b) offB[j][b] = kt_off8<BN>(r0, (wn * (BN / WN) + b * 32 + cofs) >> 3);
        } else {
            const int c = kk * 2 + (lane >> 5);
#pragma unroll
            for (int a = 0; a < TM; ++a) {
                const int r = wm * (BM / WM) + a * 32 + (lane & 31);
                offA[j][a] = r * BK + ((c ^ swz16<false, BK>(r)) << 4);
            }
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const int r = wn * (BN / WN) + b * 32 + (lane & 31);
                offB[j][b] = r * BK + ((c ^ swz16<false, BK>(r)) << 4);
            }
        }
    }

    // Fragments are double-buffered in registers: the reads for step s+1 are issued right
    // after the barrier of iteration s and fly while step s's MFMAs run.  Fragment reads are
    // inline asm: hipcc cannot tell them apart from the LDS-DMA writes still in flight to the
    // other stages and would otherwise drain vmcnt(0) before every ds_read.
    // Stage reuse: iteration s refills the stage of step s-1, whose reads every wave waited
    // for before its step s-1 MFMAs, i.e. before the barrier of iteration s.
    static_assert(STAGES >= 3, "register double buffering needs three stages");
    constexpr int READS = KT ? 2 * (TM + TN) : (TM + TN);  // per sub-step
    constexpr int RW = KW_ * READS;                        // per wave per step
    v4i fa[2][KW_][TM], fb[2][KW_][TN];
    auto read_frags = [&](auto buf_c, int step) {
        constexpr int BUF = decltype(buf_c)::value;
        const uint32_t sA = smem_base + (uint32_t)((step % STAGES) * STAGE_BYTES);
        const uint32_t sB = sA + A_BYTES;
#pragma unroll
        for (int j = 0; j < KW_; ++j) {
#pragma unroll
            for (int a = 0; a < TM; ++a)
                fa[BUF][j][a] = KT ? lds_tr8x2(sA + offA[j][a], BM * 8) : lds_b128(sA + offA[j][a]);
#pragma unroll
            for (int b = 0; b < TN; ++b)
                fb[BUF][j][b] = KT ? lds_tr8x2(sB + offB[j][b], BN * 8) : lds_b128(sB + offB[j][b]);
        }
    };
    auto body = [&](auto cur_c, int s) {
        constexpr int CUR = decltype(cur_c)::value;
        const bool more = s + 1 < nsteps;
        if (more) wait_steps<LOADS, STAGES - 3>(min(STAGES - 3, nsteps - 2 - s));  // own step s+1 loads landed
        if (NITI_ABLATE < 3) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (s + STAGES - 1 < nsteps) issue((s + STAGES - 1) % STAGES);
        if (more) {
            read_frags(std::integral_constant<int, 1 - CUR>(), s + 1);
            lgkm_wait<RW>();  // step s's fragments (requested one iteration earlier) are in
        } else {
            lgkm_wait<0>();
        }
#pragma unroll
        for (int j = 0; j < KW_; ++j) {
#pragma unroll
            for (int a = 0; a < TM; ++a) reg_fence(fa[CUR][j][a]);
#pragma unroll
            for (int b = 0; b < TN; ++b) reg_fence(fb[CUR][j][b]);
        }
#pragma unroll
        for (int j = 0; j < KW_; ++j)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b) {
                    if (NITI_ABLATE == 2) {
                        acc[a][b][0] += fa[CUR][j][a][0] ^ fb[CUR][j][b][1];
                    } else {
                        acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[CUR][j][a], fb[CUR][j][b], acc[a][b], 0,
                                                                          0, 0);
                    }
                }
        __builtin_amdgcn_sched_barrier(0);
    };

#pragma unroll
    for (int st = 0; st < STAGES - 1; ++st)
        if (st < nsteps) issue(st);
    if (nsteps > 0) {
        wait_steps<LOADS, STAGES - 2>(min(STAGES - 2, nsteps - 1));
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        read_frags(std::integral_constant<int, 0>(), 0);
    }
    for (int s = 0; s < nsteps; s += 2) {
        body(std::integral_constant<int, 0>(), s);
        if (s + 1 < nsteps) body(std::integral_constant<int, 1>(), s + 1);
    }
    // The last step waited lgkmcnt(0), but hipcc sees the fragment registers of the merged
    // "more" path as dead at the loop exit and may reuse them in the epilogue ahead of any wait;
    // drain and touch every fragment register so none is reused while an asm read could be in
    // flight (tools/isa_inflight.py scans for this).
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < KW_; ++j) {
#pragma unroll
            for (int a = 0; a < TM; ++a) reg_fence(fa[u][j][a]);
#pragma unroll
            for (int b = 0; b < TN; ++b) reg_fence(fb[u][j][b]);
        }
    __syncthreads();
    if constexpr (KG == 1) {
        gemm_epilogue<TM, TN, NW, MODE, BM, BN>(acc, m0 + wm * (BM / WM), n0 + wn * (BN / WN), M, N, epi, smem, split,
                                                m0, n0);
    } else {
        // The two wave groups hold partial sums of the same tiles: group 0 keeps tile rows
        // a < TM/2 and sends the rest, group 1 the reverse; one LDS exchange, then each wave
        // finishes half of the tiles.
        constexpr int TH = TM / 2;
        v4i* xbuf = (v4i*)smem;
        const int send_a = kg == 0 ? TH : 0;
#pragma unroll
        for (int a = 0; a < TH; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const v16i& t = acc[send_a + a][b];
                    xbuf[((wid * TH + a) * TN + b) * 256 + q * 64 + lane] = v4i{t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]};
                }
        __syncthreads();
        const int partner = (1 - kg) * WP + wq;
        const int keep_a = kg == 0 ? 0 : TH;
        v16i keep[TH][TN];
#pragma unroll
        for (int a = 0; a < TH; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                keep[a][b] = acc[keep_a + a][b];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const v4i v = xbuf[((partner * TH + a) * TN + b) * 256 + q * 64 + lane];
                    keep[a][b][4 * q] += v[0];
                    keep[a][b][4 * q + 1] += v[1];
                    keep[a][b][4 * q + 2] += v[2];
                    keep[a][b][4 * q + 3] += v[3];
                }
            }
        __syncthreads();  // exchange buffer is reused by the epilogue's block max
        gemm_epilogue<TH, TN, NW, MODE, BM, BN>(keep, m0 + wm * (BM / WM) + keep_a * 32, n0 + wn * (BN / WN), M, N,
                                                epi, smem, split, m0, n0);
    }
    span_end(epi.span, span_t0);
}

// Sum of K-split slabs -> C (+ max|C|).  A block covers 256/G v4i elements with G threads
// per element, each summing every G-th slab with 8 loads in flight; the G partials meet in
// registers (shfl_xor inside the wave).  Splits are many and outputs small for the weight
// gradient (e.g. VGG-11 L1: 160 slabs of 9 K elements), so split-level parallelism matters.
// Where a 16-byte slab chunk e lands in C: the same place (GEMM slabs are [M][N] like C), or,
// for the tap-sharing kernel's tile-blocked slabs ([tile][64 rows][NT taps][32 ch], each block's
// partial tile one contiguous 72 KiB run), row co0 + r, columns t * CIP + ci0 + 4 * part of C.
struct SlabLinear {
    __device__ bool operator()(int64_t e, int64_t* dst) const {
        *dst = e;
        return true;
    }
};
struct SlabTapsBlocked {
    int tiles_ci, cip4, c_out, ld4;  // ld4 = NT * CIP / 4
    FastDiv fTile, fRow, fPart, fTci;   // 64 * 72 v4i per tile, 72 per row, 8 per tap, tiles_ci
    __device__ bool operator()(int64_t e, int64_t* dst) const {
        const uint32_t u = (uint32_t)e;
        const uint32_t tile = fdiv(fTile, u), rem = u - tile * 4608u;
        const uint32_t row = fdiv(fRow, rem), rc = rem - row * 72u;
        const uint32_t t = fdiv(fPart, rc), part = rc - t * 8u;
        const uint32_t tco = fdiv(fTci, tile), tci = tile - tco * (uint32_t)tiles_ci;
        const int co = (int)(tco * 64u + row);
        *dst = (int64_t)co * ld4 + t * cip4 + tci * 8u + part;
        return co < c_out;
    }
};

template <class MAP>
__global__ void splitk_reduce_kernel(const int32_t* __restrict__ slab, int splits, int64_t stride, int64_t n4, int G,
                                     int32_t* __restrict__ C, uint32_t* __restrict__ amax, MAP map) {
    const int g = threadIdx.x & (G - 1);
    const int64_t e = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G;
    int64_t de = 0;
    const bool live = e < n4 && map(e, &de);
    v4i s = {0, 0, 0, 0};
    if (live) {
        const v4i* base = (const v4i*)slab + e;
        const int64_t st4 = stride / 4;
        // up to 8 independent loads in flight per pass (predicated, no dependent chain)
        for (int z0 = g; z0 < splits; z0 += 8 * G) {
            v4i v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int z = z0 + j * G;
                v[j] = z < splits ? __builtin_nontemporal_load(base + (int64_t)z * st4) : v4i{0, 0, 0, 0};
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) s += v[j];
        }
    }
    for (int o = G >> 1; o > 0; o >>= 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += __shfl_xor(s[j], o, 64);
    }
    uint32_t m = 0;
    if (g == 0 && live) {
        ((v4i*)C)[de] = s;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t u = uabs32(s[j]);
            m = m > u ? m : u;
        }
    }
    if (amax != nullptr) {
        m = wave_max(m);
        __shared__ uint32_t red[4];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < 4; ++i) m = m > red[i] ? m : red[i];
            m = m > red[0] ? m : red[0];
            publish_max(amax, m);
        }
    }
}

// =====================================================================================
// Tap-sharing weight gradient (NITI_GradientConv_Int8, NITI_GradientConv_Int8.cpp:165-298)
// for stride-1, dilation-1 convolutions with Cip % 32 == 0 and Cop % 64 == 0.
//
//   C[co][tap][ci] = sum over output pixels p of dy[p][co] * x[p + tap][ci]
//
// The generic KT GEMM stages an im2col panel per (tap, channel) column tile, so x is fetched
// once per tap.  Here a block owns 64 output channels x ALL taps x 32 input channels.  Pixels
// come in REGION STEPS of 64 output pixels (whole output rows of one image, or whole images);
// a region step stages the zero-padded input region its pixels touch (rows RH = band + KH - 1,
// cols RW = OW + KW - 1; out-of-image pixels read zeros through the buffer range check) once,
// as 32-byte LDS rows, and every tap's B fragment is the same transposed read shifted by the
// tap's region offset (ky*RW + kx rows).  32-byte rows keep each half-wave's transposed read
// (8 consecutive region rows x 32 B = 256 contiguous bytes) conflict-free at any shift.
//
// A K step is one region step.  8 waves, two per SIMD: K group kg (the step's 32-pixel half)
// x tap group tg (TapGroup: 5 or 4 of the 18 (output-channel half, tap) tiles, paired 5 + 4 on
// a SIMD), so one wave's fragment reads and barrier wait hide under the other wave's MFMAs.
// A step is one MFMA stream per wave with the next step's fragment reads (double-buffered)
// and the LDS-DMA issue in the gaps; every LDS address is a per-lane register plus a
// compile-time stage offset (the K loop is unrolled by the pipeline stages).  The two K
// groups' partial tiles meet through LDS, and the int32 tile leaves as 16-byte row chunks
// (split-K: one contiguous run of a tile-blocked slab).  Blocks: tiles (co64 x ci32) x K
// splits, split-major under the XCD remap, so a split's tiles share one XCD's L2 and each XCD
// reads only its own pixel range of x and dy.
// =====================================================================================
struct WgTaps {
    const int8_t* x;   // NHWC16 [N][H][W][CIP]
    const int8_t* dy;  // NHWC16 [N][OH][OW][COP]
    uint32_t xbytes, dybytes;
    int H, W, OH, OW, CIP, COP, KW, pt, pl;
    int c_out;         // rows of C that exist
    int RH, RW;        // region rows / columns per region image
    int PPI;           // output pixels per region image (64 in band mode)
    int imgs;          // region images per region step (1 in band mode)
    int band;          // 1: a region step is 64 / OW output rows of one image
    int rows_per_step;
    int rs_total;      // region steps (K / 64)
    int BPI;           // region steps per image group (OH / rows_per_step in band mode, else 1)
    int steps_total, steps_per_split;  // K steps of two region steps
    int tiles_ci, tiles;  // 32-channel input tiles; tiles per K split
    FastDiv fRW, fRPI, fPPI, fOW, fOHW, fTiles, fTci, fBPI;
    // segment mode (maps whose rows are not whole 64-pixel steps: 224 / 112 / 56 / 28 / 14 px): a
    // region step is 4 row segments of SW = 16 (or 14: two zero pixel slots) output pixels, each a
    // 1 x 16 region image of 3 x 18 input pixels; segment gs = 4 step + s is row gs / NS (of all
    // N * H rows), columns (gs % NS) * SW ...
    int seg, SW, NS, nseg;  // NS segments per row, nseg = N * H * NS
    FastDiv fNS, fH;
    // tile mode (seg == 2): a step is one 4-row x 16-slot tile (SW real columns) of one image, a
    // 6 x 18 region: the halo rows are shared by the tile's 4 rows (segment mode stages 3 rows per
    // row); tile t = strip (t % NS), band ((t / NS) % NB), image (t / NS / NB); nseg = tiles
    int NB;
    FastDiv fNB;
    unsigned long long* stamps;  // diagnostic builds (NITI_STAMPS): per-block s_memtime marks
    unsigned long long* span;    // kernel-span probe slot (probe_span_arm)
};
#ifndef NITI_STAMPS
#define NITI_STAMPS 0
#endif
#define TAPS_STAMP(k)                                                                                         \
    do {                                                                                                      \
        if (NITI_STAMPS && g.stamps != nullptr && tid == 0) {                                                 \
            g.stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime();                                    \
            if ((k) == 0 || (k) == 5) g.stamps[blockIdx.x * 8 + 6 + ((k) == 5)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                                     \
    } while (0)


constexpr int TAPS_THREADS = 512;

// The four tap groups of a K group's 18 (output-channel half, tap) tiles: the two waves on one
// SIMD hold 5 + 4 tiles (9 MFMAs per SIMD per step), and a wave reads both dy halves plus 2-3 x
// taps per step (18 fragments per K group, where per-channel-half waves read 22).  Tile j of
// group G is (ch(j), tap(xi(j))); x tap i is read after MFMA i + 1, both dy halves after MFMA 0.
template <int G>
struct TapGroup {
    static constexpr int NX = G < 2 ? 3 : 2;     // x taps
    static constexpr int NTILE = G < 2 ? 5 : 4;  // MFMA tiles
    static constexpr int tap(int i) { return G == 0 ? i : G == 1 ? 2 + i : G == 2 ? 5 + i : 7 + i; }
    static constexpr int ch(int j) { return G == 1 ? ((j + 1) & 1) : (j & 1); }
    static constexpr int xi(int j) { return G == 1 ? (j + 1) >> 1 : j >> 1; }
    // ds_reads a step issues before its MFMA j (its reads of the next step)
    static constexpr int cum(int j) { return j == 0 ? 0 : 4 + 2 * (j - 1 < NX ? j - 1 : NX); }
    // reads issued after the last read of MFMA j's x tap: 2 per later x tap of the previous
    // step, plus this step's reads so far
    static constexpr int wait(int j, bool more) { return 2 * (NX - 1 - xi(j)) + (more ? cum(j) : 0); }
};
#ifndef NITI_TAPS_STAGES1
#define NITI_TAPS_STAGES1 4  // pipeline stages of the one-DMA-per-wave (XPW 1) kernel
#endif
#ifndef NITI_TAPS_NT
#define NITI_TAPS_NT 0  // nontemporal (L2-bypassing) stores of the int32 tile (2: write-through sc1)
#endif
#ifndef NITI_TAPS_PRIO
#define NITI_TAPS_PRIO 0  // s_setprio 1 for the second-dispatched half (waves 4-7) over the K loop
#endif

template <int NT, int XPW, int MODE>
__global__ void __launch_bounds__(TAPS_THREADS) wgrad_taps_kernel(WgTaps g, Epi epi) {
    constexpr int NW = TAPS_THREADS / 64;
    static_assert(NW == 8, "8 waves: 4 tap groups x K group");
    static_assert(NT == 9, "3x3 taps (the tap groups of TapGroup)");
    constexpr int STAGES = XPW == 1 ? NITI_TAPS_STAGES1 : 4;  // stage offsets stay below the 64 KiB DS immediate
    static_assert(STAGES % 2 == 0, "the dy fragment buffer alternates with the step parity");
    constexpr int XB = XPW * 4096;  // region: 4 KiB x XPW of LDS-DMA (1 KiB per instruction)
    constexpr int DB = 4096;        // dy: 64 pixels x 64 bytes
    constexpr int ZB = XPW == 2 ? 4096 : 0;  // XPW 2: sink of the 4 waves without a dy chunk
    constexpr int SB = XB + DB + ZB;
    constexpr int LOADS = XPW;      // DMA instructions per wave per step
    constexpr int TA = 5;                   // most (output-channel half, tap) tiles of one wave
    constexpr int XCH = 4 * TA * 4096;      // exchange: one 32x32 int32 tile per (tap group, tile)
    constexpr int LDT = NT * 32 + 4;        // staged C tile pitch (int32)
    constexpr int CT = 64 * LDT * 4;
    constexpr int SMEM0 = STAGES * SB > XCH ? STAGES * SB : XCH;
    constexpr int SMEM = SMEM0 > CT ? SMEM0 : CT;
    static_assert((STAGES - 1) * SB + 512 < 65536, "stage offsets fit the DS immediate");
    __shared__ __attribute__((aligned(16))) int8_t smem[SMEM];

    const int tid = threadIdx.x;
    if (NITI_ABLATE == 8) {  // diagnostic: launch cost of the grid alone
        if (tid == 0 && g.span == (unsigned long long*)1) smem[0] = 1;
        return;
    }
    const unsigned long long span_t0 = span_begin(g.span);
    TAPS_STAMP(0);
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // waves w and w + 4 share a SIMD (cyclic SIMD order): tap group tg (TapGroup) and K group kg;
    // the groups paired on a SIMD (0 + 2, 1 + 3) hold 5 + 4 tiles, 9 MFMAs per SIMD per step
    const int kg = (wid >> 1) & 1, tg = (wid >> 2) * 2 + (wid & 1);
    const int logical = xcd_remap(blockIdx.x, gridDim.x);
    const int split = (int)fdiv(g.fTiles, (uint32_t)logical);
    const int tile = logical - split * g.tiles;
    const int tco = (int)fdiv(g.fTci, (uint32_t)tile), tci = tile - tco * g.tiles_ci;
    const int co0 = tco * 64, ci0 = tci * 32;
    const int s_begin = split * g.steps_per_split;
    const int s_end = min(g.steps_total, s_begin + g.steps_per_split);
    const int nsteps = s_end > s_begin ? s_end - s_begin : 0;

    const __amdgpu_buffer_rsrc_t rX = make_rsrc(g.x, g.xbytes);
    const __amdgpu_buffer_rsrc_t rD = make_rsrc(g.dy, g.dybytes);

    // DMA lanes.  XPW 1: waves 0-3 fill the region (chunk c = (w * 64 + lane) = region row
    // c >> 1, half c & 1), waves 4-7 the 64 x 64-byte dy tile.  XPW 2: every wave one region
    // chunk block; waves 0-3 also the dy tile, waves 4-7 a dummy (zeros into the stage's sink)
    // so that every wave counts the same loads.
    const int rpi = g.RH * g.RW;
    const bool xw = XPW == 2 || wid < 4;  // this wave's first DMA is a region chunk block
    const int xblk = XPW == 2 ? wid : (wid & 3);
    int xrel = 0, xry = 0, xseg = 0, xrx = 0;
    bool xok = false;
    {
        const int c = xblk * 64 + lane;
        const int q = c >> 1;
        const int img = (int)fdiv(g.fRPI, (uint32_t)q), rr = q - img * rpi;
        const int ry = (int)fdiv(g.fRW, (uint32_t)rr), rx = rr - ry * g.RW;
        const int ix = rx - g.pl;
        xok = q < g.imgs * rpi && (g.seg || (unsigned)ix < (unsigned)g.W);
        xry = ry;
        xrel = g.seg ? 16 * (c & 1) + ci0 : ((img * g.H + ry) * g.W + ix) * g.CIP + 16 * (c & 1) + ci0;
        xseg = img;
        xrx = rx;
    }
    const int dch = (wid & 3) * 64 + lane;
    const int drow = dch >> 2;
    // segment mode, SW = 14: slot drow is pixel 14 (drow / 16) + drow % 16 of the step (slots 14 and
    // 15 of a segment read zeros); SW = 16 is the plain 64-pixel run
    // tile mode: slot drow is pixel (drow / 16, drow % 16) of the tile, relative to its first
    // pixel (the step's soffset); columns past SW read zeros
    const int dpx = g.seg == 2 ? ((drow & 15) < g.SW ? (drow >> 4) * g.W + (drow & 15) : -1)
                  : g.seg && g.SW == 14 ? ((drow & 15) < 14 ? 14 * (drow >> 4) + (drow & 15) : -1) : drow;
    const uint32_t dvo = dpx < 0 ? OOB : (uint32_t)(dpx * g.COP + co0 + 16 * ((dch & 3) ^ kt_swz<64>(drow)));
    const uint32_t dstep = (uint32_t)(g.seg ? 4 * g.SW : 64) * (uint32_t)g.COP;  // dy bytes per region step
    const bool dw = XPW == 1 ? !xw : wid < 4;  // this wave loads a dy chunk block

    // LDS-DMA of region step `step` (block-relative) into `stage`; wave-uniform offsets from the
    // region index by one multiply-shift division (no per-step branches)
    auto issue = [&](int stage, int step) {
        int8_t* st0 = smem + stage * SB;
        const int r = s_begin + step;
        // tile mode: the step's tile (image, first row, first column), uniform
        int t_img = 0, t_y0 = 0, t_x0 = 0;
        if (g.seg == 2) {
            const int rest = (int)fdiv(g.fNS, (uint32_t)r);
            t_x0 = (r - rest * g.NS) * g.SW;
            t_img = (int)fdiv(g.fNB, (uint32_t)rest);
            t_y0 = (rest - t_img * g.NB) * 4;
        }
        if (xw && g.seg == 2) {
            // region pixel (xry, xrx) = input (t_y0 + xry - 1, t_x0 + xrx - 1), zero outside
            const int iy = t_y0 + xry - 1, ix = t_x0 + xrx - 1;
            const bool v = xok && r < g.nseg && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
            const int a = ((t_img * g.H + iy) * g.W + ix) * g.CIP + xrel;
            if (NITI_ABLATE != 1 && NITI_ABLATE != 7) dma16(rX, st0 + xblk * 1024, v ? (uint32_t)a : OOB, 0u);
        } else if (xw && g.seg) {
            // the chunk's segment gs: image row `row` (of all N * H), columns from (gs % NS) * SW;
            // region pixel (xry, xrx) is input (row + xry - 1, (gs % NS) * SW + xrx - 1), zero
            // outside the image (pad 1, stride 1: output and input rows coincide)
            const int gs = 4 * r + xseg;
            const int row = (int)fdiv(g.fNS, (uint32_t)gs);
            const int ix = (gs - row * g.NS) * g.SW + xrx - 1;
            const int iy = row - (int)fdiv(g.fH, (uint32_t)row) * g.H + xry - 1;
            const bool v = xok && gs < g.nseg && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
            const int a = ((row + xry - 1) * g.W + ix) * g.CIP + xrel;
            if (NITI_ABLATE != 1 && NITI_ABLATE != 7) dma16(rX, st0 + xblk * 1024, v ? (uint32_t)a : OOB, 0u);
        } else if (xw) {
            const int q = (int)fdiv(g.fBPI, (uint32_t)r);
            const int ybase = (r - q * g.BPI) * g.rows_per_step - g.pt;
            const int ub = (q * g.imgs * g.H + ybase) * g.W * g.CIP;
            const bool v = xok && (unsigned)(ybase + xry) < (unsigned)g.H;
            if (NITI_ABLATE != 1 && NITI_ABLATE != 7) dma16(rX, st0 + xblk * 1024, v ? (uint32_t)(ub + xrel) : OOB, 0u);
        }
        if (dw) {
            const uint32_t so = g.seg == 2 ? (r < g.nseg ? (uint32_t)((t_img * g.H + t_y0) * g.W + t_x0) * (uint32_t)g.COP : OOB)
                                           : (uint32_t)r * dstep;
            if (NITI_ABLATE != 1 && NITI_ABLATE != 7) dma16(rD, st0 + XB + (wid & 3) * 1024, dvo, so);
        } else if (XPW == 2) {
            if (NITI_ABLATE != 1 && NITI_ABLATE != 7) dma16(rD, st0 + XB + DB + (wid & 3) * 1024, OOB, 0u);
        }
    };

    // fragment addresses (stage 0; later stages add a compile-time offset): rows p and p + 8
    // of the wave's 32-pixel sub-step, 8-byte column cofs of the lane's 32-column block
    const uint32_t smem_base = lds_addr(smem);
    const int p0 = kg * 32 + 16 * (lane >> 5) + ((lane & 15) >> 1);
    const int cofs = 16 * ((lane >> 4) & 1) + 8 * (lane & 1);
    const uint32_t aD0 = smem_base + XB + (uint32_t)kt_off8<64>(p0, cofs >> 3);  // +8 rows: +512
    const uint32_t aD1 = smem_base + XB + (uint32_t)kt_off8<64>(p0, (32 + cofs) >> 3);
    auto qrow = [&](int p) {
        const int img = (int)fdiv(g.fPPI, (uint32_t)p), rem = p - img * g.PPI;
        const int oy = (int)fdiv(g.fOW, (uint32_t)rem), ox = rem - oy * g.OW;
        return img * rpi + oy * g.RW + ox;
    };
    const uint32_t aX0 = smem_base + (uint32_t)(qrow(p0) * 32 + cofs);
    const uint32_t aX1 = smem_base + (uint32_t)(qrow(p0 + 8) * 32 + cofs);

    // everything below runs per tap group G (compile time, TapGroup): its x taps, its
    // (output-channel half, tap) tiles and the step's fragment reads
    auto run = [&](auto g_c) {
        using TG = TapGroup<decltype(g_c)::value>;
        constexpr int NX = TG::NX, NTW = TG::NTILE;
        uint32_t aX[NX][2];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            const int t = TG::tap(i), ky = t / 3, kx = t % 3;
            const uint32_t o = (uint32_t)((ky * g.RW + kx) * 32);
            aX[i][0] = aX0 + o;
            aX[i][1] = aX1 + o;
        }
        v16i acc[NTW];
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[j][i] = 0;
        // both dy halves and the group's x taps, double-buffered by step parity: step s + 1's
        // fragments are read during step s, both dy halves after MFMA 0, x tap i after MFMA i + 1
        v4i fd[2][2], fx[2][NX];
        auto read_d = [&](auto st_c, auto buf_c) {
            constexpr int ST = decltype(st_c)::value, BUF = decltype(buf_c)::value;
            const v2i a0 = tr8_at<ST * SB>(aD0), a1 = tr8_at<ST * SB + 512>(aD0);
            const v2i b0 = tr8_at<ST * SB>(aD1), b1 = tr8_at<ST * SB + 512>(aD1);
            fd[BUF][0] = v4i{a0[0], a0[1], a1[0], a1[1]};
            fd[BUF][1] = v4i{b0[0], b0[1], b1[0], b1[1]};
        };
        auto read_x = [&](auto st_c, auto buf_c, auto i_c) {
            constexpr int ST = decltype(st_c)::value, BUF = decltype(buf_c)::value, I = decltype(i_c)::value;
            const v2i x0 = tr8_at<ST * SB>(aX[I][0]), x1 = tr8_at<ST * SB>(aX[I][1]);
            fx[BUF][I] = v4i{x0[0], x0[1], x1[0], x1[1]};
        };
        // MFMA j of step s (stage ST, buffers CUR); after it, the next step's reads of gap j
        // (into CUR ^ 1) and after MFMA 1 the LDS-DMA of step s + STAGES - 1.  The counted lgkm
        // wait before MFMA j lets through the reads issued after its x tap's (TapGroup::wait).
        auto gap = [&](auto u_c, auto j_c, auto ss_c, int s, bool more, bool dma) {
            constexpr int U = decltype(u_c)::value, J = decltype(j_c)::value;
            constexpr bool SS = decltype(ss_c)::value;
            constexpr int ST = U % STAGES, CUR = U & 1, NST = (ST + 1) % STAGES;
            constexpr int CH = TG::ch(J), XI = TG::xi(J);
            if (SS || more)
                lgkm_wait<TG::wait(J, true)>();
            else
                lgkm_wait<TG::wait(J, false)>();
            reg_fence(fx[CUR][XI]);
            reg_fence(fd[CUR][CH]);
            if (NITI_ABLATE == 2 || NITI_ABLATE == 6)
                acc[J][0] += fd[CUR][CH][0] ^ fx[CUR][XI][1];
            else
                acc[J] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fd[CUR][CH], fx[CUR][XI], acc[J], 0, 0, 0);
            if ((SS || more) && NITI_ABLATE != 9) {
                if constexpr (J == 0)
                    read_d(std::integral_constant<int, NST>(), std::integral_constant<int, CUR ^ 1>());
                else if constexpr (J - 1 < NX)
                    read_x(std::integral_constant<int, NST>(), std::integral_constant<int, CUR ^ 1>(),
                           std::integral_constant<int, J - 1>());
            }
            if constexpr (J == 1) {
                if (SS || dma) issue((ST + STAGES - 1) % STAGES, s + STAGES - 1);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        auto body = [&](auto u_c, auto ss_c, int s) {
            constexpr bool SS = decltype(ss_c)::value;
            const bool more = s + 1 < nsteps, dma = s + STAGES - 1 < nsteps;
            // own loads of step s + 1 landed (steps up to s + 2 may be in flight)
            if (SS)
                wait_vmcnt<(STAGES - 3) * LOADS>();
            else if (more)
                wait_steps<LOADS, STAGES - 3>(min(STAGES - 3, nsteps - 2 - s));
            if (NITI_ABLATE != 4) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            [&]<int... J>(std::integer_sequence<int, J...>) {
                (gap(u_c, std::integral_constant<int, J>(), ss_c, s, more, dma), ...);
            }(std::make_integer_sequence<int, NTW>());
        };

#pragma unroll
        for (int st = 0; st < STAGES - 1; ++st)
            if (st < nsteps) issue(st, st);
        if (nsteps > 0) {
            wait_steps<LOADS, STAGES - 2>(min(STAGES - 2, nsteps - 1));
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            // step 0's reads in a step's gap order (its first waits count on that order)
            read_d(std::integral_constant<int, 0>(), std::integral_constant<int, 0>());
            [&]<int... I>(std::integer_sequence<int, I...>) {
                (read_x(std::integral_constant<int, 0>(), std::integral_constant<int, 0>(),
                        std::integral_constant<int, I>()),
                 ...);
            }(std::make_integer_sequence<int, NX>());
        }
        TAPS_STAMP(1);
        if (NITI_TAPS_PRIO && wid >= 4) __builtin_amdgcn_s_setprio(1);
        // steady state: STAGES straight-line steps per iteration while every step has its DMA;
        // then the tail with run-time conditions
        int s = 0;
        for (; s + 2 * STAGES - 2 < nsteps; s += STAGES) {
            [&]<int... U>(std::integer_sequence<int, U...>) {
                (body(std::integral_constant<int, U>(), std::true_type(), s + U), ...);
            }(std::make_integer_sequence<int, STAGES>());
        }
        for (; s < nsteps; s += STAGES) {
            [&]<int... U>(std::integer_sequence<int, U...>) {
                ((s + U < nsteps ? body(std::integral_constant<int, U>(), std::false_type(), s + U) : void()), ...);
            }(std::make_integer_sequence<int, STAGES>());
        }
        lgkm_wait<0>();
        // hipcc cannot prove the tail runs at least once after the steady-state loop, so on its
        // (dead) steady-exit path the look-ahead fragments are in flight; keep every fragment
        // register live through the drain so none is reused ahead of it
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            reg_fence(fd[b][0]);
            reg_fence(fd[b][1]);
#pragma unroll
            for (int i = 0; i < NX; ++i) reg_fence(fx[b][i]);
        }
        if (NITI_TAPS_PRIO && wid >= 4) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        TAPS_STAMP(2);

        // the two K groups meet: K group 0 keeps tiles [0, KA) of the group, K group 1 the rest;
        // each sends the other part (MFMA C layout, 16-byte LDS writes), adds its partner's,
        // then writes the kept tiles row-major into the staged tile ct [64][LDT]
        constexpr int KA = (NTW + 1) / 2;
        v4i* xbuf = (v4i*)smem;
        const int xs0 = tg * TA * 256;  // v4i index of the group's first tile
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const bool mine = kg == 0 ? j < KA : j >= KA;
            if (!mine) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    xbuf[xs0 + j * 256 + q * 64 + lane] =
                        v4i{acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]};
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const bool mine = kg == 0 ? j < KA : j >= KA;
            if (mine) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const v4i v = xbuf[xs0 + j * 256 + q * 64 + lane];
                    acc[j][4 * q] += v[0];
                    acc[j][4 * q + 1] += v[1];
                    acc[j][4 * q + 2] += v[2];
                    acc[j][4 * q + 3] += v[3];
                }
            }
        }
        __syncthreads();  // ct overlays the exchange buffer
        int32_t* ct = (int32_t*)smem;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const bool mine = kg == 0 ? j < KA : j >= KA;
            if (mine) {
                const int ch = TG::ch(j), tap = TG::tap(TG::xi(j));
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int row = ch * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
                    ct[row * LDT + tap * 32 + (lane & 31)] = acc[j][i];
                }
            }
        }
    };
    switch (tg) {
        case 0: run(std::integral_constant<int, 0>()); break;
        case 1: run(std::integral_constant<int, 1>()); break;
        case 2: run(std::integral_constant<int, 2>()); break;
        default: run(std::integral_constant<int, 3>()); break;
    }
    __syncthreads();
    TAPS_STAMP(3);
    // 16-byte row chunks: 8 consecutive threads write one 128-byte (tap, 32-channel) segment
    // (SLAB: the block's partial tile as one contiguous run of its split's tile-blocked slab --
    // sequential 16-byte stores drain at HBM write speed, where 128-byte segments strided over
    // the [co][tap][ci] matrix by all 256 blocks at once drained at ~2.7 TB/s)
    const int32_t* ct = (const int32_t*)smem;
    int32_t* Cs = MODE == EPI_SLAB ? epi.C + (int64_t)split * epi.slab_stride + (int64_t)tile * (64 * NT * 32) : epi.C;
    constexpr int CPR = NT * 8;  // chunks per tile row
    const int rows = min(64, g.c_out - co0);
    uint32_t lmax = 0;
    for (int c = tid; c < rows * CPR; c += TAPS_THREADS) {
        const int row = c / CPR, rem = c - row * CPR;
        const int t = rem >> 3, part = rem & 7;
        const v4i v = *(const v4i*)(ct + row * LDT + t * 32 + part * 4);
        v4i* dst = MODE == EPI_SLAB ? (v4i*)(Cs + c * 4)
                                    : (v4i*)(Cs + (int64_t)(co0 + row) * epi.ldc + t * g.CIP + ci0 + part * 4);
        if (NITI_ABLATE >= 5)  // diagnostic: no tile stores (timing of the rest)
            asm volatile("" ::"v"(v), "v"(dst));
        else if (NITI_TAPS_NT == 2)
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
        else if (NITI_TAPS_NT)
            __builtin_nontemporal_store(v, dst);
        else
            *dst = v;
        if (MODE == EPI_STORE) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t uu = uabs32(v[j]);
                lmax = lmax > uu ? lmax : uu;
            }
        }
    }
    if (MODE == EPI_STORE) {
        lmax = wave_max(lmax);
        __syncthreads();
        uint32_t* red = (uint32_t*)smem;
        if (lane == 0) red[wid] = lmax;
        __syncthreads();
        if (tid == 0 && epi.amax != nullptr) {
            uint32_t m = red[0];
            for (int i = 1; i < NW; ++i) m = m > red[i] ? m : red[i];
            publish_max(epi.amax, m);
        }
    }
    if (NITI_STAMPS) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        TAPS_STAMP(5);
    }
    span_end(g.span, span_t0);
}


// Kernel-event probe: the next weight-gradient launch records these two events as part of its
// own dispatch (hipExtLaunchKernel), i.e. the kernel's begin / end as rocprofv3 sees them.
static hipEvent_t g_ev_next[2] = {nullptr, nullptr};
void probe_events_arm(hipEvent_t begin, hipEvent_t end) {
    g_ev_next[0] = begin;
    g_ev_next[1] = end;
}
static void take_events(hipEvent_t* b, hipEvent_t* e) {
    *b = g_ev_next[0];
    *e = g_ev_next[1];
    g_ev_next[0] = g_ev_next[1] = nullptr;
}
static unsigned long long* g_span_next = nullptr;
void probe_span_arm(unsigned long long* slot) { g_span_next = slot; }
static unsigned long long* take_span() {
    unsigned long long* p = g_span_next;
    g_span_next = nullptr;
    return p;
}

// ------------------------------------------------------------------------------ planning
// STRAT_SPEC: the speculative pair (forward / input gradient, no K split): launch A requantises
// with the layer's previous bit width and publishes the max, launch B redoes the GEMM only when
// the (all-reduced) max's bit width differs -- one GEMM pass on a hit, no int32 tensor.  Callers
// that run the two-phase entry points take it as STRAT_RECOMPUTE (same results).
// STRAT_FUSED: one launch with the rescale fused behind an in-kernel grid barrier (act_fused) where
// every tile is resident and nothing spans ranks; elsewhere it runs as STRAT_RECOMPUTE
enum Strategy { STRAT_STORE = 0, STRAT_RECOMPUTE = 1, STRAT_SLAB = 2, STRAT_SPEC = 3, STRAT_FUSED = 4 };
static bool recomputes(int strat) { return strat == STRAT_RECOMPUTE || strat == STRAT_FUSED; }

struct GemmPlan {
    int bm = 128, bn = 128, tiles = 1, splits = 1, kc_per_split = 0;
    Strategy strat = STRAT_STORE;
    bool taps = false;  // weight gradient on wgrad_taps_kernel (kc_per_split counts 64-pixel region steps)
};

// k_total: K extent in the kernel's units (16-byte chunks for KT = false, k rows for
// KT = true); k_step: units per K step; k_bytes: K in bytes (recompute threshold).
// Distance between K-split slabs: an odd number of 4 KiB pages, so the same offset in every
// slab falls in a different HBM channel (a power-of-two stride such as 8 MiB put all S reads
// of one output element on one channel: the 3-slab reduces ran at ~1 TB/s).
static size_t slab_stride_elems(int M, int N) {
    size_t pages = ((size_t)M * N * 4 + 4095) / 4096;
    if ((pages & 1) == 0) ++pages;
    return pages * 1024;
}

// Plan overrides: the model's autotuner (niti_model.hip, Model::autotune) times candidate
// plans for each of its GEMM shapes on the device and records the fastest here; plan_gemm
// consults the table first.  Every plan computes the same exact int32 sums, so an override
// changes speed only, never a result.
namespace {
std::mutex g_plan_mu;
std::map<PlanKey, PlanChoice> g_plan_tab;
std::atomic<unsigned> g_plan_epoch{1};
}  // namespace

void plan_override_set(const PlanKey& k, const PlanChoice& c) {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    g_plan_tab[k] = c;
    g_plan_epoch.fetch_add(1);
}
void plan_override_clear(const PlanKey& k) {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    g_plan_tab.erase(k);
    g_plan_epoch.fetch_add(1);
}
void plan_override_clear_all() {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    g_plan_tab.clear();
    g_plan_epoch.fetch_add(1);
}
unsigned plan_override_epoch() { return g_plan_epoch.load(); }
bool plan_override_lookup(const PlanKey& k, PlanChoice* c) {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    auto it = g_plan_tab.find(k);
    if (it == g_plan_tab.end()) return false;
    *c = it->second;
    return true;
}
// the NHWC16 planners ignore P16 weight-gradient plans (the model runs those itself)
static bool plan_override_get(const PlanKey& k, PlanChoice* c) {
    return plan_override_lookup(k, c) && c->bm != PLAN_P16_TILE;
}

static void plan_slab(GemmPlan& p, int s, int k_total, int k_step, int steps, bool recompute, int M, int N,
                      size_t ws_elems) {
    if (s > steps) s = steps;
    const size_t slab = slab_stride_elems(M, N);
    while (s > 1 && (size_t)s * slab > ws_elems) --s;
    if (s < 2) {
        p.strat = recompute ? STRAT_RECOMPUTE : STRAT_STORE;
        return;
    }
    const int per = ((steps + s - 1) / s) * k_step;
    p.splits = (k_total + per - 1) / per;
    p.kc_per_split = per;
    p.strat = p.splits > 1 ? STRAT_SLAB : (recompute ? STRAT_RECOMPUTE : STRAT_STORE);
    if (p.splits == 1) p.kc_per_split = steps * k_step;
}

static GemmPlan plan_gemm(int M, int N, int k_total, int k_step, int k_bytes, bool recompute_ok, size_t ws_elems,
                          int op = -1) {
    GemmPlan p;
    const int steps = (k_total + k_step - 1) / k_step;
    p.kc_per_split = steps * k_step;
    PlanChoice c;
    if (op >= 0 && plan_override_get(PlanKey{op, M, N, k_total}, &c)) {
        p.bm = c.bm == 64 ? 64 : (c.bm == 256 ? 256 : 128);
        p.bn = c.bn == 64 ? 64 : (c.bn == 256 ? 256 : 128);
        p.tiles = ((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
        if (c.strat == STRAT_SLAB) {
            plan_slab(p, c.splits, k_total, k_step, steps, false, M, N, ws_elems);
        } else if (c.strat == STRAT_SPEC) {
            p.strat = recompute_ok ? STRAT_SPEC : STRAT_STORE;
        } else if (c.strat == STRAT_FUSED) {
            p.strat = recompute_ok ? STRAT_FUSED : STRAT_STORE;
        } else {
            p.strat = c.strat == STRAT_RECOMPUTE && recompute_ok ? STRAT_RECOMPUTE : STRAT_STORE;
        }
        return p;
    }
    p.bn = N <= 64 ? 64 : 128;
    p.bm = (M <= 64 && p.bn >= 64) ? 64 : 128;
    if (const char* f = getenv("NITI_DIAG_TILE")) {  // diagnostics (tools/): force a tile shape
        const int v = atoi(f);
        if (v == 64 || v == 6464) p.bm = p.bn = 64;
        if (v == 12864) { p.bm = 128; p.bn = 64; }
        if (v == 64128) { p.bm = 64; p.bn = 128; }
        if (v == 256128) { p.bm = 256; p.bn = 128; }
        if (v == 128256) { p.bm = 128; p.bn = 256; }
        if (v == 256256) { p.bm = 256; p.bn = 256; }
    }
    p.tiles = ((M + p.bm - 1) / p.bm) * ((N + p.bn - 1) / p.bn);
    const bool recompute = recompute_ok && k_bytes <= 1152;
    if (p.tiles >= 160 || steps < 12) {
        // enough workgroups (or too little K to split): one pass; for small K recomputing the
        // GEMM is cheaper than an int32 round trip through HBM
        p.strat = recompute ? STRAT_RECOMPUTE : STRAT_STORE;
        return p;
    }
    // one block per CU: tiles * splits <= 256 (measured best against 320 and 512 block targets
    // on the VGG-11 weight and input gradients, tools/gpu_splits.sh)
    int s = 256 / p.tiles;
    const int max_s = steps / 4;
    if (s > max_s) s = max_s;
    if (const char* f = getenv("NITI_DIAG_SPLITS")) {  // diagnostics (tools/): force the split count
        const int v = atoi(f);
        if (v >= 1) s = v < steps ? v : steps;
    }
    plan_slab(p, s, k_total, k_step, steps, recompute, M, N, ws_elems);
    return p;
}

PlanChoice plan_query(const PlanKey& k, int k_step, bool recompute_ok, size_t ws_bytes) {
    const GemmPlan p = plan_gemm(k.M, k.N, k.K, k_step, k.K * 16, recompute_ok, ws_bytes / 4, k.op);
    PlanChoice c;
    c.bm = p.bm;
    c.bn = p.bn;
    c.splits = p.strat == STRAT_SLAB ? p.splits : 1;
    c.strat = p.strat;
    return c;
}

size_t plan_slab_bytes(int M, int N, int splits) { return (size_t)splits * slab_stride_elems(M, N) * 4; }

// the workspace of the default plan, or of a forced one (op >= 0: plan_override_set, e.g. autotuned
// plans of a caller that sizes its workspace per call) when that needs more
static size_t plan_ws_elems(int M, int N, int k_total, int k_step, int op = -1) {
    GemmPlan p = plan_gemm(M, N, k_total, k_step, 1 << 30, false, (size_t)-1);
    size_t e = p.strat == STRAT_SLAB ? (size_t)p.splits * slab_stride_elems(M, N) : 0;
    if (op >= 0) {
        const GemmPlan q = plan_gemm(M, N, k_total, k_step, 1 << 30, false, (size_t)-1, op);
        if (q.strat == STRAT_SLAB) e = std::max(e, (size_t)q.splits * slab_stride_elems(M, N));
    }
    return e;
}

template <class LA, class LB, int MODE, bool KT>
static hipError_t launch_mode(const GemmPlan& p, const LA& la, const LB& lb, int M, int N, int k_total,
                              const Epi& epi, hipStream_t st) {
    const int k_step = KT ? KT_BK : LA::BK / 16;
    const int splits = MODE == EPI_SLAB ? p.splits : 1;
    const int per = MODE == EPI_SLAB ? p.kc_per_split : ((k_total + k_step - 1) / k_step) * k_step;
    hipEvent_t ev_b = nullptr, ev_e = nullptr;
    if (KT) take_events(&ev_b, &ev_e);  // weight gradient: the kernel-event probe, if armed
#define NITI_LAUNCH(BM_, BN_, WM_, WN_, NW_)                                                                      \
    do {                                                                                                          \
        const int tm = (M + BM_ - 1) / BM_, tn = (N + BN_ - 1) / BN_;                                             \
        dim3 grid(tm * tn, splits);                                                                               \
        if (ev_b != nullptr)                                                                                      \
            hipExtLaunchKernelGGL((gemm_kernel<BM_, BN_, WM_, WN_, LA, LB, MODE, KT, NW_>), grid, dim3(NW_ * 64), \
                                  0, st, ev_b, ev_e, 0, la, lb, M, N, tn, k_total, per, epi);                     \
        else                                                                                                      \
            hipLaunchKernelGGL((gemm_kernel<BM_, BN_, WM_, WN_, LA, LB, MODE, KT, NW_>), grid, dim3(NW_ * 64), 0, \
                               st, la, lb, M, N, tn, k_total, per, epi);                                          \
    } while (0)
    // per-wave tiles: 64x64 (two wave groups over K for 128x128), 64x32 / 32x64 for the
    // 4-wave shapes, 128x64 for 256x256
    if (p.bn == 64 && p.bm == 64)
        NITI_LAUNCH(64, 64, 2, 2, 4);
    else if (p.bn == 64)
        NITI_LAUNCH(128, 64, 2, 2, 4);
    else if (p.bm == 64)
        NITI_LAUNCH(64, 128, 1, 4, 4);
    else if (p.bm == 256 && p.bn == 256) {
        // (the fully connected layers' range / update passes take 128 x 256: at 256 x 256 their
        // weight-gradient instantiations move registers an in-flight fragment read still writes,
        // tools/isa_inflight.py)
        if constexpr (KT && (MODE == EPI_AMAX || MODE == EPI_SGD))
            NITI_LAUNCH(128, 256, 2, 4, 8);
        else
            NITI_LAUNCH(256, 256, 2, 4, 8);
    }
    else if (p.bm == 256)
        NITI_LAUNCH(256, 128, 4, 2, 8);
    else if (p.bn == 256)
        NITI_LAUNCH(128, 256, 2, 4, 8);
    else
        NITI_LAUNCH(128, 128, 2, 2, 8);
#undef NITI_LAUNCH
    return hipGetLastError();
}

// The kernel launch_mode would run for plan p (same dispatch), for the occupancy query
template <class LA, class LB, int MODE, bool KT>
static std::pair<const void*, int> gemm_fn(const GemmPlan& p) {
#define NITI_FN(BM_, BN_, WM_, WN_, NW_) \
    return {(const void*)&gemm_kernel<BM_, BN_, WM_, WN_, LA, LB, MODE, KT, NW_>, NW_ * 64}
    if (p.bn == 64 && p.bm == 64) NITI_FN(64, 64, 2, 2, 4);
    if (p.bn == 64) NITI_FN(128, 64, 2, 2, 4);
    if (p.bm == 64) NITI_FN(64, 128, 1, 4, 4);
    if (p.bm == 256 && p.bn == 256) {
        if constexpr (KT && (MODE == EPI_AMAX || MODE == EPI_SGD))
            NITI_FN(128, 256, 2, 4, 8);
        else
            NITI_FN(256, 256, 2, 4, 8);
    }
    if (p.bm == 256) NITI_FN(256, 128, 4, 2, 8);
    if (p.bn == 256) NITI_FN(128, 256, 2, 4, 8);
    NITI_FN(128, 128, 2, 2, 8);
#undef NITI_FN
}

template <class MAP = SlabLinear>
static hipError_t splitk_reduce(const GemmPlan& p, const int32_t* slab, int64_t n, int64_t stride, int32_t* C,
                                uint32_t* amax, hipStream_t st, MAP map = MAP()) {
    const int64_t n4 = n / 4;
    int G = 1;  // split-level parallelism only where the output alone cannot fill the GPU
    while (G < 16 && G * 2 <= p.splits && n4 * G < 131072) G <<= 1;
    const int64_t blocks = (n4 + (256 / G) - 1) / (256 / G);
    hipLaunchKernelGGL(splitk_reduce_kernel<MAP>, dim3((unsigned)blocks), dim3(256), 0, st, slab, p.splits, stride, n4,
                       G, C, amax, map);
    return hipGetLastError();
}

// C[i] = sum over splits z of slab[z * stride + i] (+ max|C|), n elements (n % 4 == 0); the split-K
// partials of the P16 weight gradient (niti_wgrad.hip) share C's layout
hipError_t splitk_reduce_linear(const int32_t* slab, int splits, int64_t n, int64_t stride, int32_t* C,
                                uint32_t* amax, hipStream_t st) {
    GemmPlan p;
    p.splits = splits;
    return splitk_reduce(p, slab, n, stride, C, amax, st);
}

// Materialise C [M][N] int32 (+ max|C| if amax) under plan p: STORE, or SLAB + reduce.
template <class LA, class LB, bool KT = false>
static hipError_t gemm_acc_plan(const GemmPlan& p, const LA& la, const LB& lb, int M, int N, int kc_total, int32_t* C,
                                uint32_t* amax, int32_t* ws, hipStream_t st, hipEvent_t after_gemm = nullptr,
                                SgdJob* defer = nullptr) {
    Epi e;
    if (KT) e.span = take_span();  // weight gradient: the kernel-span probe slot, if armed
    if (p.strat == STRAT_SLAB) {
        e.C = ws;
        e.ldc = N;
        e.slab_stride = (int64_t)slab_stride_elems(M, N);
        if (const char* f = getenv("NITI_DIAG_SPLIT_MAJOR")) e.split_major = atoi(f);
        hipError_t r = launch_mode<LA, LB, EPI_SLAB, KT>(p, la, lb, M, N, kc_total, e, st);
        if (r == hipSuccess && after_gemm != nullptr) r = hipEventRecord(after_gemm, st);
        if (r != hipSuccess) return r;
        // the NITI_SGD launch combines the slabs -- where each split has a few 1024-element chunks;
        // a small gradient over many splits (VGG-11 conv0: 2048 elements x 256 splits) reduces faster
        // here, splitk_reduce spreading the splits over blocks (the combine sums them serially)
        if (defer != nullptr && ((int64_t)M * N) % 4 == 0 && (int64_t)M * N >= (int64_t)p.splits * 4096) {
            defer->slab = ws;
            defer->splits = p.splits;
            defer->slab_stride = e.slab_stride;
            defer->slab_n = (int64_t)M * N;
            return hipSuccess;
        }
        return splitk_reduce(p, ws, (int64_t)M * N, e.slab_stride, C, amax, st);
    }
    e.C = C;
    e.ldc = N;
    e.amax = amax;
    hipError_t r = launch_mode<LA, LB, EPI_STORE, KT>(p, la, lb, M, N, kc_total, e, st);
    if (r == hipSuccess && after_gemm != nullptr) r = hipEventRecord(after_gemm, st);
    return r;
}

template <class LA, class LB, bool KT = false>
static hipError_t gemm_acc(int op, const LA& la, const LB& lb, int M, int N, int kc_total, int32_t* C, uint32_t* amax,
                           int32_t* ws, size_t ws_elems, hipStream_t st, hipEvent_t after_gemm = nullptr,
                           SgdJob* defer = nullptr) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const int k_step = KT ? KT_BK : LA::BK / 16;
    const GemmPlan p = plan_gemm(M, N, kc_total, k_step, 1 << 30, false, ws ? ws_elems : 0, op);
    return gemm_acc_plan<LA, LB, KT>(p, la, lb, M, N, kc_total, C, amax, ws, st, after_gemm, defer);
}

// Two-phase activation GEMM (forward / input gradient): phase 1 establishes max|acc| (and
// materialises acc unless the plan recomputes); phase 2 writes the requantised int8.
template <class LA, class LB>
static hipError_t act_phase1(int op, const LA& la, const LB& lb, int M, int N, int kc_total, int32_t* acc,
                             uint32_t* amax, int32_t* ws, size_t ws_elems, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const GemmPlan p = plan_gemm(M, N, kc_total, LA::BK / 16, kc_total * 16, true, ws ? ws_elems : 0, op);
    if (recomputes(p.strat) || p.strat == STRAT_SPEC) {
        Epi e;
        e.amax = amax;
        return launch_mode<LA, LB, EPI_AMAX, false>(p, la, lb, M, N, kc_total, e, st);
    }
    return gemm_acc_plan<LA, LB, false>(p, la, lb, M, N, kc_total, acc, amax, ws, st);
}

template <class LA, class LB>
static hipError_t act_phase2(int op, const LA& la, const LB& lb, int M, int N, int kc_total, const int32_t* acc,
                             const uint32_t* amax, const ActOut& o, size_t ws_elems, hipStream_t st) {
    const GemmPlan p = plan_gemm(M, N, kc_total, LA::BK / 16, kc_total * 16, true, ws_elems, op);
    if (recomputes(p.strat) || p.strat == STRAT_SPEC) {
        if (o.pool.pool_out != nullptr || o.pool.dx != nullptr || o.out_p16 != nullptr || o.pool3.out != nullptr)
            return hipErrorInvalidValue;
        Epi e;
        e.amax = const_cast<uint32_t*>(amax);
        e.out = o.out;
        e.ldo = N;
        e.relu = o.relu;
        e.relu_mask = o.relu_mask;
        e.exp_in = o.exp_in;
        e.wscale = o.wscale;
        e.exp_out = o.exp_out;
        return launch_mode<LA, LB, EPI_REQUANT, false>(p, la, lb, M, N, kc_total, e, st);
    }
    ActRequant r;
    r.acc = acc;
    r.rows = M;
    r.ldc = N;
    r.amax = amax;
    r.exp_in = o.exp_in;
    r.wscale = o.wscale;
    r.exp_out = o.exp_out;
    r.relu = o.relu;
    r.relu_mask = o.relu_mask;
    r.out_nhwc16 = o.out;
    r.pool = o.pool;
    r.out_p16 = o.out_p16;
    r.zero_cls = o.zero_cls;
    r.zc_h = o.zc_h;
    r.zc_w = o.zc_w;
    r.pool3 = o.pool3;
    return requant_act(r, st);
}

// diagnostics: launch A of every GEMM pair guesses the hint + this bias (tests: +-1 exercises the
// alternates, 2 the redone launch)
static int g_gemm_spec_bias = 0;
void gemm_speculate_bias(int bias) { g_gemm_spec_bias = bias; }

// The speculative pair (STRAT_SPEC): pass 0 = launch A, pass 1 = launch B (see Epi::spec)
template <class LA, class LB>
static hipError_t act_spec(int op, const LA& la, const LB& lb, int M, int N, int kc_total, uint32_t* amax,
                           const ActOut& o, uint32_t* hint, int pass, int8_t* alt, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (o.pool.pool_out != nullptr || o.pool.dx != nullptr || o.out_p16 != nullptr || hint == nullptr || o.out == nullptr)
        return hipErrorInvalidValue;
    const GemmPlan p = plan_gemm(M, N, kc_total, LA::BK / 16, kc_total * 16, true, 0, op);
    Epi e;
    e.amax = amax;
    e.out = o.out;
    e.ldo = N;
    e.relu = o.relu;
    e.relu_mask = o.relu_mask;
    e.exp_in = o.exp_in;
    e.wscale = o.wscale;
    e.exp_out = o.exp_out;
    e.spec = pass == 0 ? 1 : 2;
    e.hint = hint;
    e.hint_scale = op == PLAN_FWD ? 1 : 0;
    e.alt = alt;
    e.spec_bias = g_gemm_spec_bias;
    return launch_mode<LA, LB, EPI_REQUANT, false>(p, la, lb, M, N, kc_total, e, st);
}

// STRAT_FUSED: one launch, the rescale fused behind the grid barrier (Epi::bar).  hipErrorNotSupported
// (nothing launched) unless the plan is STRAT_FUSED and every tile is resident at once -- the
// caller then runs the two-phase form, which treats the plan as STRAT_RECOMPUTE.
static std::atomic<unsigned long long> g_fused_launches{0};
unsigned long long gemm_fused_launches() { return g_fused_launches.load(); }

template <class LA, class LB>
static hipError_t act_fused(int op, const LA& la, const LB& lb, int M, int N, int kc_total, const ActOut& o,
                            const FusedBar& fb, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const GemmPlan p = plan_gemm(M, N, kc_total, LA::BK / 16, kc_total * 16, true, 0, op);
    if (p.strat != STRAT_FUSED) return hipErrorNotSupported;
    if (o.pool.pool_out != nullptr || o.pool.dx != nullptr || o.out_p16 != nullptr || o.pool3.out != nullptr ||
        o.out == nullptr || fb.bar == nullptr || fb.err == nullptr)
        return hipErrorInvalidValue;
    const auto f = gemm_fn<LA, LB, EPI_REQUANT, false>(p);
    if (p.tiles > resident_wgs(f.first, f.second)) return hipErrorNotSupported;
    Epi e;
    e.out = o.out;
    e.ldo = N;
    e.relu = o.relu;
    e.relu_mask = o.relu_mask;
    e.exp_in = o.exp_in;
    e.wscale = o.wscale;
    e.exp_out = o.exp_out;
    e.bar = fb.bar;
    e.epoch = fb.epoch;
    e.err = fb.err;
    e.spin_limit = fb.spin_limit ? fb.spin_limit : BAR_SPIN_LIMIT;
    g_fused_launches.fetch_add(1);
    return launch_mode<LA, LB, EPI_REQUANT, false>(p, la, lb, M, N, kc_total, e, st);
}

// ------------------------------------------------------------------------------ per-op wrappers
bool conv_fwd_spec_ok(const ConvGeom& g) {
    const int kc = g.kh * g.kw * g.cip / 16;
    return plan_gemm(g.n * g.oh * g.ow, g.cop, kc, 64 / 16, kc * 16, true, 0, PLAN_FWD).strat == STRAT_SPEC;
}
bool conv_dgrad_spec_ok(const ConvGeom& g) {
    const int kc = g.kh * g.kw * g.cop / 16;
    return plan_gemm(g.n * g.h * g.w, g.cip, kc, 64 / 16, kc * 16, true, 0, PLAN_DGRAD).strat == STRAT_SPEC;
}
bool conv_fwd_phase2_separate(const ConvGeom& g, size_t ws_bytes) {
    const int kc = g.kh * g.kw * g.cip / 16;  // every forward operand loader steps 64 bytes
    return !recomputes(plan_gemm(g.n * g.oh * g.ow, g.cop, kc, 64 / 16, kc * 16, true, ws_bytes / 4, PLAN_FWD).strat);
}
bool conv_dgrad_phase2_separate(const ConvGeom& g, size_t ws_bytes) {
    const int kc = g.kh * g.kw * g.cop / 16;
    return !recomputes(plan_gemm(g.n * g.h * g.w, g.cip, kc, 64 / 16, kc * 16, true, ws_bytes / 4, PLAN_DGRAD).strat);
}
static RowsK rows_k(const int8_t* p, int64_t ld, int rows, int kc_total) {
    RowsK r;
    r.p = p;
    r.ld = ld;
    r.rows = rows;
    r.kc_total = kc_total;
    r.bytes = (uint32_t)(ld * rows);
    return r;
}
static LoadConvFwd fwd_loader(const ConvGeom& g, const int8_t* x) {
    LoadConvFwd la;
    la.x = x;
    la.H = g.h;
    la.W = g.w;
    la.CPC = g.cip / 16;
    la.OH = g.oh;
    la.OW = g.ow;
    la.KW = g.kw;
    la.sh = g.sh;
    la.sw = g.sw;
    la.pt = g.pt;
    la.pl = g.pl;
    la.dh = g.dh;
    la.dw = g.dw;
    la.M = g.n * g.oh * g.ow;
    la.kc_total = g.kh * g.kw * la.CPC;
    la.img = (uint32_t)((int64_t)g.h * g.w * g.cip);
    la.bytes = (uint32_t)((int64_t)g.n * la.img);
    return la;
}
static LoadConvDgrad dgrad_loader(const ConvGeom& g, const int8_t* dy) {
    LoadConvDgrad la;
    la.dy = dy;
    la.OH = g.oh;
    la.OW = g.ow;
    la.CPC = g.cop / 16;
    la.H = g.h;
    la.W = g.w;
    la.KW = g.kw;
    la.sh = g.sh;
    la.sw = g.sw;
    la.pt = g.pt;
    la.pl = g.pl;
    la.dh = g.dh;
    la.dw = g.dw;
    la.M = g.n * g.h * g.w;
    la.kc_total = g.kh * g.kw * la.CPC;
    la.img = (uint32_t)((int64_t)g.oh * g.ow * g.cop);
    la.bytes = (uint32_t)((int64_t)g.n * la.img);
    return la;
}
// Tap-aligned operands (ConvTaps) where the channel padding allows it, else the per-lane loaders.
template <int BKB>
static ConvTaps<BKB> conv_taps(const ConvGeom& g, const int8_t* src, bool fwd) {
    ConvTaps<BKB> t;
    t.src = src;
    t.SH = fwd ? g.h : g.oh;
    t.SW = fwd ? g.w : g.ow;
    t.CPC = (fwd ? g.cip : g.cop) / 16;
    t.PH = fwd ? g.oh : g.h;
    t.PW = fwd ? g.ow : g.w;
    t.sh = fwd ? g.sh : 1;
    t.sw = fwd ? g.sw : 1;
    t.oy_add = fwd ? -g.pt : g.pt;
    t.ox_add = fwd ? -g.pl : g.pl;
    t.dh = g.dh;
    t.dw = g.dw;
    t.KH = g.kh;
    t.KW = g.kw;
    t.M = g.n * t.PH * t.PW;
    t.sgn = fwd ? 1 : -1;
    t.img = (uint32_t)((int64_t)t.SH * t.SW * t.CPC * 16);
    t.bytes = (uint32_t)((int64_t)g.n * t.img);
    return t;
}
// K bytes per step of the forward / input-gradient operand (0 = per-lane loader, 64 bytes)
static int fwd_taps_bk(const ConvGeom& g) {
    if (g.kh * g.kw > 32) return 0;
    return g.cip % 64 == 0 ? 64 : 0;  // 128-byte steps measured slower (one block per CU)
}
static int dgrad_taps_bk(const ConvGeom& g) {
    if (g.kh * g.kw > 32 || g.sh != 1 || g.sw != 1) return 0;
    return g.cop % 64 == 0 ? 64 : 0;
}
// a 1x1, stride-1, unpadded conv is a plain GEMM over the activation rows: x [pixels][cip] (forward),
// dy [pixels][cop] (input gradient) and, K-major, x again (weight gradient) -- the row-major
// loaders with no per-lane address arithmetic (ResNet-18's stem over its 160-column im2col, the fc
// heads); a per-lane conv loader gathered those rows at ~2 TB/s
static bool plain_1x1(const ConvGeom& g) {
    return g.kh == 1 && g.kw == 1 && g.sh == 1 && g.sw == 1 && g.dh == 1 && g.dw == 1 && g.pt == 0 && g.pl == 0 &&
           g.pb == 0 && g.pr == 0 && g.oh == g.h && g.ow == g.w &&
           (int64_t)g.n * g.h * g.w * (g.cip > g.cop ? g.cip : g.cop) < ((int64_t)1 << 31);
}
template <class F>
static hipError_t with_fwd_operand(const ConvGeom& g, const int8_t* x, F&& f) {
    if (plain_1x1(g)) return f(rows_k(x, g.cip, g.n * g.h * g.w, g.cip / 16));
    const int bk = fwd_taps_bk(g);
    if (bk == 64) return f(conv_taps<64>(g, x, true));
    return f(per_lane<LoadConvFwd, false>(fwd_loader(g, x)));
}
template <class F>
static hipError_t with_dgrad_operand(const ConvGeom& g, const int8_t* dy, F&& f) {
    if (plain_1x1(g)) return f(rows_k(dy, g.cop, g.n * g.h * g.w, g.cop / 16));
    const int bk = dgrad_taps_bk(g);
    if (bk == 64) return f(conv_taps<64>(g, dy, false));
    return f(per_lane<LoadConvDgrad, false>(dgrad_loader(g, dy)));
}
static void wgrad_operands(const ConvGeom& g, const int8_t* x, const int8_t* dy, KtRowsU* la, KtIm2col* lb) {
    const int K = g.n * g.oh * g.ow;
    la->p = dy;
    la->ld = g.cop;
    la->cols = g.cop;
    la->K = K;
    la->bytes = (uint32_t)((int64_t)K * g.cop);
    lb->x = x;
    lb->H = g.h;
    lb->W = g.w;
    lb->OH = g.oh;
    lb->OW = g.ow;
    lb->CIP = g.cip;
    lb->KW = g.kw;
    lb->sh = g.sh;
    lb->sw = g.sw;
    lb->pt = g.pt;
    lb->pl = g.pl;
    lb->dh = g.dh;
    lb->dw = g.dw;
    lb->ncols = g.kh * g.kw * g.cip;
    lb->K = K;
    lb->fOW = make_fastdiv((uint32_t)g.ow);
    lb->fOH = make_fastdiv((uint32_t)g.oh);
    lb->bytes = (uint32_t)((int64_t)g.n * g.h * g.w * g.cip);
}

// ------------------------------------------------------------------------------ tap-sharing wgrad
// NITI_TAPS_TILE=0: segment mode instead of 4-row tiles (A/B); NITI_TAPS_SEG_MAX_CIP: the widest input
// the segment / tile modes take
static bool taps_tile_mode() {
    static const bool on = !(getenv("NITI_TAPS_TILE") && atoi(getenv("NITI_TAPS_TILE")) == 0);
    return on;
}
static int taps_seg_max_cip() {
    static const int v = getenv("NITI_TAPS_SEG_MAX_CIP") ? atoi(getenv("NITI_TAPS_SEG_MAX_CIP")) : 128;
    return v;
}

// Geometry of wgrad_taps_kernel, or false where it does not apply (the generic KT GEMM runs).
static bool wgrad_taps_geom(const ConvGeom& g, const int8_t* x, const int8_t* dy, WgTaps* t) {
    if (const char* f = getenv("NITI_DIAG_NO_TAPS")) {  // diagnostics / tests: generic KT GEMM only
        if (atoi(f) != 0) return false;
    }
    if (g.kh != 3 || g.kw != 3 || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1) return false;
    if (g.cip % 32 != 0 || g.cop % 64 != 0) return false;
    const int64_t ohw = (int64_t)g.oh * g.ow;
    const int64_t K = (int64_t)g.n * ohw;
    const int64_t xbytes = (int64_t)g.n * g.h * g.w * g.cip, dybytes = K * g.cop;
    if (xbytes >= (int64_t)OOB || dybytes >= (int64_t)OOB) return false;
    WgTaps w{};
    // segment / tile modes: rows of 16-pixel (or 14-pixel) segments, pad 1 (output rows = input
    // rows), inputs up to 128 channels: faster than the K-major GEMM at 64 (VGG-16 conv1_2 180 vs
    // 378 us, conv2_1 93 vs 106 us), level with it at 128 (conv2_2 in tile mode 171.5 vs 166-169 us,
    // with a fraction of its traffic: the GEMM fetches x once per tap), 13 - 40 % slower at 256 - 512
    // in segment mode (tools/gpu_r04g.sh, gpu_r04p.sh); the autotuner picks per layer
    const int sw = g.ow % 16 == 0 ? 16 : (g.ow % 14 == 0 ? 14 : 0);
    const bool seg_ok = sw > 0 && g.cip <= taps_seg_max_cip() && g.oh == g.h && g.ow == g.w && g.pt == 1 && g.pl == 1 && g.pb == 1 && g.pr == 1 &&
                        g.kh == 3 && g.kw == 3 && !getenv("NITI_DIAG_NO_TAPS_SEG");
    if (64 % g.ow == 0 && ohw % 64 == 0) {
        w.band = 1;
        w.rows_per_step = 64 / g.ow;
        w.RH = w.rows_per_step + g.kh - 1;
        w.imgs = 1;
        w.PPI = 64;
    } else if (64 % ohw == 0 && K % 64 == 0) {
        w.band = 0;
        w.rows_per_step = 0;
        w.RH = g.oh + g.kh - 1;
        w.imgs = (int)(64 / ohw);
        w.PPI = (int)ohw;
    } else if (seg_ok && g.oh % 4 == 0 && taps_tile_mode()) {  // 4-row tiles
        w.seg = 2;
        w.SW = sw;
        w.NS = g.ow / sw;
        w.NB = g.oh / 4;
        w.nseg = g.n * w.NB * w.NS;
        w.band = 0;
        w.rows_per_step = 0;
        w.RH = 6;
        w.imgs = 1;
        w.PPI = 64;
    } else if (seg_ok) {
        w.seg = 1;
        w.SW = sw;
        w.NS = g.ow / sw;
        w.nseg = g.n * g.oh * w.NS;
        w.band = 0;
        w.rows_per_step = 0;
        w.RH = 3;
        w.imgs = 4;
        w.PPI = 16;
    } else {
        return false;
    }
    w.RW = (w.seg ? 16 : g.ow) + g.kw - 1;
    if (w.imgs * w.RH * w.RW > 256) return false;  // region rows (XPW <= 2)
    w.x = x;
    w.dy = dy;
    w.xbytes = (uint32_t)xbytes;
    w.dybytes = (uint32_t)dybytes;
    w.H = g.h;
    w.W = g.w;
    w.OH = g.oh;
    w.OW = g.ow;
    w.CIP = g.cip;
    w.COP = g.cop;
    w.KW = g.kw;
    w.pt = g.pt;
    w.pl = g.pl;
    w.c_out = g.c_out;
    w.rs_total = w.seg == 2 ? w.nseg : w.seg ? (w.nseg + 3) / 4 : (int)(K / 64);
    w.steps_total = w.rs_total;
    w.steps_per_split = w.steps_total;
    w.tiles_ci = g.cip / 32;
    w.tiles = (g.cop / 64) * w.tiles_ci;
    w.fRW = make_fastdiv((uint32_t)w.RW);
    w.fRPI = make_fastdiv((uint32_t)(w.RH * w.RW));
    w.fPPI = make_fastdiv((uint32_t)w.PPI);
    w.fOW = make_fastdiv((uint32_t)(w.seg ? 16 : g.ow));
    if (w.seg) {  // a region image is one 16-slot segment (tile mode: 4 of them stacked)
        w.OW = 16;
        w.fNS = make_fastdiv((uint32_t)w.NS);
        w.fH = make_fastdiv((uint32_t)g.h);
        if (w.seg == 2) w.fNB = make_fastdiv((uint32_t)w.NB);
    }
    w.fOHW = make_fastdiv((uint32_t)ohw);
    w.fTiles = make_fastdiv((uint32_t)w.tiles);
    w.fTci = make_fastdiv((uint32_t)w.tiles_ci);
    w.BPI = w.band ? g.oh / w.rows_per_step : 1;
    w.fBPI = make_fastdiv((uint32_t)w.BPI);
    *t = w;
    return true;
}

bool conv_wgrad_taps_ok(const ConvGeom& g) {
    WgTaps t;
    return wgrad_taps_geom(g, nullptr, nullptr, &t);
}

// splits: override (ov) or one block per CU with >= 4 steps per split
// rows of a tile-blocked taps slab: whole 64-row output-channel tiles
static int taps_slab_rows(const WgTaps& t) { return t.COP / 64 * 64; }

static GemmPlan plan_taps(const WgTaps& t, int M, int N, size_t ws_elems, const PlanChoice* ov) {
    GemmPlan p;
    p.taps = true;
    p.bm = p.bn = PLAN_TAPS_TILE;
    p.tiles = t.tiles;
    int s;
    if (ov != nullptr) {
        s = ov->strat == STRAT_SLAB ? ov->splits : 1;
    } else {
        s = 256 / t.tiles;
        if (s > t.steps_total / 4) s = t.steps_total / 4;
        if (const char* f = getenv("NITI_DIAG_SPLITS")) s = atoi(f);  // diagnostics / tests
    }
    if (s < 1) s = 1;
    p.kc_per_split = t.steps_total;
    p.strat = STRAT_STORE;
    if (s >= 2) plan_slab(p, s, t.steps_total, 1, t.steps_total, false, taps_slab_rows(t), N, ws_elems);
    (void)M;
    return p;
}

#if NITI_STAMPS
// diagnostic builds only: medians over blocks of the stamp intervals (us at the kernel's clock)
static void taps_stamp_report(const unsigned long long* d, int blocks, hipStream_t st) {
    std::vector<unsigned long long> h((size_t)blocks * 8);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return;
    auto med = [&](int a, int b) {
        std::vector<double> v;
        for (int i = 0; i < blocks; ++i) v.push_back((double)(h[i * 8 + b] - h[i * 8 + a]));
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    unsigned long long t0 = ~0ull, t1 = 0, r0 = ~0ull, r1 = 0;
    for (int i = 0; i < blocks; ++i) {
        t0 = std::min(t0, h[i * 8]);
        t1 = std::max(t1, h[i * 8 + 5]);
        r0 = std::min(r0, h[i * 8 + 6]);
        r1 = std::max(r1, h[i * 8 + 7]);
    }
    const double ghz = (double)(t1 - t0) / ((double)(r1 - r0) * 10.0);  // memrealtime = 100 MHz
    fprintf(stderr, "taps stamps: blocks %d clk %.2f GHz span %.2f us | prologue %.0f loop %.0f xchg %.0f store %.0f cyc\n",
            blocks, ghz, (r1 - r0) / 100.0, med(0, 1), med(1, 2), med(2, 3), med(3, 5));
}
#endif

template <int MODE>
static hipError_t launch_taps(const GemmPlan& p, WgTaps t, const Epi& e, hipStream_t st) {
    const int splits = MODE == EPI_SLAB ? p.splits : 1;
    t.steps_per_split = MODE == EPI_SLAB ? p.kc_per_split : t.steps_total;
    const dim3 grid((unsigned)(t.tiles * splits));
    t.stamps = nullptr;
    t.span = e.span;
#if NITI_STAMPS
    static unsigned long long* sbuf = nullptr;
    if (sbuf == nullptr && hipMalloc(&sbuf, 4096 * 8 * 8) != hipSuccess) sbuf = nullptr;
    if (grid.x <= 4096) t.stamps = sbuf;
#endif
    hipEvent_t ev_b = nullptr, ev_e = nullptr;
    take_events(&ev_b, &ev_e);  // the kernel-event probe, if armed
    if (t.imgs * t.RH * t.RW * 32 > 4096) {
        if (ev_b != nullptr)
            hipExtLaunchKernelGGL((wgrad_taps_kernel<9, 2, MODE>), grid, dim3(TAPS_THREADS), 0, st, ev_b, ev_e, 0, t, e);
        else
            hipLaunchKernelGGL((wgrad_taps_kernel<9, 2, MODE>), grid, dim3(TAPS_THREADS), 0, st, t, e);
    } else {
        if (ev_b != nullptr)
            hipExtLaunchKernelGGL((wgrad_taps_kernel<9, 1, MODE>), grid, dim3(TAPS_THREADS), 0, st, ev_b, ev_e, 0, t, e);
        else
            hipLaunchKernelGGL((wgrad_taps_kernel<9, 1, MODE>), grid, dim3(TAPS_THREADS), 0, st, t, e);
    }
#if NITI_STAMPS
    if (t.stamps) taps_stamp_report(t.stamps, (int)grid.x, st);
#endif
    return hipGetLastError();
}

static hipError_t wgrad_taps_run(const GemmPlan& p, const WgTaps& t, int M, int N, int32_t* C, uint32_t* amax,
                                 int32_t* ws, hipStream_t st, hipEvent_t after_gemm, SgdJob* defer = nullptr) {
    Epi e;
    e.span = take_span();
    if (p.strat == STRAT_SLAB) {
        const int mb = taps_slab_rows(t);
        e.C = ws;
        e.ldc = N;
        e.slab_stride = (int64_t)slab_stride_elems(mb, N);
        hipError_t r = launch_taps<EPI_SLAB>(p, t, e, st);
        if (r == hipSuccess && after_gemm != nullptr) r = hipEventRecord(after_gemm, st);
        if (r != hipSuccess) return r;
        SlabTapsBlocked map;
        map.tiles_ci = t.tiles_ci;
        map.cip4 = t.CIP / 4;
        map.c_out = M;
        map.ld4 = N / 4;
        map.fTile = make_fastdiv(4608);
        map.fRow = make_fastdiv(72);
        map.fPart = make_fastdiv(8);
        map.fTci = make_fastdiv((uint32_t)t.tiles_ci);
        // the NITI_SGD launch's combine sums the tile-blocked slabs (as gemm_acc_plan's C-shaped ones)
        if (defer != nullptr && (int64_t)mb * N >= (int64_t)p.splits * 4096 && (int64_t)mb * N < ((int64_t)1 << 32)) {
            defer->slab = ws;
            defer->splits = p.splits;
            defer->slab_stride = e.slab_stride;
            defer->slab_n = (int64_t)mb * N;
            defer->slab_map = 1;
            defer->tb_tiles_ci = map.tiles_ci;
            defer->tb_cip4 = map.cip4;
            defer->tb_ld4 = map.ld4;
            defer->tb_m = map.fTci.m;
            defer->tb_s = map.fTci.s;
            return hipSuccess;
        }
        return splitk_reduce(p, ws, (int64_t)mb * N, e.slab_stride, C, amax, st, map);
    }
    e.C = C;
    e.ldc = N;
    e.amax = amax;
    hipError_t r = launch_taps<EPI_STORE>(p, t, e, st);
    if (r == hipSuccess && after_gemm != nullptr) r = hipEventRecord(after_gemm, st);
    return r;
}

// bytes of the K-split slabs a weight-gradient plan writes (the tap-sharing kernel's tile-blocked
// slabs pad the output channels to whole 64-row tiles)
size_t conv_wgrad_slab_bytes(const ConvGeom& g, const PlanChoice& c) {
    const PlanKey k = conv_plan_key(PLAN_WGRAD, g);
    WgTaps t;
    if (c.bm == PLAN_TAPS_TILE && wgrad_taps_geom(g, nullptr, nullptr, &t))
        return (size_t)c.splits * slab_stride_elems(taps_slab_rows(t), k.N) * 4;
    return plan_slab_bytes(k.M, k.N, c.splits);
}

PlanChoice conv_plan_query(int op, const ConvGeom& g, bool recompute_ok, size_t ws_bytes) {
    const PlanKey key = conv_plan_key(op, g);
    WgTaps t;
    PlanChoice c;
    if (op == PLAN_WGRAD && wgrad_taps_geom(g, nullptr, nullptr, &t)) {
        const bool has = plan_override_get(key, &c);
        if (!has || c.bm == PLAN_TAPS_TILE) {
            const GemmPlan p = plan_taps(t, key.M, key.N, ws_bytes / 4, has ? &c : nullptr);
            c.bm = c.bn = PLAN_TAPS_TILE;
            c.splits = p.strat == STRAT_SLAB ? p.splits : 1;
            c.strat = p.strat;
            return c;
        }
    }
    return plan_query(key, conv_plan_k_step(op, g), recompute_ok, ws_bytes);
}

PlanKey conv_plan_key(int op, const ConvGeom& g) {
    if (op == PLAN_FWD) return PlanKey{op, g.n * g.oh * g.ow, g.cop, g.kh * g.kw * g.cip / 16};
    if (op == PLAN_DGRAD) return PlanKey{op, g.n * g.h * g.w, g.cip, g.kh * g.kw * g.cop / 16};
    return PlanKey{PLAN_WGRAD, g.c_out, g.kh * g.kw * g.cip, g.n * g.oh * g.ow};
}
int conv_plan_k_step(int op, const ConvGeom& g) {
    if (op == PLAN_FWD) return (fwd_taps_bk(g) ? fwd_taps_bk(g) : 64) / 16;
    if (op == PLAN_DGRAD) return (dgrad_taps_bk(g) ? dgrad_taps_bk(g) : 64) / 16;
    return KT_BK;
}

size_t conv_fwd_workspace(const ConvGeom& g) {
    const int bk = fwd_taps_bk(g) ? fwd_taps_bk(g) : 64;
    return plan_ws_elems(g.n * g.oh * g.ow, g.cop, g.kh * g.kw * g.cip / 16, bk / 16, PLAN_FWD) * sizeof(int32_t);
}
size_t conv_dgrad_workspace(const ConvGeom& g) {
    const int bk = dgrad_taps_bk(g) ? dgrad_taps_bk(g) : 64;
    return plan_ws_elems(g.n * g.h * g.w, g.cip, g.kh * g.kw * g.cop / 16, bk / 16, PLAN_DGRAD) * sizeof(int32_t);
}
size_t conv_wgrad_workspace(const ConvGeom& g) {
    const int M = g.c_out, N = g.kh * g.kw * g.cip;
    size_t e = plan_ws_elems(M, N, g.n * g.oh * g.ow, KT_BK, PLAN_WGRAD);
    WgTaps t;
    if (wgrad_taps_geom(g, nullptr, nullptr, &t)) {
        const GemmPlan p = plan_taps(t, M, N, (size_t)-1, nullptr);
        if (p.strat == STRAT_SLAB) e = std::max(e, (size_t)p.splits * slab_stride_elems(taps_slab_rows(t), N));
    }
    return e * sizeof(int32_t);
}
size_t matmul_workspace(int M, int ldc, int k16) {
    return plan_ws_elems(M, ldc, k16 / 16, RowsK::BK / 16) * sizeof(int32_t);
}

hipError_t conv_fwd_acc(const ConvGeom& g, const int8_t* x, const int8_t* w, int32_t* acc, uint32_t* amax,
                        void* ws, size_t ws_bytes, hipStream_t st) {
    const int kc_total = g.kh * g.kw * g.cip / 16;
    const RowsK lb = rows_k(w, (int64_t)g.kh * g.kw * g.cip, g.c_out, kc_total);
    return with_fwd_operand(g, x, [&](const auto& la) {
        return gemm_acc(PLAN_FWD, la, lb, g.n * g.oh * g.ow, g.cop, kc_total, acc, amax, (int32_t*)ws, ws_bytes / 4, st);
    });
}

hipError_t conv_dgrad_acc(const ConvGeom& g, const int8_t* dy, const int8_t* wt, int32_t* acc, uint32_t* amax,
                          void* ws, size_t ws_bytes, hipStream_t st) {
    const int kc_total = g.kh * g.kw * g.cop / 16;
    const RowsK lb = rows_k(wt, (int64_t)g.kh * g.kw * g.cop, g.c_in, kc_total);
    return with_dgrad_operand(g, dy, [&](const auto& la) {
        return gemm_acc(PLAN_DGRAD, la, lb, g.n * g.h * g.w, g.cip, kc_total, acc, amax, (int32_t*)ws, ws_bytes / 4, st);
    });
}

hipError_t conv_wgrad_acc(const ConvGeom& g, const int8_t* x, const int8_t* dy, int32_t* acc, uint32_t* amax,
                          void* ws, size_t ws_bytes, hipStream_t st, hipEvent_t after_gemm, SgdJob* defer) {
    WgTaps tg;
    if (wgrad_taps_geom(g, x, dy, &tg)) {
        const int M = g.c_out, N = g.kh * g.kw * g.cip;
        PlanChoice c;
        const bool has = plan_override_get(conv_plan_key(PLAN_WGRAD, g), &c);
        if (!has || c.bm == PLAN_TAPS_TILE) {
            const GemmPlan p = plan_taps(tg, M, N, ws ? ws_bytes / 4 : 0, has ? &c : nullptr);
            return wgrad_taps_run(p, tg, M, N, acc, amax, (int32_t*)ws, st, after_gemm, defer);
        }
    }
    KtRowsU la;
    KtIm2col lg;
    wgrad_operands(g, x, dy, &la, &lg);
    if (plain_1x1(g)) {  // the im2col is x itself: K-major rows of [pixels][cip]
        KtRowsU lx;
        lx.p = x;
        lx.ld = g.cip;
        lx.cols = g.cip;
        lx.K = lg.K;
        lx.bytes = lg.bytes;
        return gemm_acc<KtRowsU, KtRowsU, true>(PLAN_WGRAD, la, lx, g.c_out, lg.ncols, lg.K, acc, amax, (int32_t*)ws,
                                                ws_bytes / 4, st, after_gemm, defer);
    }
    const int ohw = g.oh * g.ow;
    const bool rows_mode = ohw % KT_BK == 0 && KT_BK % g.ow == 0;
    if (rows_mode || KT_BK % ohw == 0) {
        KtIm2colU lb;
        lb.x = x;
        lb.bytes = lg.bytes;
        lb.H = g.h;
        lb.W = g.w;
        lb.OH = g.oh;
        lb.OW = g.ow;
        lb.CIP = g.cip;
        lb.KW = g.kw;
        lb.sh = g.sh;
        lb.sw = g.sw;
        lb.pt = g.pt;
        lb.pl = g.pl;
        lb.dh = g.dh;
        lb.dw = g.dw;
        lb.ncols = lg.ncols;
        lb.K = lg.K;
        lb.rows_mode = rows_mode;
        return gemm_acc<KtRowsU, KtIm2colU, true>(PLAN_WGRAD, la, lb, g.c_out, lg.ncols, lg.K, acc, amax, (int32_t*)ws,
                                                  ws_bytes / 4, st, after_gemm, defer);
    }
    return gemm_acc<KtRowsU, PerLane<KtIm2col, true>, true>(PLAN_WGRAD, la, per_lane<KtIm2col, true>(lg), g.c_out, lg.ncols, lg.K,
                                                            acc, amax, (int32_t*)ws, ws_bytes / 4, st, after_gemm, defer);
}

// A fully connected layer's weight gradient in two GEMM passes with no int32 tensor: pass 0 takes
// its range (EPI_AMAX), pass 1 recomputes it and applies NITI_SGD in the epilogue (EPI_SGD).  The
// reduction is the batch, so the second pass costs a few microseconds against the gradient's
// int32 write + read (411 MB for VGG-16's first FC layer).
bool conv_wgrad_fc_sgd_ok(const ConvGeom& g) {
    return g.kh == 1 && g.kw == 1 && g.h == 1 && g.w == 1 && g.oh == 1 && g.ow == 1 && plain_1x1(g);
}
hipError_t conv_wgrad_fc_sgd(const ConvGeom& g, const int8_t* x, const int8_t* dy, uint32_t* amax, const SgdJob& j,
                             int pass, hipStream_t st) {
    if (!conv_wgrad_fc_sgd_ok(g) || amax == nullptr || (pass == 1 && j.w == nullptr)) return hipErrorInvalidValue;
    // the EPI_SGD epilogue writes w, wT and the int8 gradient only: a job carrying the row kernels'
    // fragment-major copies, sub-pixel class weights or deferred slabs would leave them stale
    if (pass == 1 && (j.wf != nullptr || j.wft != nullptr || j.subw != nullptr || j.slab != nullptr))
        return hipErrorInvalidValue;
    KtRowsU la;
    KtIm2col lg;
    wgrad_operands(g, x, dy, &la, &lg);
    KtRowsU lx;
    lx.p = x;
    lx.ld = g.cip;
    lx.cols = g.cip;
    lx.K = lg.K;
    lx.bytes = lg.bytes;
    const int M = g.c_out, N = lg.ncols;
    GemmPlan p = plan_gemm(M, N, lg.K, KT_BK, 1 << 30, false, 0, PLAN_WGRAD);
    // diagnostics: the update pass's tile (NITI_DIAG_FC_SGD_TILE=64 / 128 / 256: bm = bn)
    static const int tile = getenv("NITI_DIAG_FC_SGD_TILE") ? atoi(getenv("NITI_DIAG_FC_SGD_TILE")) : 0;
    if (pass == 1 && (tile == 64 || tile == 128)) p.bm = p.bn = tile;
    Epi e;
    e.amax = amax;
    if (pass == 0) return launch_mode<KtRowsU, KtRowsU, EPI_AMAX, true>(p, la, lx, M, N, lg.K, e, st);
    e.ldo = N;
    e.sgd_w = j.w;
    e.sgd_wT = j.wT;
    e.sgd_g = j.g_out;
    e.sgd_rule = j.rule;
    e.sgd_ci = j.ci;
    e.sgd_ldt = j.cop;
    return launch_mode<KtRowsU, KtRowsU, EPI_SGD, true>(p, la, lx, M, N, lg.K, e, st);
}

hipError_t matmul_acc(int M, int O, int k16, const int8_t* B, int64_t ldb, const int8_t* A, int64_t lda, int32_t* acc,
                      int64_t ldc, uint32_t* amax, void* ws, size_t ws_bytes, hipStream_t st) {
    const int kc_total = k16 / 16;
    const RowsK la = rows_k(B, ldb, M, kc_total);
    const RowsK lb = rows_k(A, lda, O, kc_total);  // rows >= O read as zero, so columns O..ldc are 0
    return gemm_acc(PLAN_MATMUL, la, lb, M, (int)ldc, kc_total, acc, amax, (int32_t*)ws, ws_bytes / 4, st);
}

hipError_t conv_fwd_phase1(const ConvGeom& g, const int8_t* x, const int8_t* w, int32_t* acc, uint32_t* amax,
                           void* ws, size_t ws_bytes, hipStream_t st) {
    const int kc_total = g.kh * g.kw * g.cip / 16;
    const RowsK lb = rows_k(w, (int64_t)g.kh * g.kw * g.cip, g.c_out, kc_total);
    return with_fwd_operand(g, x, [&](const auto& la) {
        return act_phase1(PLAN_FWD, la, lb, g.n * g.oh * g.ow, g.cop, kc_total, acc, amax, (int32_t*)ws, ws_bytes / 4, st);
    });
}
hipError_t conv_fwd_phase2(const ConvGeom& g, const int8_t* x, const int8_t* w, const int32_t* acc,
                           const uint32_t* amax, const ActOut& o, size_t ws_bytes, hipStream_t st) {
    const int kc_total = g.kh * g.kw * g.cip / 16;
    const RowsK lb = rows_k(w, (int64_t)g.kh * g.kw * g.cip, g.c_out, kc_total);
    return with_fwd_operand(g, x, [&](const auto& la) {
        return act_phase2(PLAN_FWD, la, lb, g.n * g.oh * g.ow, g.cop, kc_total, acc, amax, o, ws_bytes / 4, st);
    });
}
hipError_t conv_fwd_spec(const ConvGeom& g, const int8_t* x, const int8_t* w, uint32_t* amax, const ActOut& o,
                         uint32_t* slot, int pass, hipStream_t st, int8_t* alt) {
    const int kc_total = g.kh * g.kw * g.cip / 16;
    const RowsK lb = rows_k(w, (int64_t)g.kh * g.kw * g.cip, g.c_out, kc_total);
    return with_fwd_operand(g, x, [&](const auto& la) {
        return act_spec(PLAN_FWD, la, lb, g.n * g.oh * g.ow, g.cop, kc_total, amax, o, slot, pass, alt, st);
    });
}
hipError_t conv_dgrad_spec(const ConvGeom& g, const int8_t* dy, const int8_t* wt, uint32_t* amax, const ActOut& o,
                           uint32_t* slot, int pass, hipStream_t st, int8_t* alt) {
    const int kc_total = g.kh * g.kw * g.cop / 16;
    const RowsK lb = rows_k(wt, (int64_t)g.kh * g.kw * g.cop, g.c_in, kc_total);
    return with_dgrad_operand(g, dy, [&](const auto& la) {
        return act_spec(PLAN_DGRAD, la, lb, g.n * g.h * g.w, g.cip, kc_total, amax, o, slot, pass, alt, st);
    });
}
hipError_t conv_fwd_fused(const ConvGeom& g, const int8_t* x, const int8_t* w, const ActOut& o, const FusedBar& fb,
                          hipStream_t st) {
    const int kc_total = g.kh * g.kw * g.cip / 16;
    const RowsK lb = rows_k(w, (int64_t)g.kh * g.kw * g.cip, g.c_out, kc_total);
    return with_fwd_operand(g, x, [&](const auto& la) {
        return act_fused(PLAN_FWD, la, lb, g.n * g.oh * g.ow, g.cop, kc_total, o, fb, st);
    });
}
hipError_t conv_dgrad_fused(const ConvGeom& g, const int8_t* dy, const int8_t* wt, const ActOut& o, const FusedBar& fb,
                            hipStream_t st) {
    if (g.sh != 1 || g.sw != 1) return hipErrorNotSupported;  // (strided: the sub-pixel class GEMMs)
    const int kc_total = g.kh * g.kw * g.cop / 16;
    const RowsK lb = rows_k(wt, (int64_t)g.kh * g.kw * g.cop, g.c_in, kc_total);
    return with_dgrad_operand(g, dy, [&](const auto& la) {
        return act_fused(PLAN_DGRAD, la, lb, g.n * g.h * g.w, g.cip, kc_total, o, fb, st);
    });
}
size_t conv_fwd_spec_alt_bytes(const ConvGeom& g) { return (size_t)2 * g.n * g.oh * g.ow * g.cop; }
size_t conv_dgrad_spec_alt_bytes(const ConvGeom& g) { return (size_t)2 * g.n * g.h * g.w * g.cip; }
// ---- the stride-2 input gradient as four sub-pixel classes ------------------------------------
// dx[iy][ix] gathers dy[(iy + pt - ky) / 2][(ix + pl - kx) / 2] over the taps where both divisions
// are exact: the taps of pixel (2 my + py, 2 mx + px) are ky = ky0(py), ky0 + 2, ... and kx alike,
// the same for the whole class.  Each class is a stride-1 input gradient over dy with a 1- or 2-tap
// kernel per axis (pad (py + pt - ky0) / 2), written into dx through a row map: the generic per-lane
// loader instead walked all kh x kw taps for every pixel with 3/4 of them masked to zero.  The
// class weights [class][ci][kh_c][kw_c][cop] are kept beside wT: built from it when the weights are
// set (conv_dgrad_subpix_weights) and rewritten by NITI_SGD (SgdJob::subw, sgd_tile_finish).
struct SubpixAxis {
    int n, k0;  // taps of the class (k0, k0 + 2, ...), n may be 0
    int pad;    // the class conv's pad: (p + parity - k0) / 2
};
static SubpixAxis subpix_axis(int k, int pad, int parity) {
    SubpixAxis a;
    a.k0 = ((parity + pad) % 2 + 2) % 2;
    a.n = a.k0 < k ? (k - a.k0 + 1) / 2 : 0;
    a.pad = (parity + pad - a.k0) / 2;
    return a;
}
bool conv_dgrad_subpix_ok(const ConvGeom& g) {
    return g.sh == 2 && g.sw == 2 && g.dh == 1 && g.dw == 1 && g.h % 2 == 0 && g.w % 2 == 0 && g.kh <= 8 &&
           g.kw <= 8 && g.pt >= 0 && g.pl >= 0 && g.cop % 64 == 0 && g.cip % 16 == 0 &&
           (int64_t)g.n * g.h * g.w * g.cip < ((int64_t)1 << 31) && (int64_t)g.n * g.oh * g.ow * g.cop < ((int64_t)1 << 31);
}
size_t conv_dgrad_subpix_bytes(const ConvGeom& g) { return (size_t)g.kh * g.kw * g.c_in * g.cop; }

struct SubpixW {
    const int8_t* wt;
    int8_t* out;
    int ci, kh, kw, cop16;  // cop16: 16-byte chunks per tap row
    int ny[4], nx[4], ky0[4], kx0[4];
    int64_t off[5];  // chunk offsets of the classes (prefix)
};
__global__ void subpix_weights_kernel(SubpixW p) {
    const int64_t total = p.off[4];
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        int c = 0;
        while (c < 3 && t >= p.off[c + 1]) ++c;
        int64_t r = t - p.off[c];
        const int cc = (int)(r % p.cop16);
        r /= p.cop16;
        const int jx = (int)(r % p.nx[c]);
        r /= p.nx[c];
        const int jy = (int)(r % p.ny[c]);
        const int ci = (int)(r / p.ny[c]);
        const int ky = p.ky0[c] + 2 * jy, kx = p.kx0[c] + 2 * jx;
        ((v4i*)p.out)[t] = ((const v4i*)p.wt)[((int64_t)(ci * p.kh + ky) * p.kw + kx) * p.cop16 + cc];
    }
}

// the classes in order (py, px) = (0,0), (0,1), (1,0), (1,1): axes and weight offsets (bytes)
struct SubpixPlan {
    SubpixAxis ay[2], ax[2];
    int64_t woff[4];
};
static SubpixPlan subpix_plan(const ConvGeom& g) {
    SubpixPlan q;
    for (int p = 0; p < 2; ++p) {
        q.ay[p] = subpix_axis(g.kh, g.pt, p);
        q.ax[p] = subpix_axis(g.kw, g.pl, p);
    }
    int64_t o = 0;
    for (int c = 0; c < 4; ++c) {
        q.woff[c] = o;
        o += (int64_t)q.ay[c >> 1].n * q.ax[c & 1].n * g.c_in * g.cop;
    }
    return q;
}
hipError_t conv_dgrad_subpix_weights(const ConvGeom& g, const int8_t* wt, int8_t* out, hipStream_t st) {
    if (!conv_dgrad_subpix_ok(g) || wt == nullptr || out == nullptr) return hipErrorInvalidValue;
    const SubpixPlan q = subpix_plan(g);
    SubpixW p;
    p.wt = wt;
    p.out = out;
    p.ci = g.c_in;
    p.kh = g.kh;
    p.kw = g.kw;
    p.cop16 = g.cop / 16;
    p.off[0] = 0;
    for (int c = 0; c < 4; ++c) {
        p.ny[c] = q.ay[c >> 1].n;
        p.nx[c] = q.ax[c & 1].n;
        p.ky0[c] = q.ay[c >> 1].k0;
        p.kx0[c] = q.ax[c & 1].k0;
        p.off[c + 1] = p.off[c] + (int64_t)p.ny[c] * p.nx[c] * g.c_in * p.cop16;
    }
    if (p.off[4] == 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((p.off[4] + 255) / 256, 1024);
    hipLaunchKernelGGL(subpix_weights_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p);
    return hipGetLastError();
}

// one pass over the four classes: MODE EPI_STORE (acc), EPI_AMAX (max only) or EPI_REQUANT (o)
template <int MODE>
static hipError_t subpix_pass(const ConvGeom& g, const GemmPlan& plan, const int8_t* dy, const int8_t* subw,
                              int32_t* acc, uint32_t* amax, const ActOut* o, hipStream_t st, bool zero_fill = false) {
    const SubpixPlan q = subpix_plan(g);
    for (int c = 0; c < 4; ++c) {
        if (zero_fill && q.ay[c >> 1].n * q.ax[c & 1].n != 0) continue;  // only the tap-less classes' zeros
        const SubpixAxis& ay = q.ay[c >> 1];
        const SubpixAxis& ax = q.ax[c & 1];
        ConvGeom gc = g;
        gc.h = g.h / 2;
        gc.w = g.w / 2;
        gc.kh = ay.n > 0 ? ay.n : 1;
        gc.kw = ax.n > 0 ? ax.n : 1;
        gc.sh = gc.sw = 1;
        gc.pt = ay.pad;
        gc.pl = ax.pad;
        gc.dh = gc.dw = 1;
        const int kc = ay.n * ax.n * g.cop / 16;  // 0: the class gets no tap (its dx is zero)
        const int M = g.n * gc.h * gc.w;
        GemmPlan p = plan;
        p.splits = 1;
        Epi e;
        e.rmap.on = 1;
        e.rmap.hc = gc.h;
        e.rmap.wc = gc.w;
        e.rmap.h = g.h;
        e.rmap.w = g.w;
        e.rmap.py = c >> 1;
        e.rmap.px = c & 1;
        e.amax = amax;
        if (MODE == EPI_STORE) {
            e.C = acc;
            e.ldc = g.cip;
        }
        if (MODE == EPI_REQUANT) {
            e.out = o->out;
            e.ldo = g.cip;
            e.relu = o->relu;
            e.relu_mask = o->relu_mask;
            e.exp_in = o->exp_in;
            e.wscale = o->wscale;
            e.exp_out = o->exp_out;
        }
        if ((MODE == EPI_AMAX || MODE == EPI_STORE) && kc == 0 && !zero_fill) continue;  // (requant: zero_cls)
        const RowsK lb = rows_k(subw + q.woff[c], (int64_t)gc.kh * gc.kw * g.cop, g.c_in, kc);
        const hipError_t r = launch_mode<ConvTaps<64>, RowsK, MODE, false>(p, conv_taps<64>(gc, dy, false), lb, M, g.cip,
                                                                          kc, e, st);
        if (r != hipSuccess) return r;
    }
    return hipSuccess;
}

hipError_t conv_dgrad_phase1(const ConvGeom& g, const int8_t* dy, const int8_t* wt, int32_t* acc, uint32_t* amax,
                             void* ws, size_t ws_bytes, hipStream_t st, const int8_t* subw) {
    const int kc_total = g.kh * g.kw * g.cop / 16;
    if (subw != nullptr && conv_dgrad_subpix_ok(g)) {  // (the strategy phase 2 will see: same workspace rule)
        const GemmPlan p = plan_gemm(g.n * g.h * g.w, g.cip, kc_total, 64 / 16, kc_total * 16, true,
                                     ws ? ws_bytes / 4 : 0, PLAN_DGRAD);
        if (p.strat != STRAT_SPEC) {
            if (recomputes(p.strat)) return subpix_pass<EPI_AMAX>(g, p, dy, subw, nullptr, amax, nullptr, st);
            return subpix_pass<EPI_STORE>(g, p, dy, subw, acc, amax, nullptr, st);
        }
    }
    const RowsK lb = rows_k(wt, (int64_t)g.kh * g.kw * g.cop, g.c_in, kc_total);
    return with_dgrad_operand(g, dy, [&](const auto& la) {
        return act_phase1(PLAN_DGRAD, la, lb, g.n * g.h * g.w, g.cip, kc_total, acc, amax, (int32_t*)ws, ws_bytes / 4, st);
    });
}
hipError_t conv_dgrad_phase2(const ConvGeom& g, const int8_t* dy, const int8_t* wt, const int32_t* acc,
                             const uint32_t* amax, const ActOut& o, size_t ws_bytes, hipStream_t st,
                             const int8_t* subw) {
    const int kc_total = g.kh * g.kw * g.cop / 16;
    if (subw != nullptr && conv_dgrad_subpix_ok(g)) {
        const GemmPlan p = plan_gemm(g.n * g.h * g.w, g.cip, kc_total, 64 / 16, kc_total * 16, true, ws_bytes / 4,
                                     PLAN_DGRAD);
        if (recomputes(p.strat)) {
            if (o.pool.pool_out != nullptr || o.pool.dx != nullptr || o.out_p16 != nullptr) return hipErrorInvalidValue;
            return subpix_pass<EPI_REQUANT>(g, p, dy, subw, nullptr, const_cast<uint32_t*>(amax), &o, st);
        }
        // phase 1 left the tap-less classes' accumulators unwritten: the plain requantise pass
        // writes their zeros without reading them, any other pass gets them zero-filled first
        const SubpixPlan q = subpix_plan(g);
        int zc = 0;
        for (int c = 0; c < 4; ++c)
            if (q.ay[c >> 1].n * q.ax[c & 1].n == 0) zc |= 1 << c;
        if (zc != 0 && p.strat != STRAT_SPEC) {  // (a speculative plan runs phase 1 as one GEMM)
            if (o.pool.pool_out == nullptr && o.pool.dx == nullptr && o.out_p16 == nullptr) {
                ActOut oz = o;
                oz.zero_cls = zc;
                oz.zc_h = g.h;
                oz.zc_w = g.w;
                return with_dgrad_operand(g, dy, [&](const auto& la) {
                    const RowsK lb = rows_k(wt, (int64_t)g.kh * g.kw * g.cop, g.c_in, kc_total);
                    return act_phase2(PLAN_DGRAD, la, lb, g.n * g.h * g.w, g.cip, kc_total, acc, amax, oz, ws_bytes / 4, st);
                });
            }
            const hipError_t r = subpix_pass<EPI_STORE>(g, p, dy, subw, const_cast<int32_t*>(acc), nullptr, nullptr, st, true);
            if (r != hipSuccess) return r;
        }
    }
    const RowsK lb = rows_k(wt, (int64_t)g.kh * g.kw * g.cop, g.c_in, kc_total);
    return with_dgrad_operand(g, dy, [&](const auto& la) {
        return act_phase2(PLAN_DGRAD, la, lb, g.n * g.h * g.w, g.cip, kc_total, acc, amax, o, ws_bytes / 4, st);
    });
}

// =====================================================================================
// Range estimate and requantisation
// =====================================================================================

// max|a| of one range over blocks [0, nb) of the grid (block b of them), published to amax
__device__ __forceinline__ void absmax_body(const int32_t* __restrict__ a, int64_t n, uint32_t* __restrict__ amax,
                                            int64_t b, int64_t nb) {
    uint32_t m = 0;
    const int64_t n4 = n / 4;
    const v4i* a4 = (const v4i*)a;
    for (int64_t i = b * blockDim.x + threadIdx.x; i < n4; i += nb * blockDim.x) {
        const v4i v = a4[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t u = uabs32(v[j]);
            m = m > u ? m : u;
        }
    }
    for (int64_t i = n4 * 4 + b * blockDim.x + threadIdx.x; i < n; i += nb * blockDim.x) {
        const uint32_t u = uabs32(a[i]);
        m = m > u ? m : u;
    }
    m = wave_max(m);
    __shared__ uint32_t red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = m > red[i] ? m : red[i];
        m = m > red[0] ? m : red[0];
        publish_max(amax, m);
    }
}

__global__ void absmax_kernel(const int32_t* __restrict__ a, int64_t n, uint32_t* __restrict__ amax) {
    absmax_body(a, n, amax, blockIdx.x, gridDim.x);
}

// several ranges in one launch: job k owns workgroups [b0_k, b0_{k+1})
__global__ void absmax_many_kernel(AbsmaxJobs J) {
    int k = 0;
    while (k + 1 < J.n && blockIdx.x >= J.j[k + 1].b0) ++k;
    const AbsmaxJob jb = J.j[k];
    const uint32_t end = k + 1 < J.n ? J.j[k + 1].b0 : gridDim.x;
    absmax_body(jb.a, jb.n, jb.amax, blockIdx.x - jb.b0, end - jb.b0);
}

hipError_t absmax_many(const AbsmaxJob* jobs, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (n > ABSMAX_MAX_JOBS) return hipErrorInvalidValue;
    AbsmaxJobs J{};
    uint32_t wg = 0;
    for (int i = 0; i < n; ++i) {
        if (jobs[i].n <= 0) continue;
        int64_t blocks = (jobs[i].n / 4 + 255) / 256;
        if (blocks > 128) blocks = 128;
        if (blocks < 1) blocks = 1;
        J.j[J.n] = jobs[i];
        J.j[J.n++].b0 = wg;
        wg += (uint32_t)blocks;
    }
    if (J.n == 0) return hipSuccess;
    hipLaunchKernelGGL(absmax_many_kernel, dim3(wg), dim3(256), 0, st, J);
    return hipGetLastError();
}

hipError_t absmax_i32(const int32_t* a, int64_t n, uint32_t* amax, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n / 4 + 255) / 256;
    if (blocks > 512) blocks = 512;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, n, amax);
    return hipGetLastError();
}

// forward / deconv rule, NITI_Conv_Int8.cpp:262-307: shift>1 PSTO(shift); ==1 PSTO(2); else raw cast
// NITI forward shift rule on 16 consecutive channels of one accumulator row
__device__ __forceinline__ v16c requant16(const int32_t* src, bool raw, int s, int relu) {
    const v4i* p = (const v4i*)src;
    v16c q;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const v4i v = p[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            int32_t o = raw ? (int32_t)(int8_t)v[e] : psto_any(v[e], s);
            if (relu && o < 0) o = 0;
            q[j * 4 + e] = (signed char)o;
        }
    }
    return q;
}

__global__ void requant_act_kernel(ActRequant r) {
    const int bw = bitwidth_of(read_max(r.amax));
    const int shift = bw - 7;
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    const int groups = r.ldc / 16;
    if (blockIdx.x == 0 && threadIdx.x == 0 && r.exp_out != nullptr) {
        const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
        const int ein = r.exp_in ? (int)*r.exp_in : 0;
        const int ws = r.wscale ? (int)*r.wscale : 0;
        *r.exp_out = (int8_t)(ein + ws + inc);
    }
    if (r.pool.pool_out != nullptr || r.pool.dx != nullptr) {
        // one thread per (pooled pixel, 16-channel group)
        const int H = r.pool.H, W = r.pool.W, ph = H / 2, pw = W / 2;
        const int64_t np = r.pool.dx != nullptr ? r.rows : r.rows / 4;  // pooled pixels
        const int64_t total = np * groups;
        for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
             t += (int64_t)gridDim.x * blockDim.x) {
            const int64_t pp = t / groups;
            const int gi = (int)(t - pp * groups);
            const int px = (int)(pp % pw);
            const int64_t rest = pp / pw;
            const int py = (int)(rest % ph);
            const int64_t b = rest / ph;
            const int64_t m0 = (b * H + 2 * py) * W + 2 * px;  // window's first pixel
            const int64_t win[4] = {m0, m0 + 1, m0 + W, m0 + W + 1};
            if (r.pool.pool_out != nullptr) {
                v16c mx;
#pragma unroll
                for (int j = 0; j < 16; ++j) mx[j] = (signed char)-128;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const v16c q = requant16(r.acc + win[k] * r.ldc + gi * 16, raw, s, r.relu);
                    *(v16c*)(r.out_nhwc16 + win[k] * r.ldc + gi * 16) = q;
#pragma unroll
                    for (int j = 0; j < 16; ++j) mx[j] = q[j] > mx[j] ? q[j] : mx[j];
                }
                *(v16c*)(r.pool.pool_out + pp * r.ldc + gi * 16) = mx;
            } else {
                const v16c q = requant16(r.acc + pp * r.ldc + gi * 16, raw, s, 0);
                if (r.out_nhwc16 != nullptr) *(v16c*)(r.out_nhwc16 + pp * r.ldc + gi * 16) = q;
                const v16c mv = *(const v16c*)(r.pool.y + pp * r.ldc + gi * 16);
                unsigned done = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const v16c xv = *(const v16c*)(r.pool.x + win[k] * r.ldc + gi * 16);
                    v16c o;
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const bool take = !((done >> j) & 1u) && xv[j] >= mv[j];
                        if (take) done |= 1u << j;
                        signed char d = take ? q[j] : (signed char)0;
                        if (r.pool.relu && xv[j] <= 0) d = 0;
                        o[j] = d;
                    }
                    *(v16c*)(r.pool.dx + win[k] * r.ldc + gi * 16) = o;
                }
            }
        }
        return;
    }
    const int64_t total = r.rows * groups;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = t / groups;
        const int gi = (int)(t - m * groups);
        const v4i* src = (const v4i*)(r.acc + m * r.ldc + gi * 16);
        v16c q;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const v4i v = src[j];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                int32_t o = raw ? (int32_t)(int8_t)v[e] : psto_any(v[e], s);
                if (r.relu && o < 0) o = 0;
                q[j * 4 + e] = (signed char)o;
            }
        }
        if (r.relu_mask != nullptr) {
            const v16c mk = *(const v16c*)(r.relu_mask + m * r.ldc + gi * 16);
#pragma unroll
            for (int j = 0; j < 16; ++j) q[j] = mk[j] > 0 ? q[j] : (signed char)0;
        }
        if (r.out_nhwc16 != nullptr) *(v16c*)(r.out_nhwc16 + m * r.ldc + gi * 16) = q;
        if (r.out_c4 != nullptr) {
            const int64_t b = m / r.hw, p = m - b * r.hw;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int c = gi * 16 + j;
                if (c < r.c_real) r.out_c4[(((int64_t)(c >> 2) * r.n + b) * r.hw + p) * 4 + (c & 3)] = q[j];
            }
        }
    }
}

// Streaming requantisation (the training step's path; out_c4 uses requant_act_kernel above).
// A unit is 4 channels (one 16-byte int32 load, one 4-byte int8 store): consecutive lanes take
// consecutive channel quads, so every wave instruction moves whole contiguous runs (a full
// 1 KiB of accumulator per load), and each thread keeps RQ_U units' loads in flight.
//   RQ_PLAIN     unit over [rows][ldc/4]: out = requant (+relu) (& relu_mask > 0)
//   RQ_POOL_FWD  unit over [pooled pixel][ldc/4]: requant (+relu) the 2x2 window -> out, max -> pool_out
//   RQ_POOL_BWD  unit over [pooled pixel = row][ldc/4]: requant, route to the window's first max
//                of x (relu: and x > 0) in dx, zero elsewhere (+ optional out)
enum { RQ_PLAIN = 0, RQ_POOL_FWD = 1, RQ_POOL_BWD = 2 };
constexpr int RQ_U = 4;

struct RqGeom {
    FastDiv fq, fpw, fph;  // by quads per row, pooled width, pooled height
    int qpr, W;            // quads per row, pre-pool width
    uint32_t units;
    FastDiv fzw, fzh;      // ActRequant::zc_w / zc_h (zero_cls)
};

__device__ __forceinline__ uint32_t rq4(v4i v, bool raw, int s, int relu) {
    uint32_t o = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        int32_t q = raw ? (int32_t)(int8_t)v[e] : psto_fast(v[e], s);
        if (relu && q < 0) q = 0;
        o |= ((uint32_t)q & 0xffu) << (8 * e);
    }
    return o;
}
__device__ __forceinline__ uint32_t bmax4(uint32_t a, uint32_t b) {
    uint32_t o = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int x = (int8_t)(a >> (8 * e)), y = (int8_t)(b >> (8 * e));
        o |= ((uint32_t)(x > y ? x : y) & 0xffu) << (8 * e);
    }
    return o;
}

template <int MODE>
__global__ void __launch_bounds__(256) requant_quad_kernel(ActRequant r, RqGeom g) {
    const int bw = bitwidth_of(read_max(r.amax));  // whole wave active
    const int shift = bw - 7;
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && r.exp_out != nullptr) {
        const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
        const int ein = r.exp_in ? (int)*r.exp_in : 0;
        const int ws = r.wscale ? (int)*r.wscale : 0;
        *r.exp_out = (int8_t)(ein + ws + inc);
    }
    const uint32_t stride = gridDim.x * 256u;
    const int ldc = r.ldc;
    for (uint32_t u0 = blockIdx.x * 256u + threadIdx.x; u0 < g.units; u0 += stride * RQ_U) {
        if (MODE == RQ_PLAIN) {
            v4i v[RQ_U];
            uint32_t mk[RQ_U];
#pragma unroll
            for (int j = 0; j < RQ_U; ++j) {
                const uint32_t u = u0 + j * stride;
                bool ld = u < g.units;
                if (ld && r.zero_cls != 0) {  // a tap-less sub-pixel class: 0, its accumulators unread
                    const uint32_t row = fdiv(g.fq, u), t = fdiv(g.fzw, row);
                    const uint32_t x = row - t * g.fzw.d, y = t - fdiv(g.fzh, t) * g.fzh.d;
                    ld = !((r.zero_cls >> (2 * (y & 1u) + (x & 1u))) & 1);
                }
                v[j] = ld ? __builtin_nontemporal_load((const v4i*)r.acc + u) : v4i{0, 0, 0, 0};
                mk[j] = (r.relu_mask != nullptr && u < g.units) ? ((const uint32_t*)r.relu_mask)[u] : 0x01010101u;
            }
#pragma unroll
            for (int j = 0; j < RQ_U; ++j) {
                const uint32_t u = u0 + j * stride;
                if (u >= g.units) break;
                uint32_t o = rq4(v[j], raw, s, r.relu);
                if (r.relu_mask != nullptr) {
                    uint32_t keep = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if ((int8_t)(mk[j] >> (8 * e)) > 0) keep |= 0xffu << (8 * e);
                    o &= keep;
                }
                ((uint32_t*)r.out_nhwc16)[u] = o;
            }
        } else {
            // window rows of each unit
            int64_t wrow[RQ_U];
            uint32_t pp_[RQ_U], img_[RQ_U];
            int cq_[RQ_U];
#pragma unroll
            for (int j = 0; j < RQ_U; ++j) {
                const uint32_t u = u0 + j * stride;
                const uint32_t uu = u < g.units ? u : 0u;
                const uint32_t pp = fdiv(g.fq, uu);
                cq_[j] = (int)(uu - pp * (uint32_t)g.qpr);
                const uint32_t rest = fdiv(g.fpw, pp);
                const int px = (int)(pp - rest * g.fpw.d);
                const uint32_t b = fdiv(g.fph, rest);
                const int py = (int)(rest - b * g.fph.d);
                wrow[j] = ((int64_t)b * (2 * g.fph.d) + 2 * py) * g.W + 2 * px;
                pp_[j] = pp;
                img_[j] = b;
            }
            if (MODE == RQ_POOL_FWD) {
                v4i v[RQ_U][4];
#pragma unroll
                for (int j = 0; j < RQ_U; ++j)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int64_t row = wrow[j] + (k & 1) + (k >> 1) * g.W;
                        v[j][k] = u0 + j * stride < g.units
                                      ? __builtin_nontemporal_load((const v4i*)(r.acc + row * ldc) + cq_[j])
                                      : v4i{0, 0, 0, 0};
                    }
#pragma unroll
                for (int j = 0; j < RQ_U; ++j) {
                    if (u0 + j * stride >= g.units) break;
                    uint32_t mx = 0x80808080u;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int64_t row = wrow[j] + (k & 1) + (k >> 1) * g.W;
                        const uint32_t o = rq4(v[j][k], raw, s, r.relu);
                        ((uint32_t*)(r.out_nhwc16 + row * ldc))[cq_[j]] = o;
                        mx = bmax4(mx, o);
                    }
                    ((uint32_t*)(r.pool.pool_out + (int64_t)pp_[j] * ldc))[cq_[j]] = mx;
                }
            } else {
                v4i v[RQ_U];
                uint32_t yv[RQ_U], xv[RQ_U][4];
#pragma unroll
                for (int j = 0; j < RQ_U; ++j) {
                    const bool ok = u0 + j * stride < g.units;
                    v[j] = ok ? __builtin_nontemporal_load((const v4i*)(r.acc + (int64_t)pp_[j] * ldc) + cq_[j])
                              : v4i{0, 0, 0, 0};
                    yv[j] = ok ? ((const uint32_t*)(r.pool.y + (int64_t)pp_[j] * ldc))[cq_[j]] : 0u;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int64_t row = wrow[j] + (k & 1) + (k >> 1) * g.W;
                        xv[j][k] = ok ? ((const uint32_t*)(r.pool.x + row * ldc))[cq_[j]] : 0u;
                    }
                }
#pragma unroll
                for (int j = 0; j < RQ_U; ++j) {
                    if (u0 + j * stride >= g.units) break;
                    const uint32_t q = rq4(v[j], raw, s, 0);
                    if (r.out_nhwc16 != nullptr) ((uint32_t*)(r.out_nhwc16 + (int64_t)pp_[j] * ldc))[cq_[j]] = q;
                    uint32_t done = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        uint32_t o = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int x = (int8_t)(xv[j][k] >> (8 * e)), m = (int8_t)(yv[j] >> (8 * e));
                            const bool take = !((done >> e) & 1u) && x >= m;
                            if (take) done |= 1u << e;
                            if (take && !(r.pool.relu && x <= 0)) o |= q & (0xffu << (8 * e));
                        }
                        const int64_t row = wrow[j] + (k & 1) + (k >> 1) * g.W;
                        ((uint32_t*)(r.pool.dx + row * ldc))[cq_[j]] = o;
                        if (r.pool.dx_c32 != nullptr) {  // [img][c / 32][H][W][32]: 4 channels of one pixel
                            const int64_t hw = (int64_t)(2 * g.fph.d) * g.W;
                            const int64_t pix = row - (int64_t)img_[j] * hw;
                            const int c = 4 * cq_[j];
                            *(uint32_t*)(r.pool.dx_c32 + (((int64_t)img_[j] * (ldc / 32) + c / 32) * hw + pix) * 32 + (c & 31)) = o;
                        }
                    }
                }
            }
        }
    }
}

// Requantisation passes that also leave the P16 copy ([pixels/16][ldc][16], niti_wgrad.hip) of
// their output, so the input-gradient chain hands dy to the P16 weight gradient without a layout
// launch of its own.  A thread takes one channel quad of a run of output pixels covering whole
// 16-pixel blocks -- G pooled pixels whose 2x2 windows are 4G consecutive dx pixels (G = 4: a pooled row of an 8x8 image, one 4x4 image, four 2x2 images;
// G = 8: a pooled row of a 16x16 image).  It computes and stores the NHWC16 output exactly as
// requant_quad_kernel does, then transposes each 4 pixels x 4 channels in registers (v_perm) and
// writes every block's 4 channels x 16 pixels as 64 contiguous bytes (consecutive lanes,
// consecutive quads: a wave stores whole 4 KiB runs).
template <int W>
__host__ __device__ constexpr int p16_group() { return W == 16 ? 8 : 4; }
// position, inside the run, of corner k (0: top left, 1: top right, 2, 3: bottom) of pooled pixel j
template <int W>
__device__ constexpr int p16_loc(int j, int k) {
    if constexpr (W >= 8) return (k >> 1) * W + 2 * j + (k & 1);               // one pooled row
    else if constexpr (W == 4) return (2 * (j >> 1) + (k >> 1)) * 4 + 2 * (j & 1) + (k & 1);  // one image
    else return 4 * j + 2 * (k >> 1) + (k & 1);                                  // four 2x2 images
}

template <int MODE, int W>
__global__ void __launch_bounds__(256) requant_p16_kernel(ActRequant r, RqGeom g) {
    static_assert(MODE == RQ_POOL_BWD, "the plain pass is requant_p16_plain_kernel");
    constexpr int G = p16_group<W>();  // pooled pixels per thread
    constexpr int NPX = 4 * G;         // dx pixels per thread
    const int bw = bitwidth_of(read_max(r.amax));
    const int shift = bw - 7;
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && r.exp_out != nullptr) {
        const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
        const int ein = r.exp_in ? (int)*r.exp_in : 0;
        const int ws = r.wscale ? (int)*r.wscale : 0;
        *r.exp_out = (int8_t)(ein + ws + inc);
    }
    const int ldc = r.ldc;
    for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < g.units; u += gridDim.x * 256u) {
        const uint32_t grp = fdiv(g.fq, u);
        const int cq = (int)(u - grp * (uint32_t)g.qpr);
        const int64_t d0 = (int64_t)grp * NPX;  // the run's first output pixel
        uint32_t d[NPX];
        {
            const int64_t p0 = (int64_t)grp * G;  // the run's first pooled pixel
            v4i v[G];
            uint32_t yv[G], xv[G][4];
#pragma unroll
            for (int j = 0; j < G; ++j) {
                v[j] = __builtin_nontemporal_load((const v4i*)(r.acc + (p0 + j) * ldc) + cq);
                yv[j] = ((const uint32_t*)(r.pool.y + (p0 + j) * ldc))[cq];
#pragma unroll
                for (int k = 0; k < 4; ++k) xv[j][k] = ((const uint32_t*)(r.pool.x + (d0 + p16_loc<W>(j, k)) * ldc))[cq];
            }
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const uint32_t q = rq4(v[j], raw, s, 0);
                if (r.out_nhwc16 != nullptr) ((uint32_t*)(r.out_nhwc16 + (p0 + j) * ldc))[cq] = q;
                uint32_t done = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    uint32_t o = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int x = (int8_t)(xv[j][k] >> (8 * e)), m = (int8_t)(yv[j] >> (8 * e));
                        const bool take = !((done >> e) & 1u) && x >= m;
                        if (take) done |= 1u << e;
                        if (take && !(r.pool.relu && x <= 0)) o |= q & (0xffu << (8 * e));
                    }
                    ((uint32_t*)(r.pool.dx + (d0 + p16_loc<W>(j, k)) * ldc))[cq] = o;
                    d[p16_loc<W>(j, k)] = o;
                }
            }
        }
#pragma unroll
        for (int b = 0; b < NPX / 16; ++b) {
            v4i c[4];  // channel e: the block's 16 pixels
#pragma unroll
            for (int t = 0; t < 4; ++t) {  // 4x4 byte transpose of pixels 16b + 4t .. 4t + 3
                const uint32_t a0 = d[16 * b + 4 * t], a1 = d[16 * b + 4 * t + 1], a2 = d[16 * b + 4 * t + 2],
                               a3 = d[16 * b + 4 * t + 3];
                const uint32_t t0 = __builtin_amdgcn_perm(a1, a0, 0x05010400u);  // a0.0 a1.0 a0.1 a1.1
                const uint32_t t1 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);  // a0.2 a1.2 a0.3 a1.3
                const uint32_t t2 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);
                const uint32_t t3 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
                c[0][t] = (int)__builtin_amdgcn_perm(t2, t0, 0x05040100u);
                c[1][t] = (int)__builtin_amdgcn_perm(t2, t0, 0x07060302u);
                c[2][t] = (int)__builtin_amdgcn_perm(t3, t1, 0x05040100u);
                c[3][t] = (int)__builtin_amdgcn_perm(t3, t1, 0x07060302u);
            }
            int8_t* o = r.out_p16 + ((d0 / 16 + b) * ldc + 4 * cq) * 16;
#pragma unroll
            for (int e = 0; e < 4; ++e) *(v4i*)(o + 16 * e) = c[e];
        }
    }
}

// The plain pass with 4 rows per thread (4x the threads of the 16-row form above, which ran
// latency-bound at one block per CU): lanes 4 cq + sub take rows 4 sub .. 4 sub + 3 of a 16-row
// block and channel quad cq, so the four lanes of a quad write each channel's 16 P16 bytes as
// four adjacent dwords.
__global__ void __launch_bounds__(256) requant_p16_plain_kernel(ActRequant r, RqGeom g) {
    const int bw = bitwidth_of(read_max(r.amax));
    const int shift = bw - 7;
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && r.exp_out != nullptr) {
        const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
        const int ein = r.exp_in ? (int)*r.exp_in : 0;
        const int ws = r.wscale ? (int)*r.wscale : 0;
        *r.exp_out = (int8_t)(ein + ws + inc);
    }
    const int ldc = r.ldc;
    for (uint32_t u = blockIdx.x * 256u + threadIdx.x; u < g.units; u += gridDim.x * 256u) {
        const int sub = (int)(u & 3u);
        const uint32_t qu = u >> 2;
        const uint32_t blk = fdiv(g.fq, qu);
        const int cq = (int)(qu - blk * (uint32_t)g.qpr);
        const int64_t row0 = (int64_t)blk * 16 + 4 * sub;
        v4i v[4];
        uint32_t mk[4], d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[i] = __builtin_nontemporal_load((const v4i*)(r.acc + (row0 + i) * ldc) + cq);
            mk[i] = r.relu_mask != nullptr ? ((const uint32_t*)(r.relu_mask + (row0 + i) * ldc))[cq] : 0x01010101u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t o = rq4(v[i], raw, s, r.relu);
            if (r.relu_mask != nullptr) {
                uint32_t keep = 0;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if ((int8_t)(mk[i] >> (8 * e)) > 0) keep |= 0xffu << (8 * e);
                o &= keep;
            }
            ((uint32_t*)(r.out_nhwc16 + (row0 + i) * ldc))[cq] = o;
            d[i] = o;
        }
        const uint32_t t0 = __builtin_amdgcn_perm(d[1], d[0], 0x05010400u);
        const uint32_t t1 = __builtin_amdgcn_perm(d[1], d[0], 0x07030602u);
        const uint32_t t2 = __builtin_amdgcn_perm(d[3], d[2], 0x05010400u);
        const uint32_t t3 = __builtin_amdgcn_perm(d[3], d[2], 0x07030602u);
        uint32_t* o = (uint32_t*)(r.out_p16 + ((int64_t)blk * ldc + 4 * cq) * 16) + sub;
        o[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);
        o[4] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);
        o[8] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
        o[12] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
    }
}

template <int MODE>
static void launch_requant_p16(const ActRequant& r, RqGeom g, int64_t blocks, hipStream_t st) {
    switch (r.pool.W) {
        case 2: hipLaunchKernelGGL((requant_p16_kernel<RQ_POOL_BWD, 2>), dim3((unsigned)blocks), dim3(256), 0, st, r, g); break;
        case 4: hipLaunchKernelGGL((requant_p16_kernel<RQ_POOL_BWD, 4>), dim3((unsigned)blocks), dim3(256), 0, st, r, g); break;
        case 8: hipLaunchKernelGGL((requant_p16_kernel<RQ_POOL_BWD, 8>), dim3((unsigned)blocks), dim3(256), 0, st, r, g); break;
        default: hipLaunchKernelGGL((requant_p16_kernel<RQ_POOL_BWD, 16>), dim3((unsigned)blocks), dim3(256), 0, st, r, g); break;
    }
}

bool requant_p16_ok(const ActRequant& r) {
    if (r.ldc % 16 != 0 || r.out_c4 != nullptr || r.pool.pool_out != nullptr) return false;
    if (r.pool.dx == nullptr) return r.out_nhwc16 != nullptr && r.rows % 16 == 0;
    const int W = r.pool.W;
    if (r.pool.H != W || !(W == 2 || W == 4 || W == 8 || W == 16)) return false;
    const int gsz = W == 16 ? p16_group<16>() : p16_group<8>();
    return r.rows % gsz == 0;
}

// Residual add fused with its requantisation (the rule of niti_resnet.hip): the range comes from a
// residual_add pass that stores no z (and, data parallel, a MAX all-reduce); this pass recomputes z
// from the int8 operands and applies the forward rule exactly as requant_act (RQ_PLAIN) on z:
// out = relu?(PSTO(z, shift) | (int8) z), *ez = e_hi - d, *exp_out = *ez + inc.
__global__ void __launch_bounds__(256) residual_requant_kernel(const int8_t* __restrict__ a, const int8_t* __restrict__ ea,
                                                               const int8_t* __restrict__ b, const int8_t* __restrict__ eb,
                                                               int64_t n16, const uint32_t* __restrict__ amax,
                                                               int8_t* __restrict__ ez, int8_t* __restrict__ exp_out,
                                                               int relu, const int8_t* __restrict__ relu_mask,
                                                               int8_t* __restrict__ out, int spec,
                                                               uint32_t* __restrict__ hint, int pk) {
    const int xa = *ea, xb = *eb;
    const bool a_hi = xa >= xb;
    const int diff = a_hi ? xa - xb : xb - xa;
    const int d = diff < 23 ? diff : 23, r = diff - d;
    int bw;
    if (spec == 1) {  // launch A: the guess; the range is published below
        bw = (int)spec_pick(hint, relu ? (a_hi ? xa : xb) - d : 0) - 1;  // forward: on z's scale
        if (bw < 0) bw = 0;  // (no hint yet: B redoes unless the max is 0)
        if (blockIdx.x == 0 && threadIdx.x == 0)
            __hip_atomic_store(hint + 1, (uint32_t)bw + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        bw = bitwidth_of(read_max(amax));  // whole wave active
        if (spec == 2) {  // launch B: A's output stands unless the (all-reduced) range differs
            const int used = __builtin_amdgcn_readfirstlane(
                                 (int)__hip_atomic_load(hint + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - 1;
            if (blockIdx.x == 0 && threadIdx.x < 64) spec_learn(hint, bw, relu ? (a_hi ? xa : xb) - d : 0, threadIdx.x);
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                if (bw != used) __hip_atomic_fetch_add(hint + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int shift = bw - 7;
                const int e_z = (a_hi ? xa : xb) - d;
                if (ez != nullptr) *ez = (int8_t)e_z;
                if (exp_out != nullptr) *exp_out = (int8_t)(e_z + (shift > 1 ? shift : (shift == 1 ? 2 : 0)));
            }
            if (bw == used) return;
        }
    }
    const int shift = bw - 7;
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    if (spec == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        const int e_z = (a_hi ? xa : xb) - d;
        if (ez != nullptr) *ez = (int8_t)e_z;
        if (exp_out != nullptr) *exp_out = (int8_t)(e_z + (shift > 1 ? shift : (shift == 1 ? 2 : 0)));
    }
    uint32_t m = 0;
    if (pk && !raw) {  // the bit-field form (res_rule4)
        const ResRule k = res_rule(d, r, s);
        const int8_t* hi = a_hi ? a : b;
        const int8_t* lo = a_hi ? b : a;
        int mx = 0, mn = 0;
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
            const v4i vh = ((const v4i*)hi)[i], vl = ((const v4i*)lo)[i];
            v4i mk;
            if (relu_mask != nullptr) mk = ((const v4i*)relu_mask)[i];
            v4i q;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t o = relu ? res_rule4<true>((uint32_t)vh[w], (uint32_t)vl[w], k, mx, mn, spec == 1)
                                  : res_rule4<false>((uint32_t)vh[w], (uint32_t)vl[w], k, mx, mn, spec == 1);
                if (relu_mask != nullptr) o &= sw_expand(sw_pos_hi((uint32_t)mk[w]));
                q[w] = (int)o;
            }
            ((v4i*)out)[i] = q;
        }
        m = max(uabs32(mx), uabs32(mn));
    } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const v16c va = ((const v16c*)a)[i], vb = ((const v16c*)b)[i];
        v16c mk;
        if (relu_mask != nullptr) mk = ((const v16c*)relu_mask)[i];
        v16c q;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int32_t z = residual_z(a_hi ? va[e] : vb[e], a_hi ? vb[e] : va[e], d, r);
            if (spec == 1) {
                const uint32_t u = uabs32(z);
                m = m > u ? m : u;
            }
            int32_t o = raw ? (int32_t)(int8_t)z : psto_fast(z, s);
            if (relu && o < 0) o = 0;
            if (relu_mask != nullptr && mk[e] <= 0) o = 0;  // the next op's NITI_ReluGrad_Int8, fused
            q[e] = (signed char)o;
        }
        ((v16c*)out)[i] = q;
    }
    }
    if (spec == 1) {  // NITI_RangeEstimate of z for launch B
        m = wave_max(m);
        __shared__ uint32_t red[4];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(const_cast<uint32_t*>(amax), max(max(red[0], red[1]), max(red[2], red[3])));
    }
}

hipError_t residual_requant(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                            const uint32_t* amax, int8_t* ez, int8_t* exp_out, int relu, int8_t* out, hipStream_t st,
                            const int8_t* relu_mask, int spec, uint32_t* slot) {
    if (n < 0 || n % 16 != 0 || !a || !b || !ea || !eb || !amax || !out) return hipErrorInvalidValue;
    if (spec < 0 || spec > 2 || (spec != 0 && slot == nullptr)) return hipErrorInvalidValue;
    const int64_t n16 = n / 16;
    int64_t blocks = (n16 + 255) / 256;
    blocks = blocks < 1 ? 1 : blocks > 2048 ? 2048 : blocks;
    // NITI_RES_PK=0: the 32-bit loop only (an A/B switch for the packed form)
    static const int pk = getenv("NITI_RES_PK") ? atoi(getenv("NITI_RES_PK")) : 1;
    hipLaunchKernelGGL(residual_requant_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, ea, b, eb, n16, amax, ez,
                       exp_out, relu, relu_mask, out, spec, slot, pk);
    return hipGetLastError();
}

// ---- first layer on its im2col copy (K = 32) -------------------------------------------------
// y[p][co] = sum_k xcol[p][k] * w[co][k], k < 32: one v_mfma_i32_32x32x32_i8 per 32 pixels x 32
// output channels, both operands straight from memory (a lane's 16-byte fragment is 16
// consecutive k of one row).  Pass 0 publishes max|y| (NITI_RangeEstimate); pass 1 recomputes y
// and requantises it with the forward rule (as requant_quad_kernel), relu, stores the NHWC16
// output and, with pool_out, the 2x2 max pool of the relu'd values.  A wave takes a pair of
// output rows segment by segment (32 pixels of each row), so each pooled pixel's four inputs
// sit in one lane: the x pairs in adjacent accumulator registers, the y pair in the two rows'
// accumulators.  Requires OW % 32 == 0 and OH even (VGG's 32x32 and 224x224 first layers).
struct Conv0 {
    const int8_t* x;  // xcol [P][32]
    const int8_t* w;  // [co][32]
    uint32_t wbytes;
    int co, cop, oh, ow;
    int64_t units;    // (image, row pair, 32-pixel segment)
    uint32_t* amax;   // pass 0 out / pass 1 in
    int8_t* out;      // NHWC16 [P][cop]
    int8_t* pool_out; // [P / 4][cop] or null
    int8_t* pool_c32; // the pooled output as the next layer's C32 input [n][cop/32][oh/2][ow/2][32], or null
    int8_t* out_c32;  // the (unpooled) output as the next layer's C32 input [n][cop/32][oh][ow][32], or null
    int8_t* pool_code; // the pool gradient's route (pool_code4) [P / 4][cop], or null
    const int8_t *exp_in, *wscale;
    int8_t* exp_out;
    int relu;
};

template <int PASS>
__global__ void __launch_bounds__(256) conv0_kernel(Conv0 g) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = gridDim.x * 4;
    const int h = lane >> 5, c = lane & 31;
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(g.w, g.wbytes);
    int s = 2, shift = 0;
    bool raw = false;
    if (PASS == 1) {
        const int bw = bitwidth_of(read_max(g.amax));
        shift = bw - 7;
        s = shift > 1 ? shift : 2;
        raw = shift <= 0;
        if (blockIdx.x == 0 && threadIdx.x == 0 && g.exp_out != nullptr) {
            const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
            *g.exp_out = (int8_t)((g.exp_in ? (int)*g.exp_in : 0) + (g.wscale ? (int)*g.wscale : 0) + inc);
        }
    }
    const int tiles = g.cop / 32;
    uint32_t m = 0;
    const int segs = g.ow / 32, pairs = g.oh / 2;
    for (int64_t u = wave; u < g.units; u += nwaves) {
        const int seg = (int)(u % segs);
        const int64_t rest = u / segs;
        const int pr = (int)(rest % pairs);
        const int64_t img = rest / pairs;
        const int64_t p0 = (img * g.oh + 2 * pr) * g.ow + seg * 32;  // first pixel of the top row segment
        v4i a[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) a[r] = *(const v4i*)(g.x + (p0 + (int64_t)r * g.ow + c) * 32 + 16 * h);
        for (int t = 0; t < tiles; ++t) {
            const v4i b = buf_load16(rw, (uint32_t)((t * 32 + c) * 32 + 16 * h));
            v16i acc[2];
#pragma unroll
            for (int r = 0; r < 2; ++r)
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a[r], v16i{}, 0, 0, 0);
            // acc[r][i]: output channel t * 32 + (i & 3) + 8 (i >> 2) + 4 h, pixel p0 + r * ow + c
            if (PASS == 0) {
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int ch = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                        const uint32_t v = ch < g.co ? uabs32(acc[r][i]) : 0u;
                        m = m > v ? m : v;
                    }
            } else {
                int8_t q[2][16];
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        int32_t v;
                        if (raw) {
                            v = (int32_t)(int8_t)acc[r][i];
                        } else if (g.relu) {  // PSTO of max(acc, 0): a negative value is 0 whatever its rounding
                            const uint32_t x = (uint32_t)max(acc[r][i], 0);
                            const uint32_t qp = __builtin_amdgcn_ubfe(x, s >> 1, s - (s >> 1));
                            const uint32_t pr = __builtin_amdgcn_ubfe(x, 0, s >> 1) << (s & 1);
                            v = (int32_t)min((x >> s) + (qp > pr ? 1u : 0u), 127u);
                        } else {
                            v = psto_fast(acc[r][i], s);
                        }
                        if (g.relu && v < 0) v = 0;
                        q[r][i] = (int8_t)v;
                    }
                // lane (pixel c, half h) holds channels 8j + 4h + 0..3 as dword D[j]; one half-wave
                // swap per pair (D0, D2), (D1, D3) gives the lower half channels 0..15 and the
                // upper half 16..31 of its pixel: one 16-byte store per lane and tile
                auto pack = [&](const int8_t* v) {
                    uint32_t d[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        d[j] = (uint32_t)(uint8_t)v[4 * j] | (uint32_t)(uint8_t)v[4 * j + 1] << 8 |
                               (uint32_t)(uint8_t)v[4 * j + 2] << 16 | (uint32_t)(uint8_t)v[4 * j + 3] << 24;
                    const auto x02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
                    const auto x13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
                    return v4i{(int)x02[0], (int)x02[1], (int)x13[0], (int)x13[1]};
                };
                v4i qv[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const v4i v = pack(q[r]);
                    qv[r] = v;
                    if (g.out != nullptr) *(v4i*)(g.out + (p0 + (int64_t)r * g.ow + c) * g.cop + t * 32 + 16 * h) = v;
                    if (g.out_c32 != nullptr)
                        *(v4i*)(g.out_c32 + (((img * tiles + t) * g.oh + 2 * pr + r) * (int64_t)g.ow + seg * 32 + c) * 32 +
                                16 * h) = v;
                }
                if (g.pool_out != nullptr) {
                    // vertical max in the lane, horizontal with the neighbour pixel (lane c ^ 1);
                    // even lanes store their pooled pixel
                    int8_t pm[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int v0 = q[0][i] > q[1][i] ? q[0][i] : q[1][i];
                        const int v1 = __shfl_xor(v0, 1, 64);
                        pm[i] = (int8_t)(v0 > v1 ? v0 : v1);
                    }
                    const v4i v = pack(pm);
                    v4i code{0, 0, 0, 0};
                    if (g.pool_code != nullptr) {  // the window: (top, bottom) here, the odd neighbour's
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t t1 = (uint32_t)__builtin_amdgcn_mov_dpp(qv[0][k], 0xB1, 0xF, 0xF, false);
                            const uint32_t t3 = (uint32_t)__builtin_amdgcn_mov_dpp(qv[1][k], 0xB1, 0xF, 0xF, false);
                            code[k] = (int)pool_code4((uint32_t)qv[0][k], t1, (uint32_t)qv[1][k], t3, (uint32_t)v[k],
                                                      g.relu != 0);
                        }
                    }
                    if ((c & 1) == 0) {
                        const int64_t pp = (img * (g.oh / 2) + pr) * (g.ow / 2) + seg * 16 + (c >> 1);
                        *(v4i*)(g.pool_out + pp * g.cop + t * 32 + 16 * h) = v;
                        if (g.pool_code != nullptr) *(v4i*)(g.pool_code + pp * g.cop + t * 32 + 16 * h) = code;
                        if (g.pool_c32 != nullptr) {
                            const int64_t hw2 = (int64_t)(g.oh / 2) * (g.ow / 2);
                            *(v4i*)(g.pool_c32 + ((img * tiles + t) * hw2 + pp - img * hw2) * 32 + 16 * h) = v;
                        }
                    }
                }
            }
        }
    }
    if (PASS == 0) {
        m = wave_max(m);
        __shared__ uint32_t red[4];
        if (lane == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(g.amax, max(max(red[0], red[1]), max(red[2], red[3])));
    }
}

bool conv0_ok(const ConvGeom& g) {
    return g.kh == 1 && g.kw == 1 && g.c_in == 32 && g.cip == 32 && g.ow % 32 == 0 && g.oh % 2 == 0 && g.sh == 1 &&
           g.pt == 0 && g.cop % 32 == 0;
}

hipError_t conv0_fwd(const ConvGeom& g, const int8_t* xcol, const int8_t* w, uint32_t* amax, const ActOut& o,
                     int pass, hipStream_t st, int8_t* pool_c32, int8_t* out_c32, int8_t* pool_code) {
    // (out may be null when the pooled output is kept: pool_out + pool_code carry everything the
    // backward pass reads)
    if (!conv0_ok(g) || o.relu_mask != nullptr) return hipErrorInvalidValue;
    if (o.out == nullptr && (pass == 1 && (o.pool.pool_out == nullptr || pool_code == nullptr))) return hipErrorInvalidValue;
    if ((pool_c32 != nullptr || pool_code != nullptr) && o.pool.pool_out == nullptr) return hipErrorInvalidValue;
    Conv0 k{};
    k.x = xcol;
    k.w = w;
    k.wbytes = (uint32_t)((int64_t)g.c_out * 32);
    k.co = g.c_out;
    k.cop = g.cop;
    k.oh = g.oh;
    k.ow = g.ow;
    k.units = (int64_t)g.n * (g.oh / 2) * (g.ow / 32);
    k.amax = amax;
    k.out = o.out;
    k.pool_out = o.pool.pool_out;
    k.pool_c32 = pool_c32;
    k.out_c32 = out_c32;
    k.pool_code = pool_code;
    k.exp_in = o.exp_in;
    k.wscale = o.wscale;
    k.exp_out = o.exp_out;
    k.relu = o.relu;
    int64_t blocks = (k.units + 3) / 4;
    blocks = blocks > 1024 ? 1024 : blocks;
    if (pass == 0)
        hipLaunchKernelGGL(conv0_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, st, k);
    else
        hipLaunchKernelGGL(conv0_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st, k);
    return hipGetLastError();
}

// The requantisation with the 3x3 / 2 (pad 1) max pool fused (ActRequant::pool3, ResNet-18's
// stem: NITI_Conv_Int8.cpp:266-307's rescale + relu, then NITI_Maxpool_Int8.cpp:24-72 over the
// int8 result, first maximum in (ky, kx) order), so the pre-pool int8 image is neither written
// (unless out_nhwc16) nor read back by a pool pass.  One thread per pooled column strip of
// RQ3_ROWS pooled rows and 4 channels: each step requantises the two new input rows' three
// columns and carries the last one down as the next window's top row, so the accumulators are
// read once vertically (plus one row per strip); the horizontal overlap (the shared column of
// neighbouring windows) is the neighbouring lanes' load of the same lines.  VALU-bound before
// the relu forms below (~700 operations per pooled quad: 160 us for the batch-128 stem).
constexpr int RQ3_ROWS = 4;  // (2-28 measured: 103-113 us, profiles/r05_stem_pool.txt)
struct Rq3Geom {
    FastDiv fq, fow, fch;  // by quads per row, pooled width, strips per image
    int qpr, H, W, OH, rows;  // rows: pooled rows per strip
    uint32_t units;
    int remap;  // one thread per unit, blocks XCD-remapped (else grid-stride)
};
__device__ __forceinline__ void pool3_take(uint32_t o, int k, uint32_t& m, uint32_t& a) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int ov = (int8_t)(o >> (8 * e)), mv = (int8_t)(m >> (8 * e)), av = (int8_t)(a >> (8 * e));
        if (av < 0 || ov > mv) {
            m = (m & ~(0xffu << (8 * e))) | (o & (0xffu << (8 * e)));
            a = (a & ~(0xffu << (8 * e))) | ((uint32_t)k << (8 * e));
        }
    }
}
// relu(PSTO(v, s)) of four accumulators, packed (rq4 with relu and s >= 2, in fewer VALU
// operations: a <= 0 gives 0 either way, so the sign paths go; the pool is VALU-bound otherwise)
__device__ __forceinline__ uint32_t rq4_relu(v4i v, int s) {
    const int h = s >> 1, odd = s & 1;
    uint32_t o = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const uint32_t x = (uint32_t)max(v[e], 0);
        const uint32_t qp = __builtin_amdgcn_ubfe(x, h, s - h), pr = __builtin_amdgcn_ubfe(x, 0, h) << odd;
        const uint32_t q = min((x >> s) + (qp > pr ? 1u : 0u), 127u);
        o |= q << (8 * e);
    }
    return o;
}
// pool3_take for bytes in [0, 127] (relu outputs), four at once: where o > m (strict: the first
// maximum stays), m = o and a = k
__device__ __forceinline__ void pool3_take_u7(uint32_t o, uint32_t k4, uint32_t& m, uint32_t& a) {
    const uint32_t gt = ((o | 0x80808080u) - m - 0x01010101u) & 0x80808080u;  // bytes: 127 + o - m >= 128
    const uint32_t mask = (gt >> 7) * 0xffu;
    m = (m & ~mask) | (o & mask);
    a = (a & ~mask) | (k4 & mask);
}

template <bool RELU>
__global__ void __launch_bounds__(256) requant_pool3_kernel(ActRequant r, Rq3Geom g) {
    // (wave-uniform: scalar branches below)
    const int bw = __builtin_amdgcn_readfirstlane(bitwidth_of(read_max(r.amax)));
    const int shift = bw - 7;
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && r.exp_out != nullptr) {
        const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
        const int ein = r.exp_in ? (int)*r.exp_in : 0;
        const int ws = r.wscale ? (int)*r.wscale : 0;
        *r.exp_out = (int8_t)(ein + ws + inc);
    }
    const uint32_t qpr = (uint32_t)g.qpr;
    const int OW = (int)g.fow.d;
    const int64_t RS = (int64_t)g.W * qpr;  // input row stride, quads
    const uint32_t bid = g.remap ? (uint32_t)xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    auto rq = [&](const v4i& v) { return RELU && !raw ? rq4_relu(v, s) : rq4(v, raw, s, RELU); };
    auto take = [&](uint32_t o, int k, uint32_t& m, uint32_t& a) {
        if (RELU)
            pool3_take_u7(o, 0x01010101u * (uint32_t)k, m, a);
        else
            pool3_take(o, k, m, a);
    };
    for (uint32_t u = bid * 256u + threadIdx.x; u < g.units; u += g.remap ? g.units : gridDim.x * 256u) {
        const uint32_t pix = fdiv(g.fq, u), q = u - pix * qpr;
        const uint32_t t = fdiv(g.fow, pix), ox = pix - t * g.fow.d;
        const uint32_t b = fdiv(g.fch, t), ch = t - b * g.fch.d;
        const int oy0 = (int)ch * g.rows, oy1 = min(g.OH, oy0 + g.rows);
        const int x0 = 2 * (int)ox - 1;
        const bool c0 = x0 >= 0, c2 = x0 + 2 < g.W;
        // columns x0, x0 + 1, x0 + 2 of a row as offsets from column x0 + 1 (a column outside the
        // image reads column x0 + 1 instead: loaded, never taken)
        const int64_t o0 = c0 ? -(int64_t)qpr : 0, o2 = c2 ? (int64_t)qpr : 0;
        const v4i* p = (const v4i*)r.acc + ((int64_t)b * g.H * g.W + 2 * oy0 * g.W + x0 + 1) * qpr + q;
        uint32_t* y0 = r.out_nhwc16 ? (uint32_t*)r.out_nhwc16 + (p - (const v4i*)r.acc) : nullptr;
        // the two input rows 2 oy, 2 oy + 1 at p (the second: the first again past the image)
        auto load = [&](const v4i* p, int oy, v4i* a) {
            const v4i* p1 = 2 * oy + 1 < g.H ? p + RS : p;
            a[0] = p[o0];
            a[1] = p[0];
            a[2] = p[o2];
            a[3] = p1[o0];
            a[4] = p1[0];
            a[5] = p1[o2];
        };
        uint32_t top[3] = {0, 0, 0};
        if (oy0 > 0) {
            const v4i* pt = p - RS;
            top[0] = rq(pt[o0]);
            top[1] = rq(pt[0]);
            top[2] = rq(pt[o2]);
        }
        auto step = [&](const v4i* a, int oy) {
            const bool r2 = 2 * oy + 1 < g.H;
            uint32_t mid[3], bot[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                mid[k] = rq(a[k]);
                bot[k] = rq(a[3 + k]);
            }
            // bytes: max, position.  With relu every value is >= 0: start from 0 at the window's
            // first position, later positions taken where strictly greater (the first maximum)
            uint32_t m = RELU ? 0u : 0x80808080u;
            uint32_t am = RELU ? 0x01010101u * (uint32_t)((oy > 0 ? 0 : 3) + (c0 ? 0 : 1)) : 0xffffffffu;
            if (oy > 0) {
                if (c0) take(top[0], 0, m, am);
                take(top[1], 1, m, am);
                if (c2) take(top[2], 2, m, am);
            }
            if (c0) take(mid[0], 3, m, am);
            take(mid[1], 4, m, am);
            if (c2) take(mid[2], 5, m, am);
            if (r2) {
                if (c0) take(bot[0], 6, m, am);
                take(bot[1], 7, m, am);
                if (c2) take(bot[2], 8, m, am);
            }
            const int64_t po = (((int64_t)b * g.OH + oy) * OW + ox) * qpr + q;
            ((uint32_t*)r.pool3.out)[po] = m;
            ((uint32_t*)r.pool3.arg)[po] = am;
            if (y0 != nullptr) {  // each pre-pool pixel once: rows 2 oy, 2 oy + 1 x columns x0 + 1, x0 + 2
                uint32_t* d = y0 + (int64_t)(oy - oy0) * 2 * RS;
                d[0] = mid[1];
                if (c2) d[qpr] = mid[2];
                if (r2) {
                    d[RS] = bot[1];
                    if (c2) d[RS + qpr] = bot[2];
                }
            }
            top[0] = bot[0];
            top[1] = bot[1];
            top[2] = bot[2];
        };
        // two register sets, each step's rows loaded one step ahead
        v4i A[6], B[6];
        load(p, oy0, A);
        for (int oy = oy0;;) {
            if (oy + 1 < oy1) load(p + 2 * RS, oy + 1, B);
            step(A, oy);
            if (++oy >= oy1) break;
            p += 2 * RS;
            if (oy + 1 < oy1) load(p + 2 * RS, oy + 1, A);
            step(B, oy);
            if (++oy >= oy1) break;
            p += 2 * RS;
        }
    }
}

hipError_t requant_act(const ActRequant& r, hipStream_t st) {
    if (r.ldc % 16 != 0 || r.acc == nullptr || r.amax == nullptr) return hipErrorInvalidValue;
    if (r.pool.pool_out != nullptr || r.pool.dx != nullptr) {
        if (r.pool.H % 2 || r.pool.W % 2 || r.pool.H <= 0 || r.pool.W <= 0) return hipErrorInvalidValue;
        if (r.pool.pool_out != nullptr && (r.out_nhwc16 == nullptr || r.rows % ((int64_t)r.pool.H * r.pool.W)))
            return hipErrorInvalidValue;
        if (r.pool.dx != nullptr && (r.pool.x == nullptr || r.pool.y == nullptr ||
                                     r.rows % ((int64_t)(r.pool.H / 2) * (r.pool.W / 2))))
            return hipErrorInvalidValue;
    }
    if (r.pool.dx_c32 != nullptr && (r.pool.dx == nullptr || r.out_p16 != nullptr || r.ldc % 32 != 0))
        return hipErrorInvalidValue;
    if (r.zero_cls != 0 && (r.out_p16 != nullptr || r.out_c4 != nullptr)) return hipErrorInvalidValue;
    if (r.pool3.out != nullptr) {
        const Pool3& p = r.pool3;
        if (r.out_p16 != nullptr || r.out_c4 != nullptr || r.zero_cls != 0 || r.pool.pool_out != nullptr ||
            r.pool.dx != nullptr || r.relu_mask != nullptr || p.arg == nullptr || r.ldc % 4 != 0 || p.H <= 0 ||
            p.W <= 0 || p.OH != (p.H - 1) / 2 + 1 || p.OW != (p.W - 1) / 2 + 1 || r.rows % ((int64_t)p.H * p.W) != 0)
            return hipErrorInvalidValue;
        Rq3Geom g;
        g.qpr = r.ldc / 4;
        g.H = p.H;
        g.W = p.W;
        g.OH = p.OH;
        static const int rows_env = getenv("NITI_RQ3_ROWS") ? atoi(getenv("NITI_RQ3_ROWS")) : RQ3_ROWS;
        static const int remap_env = getenv("NITI_RQ3_REMAP") ? atoi(getenv("NITI_RQ3_REMAP")) : 0;
        g.rows = rows_env > 0 ? rows_env : RQ3_ROWS;
        const int strips = (p.OH + g.rows - 1) / g.rows;
        const int64_t units = r.rows / ((int64_t)p.H * p.W) * strips * p.OW * g.qpr;
        if (units >= (int64_t)1 << 31) return hipErrorInvalidValue;
        g.units = (uint32_t)units;
        g.fq = make_fastdiv((uint32_t)g.qpr);
        g.fow = make_fastdiv((uint32_t)p.OW);
        g.fch = make_fastdiv((uint32_t)strips);
        int64_t blocks = (units + 255) / 256;
        g.remap = remap_env != 0 && blocks <= ((int64_t)1 << 24);
        if (!g.remap && blocks > 8192) blocks = 8192;
        if (blocks < 1) blocks = 1;
        if (r.relu)
            hipLaunchKernelGGL(requant_pool3_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, r, g);
        else
            hipLaunchKernelGGL(requant_pool3_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, r, g);
        return hipGetLastError();
    }
    if (r.out_p16 != nullptr) {  // the output (dx with the pool gradient) also as its P16 copy
        if (!requant_p16_ok(r)) return hipErrorInvalidValue;
        RqGeom g{};
        g.qpr = r.ldc / 4;
        g.W = r.pool.W;
        const int gsz = r.pool.dx == nullptr ? 16 : (r.pool.W == 16 ? p16_group<16>() : p16_group<8>());
        // plain: a thread per (16-row block, quad, quarter); pool gradient: per (run, quad)
        const int64_t units = r.rows / gsz * g.qpr * (r.pool.dx == nullptr ? 4 : 1);
        if (units >= (int64_t)1 << 31) return hipErrorInvalidValue;
        if (units == 0) return hipSuccess;
        g.units = (uint32_t)units;
        g.fq = make_fastdiv((uint32_t)g.qpr);
        int64_t blocks = (units + 255) / 256;
        if (blocks > 2048) blocks = 2048;
        if (r.pool.dx == nullptr)
            hipLaunchKernelGGL(requant_p16_plain_kernel, dim3((unsigned)blocks), dim3(256), 0, st, r, g);
        else
            launch_requant_p16<RQ_POOL_BWD>(r, g, blocks, st);
        return hipGetLastError();
    }
    if (r.out_c4 == nullptr) {
        const bool pf = r.pool.pool_out != nullptr, pb = r.pool.dx != nullptr;
        if (!pf && !pb && r.out_nhwc16 == nullptr) return hipErrorInvalidValue;
        RqGeom g;
        g.qpr = r.ldc / 4;
        g.W = r.pool.W;
        const int64_t rows = pf ? r.rows / 4 : r.rows;  // pooled pixels for the pool modes
        const int64_t units = rows * g.qpr;
        if (units >= (int64_t)1 << 31) return hipErrorInvalidValue;
        g.units = (uint32_t)units;
        g.fq = make_fastdiv((uint32_t)g.qpr);
        if (pf || pb) {
            g.fpw = make_fastdiv((uint32_t)(r.pool.W / 2));
            g.fph = make_fastdiv((uint32_t)(r.pool.H / 2));
        }
        if (r.zero_cls != 0) {
            if (pf || pb || r.zc_h <= 0 || r.zc_w <= 0 || r.rows % ((int64_t)r.zc_h * r.zc_w)) return hipErrorInvalidValue;
            g.fzw = make_fastdiv((uint32_t)r.zc_w);
            g.fzh = make_fastdiv((uint32_t)r.zc_h);
        }
        int64_t blocks = (units + 256 * RQ_U - 1) / (256 * RQ_U);
        if (blocks > 2048) blocks = 2048;
        if (blocks < 1) blocks = 1;
        if (pf)
            hipLaunchKernelGGL(requant_quad_kernel<RQ_POOL_FWD>, dim3((unsigned)blocks), dim3(256), 0, st, r, g);
        else if (pb)
            hipLaunchKernelGGL(requant_quad_kernel<RQ_POOL_BWD>, dim3((unsigned)blocks), dim3(256), 0, st, r, g);
        else
            hipLaunchKernelGGL(requant_quad_kernel<RQ_PLAIN>, dim3((unsigned)blocks), dim3(256), 0, st, r, g);
        return hipGetLastError();
    }
    const int64_t total = r.rows * (r.ldc / 16);
    int64_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(requant_act_kernel, dim3((unsigned)blocks), dim3(256), 0, st, r);
    return hipGetLastError();
}

__global__ void requant_grad_kernel(const int32_t* __restrict__ acc, int64_t n, const uint32_t* __restrict__ amax,
                                    int rule, int8_t* __restrict__ g_out, int8_t* __restrict__ w) {
    const int bw = bitwidth_of(read_max(amax));
    const int s = bw - rule;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t g = bw == 0 ? 0 : psto_any(acc[i], s);
        if (g_out) g_out[i] = (int8_t)g;
        if (w) w[i] = (int8_t)clip127((int32_t)w[i] - g);
    }
}

hipError_t requant_grad(const int32_t* acc, int64_t n, const uint32_t* amax, int rule, int8_t* g_out, int8_t* w,
                        hipStream_t st) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(requant_grad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, acc, n, amax, rule, g_out, w);
    return hipGetLastError();
}

// Fused NITI_SGD step on a 64(co) x 64(ci) tile of one tap: g = gradient rule(acc), w <- clip(w - g)
// in OHWI16, and the updated weights also written transposed (IHWO16, the input-gradient B
// operand) through an LDS tile -- the transposed copy never needs a pass of its own.
// One 64 (co) x 64 (ci) tile of one tap: g = rule(acc, range), w <- clip(w - g, +-127) in OHWI16,
// the same tile transposed through LDS into IHWO16 (the input-gradient operand), g to g_out.
// bw: NITI_RangeEstimate of the job's gradient (read once per job by the caller)
// (sgd_tile: niti_sgd.hpp)

// Every layer's NITI_SGD update of a step in one launch: block b belongs to the job whose
// [start, start + tiles) range holds it (the updates are independent; the input gradients
// that read the old weights have all run by then).
// The deferred split-K combines of a step's P16 weight gradients, all layers in one launch ahead
// of the update (one launch instead of one reduce per layer, each of which left the chip mostly
// idle: 576 blocks of a few loads each): chunk c (1024 elements of one job's acc, 4 per thread) =
// the sum of the job's slabs, its max into the job's range.  (A grid barrier inside the update
// launch instead measured +275 us per VGG-11 step: 1536-2048 arrivals on one counter.)
__global__ void __launch_bounds__(256) sgd_combine_kernel(SgdJobs jobs) {
    const int chunks = jobs.cstart[jobs.n];
    // a block's chunks ascend, so its jobs do too: the running max of the current job is
    // published once when the block leaves it (one atomic per wave per job, not per chunk --
    // ResNet-18's ~15 K chunks of per-chunk atomics on a few range words cost ~50 us)
    uint32_t m = 0;
    int cur = -1;
    for (int c = blockIdx.x; c < chunks; c += gridDim.x) {
        int j = 0;
        while (j + 1 < jobs.n && c >= jobs.cstart[j + 1]) ++j;
        if (j != cur) {
            if (cur >= 0) {
                const uint32_t w = wave_max(m);
                if ((threadIdx.x & 63) == 0) publish_max(const_cast<uint32_t*>(jobs.job[cur].amax), w);
            }
            cur = j;
            m = 0;
        }
        const SgdJob& J = jobs.job[j];
        const int64_t e = (int64_t)(c - jobs.cstart[j]) * 1024 + threadIdx.x * 4;
        int64_t de = e;  // the acc element this slab element sums into
        bool live = J.slab != nullptr && e < J.slab_n;
        if (live && J.slab_map == 1) {  // SlabTapsBlocked (splitk_reduce's map), on 16-byte units
            const uint32_t u = (uint32_t)(e >> 2);
            const uint32_t tile = u / 4608u, rem = u - tile * 4608u;
            const uint32_t row = rem / 72u, rc = rem - row * 72u;
            const uint32_t t = rc / 8u, part = rc - t * 8u;
            FastDiv ft;
            ft.m = J.tb_m;
            ft.s = J.tb_s;
            const uint32_t tco = fdiv(ft, tile), tci = tile - tco * (uint32_t)J.tb_tiles_ci;
            const int co = (int)(tco * 64u + row);
            live = co < J.co;
            de = ((int64_t)co * J.tb_ld4 + t * J.tb_cip4 + tci * 8u + part) * 4;
        }
        if (live) {
            const v4i* base = (const v4i*)(J.slab + e);
            const int64_t st4 = J.slab_stride / 4;
            v4i s = {0, 0, 0, 0};
            for (int z0 = 0; z0 < J.splits; z0 += 8) {  // up to 8 independent loads in flight
                v4i v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    v[q] = z0 + q < J.splits ? __builtin_nontemporal_load(base + (int64_t)(z0 + q) * st4) : v4i{0, 0, 0, 0};
#pragma unroll
                for (int q = 0; q < 8; ++q) s += v[q];
            }
            *(v4i*)(const_cast<int32_t*>(J.acc) + de) = s;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t u = uabs32(s[q]);
                m = m > u ? m : u;
            }
        }
    }
    if (cur >= 0) {
        const uint32_t w = wave_max(m);
        if ((threadIdx.x & 63) == 0) publish_max(const_cast<uint32_t*>(jobs.job[cur].amax), w);
    }
}

__global__ void sgd_update_kernel(SgdJobs jobs, int total) {
    __shared__ int8_t T[64][64 + 4];
    // a block takes tiles b, b + gridDim, ...: one resident wave of blocks instead of a full
    // wave plus a straggling partial one.  The next tile's operands are loaded before this one is
    // finished, and a tile's loads are issued before its job's range is read (the range word's
    // dependent read and wave reduction then overlap the operand fetch).
    struct Tile {
        int j, ci0, co0, k;
    };
    auto locate = [&](int bb) {
        Tile t;
        int b = bb, j = 0;
        while (j + 1 < jobs.n && b >= jobs.start[j + 1]) ++j;
        const SgdJob& J = jobs.job[j];
        b -= jobs.start[j];
        const int tx = (J.cip + 63) / 64, ty = (J.cop + 63) / 64;
        const int k = b / (tx * ty), rem = b - k * tx * ty;
        t.j = j;
        t.ci0 = (rem % tx) * 64;
        t.co0 = (rem / tx) * 64;
        t.k = k;
        return t;
    };
    int bb = blockIdx.x;
    if (bb >= total) return;
    if (!NITI_SGD_PREFETCH) {  // one tile at a time
        int last_j = -1, bw = 0;
        for (; bb < total; bb += gridDim.x) {
            const Tile t = locate(bb);
            if (t.j != last_j) {
                bw = bitwidth_of(read_max(jobs.job[t.j].amax));
                last_j = t.j;
            }
            if (bb != (int)blockIdx.x) __syncthreads();  // the previous tile's transposed reads are done
            sgd_tile(jobs.job[t.j], bw, t.ci0, t.co0, t.k, T);
        }
        return;
    }
    Tile cur = locate(bb);
    SgdTileIn cin, nin;  // (named, not an indexed pair: a dynamically indexed array would live in scratch)
    sgd_tile_load(jobs.job[cur.j], cur.ci0, cur.co0, cur.k, cin);
    int last_j = -1, bw = 0;
    for (; bb < total; bb += gridDim.x) {
        const int nb = bb + gridDim.x;
        Tile nxt = cur;
        if (nb < total) {
            nxt = locate(nb);
            sgd_tile_load(jobs.job[nxt.j], nxt.ci0, nxt.co0, nxt.k, nin);
        }
        if (cur.j != last_j) {
            bw = bitwidth_of(read_max(jobs.job[cur.j].amax));
            last_j = cur.j;
        }
        if (bb != (int)blockIdx.x) __syncthreads();  // the previous tile's transposed reads are done
        sgd_tile_finish(jobs.job[cur.j], bw, cur.ci0, cur.co0, cur.k, cin, T);
        cur = nxt;
        cin = nin;
    }
}

hipError_t sgd_update_many(const SgdJob* jobs, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (n > SGD_MAX_JOBS) return hipErrorInvalidValue;
    SgdJobs J{};
    J.n = n;
    int total = 0, chunks = 0;
    for (int i = 0; i < n; ++i) {
        J.job[i] = jobs[i];
        J.start[i] = total;
        J.cstart[i] = chunks;
        total += ((jobs[i].cip + 63) / 64) * ((jobs[i].cop + 63) / 64) * jobs[i].kk;
        if (jobs[i].slab != nullptr) {
            if (jobs[i].splits < 1 || jobs[i].slab_stride % 4 != 0 || jobs[i].slab_n % 4 != 0) return hipErrorInvalidValue;
            chunks += (int)((jobs[i].slab_n + 1023) / 1024);
        }
    }
    J.cstart[n] = chunks;
    if (chunks > 0) {  // the deferred combines first (same stream: the update reads their sums)
        const int cgrid = chunks < 2048 ? chunks : 2048;
        hipLaunchKernelGGL(sgd_combine_kernel, dim3(cgrid), dim3(256), 0, st, J);
    }
    const int grid = total < 1536 ? total : 1536;  // 6 blocks per CU
    hipLaunchKernelGGL(sgd_update_kernel, dim3(grid), dim3(256), 0, st, J, total);
    return hipGetLastError();
}

hipError_t sgd_update(const int32_t* acc, const uint32_t* amax, int rule, int co, int ci, int kk, int cip, int cop,
                      int8_t* w, int8_t* wT, int8_t* g_out, hipStream_t st) {
    SgdJob j{acc, amax, rule, co, ci, kk, cip, cop, w, wT, g_out};
    return sgd_update_many(&j, 1, st);
}

// =====================================================================================
// The rest of the step: pool / relu-grad / loss-grad
// =====================================================================================

// NITI_Maxpool_Int8.cpp:24-72 (kernel clipped to the input); one thread per 16 channels (32-bit
// index math: the host keeps the thread count below 2^31).  With `arg`, each window's first-max
// position (ky * k + kx, in NITI_CPUPoolGrad_Int8.cpp:21-77's order) goes there too: the first
// element equal to the max is the first one >= it, the backward pass's choice.
__global__ void maxpool_kernel(const int8_t* __restrict__ x, int n, int h, int w, int cp, int k, int s, int p,
                               int8_t* __restrict__ y, int oh, int ow, int8_t* __restrict__ arg) {
    const uint32_t groups = cp / 16;
    const uint32_t total = (uint32_t)n * oh * ow * groups;
    const int kh = k < h ? k : h, kw = k < w ? k : w;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        uint32_t r = t;
        const int gi = (int)(r % groups);
        r /= groups;
        const int ox = (int)(r % (uint32_t)ow);
        r /= (uint32_t)ow;
        const int oy = (int)(r % (uint32_t)oh);
        const int b = (int)(r / (uint32_t)oh);
        const int sx0 = ox * s - p, sy0 = oy * s - p;
        v16c m, a;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            m[j] = (signed char)-128;
            a[j] = (signed char)-1;
        }
        for (int yy = max(0, -sy0); yy < min(kh, h - sy0); ++yy)
            for (int xx = max(0, -sx0); xx < min(kw, w - sx0); ++xx) {
                const v16c v = *(const v16c*)(x + (((int64_t)b * h + sy0 + yy) * w + sx0 + xx) * cp + gi * 16);
                const signed char pos = (signed char)(yy * k + xx);
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const bool take = a[j] < 0 || v[j] > m[j];
                    m[j] = take ? v[j] : m[j];
                    a[j] = take ? pos : a[j];
                }
            }
        *(v16c*)(y + (int64_t)t * 16) = m;
        if (arg != nullptr) *(v16c*)(arg + (int64_t)t * 16) = a;
    }
}

hipError_t maxpool_nhwc16(const int8_t* x, int n, int h, int w, int cp, int k, int s, int p, int8_t* y, int oh, int ow,
                          hipStream_t st, int8_t* arg) {
    const int64_t total = (int64_t)n * oh * ow * (cp / 16);
    if (total >= ((int64_t)1 << 31) || cp % 16 != 0) return hipErrorInvalidValue;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(maxpool_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, h, w, cp, k, s, p, y, oh, ow, arg);
    return hipGetLastError();
}

// NITI_CPUPoolGrad_Int8.cpp:21-77 in gather form: input pixel (iy,ix) receives, from every
// window containing it, dy if it is that window's first (ky,kx) element with x >= max.
// Optionally fused NITI_CPUReluGrad_Int8 (out = x > 0 ? dx : 0).
__global__ void maxpool_grad_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ y,
                                    const int8_t* __restrict__ dy, int n, int h, int w, int cp, int k, int s,
                                    int p, int oh, int ow, int relu, int8_t* __restrict__ dx) {
    const int groups = cp / 16;
    const int64_t total = (int64_t)n * h * w * groups;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t r = t;
        const int gi = (int)(r % groups);
        r /= groups;
        const int ix = (int)(r % w);
        r /= w;
        const int iy = (int)(r % h);
        const int b = (int)(r / h);
        const v16c xv = *(const v16c*)(x + (((int64_t)b * h + iy) * w + ix) * cp + gi * 16);
        v16c acc;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = 0;
        // windows (oy, ox) with oy*s - p <= iy < oy*s - p + k
        const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(oh - 1, (iy + p) / s);
        const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(ow - 1, (ix + p) / s);
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const int sy0 = oy * s - p, sx0 = ox * s - p;
                if (iy < sy0 || iy >= sy0 + k || ix < sx0 || ix >= sx0 + k) continue;
                const int64_t po = (((int64_t)b * oh + oy) * ow + ox) * cp + gi * 16;
                const v16c mv = *(const v16c*)(y + po);
                const v16c dv = *(const v16c*)(dy + po);
                // is (iy,ix) the first element >= max in this window, per channel?
                unsigned first = 0xffffu;
                for (int ky = 0; ky < k; ++ky) {
                    const int sy = sy0 + ky;
                    if (sy < 0 || sy >= h) continue;
                    for (int kx = 0; kx < k; ++kx) {
                        const int sx = sx0 + kx;
                        if (sx < 0 || sx >= w) continue;
                        if (sy == iy && sx == ix) goto done;
                        {
                            const v16c ov = *(const v16c*)(x + (((int64_t)b * h + sy) * w + sx) * cp + gi * 16);
#pragma unroll
                            for (int j = 0; j < 16; ++j)
                                if (ov[j] >= mv[j]) first &= ~(1u << j);
                        }
                    }
                }
            done:
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (((first >> j) & 1u) && xv[j] >= mv[j]) acc[j] = (signed char)(acc[j] + dv[j]);
            }
        if (relu) {
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] = xv[j] > 0 ? acc[j] : (signed char)0;
        }
        *(v16c*)(dx + (((int64_t)b * h + iy) * w + ix) * cp + gi * 16) = acc;
    }
}

// Non-overlapping windows (k == s, no padding, windows tile the input): one thread per window
// and 16 channels scans its k*k pixels once in the reference's (ky, kx) order.
__global__ void maxpool_grad_tiled_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ y,
                                          const int8_t* __restrict__ dy, int n, int h, int w, int cp, int k,
                                          int oh, int ow, int relu, int8_t* __restrict__ dx) {
    const int groups = cp / 16;
    const int64_t total = (int64_t)n * oh * ow * groups;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t r = t;
        const int gi = (int)(r % groups);
        r /= groups;
        const int ox = (int)(r % ow);
        r /= ow;
        const int oy = (int)(r % oh);
        const int b = (int)(r / oh);
        const int64_t po = (((int64_t)b * oh + oy) * ow + ox) * cp + gi * 16;
        const v16c mv = *(const v16c*)(y + po);
        const v16c dv = *(const v16c*)(dy + po);
        unsigned done = 0;
        for (int ky = 0; ky < k; ++ky)
            for (int kx = 0; kx < k; ++kx) {
                const int64_t pi = (((int64_t)b * h + oy * k + ky) * w + ox * k + kx) * cp + gi * 16;
                const v16c xv = *(const v16c*)(x + pi);
                v16c o;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const bool take = !((done >> j) & 1u) && xv[j] >= mv[j];
                    if (take) done |= 1u << j;
                    signed char d = take ? dv[j] : (signed char)0;
                    if (relu && xv[j] <= 0) d = 0;
                    o[j] = d;
                }
                *(v16c*)(dx + pi) = o;
            }
    }
}

hipError_t maxpool_relu_grad_nhwc16(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h, int w, int cp,
                                    int k, int s, int p, int oh, int ow, int relu, int8_t* dx, hipStream_t st) {
    if (k == s && p == 0 && oh * k == h && ow * k == w) {
        const int64_t total = (int64_t)n * oh * ow * (cp / 16);
        int64_t blocks = (total + 255) / 256;
        if (blocks > 4096) blocks = 4096;
        if (blocks < 1) blocks = 1;
        hipLaunchKernelGGL(maxpool_grad_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, y, dy, n, h, w, cp,
                           k, oh, ow, relu, dx);
        return hipGetLastError();
    }
    const int64_t total = (int64_t)n * h * w * (cp / 16);
    int64_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(maxpool_grad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, y, dy, n, h, w, cp, k, s, p,
                       oh, ow, relu, dx);
    return hipGetLastError();
}

// Overlapping windows in two passes over a caller workspace (the generic kernel above re-reads up
// to 8 x vectors per window for every input pixel).  Pass 1, per window and 16 channels: the
// position (ky * k + kx, in NITI_CPUPoolGrad_Int8.cpp's order, in-image elements only) of the
// first element >= the window max y.  Pass 2, per input pixel: the sum (int8, wrapping, as the
// reference's accumulation) of dy over the windows whose first max is this pixel, then the relu
// mask.  Results equal maxpool_grad_kernel's.
__global__ void maxpool_argmax_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ y, int n, int h, int w,
                                      int cp, int k, int s, int p, int oh, int ow, int8_t* __restrict__ arg) {
    const int groups = cp / 16;
    const int64_t total = (int64_t)n * oh * ow * groups;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t r = t;
        const int gi = (int)(r % groups);
        r /= groups;
        const int ox = (int)(r % ow);
        r /= ow;
        const int oy = (int)(r % oh);
        const int b = (int)(r / oh);
        const v16c mv = *(const v16c*)(y + t * 16);
        v16c a;
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = (signed char)-1;
        uint32_t open = 0xffffu;
        const int sy0 = oy * s - p, sx0 = ox * s - p;
        for (int ky = 0; ky < k && open; ++ky) {
            const int sy = sy0 + ky;
            if (sy < 0 || sy >= h) continue;
            for (int kx = 0; kx < k && open; ++kx) {
                const int sx = sx0 + kx;
                if (sx < 0 || sx >= w) continue;
                const v16c xv = *(const v16c*)(x + (((int64_t)b * h + sy) * w + sx) * cp + gi * 16);
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (((open >> j) & 1u) && xv[j] >= mv[j]) {
                        a[j] = (signed char)(ky * k + kx);
                        open &= ~(1u << j);
                    }
            }
        }
        *(v16c*)(arg + t * 16) = a;
    }
}

__global__ void maxpool_grad_gather_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ arg,
                                           const int8_t* __restrict__ dy, int n, int h, int w, int cp, int k, int s,
                                           int p, int oh, int ow, int relu, int8_t* __restrict__ dx,
                                           const int8_t* __restrict__ pooled) {
    const bool ymask = relu && pooled != nullptr;  // the relu mask from the window's pooled value
    const uint32_t groups = cp / 16;
    const uint32_t total = (uint32_t)n * h * w * groups;  // < 2^31 (host)
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        uint32_t r = t;
        const int gi = (int)(r % groups);
        r /= groups;
        const int ix = (int)(r % (uint32_t)w);
        r /= (uint32_t)w;
        const int iy = (int)(r % (uint32_t)h);
        const int b = (int)(r / (uint32_t)h);
        v16c acc;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = 0;
        const int oy_lo = max(0, (iy + p - k + s) / s), oy_hi = min(oh - 1, (iy + p) / s);
        const int ox_lo = max(0, (ix + p - k + s) / s), ox_hi = min(ow - 1, (ix + p) / s);
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const int ky = iy - (oy * s - p), kx = ix - (ox * s - p);
                if (ky < 0 || ky >= k || kx < 0 || kx >= k) continue;
                const int64_t po = (((int64_t)b * oh + oy) * ow + ox) * cp + gi * 16;
                const v16c av = *(const v16c*)(arg + po);
                const v16c dv = *(const v16c*)(dy + po);
                v16c pv;
                if (ymask) pv = *(const v16c*)(pooled + po);
                const signed char me = (signed char)(ky * k + kx);
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (av[j] == me && (!ymask || pv[j] > 0)) acc[j] = (signed char)(acc[j] + dv[j]);
            }
        if (relu && !ymask) {
            const v16c xv = *(const v16c*)(x + (int64_t)t * 16);
#pragma unroll
            for (int j = 0; j < 16; ++j) acc[j] = xv[j] > 0 ? acc[j] : (signed char)0;
        }
        *(v16c*)(dx + (int64_t)t * 16) = acc;
    }
}

// The same gather for the 3x3 / 2 pad-1 pool with the relu mask from the pooled output (ResNet-18's
// stem): four bytes at a time per 32-bit word (first-max match, pooled > 0, wrapping int8 sum)
// instead of a byte loop -- the byte form is VALU-bound.  Pooled values are relu outputs (>= 0).
struct PoolGradGeom {
    FastDiv fg, fw, fh;  // by 16-channel groups, input width, input height
    int oh, ow;
    uint32_t total;
};
__global__ void __launch_bounds__(256) maxpool3_grad_pooled_kernel(const uint4* __restrict__ arg, const uint4* __restrict__ dy,
                                                                   const uint4* __restrict__ pooled, PoolGradGeom g,
                                                                   uint4* __restrict__ dx) {
    const uint32_t groups = g.fg.d, w = g.fw.d, h = g.fh.d;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < g.total; t += gridDim.x * 256u) {
        const uint32_t r0 = fdiv(g.fg, t), gi = t - r0 * groups;
        const uint32_t r1 = fdiv(g.fw, r0), ix = r0 - r1 * w;
        const uint32_t b = fdiv(g.fh, r1), iy = r1 - b * h;
        uint32_t acc[4] = {0, 0, 0, 0};
        // windows oy with 2 oy - 1 <= iy <= 2 oy + 1 (ky = iy + 1 - 2 oy), likewise ox
        const int oy_lo = ((int)iy) >> 1, oy_hi = min(g.oh - 1, ((int)iy + 1) >> 1);
        const int ox_lo = ((int)ix) >> 1, ox_hi = min(g.ow - 1, ((int)ix + 1) >> 1);
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const uint32_t me = (uint32_t)(((int)iy + 1 - 2 * oy) * 3 + ((int)ix + 1 - 2 * ox)) * 0x01010101u;
                const int64_t po = (((int64_t)b * g.oh + oy) * g.ow + ox) * groups + gi;
                const uint4 av = arg[po], dv = dy[po], pv = pooled[po];
                const uint32_t aw[4] = {av.x, av.y, av.z, av.w}, dw[4] = {dv.x, dv.y, dv.z, dv.w},
                               pw[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t d = aw[e] ^ me;  // 0 bytes: this pixel is the window's first max
                    const uint32_t hit = ~(((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d | 0x7f7f7f7fu);
                    const uint32_t pos = ((pw[e] & 0x7f7f7f7fu) + 0x7f7f7f7fu) & ~pw[e] & 0x80808080u;  // pooled > 0
                    const uint32_t c = dw[e] & (((hit & pos) >> 7) * 0xffu);
                    acc[e] = ((acc[e] & 0x7f7f7f7fu) + (c & 0x7f7f7f7fu)) ^ ((acc[e] ^ c) & 0x80808080u);
                }
            }
        dx[t] = uint4{acc[0], acc[1], acc[2], acc[3]};
    }
}

hipError_t maxpool_relu_grad_ws(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int h, int w, int cp, int k,
                                int s, int p, int oh, int ow, int relu, int8_t* ws, int8_t* dx, hipStream_t st) {
    if (cp % 16 != 0 || k <= 0 || k > 11 || s <= 0 || ws == nullptr) return hipErrorInvalidValue;
    const int64_t tw = (int64_t)n * oh * ow * (cp / 16), tx = (int64_t)n * h * w * (cp / 16);
    if (tx >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    auto blocks = [](int64_t t) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((t + 255) / 256, 8192)); };
    hipLaunchKernelGGL(maxpool_argmax_kernel, dim3(blocks(tw)), dim3(256), 0, st, x, y, n, h, w, cp, k, s, p, oh, ow, ws);
    hipLaunchKernelGGL(maxpool_grad_gather_kernel, dim3(blocks(tx)), dim3(256), 0, st, x, ws, dy, n, h, w, cp, k, s, p,
                       oh, ow, relu, dx, (const int8_t*)nullptr);
    return hipGetLastError();
}

// the same gradient from the first-max positions the forward maxpool_nhwc16 wrote (`arg`): one pass
hipError_t maxpool_relu_grad_arg(const int8_t* x, const int8_t* arg, const int8_t* dy, int n, int h, int w, int cp,
                                 int k, int s, int p, int oh, int ow, int relu, int8_t* dx, hipStream_t st,
                                 const int8_t* pooled) {
    if (cp % 16 != 0 || k <= 0 || k > 11 || s <= 0 || arg == nullptr) return hipErrorInvalidValue;
    if (relu && pooled == nullptr && x == nullptr) return hipErrorInvalidValue;
    const int64_t tx = (int64_t)n * h * w * (cp / 16);
    if (tx >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    if (relu && pooled != nullptr && k == 3 && s == 2 && p == 1 && oh == (h - 1) / 2 + 1 && ow == (w - 1) / 2 + 1) {
        PoolGradGeom g;
        g.fg = make_fastdiv((uint32_t)(cp / 16));
        g.fw = make_fastdiv((uint32_t)w);
        g.fh = make_fastdiv((uint32_t)h);
        g.oh = oh;
        g.ow = ow;
        g.total = (uint32_t)tx;
        const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((tx + 255) / 256, 8192));
        hipLaunchKernelGGL(maxpool3_grad_pooled_kernel, dim3(blocks), dim3(256), 0, st, (const uint4*)arg,
                           (const uint4*)dy, (const uint4*)pooled, g, (uint4*)dx);
        return hipGetLastError();
    }
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((tx + 255) / 256, 8192));
    hipLaunchKernelGGL(maxpool_grad_gather_kernel, dim3(blocks), dim3(256), 0, st, x, arg, dy, n, h, w, cp, k, s, p, oh,
                       ow, relu, dx, pooled);
    return hipGetLastError();
}

__global__ void relu_grad_kernel(const int8_t* __restrict__ x, const int8_t* __restrict__ dy, int64_t n16,
                                 int64_t n, int8_t* __restrict__ out) {
    const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (int64_t i = t0; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const v16c xv = ((const v16c*)x)[i];
        const v16c dv = ((const v16c*)dy)[i];
        v16c o;
#pragma unroll
        for (int j = 0; j < 16; ++j) o[j] = xv[j] > 0 ? dv[j] : (signed char)0;
        ((v16c*)out)[i] = o;
    }
    const int64_t e = n16 * 16 + t0;  // the last n % 16 elements
    if (e < n) out[e] = x[e] > 0 ? dy[e] : (int8_t)0;
}

hipError_t relu_grad_nhwc16(const int8_t* x, const int8_t* dy, int64_t n, int8_t* out, hipStream_t st) {
    if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)out) & 15) return hipErrorInvalidValue;  // 16-byte vectors
    const int64_t n16 = n / 16;
    int64_t blocks = (n16 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(relu_grad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, dy, n16, n, out);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) loss_grad_kernel(const int8_t* __restrict__ logits, int batch, int classes,
                                                        int ld, const int8_t* __restrict__ ascale_p,
                                                        const int32_t* __restrict__ labels, int8_t* __restrict__ out) {
    loss_rows16(logits, batch, classes, ld, ascale_p, labels, out, blockIdx.x * blockDim.x + threadIdx.x);
}
// The loss gradient and the backward pass's P16 copies of the layer inputs in one launch: the
// first lw workgroups take the loss rows, the rest the conversion jobs (independent data: the
// copies read forward activations only).  Saves a launch at the head of the backward pass.
__global__ void __launch_bounds__(256) loss_grad_p16_kernel(const int8_t* __restrict__ logits, int batch, int classes,
                                                            int ld, const int8_t* __restrict__ ascale_p,
                                                            const int32_t* __restrict__ labels,
                                                            int8_t* __restrict__ out, int lw, P16Jobs J) {
    __shared__ __attribute__((aligned(16))) int8_t tile[16 * 1024];
    if ((int)blockIdx.x < lw)
        loss_rows16(logits, batch, classes, ld, ascale_p, labels, out, blockIdx.x * blockDim.x + threadIdx.x);
    else
        p16_convert_block(J, blockIdx.x - lw, tile);
}

// Exponent of a requantised weight gradient, for the DSP op slots whose graph carries one:
// the applied PSTO shift bw - rule (0 when the gradient is all zero), as the DSP ops add their
// requantisation shift to exp_in + wscale (NITI_DSPTransposeGradientConv_Int8.cpp:438-439).
__global__ void grad_exponent_kernel(const uint32_t* __restrict__ amax, int rule, int8_t* __restrict__ out) {
    const int bw = bitwidth_of(read_max(amax));  // whole wave active
    if (threadIdx.x == 0) *out = (int8_t)(bw == 0 ? 0 : bw - rule);
}
hipError_t grad_exponent(const uint32_t* amax, int rule, int8_t* out, hipStream_t st) {
    hipLaunchKernelGGL(grad_exponent_kernel, dim3(1), dim3(64), 0, st, amax, rule, out);
    return hipGetLastError();
}

// The same arithmetic for wide class rows (ImageNet heads, up to LOSS_WIDE_MAXC classes): one
// 256-thread block per sample, the row's max / sums reduced in LDS (int64, exact).
constexpr int LOSS_WIDE_PER = 8;
constexpr int LOSS_WIDE_MAXC = 256 * LOSS_WIDE_PER;
__device__ int64_t block_reduce_i64(int64_t v, bool is_max, int64_t* red) {
    const int tid = threadIdx.x;
    red[tid] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) red[tid] = is_max ? (red[tid] > red[tid + o] ? red[tid] : red[tid + o]) : red[tid] + red[tid + o];
        __syncthreads();
    }
    const int64_t r = red[0];
    __syncthreads();
    return r;
}
__global__ void __launch_bounds__(256) loss_grad_wide_kernel(const int8_t* __restrict__ logits, int classes, int ld,
                                                             const int8_t* __restrict__ ascale_p,
                                                             const int32_t* __restrict__ labels,
                                                             int8_t* __restrict__ out) {
    __shared__ int64_t red[256];
    const int i = blockIdx.x, tid = threadIdx.x;
    const int as = (int)*ascale_p;
    const int8_t* L = logits + (int64_t)i * ld;
    int64_t o[LOSS_WIDE_PER];
    if (as > -7) {
        int64_t sv[LOSS_WIDE_PER];
        int64_t mx = INT64_MIN;
#pragma unroll
        for (int k = 0; k < LOSS_WIDE_PER; ++k) {
            const int j = tid + 256 * k;
            if (j < classes) {
                int64_t t = (int64_t)L[j] * 47274;
                t = t / (1 << 15);
                sv[k] = as >= 0 ? t * ipow2_64(as) : t / ipow2_64(-as);
                mx = mx > sv[k] ? mx : sv[k];
            }
        }
        mx = block_reduce_i64(mx, true, red) - 10;
#pragma unroll
        for (int k = 0; k < LOSS_WIDE_PER; ++k) {
            const int j = tid + 256 * k;
            int64_t t = j < classes ? sv[k] - mx : 0;
            t = t > 0 ? t : 0;
            o[k] = j < classes ? ipow2_64(t) - 1 : 0;
        }
    } else {
        const int64_t base = ipow2_64(1 - 2 * (int64_t)as);
        const int64_t sb = ipow2_64(1 - (int64_t)as);
#pragma unroll
        for (int k = 0; k < LOSS_WIDE_PER; ++k) {
            const int j = tid + 256 * k;
            const int64_t t = j < classes ? L[j] : 0;
            o[k] = j < classes ? base + t * sb + t * t : 0;
        }
    }
    int64_t part = 0;
#pragma unroll
    for (int k = 0; k < LOSS_WIDE_PER; ++k) part += o[k];
    const int64_t sum = block_reduce_i64(part, false, red);
    part = 0;
#pragma unroll
    for (int k = 0; k < LOSS_WIDE_PER; ++k) {
        const int j = tid + 256 * k;
        o[k] = j < classes ? (o[k] * (1 << 11)) / sum : 0;
        part += o[k];
    }
    const int64_t gs = block_reduce_i64(part, false, red);
    const int tgt = labels[i];
    int8_t* O = out + (int64_t)i * ld;
    for (int j = tid; j < ld; j += 256) {
        const int k = j >> 8;
        int32_t gf = 0;
#pragma unroll
        for (int q = 0; q < LOSS_WIDE_PER; ++q)
            if (q == k) gf = (int32_t)(j == tgt ? o[q] - gs : o[q]);
        O[j] = j < classes ? (int8_t)psto_any(gf, 4) : (int8_t)0;
    }
}

hipError_t p16_jobs_build(const P16Conv* jobs, int n, hipStream_t st, P16Jobs* out, uint32_t* wgs_out);

hipError_t loss_grad_p16(const int8_t* logits, int batch, int classes, int ld, const int8_t* ascale,
                         const int32_t* labels, int8_t* out, const P16Conv* jobs, int n, hipStream_t st) {
    if (classes > LOSS_MAXC || ld > LOSS_WIDE_MAXC || classes > ld) {
        hipError_t e = loss_grad(logits, batch, classes, ld, ascale, labels, out, st);
        return e != hipSuccess ? e : nhwc16_to_p16_many(jobs, n, st);
    }
    P16Jobs J;
    uint32_t wg = 0;
    hipError_t e = p16_jobs_build(jobs, n, st, &J, &wg);
    if (e != hipSuccess) return e;
    const int lw = (batch + 15) / 16;
    if (J.n == 0) wg = 0;
    hipLaunchKernelGGL(loss_grad_p16_kernel, dim3((unsigned)lw + wg), dim3(256), 0, st, logits, batch, classes, ld,
                       ascale, labels, out, lw, J);
    return hipGetLastError();
}

hipError_t loss_grad(const int8_t* logits, int batch, int classes, int ld, const int8_t* ascale, const int32_t* labels,
                     int8_t* out, hipStream_t st) {
    if (classes > ld || classes > LOSS_WIDE_MAXC || ld > LOSS_WIDE_MAXC) return hipErrorInvalidValue;
    if (classes > LOSS_MAXC) {
        hipLaunchKernelGGL(loss_grad_wide_kernel, dim3((unsigned)batch), dim3(256), 0, st, logits, classes, ld, ascale,
                           labels, out);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(loss_grad_kernel, dim3((batch + 15) / 16), dim3(256), 0, st, logits, batch, classes, ld, ascale,
                       labels, out);
    return hipGetLastError();
}

// =====================================================================================
// Layout transforms
// =====================================================================================

// NHWC16 -> CHWN16 through an LDS tile: block = (pixel, 64 images, 64 channels).
__global__ void nhwc16_to_chwn16_kernel(const int8_t* __restrict__ in, int n, int hw, int cp, int np,
                                        int8_t* __restrict__ out) {
    __shared__ int8_t tile[64][64 + 4];
    const int pix = blockIdx.x;
    const int n0 = blockIdx.y * 64, c0 = blockIdx.z * 64;
    const int t = threadIdx.x;
    {   // read: row = image, 4 x 16B chunks of channels
        const int r = t >> 2, ch = (t & 3) * 16;
        v16c v;
        if (n0 + r < n && c0 + ch < cp)
            v = *(const v16c*)(in + ((int64_t)(n0 + r) * hw + pix) * cp + c0 + ch);
        else
            for (int j = 0; j < 16; ++j) v[j] = 0;
        for (int j = 0; j < 16; ++j) tile[r][ch + j] = v[j];
    }
    __syncthreads();
    {   // write: row = channel, 4 x 16B chunks of images
        const int c = t >> 2, nb = (t & 3) * 16;
        if (c0 + c < cp && n0 + nb < np) {
            v16c v;
            for (int j = 0; j < 16; ++j) v[j] = tile[nb + j][c];
            *(v16c*)(out + ((int64_t)(c0 + c) * hw + pix) * np + n0 + nb) = v;
        }
    }
}

hipError_t nhwc16_to_chwn16(const int8_t* in, int n, int hw, int cp, int np, int8_t* out, hipStream_t st) {
    dim3 grid(hw, (np + 63) / 64, (cp + 63) / 64);
    hipLaunchKernelGGL(nhwc16_to_chwn16_kernel, grid, dim3(256), 0, st, in, n, hw, cp, np, out);
    return hipGetLastError();
}

struct OhwiToIhwo {
    const int8_t* w;
    int co, ci, kk, cip, cop;
    int8_t* wt;
    __device__ void operator()(int64_t i) const {  // i over [ci][kk][cop]
        const int o = (int)(i % cop);
        const int64_t r = i / cop;
        const int k = (int)(r % kk);
        const int c = (int)(r / kk);
        wt[i] = o < co ? w[((int64_t)o * kk + k) * cip + c] : (int8_t)0;
    }
};
hipError_t ohwi16_to_ihwo16(const int8_t* w, int co, int ci, int kk, int cip, int cop, int8_t* wt, hipStream_t st) {
    return launch_map((int64_t)ci * kk * cop, OhwiToIhwo{w, co, ci, kk, cip, cop, wt}, st);
}

struct C4ToNhwc16 {
    const int8_t* x;
    int n, c, hw, cp;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [n][hw][cp]
        const int ch = (int)(i % cp);
        const int64_t r = i / cp;
        const int64_t p = r % hw;
        const int64_t b = r / hw;
        out[i] = ch < c ? x[(((int64_t)(ch >> 2) * n + b) * hw + p) * 4 + (ch & 3)] : (int8_t)0;
    }
};
hipError_t c4_to_nhwc16(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)n * hw * cp, C4ToNhwc16{x, n, c, hw, cp, out}, st);
}

struct NchwToNhwc16 {
    const int8_t* x;
    int n, c, hw, cp;
    int8_t* out;
    __device__ void operator()(int64_t i) const {
        const int ch = (int)(i % cp);
        const int64_t r = i / cp;
        const int64_t p = r % hw;
        const int64_t b = r / hw;
        out[i] = ch < c ? x[((int64_t)b * c + ch) * hw + p] : (int8_t)0;
    }
};
hipError_t nchw_to_nhwc16(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)n * hw * cp, NchwToNhwc16{x, n, c, hw, cp, out}, st);
}

struct NchwToChwn16 {
    const int8_t* x;
    int n, c, hw, cp, np;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [cp][hw][np]
        const int b = (int)(i % np);
        const int64_t r = i / np;
        const int64_t p = r % hw;
        const int ch = (int)(r / hw);
        out[i] = (ch < c && b < n) ? x[((int64_t)b * c + ch) * hw + p] : (int8_t)0;
    }
};
hipError_t nchw_to_chwn16(const int8_t* x, int n, int c, int hw, int cp, int np, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)cp * hw * np, NchwToChwn16{x, n, c, hw, cp, np, out}, st);
}

struct C4ToChwn16 {
    const int8_t* x;
    int n, c, hw, cp, np;
    int8_t* out;
    __device__ void operator()(int64_t i) const {
        const int b = (int)(i % np);
        const int64_t r = i / np;
        const int64_t p = r % hw;
        const int ch = (int)(r / hw);
        out[i] = (ch < c && b < n) ? x[(((int64_t)(ch >> 2) * n + b) * hw + p) * 4 + (ch & 3)] : (int8_t)0;
    }
};
hipError_t c4_to_chwn16(const int8_t* x, int n, int c, int hw, int cp, int np, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)cp * hw * np, C4ToChwn16{x, n, c, hw, cp, np, out}, st);
}

struct Nhwc16ToNchw {
    const int8_t* x;
    int n, c, hw, cp;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [n][c][hw]
        const int64_t p = i % hw;
        const int64_t r = i / hw;
        const int ch = (int)(r % c);
        const int64_t b = r / c;
        out[i] = x[(b * hw + p) * cp + ch];
    }
};
hipError_t nhwc16_to_nchw(const int8_t* x, int n, int c, int hw, int cp, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)n * c * hw, Nhwc16ToNchw{x, n, c, hw, cp, out}, st);
}

struct OihwToOhwi16 {
    const int8_t* w;
    int co, ci, kk, cip, rev;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [co][kk][cip]
        const int c = (int)(i % cip);
        const int64_t r = i / cip;
        const int k = (int)(r % kk);
        const int64_t o = r / kk;
        const int ks = rev ? kk - 1 - k : k;  // rotate180 == reversing the KH*KW plane
        out[i] = c < ci ? w[(o * ci + c) * kk + ks] : (int8_t)0;
    }
};
hipError_t oihw_to_ohwi16(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, hipStream_t st,
                          bool reverse_taps) {
    return launch_map((int64_t)co * kk * cip, OihwToOhwi16{w, co, ci, kk, cip, reverse_taps ? 1 : 0, out}, st);
}

struct OihwToIhwo16 {
    const int8_t* w;
    int co, ci, kk, cop;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [ci][kk][cop]
        const int o = (int)(i % cop);
        const int64_t r = i / cop;
        const int k = (int)(r % kk);
        const int64_t c = r / kk;
        out[i] = o < co ? w[((int64_t)o * ci + c) * kk + k] : (int8_t)0;
    }
};
hipError_t oihw_to_ihwo16(const int8_t* w, int co, int ci, int kk, int cop, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)ci * kk * cop, OihwToIhwo16{w, co, ci, kk, cop, out}, st);
}

struct Ohwi16ToOihw {
    const int8_t* w;
    int co, ci, kk, cip;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over [co][ci][kk]
        const int k = (int)(i % kk);
        const int64_t r = i / kk;
        const int c = (int)(r % ci);
        const int64_t o = r / ci;
        out[i] = w[(o * kk + k) * cip + c];
    }
};
hipError_t ohwi16_to_oihw(const int8_t* w, int co, int ci, int kk, int cip, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)co * ci * kk, Ohwi16ToOihw{w, co, ci, kk, cip, out}, st);
}

struct PadRows {
    const int8_t* in;
    int rows, cols, ld;
    int8_t* out;
    __device__ void operator()(int64_t i) const {
        const int c = (int)(i % ld);
        const int64_t r = i / ld;
        out[i] = c < cols ? in[r * cols + c] : (int8_t)0;
    }
};
hipError_t pad_rows(const int8_t* in, int rows, int cols, int ld, int8_t* out, hipStream_t st) {
    return launch_map((int64_t)rows * ld, PadRows{in, rows, cols, ld, out}, st);
}

struct TransposeI32 {
    const int32_t* in;
    int rows, cols, ld;
    int32_t* out;
    __device__ void operator()(int64_t i) const {  // out [cols][rows]
        const int r = (int)(i % rows);
        const int64_t c = i / rows;
        out[i] = in[(int64_t)r * ld + c];
    }
};
hipError_t transpose_i32(const int32_t* in, int rows, int cols, int ld, int32_t* out, hipStream_t st) {
    return launch_map((int64_t)rows * cols, TransposeI32{in, rows, cols, ld, out}, st);
}

}  // namespace niti
