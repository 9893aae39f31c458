// niti_rowconv.hip -- NITI_Conv_Int8 forward (execution-engine/source/backend/cpu/NITI_Conv_Int8.cpp:
// 162-310) of stride-1, pad-1 3x3 layers as register-fed MFMAs with the per-layer rescale fused.
//
//   y[co][p] = sum over (tap, ci) of w[co][tap][ci] * x[p + tap][ci]                 (exact int32)
//
// One wave owns 32 output channels x R output rows x 32 pixel columns: the 32 columns of a
// v_mfma_i32_32x32x32_i8 B operand are G = 32 / W images side by side, one image row of W pixels
// each (W = 2, 4, 8, 16), and a wave's R rows live in R accumulator tiles.  The taps never touch
// memory twice:
//   ky  selects which of the R + 2 loaded input rows feeds an output row (registers);
//   kx  moves pixels one lane left or right inside each image row: a DPP row shift of the
//       B fragment, zero filled where the shift leaves the image row (ox = 0 or W - 1).
// So a 32-channel chunk of input is loaded once per wave (R + 2 rows, 16 bytes per lane each) and
// feeds 9 R MFMAs; the weights come as 9 fragments per chunk from a fragment-major copy in which
// each 32 x 32 fragment is 1 KiB contiguous (a wave load = 8 whole cache lines).
//
// Layouts (rowconv.hpp terms):
//   C32 activations  [n][C/32][H][W][32]      a fragment row = W x 32 contiguous bytes per image
//   WF weights       [Co/32][Ci/32][9][2][32][16]  fragment (co block, ci block, tap) = 1 KiB
//
// The NITI rule needs max|y| over the whole tensor (NITI_RangeEstimate, NITI_Conv_Int8.cpp:260)
// before any output can be requantised (:266-307).  Mode FUSED keeps every wave's accumulators
// in registers across an in-kernel grid barrier that also reduces the max (one unit per wave,
// every workgroup resident); RANGE publishes the max and exits and REQUANT recomputes the GEMM
// and requantises with a given max (data parallel: the MAX all-reduce sits between the two).
// The epilogue requantises (PSTO, the shift==1 and raw-cast branches), applies relu, and writes
// the NHWC16 output, the fused 2x2 max pool and the next layer's C32 input.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "niti_device.hpp"
#include "niti_gridbar.hpp"
#include "niti_kernels.hpp"
#include "niti_map.hpp"

#ifndef RC_EXP
#define RC_EXP 0
#endif
namespace niti {

__device__ __forceinline__ int bitwidth_rc(uint32_t m) { return m <= 1u ? 0 : 32 - __clz((int)(m - 1u)); }

// NITI_MNNPstoShiftInt32 (CommonOptFunction.cpp:1595-1627) for 2 <= s <= 30, clipped to +-127
__device__ __forceinline__ int32_t psto_rc(int32_t a, int s) {
    const uint32_t ua = a < 0 ? 0u - (uint32_t)a : (uint32_t)a;
    const uint32_t q = ua >> s;
    const uint32_t prob = ua & ((1u << s) - 1u);
    const int h = s >> 1;
    const uint32_t qp = prob >> h;
    uint32_t pr = prob & ((1u << h) - 1u);
    if (s & 1) pr <<= 1;
    int32_t r = (int32_t)q + (qp > pr ? 1 : 0);
    r = r > 127 ? 127 : r;
    return a < 0 ? -r : r;
}

// lane i <- lane i - 1 inside each image row of W pixels (zero at ox = 0): the kx = 0 tap
template <int W>
__device__ __forceinline__ v4i shift_in_left(v4i v, bool row_start) {
    v4i r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // row_shr:1 with bound_ctrl: lane 0 of each 16-lane DPP row reads zero
        int t = __builtin_amdgcn_update_dpp(0, v[k], 0x111, 0xF, 0xF, true);
        if constexpr (W < 16) t = row_start ? 0 : t;
        r[k] = t;
    }
    return r;
}
// lane i <- lane i + 1 inside each image row (zero at ox = W - 1): the kx = 2 tap
template <int W>
__device__ __forceinline__ v4i shift_in_right(v4i v, bool row_end) {
    v4i r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int t = __builtin_amdgcn_update_dpp(0, v[k], 0x101, 0xF, 0xF, true);  // row_shl:1
        if constexpr (W < 16) t = row_end ? 0 : t;
        r[k] = t;
    }
    return r;
}

// Speculative epilogue: the bit width a layer's output had at this state's previous fused launch
// (forward and input-gradient launches keep separate slots: lines 16 / 17 of the parity-0 word
// set, which the shard resets never touch), stored as bw + 1 (0: none yet).  A launch requantises
// with it while its grid barrier completes and redoes the epilogue only if the barrier's bw
// differs: per layer the bit width is stable from step to step, so the barrier's release latency
// overlaps the epilogue instead of preceding it.  The results are the rule's whatever the guess.


struct RowConvArgs {
    const int8_t* x;  // C32 [n][CB][H][W][32]
    const int8_t* wf; // WF [COB][CB][9][2][32][16]
    uint32_t xbytes, wbytes;
    int n, CB, COB;
    int ngb, ngb4;    // (image group, band) pairs; rounded up to whole workgroups of 4
    int nbands;
    int wgs;          // workgroup tiles: COB * ngb4 / 4
    int wmajor;       // 1: consecutive tiles (one co block) on one XCD (xcd_remap), so a co block's
                      // weight panel is fetched into one L2; 0: dispatch order, which deals every
                      // co block's image groups over the 8 XCDs alike, so each XCD reads 1/8 of x
    int8_t* out;      // NHWC16 [n][H][W][cop]
    int cop;
    int8_t* pool_out; // NHWC16 [n][H/2][W/2][cop] or null
    int8_t* next;     // C32 [n][COB][Ho][Wo][32] of the (pooled) output, or null
    const int8_t* exp_in;
    const int8_t* wscale;
    int8_t* exp_out;
    int relu;
    int hint_scale;   // the pair's hint on the input's scale (forward slot) or bare (input gradient)
    uint32_t* amax;   // RANGE: published; REQUANT: read
    uint32_t* bar;    // FUSED: barrier state
    uint32_t epoch;
    uint32_t* err;
    uint32_t spin_limit;         // FUSED: polls before the barrier gives up and sets *err
    uint32_t expect_extra;       // diagnostics (niti_diag_rowconv_barrier): arrivals that never come
    int spec;                    // FUSED: 1 speculative epilogue (hint slot), 0 off, 2 diagnostics:
                                 // guess one bit wide of the hint (every launch redoes its epilogue)
    unsigned long long* stamps;  // diagnostics (niti_diag_rowconv_stamps): 8 per wave, or null
    const int8_t* relu_mask;     // input gradient: RowConvOut's relu / pool gradients
    const int8_t* pool_x;
    const int8_t* pool_y;
    int8_t* pool_dx;
    int8_t* pool_dx_next;
    int pool_relu;
    const int8_t* pool_code;     // the recorded route (pool_code4) instead of pool_x / pool_y, or null
    int8_t* pool_code_out;       // forward with pool_out: the route recorded, or null
    int pool_dx_nhwc;            // 0: the NHWC16 pool_dx is not written (its consumers read the C32 / P16 copies)
    int8_t* p16;                 // P16 [pixels/16][cop][16] copy of out / pool_dx, or null
    int64_t p16_pixels;          // pixels of that tensor
    int32_t* acc_store;          // RANGE writes / REQUANT reads every unit's accumulators, or null
    // REQUANT as a speculative pair (spec_hint, below): 1 = launch A, requantise with the hinted bit
    // width and publish the max; 2 = launch B, redo only if the (all-reduced) max's bit width differs
    int spec2;
    uint32_t spec_cooldown;      // spec2: pairs in store mode after a change (spec_cooldown())
    uint32_t* hint;              // spec2: the slot (spec_hint); its word 0 the hint, 1 the guess A used, 2 misses
    // W = 1 (1x1 maps, the classifier head): x is row-major [n][xld], the weights row-major
    // [rows][wld] (OHWI16 forward, IHWO16 input gradient), K the reduced channels
    int xld, wld, K, rows;
    // W = 0, the row-segment form (maps of 224 / 112 / 56 / 28 / 14 / 7 px): hw the map's side,
    // gw images per unit (1: two 14-px segments of one row, 2: one 14-px row of two images, 4: two
    // 7-px rows of two images per 16 lanes), nsp segment pairs per row, upc4 units per co block
    // rounded up to whole workgroups of 4
    int hw, gw, nsp, upc4;
    // the row-segment form's input layout as byte strides: pixel, image row, image, 32-channel
    // chunk -- C32 (32, W*32, CB*H*W*32, H*W*32) or NHWC16 with cip % 32 == 0 (cip, W*cip,
    // H*W*cip, 32: a lane's 16 bytes are still one pixel's 16 channels, so no C32 copy is needed)
    uint32_t xps, xrs, xis, xcs;
};

// diagnostic stamps, 16 per wave: [0] start, [1] prologue issued, [2] cycles issuing loads, [3] K
// loop done, [4] max reduced (+ grid barrier), [5] end, [6] cycles in the per-step waits +
// barriers, [7] cycles in the per-step fragment reads (s_memtime, per-XCD clock); wave 0 of each
// workgroup: [8] / [9] s_memrealtime (chip-wide 100 MHz) at the grid barrier's arrival / release
#define RC_STAMP(k)                                                                                  \
    do {                                                                                             \
        if (a.stamps != nullptr && lane == 0)                                                        \
            a.stamps[(blockIdx.x * 4 + wid) * 16 + (k)] = __builtin_amdgcn_s_memtime();              \
    } while (0)

enum RowMode { RC_FUSED = 0, RC_RANGE = 1, RC_REQUANT = 2 };
// host modes RC_SPEC_A / RC_SPEC_B of rowconv_fwd / rowconv_fc (niti_kernels.hpp): the speculative
// two-launch pair (spec_guess), both on the RC_REQUANT instantiation

// A workgroup tile is one co block x 4 consecutive (image group, band) pairs, one per wave: the
// four waves share the co block's weight fragments, which the workgroup stages through LDS once
// per 32-channel chunk (a 9 KiB contiguous run of WF) instead of each wave loading them.
template <int W, int R>
struct RowUnit {
    static constexpr int G = W > 0 ? 32 / W : 1, H = W, NR = R + 2;
    int cob, b, img;
    bool valid, img_ok;
    // the row-segment form (W = 0): the lane's input column x (-1 / hw: a zero halo), whether x is
    // in the map, and whether the lane's MFMA column is an output pixel (not a halo lane)
    int x = 0;
    bool x_ok = true, out_ok = true;
    // ks: the K-split form -- one unit per workgroup, its four waves splitting the channel chunks
    __device__ RowUnit(const RowConvArgs& a, int wg, int wid, int c, bool ks = false) {
        if constexpr (W == 0) {
            // units of a co block: ((image group, band), segment pair), whole workgroups of four; the
            // co block varies fastest, so the co blocks of one pixel tile run side by side and its
            // input rows (tens to hundreds of MB per layer) come from HBM once, not once per co block
            cob = wg % a.COB;
            const int u = (wg / a.COB) * 4 + wid;
            const int nu = a.ngb * a.nsp;  // ngb = image groups x bands
            valid = u < nu;
            const int uc = valid ? u : 0;
            const int sp = uc % a.nsp, gb = uc / a.nsp;
            b = gb % a.nbands;
            const int ig = gb / a.nbands;
            const int sgi = c >> 4, q = c & 15;
            if (a.gw == 1) {  // two 14-px segments of one row: lanes 0 / 15 (16 / 31) are halos
                img = ig;
                x = 28 * sp + 14 * sgi + q - 1;
                out_ok = q >= 1 && q <= 14;
            } else if (a.gw == 2) {  // one 14-px row per 16 lanes, two images
                img = 2 * ig + sgi;
                x = q - 1;
                out_ok = q >= 1 && q <= 14;
            } else {  // two 7-px rows per 16 lanes (lanes 0 and 8 zero halos), four images
                img = 4 * ig + 2 * sgi + (q >> 3);
                x = (q & 7) - 1;
                out_ok = (q & 7) >= 1;
            }
            x_ok = x >= 0 && x < a.hw;
            img_ok = valid && img < a.n;
            out_ok = out_ok && img_ok;
            return;
        }
        const int per = ks ? a.ngb : a.ngb4 / 4;
        cob = wg / per;
        const int gb = ks ? wg - cob * per : (wg - cob * per) * 4 + wid;
        valid = gb < a.ngb;
        const int gbc = valid ? gb : 0;
        b = gbc % a.nbands;
        img = (gbc / a.nbands) * G + c / W;
        img_ok = valid && img < a.n;
    }
};

constexpr int RC_MAX_STAGES = 4;
constexpr int RC_PIECES = 12;               // 9 KiB of fragments as 3 x 1 KiB DMA per wave (3 dummies)
constexpr int RC_STAGE_BYTES = RC_PIECES * 1024;
constexpr int RC_LDS_BYTES = RC_MAX_STAGES * RC_STAGE_BYTES;
// after the K loop the ring holds each wave's output tile for the P16 transpose: 32 channels x
// (the wave's pixels: 32 R, or 128 R at the pool's input resolution) -- 16 KiB per wave at R = 4
constexpr int RC_P16_WAVE_BYTES = 16 * 1024;
constexpr int RC_SMEM_BYTES = RC_LDS_BYTES > 4 * RC_P16_WAVE_BYTES ? RC_LDS_BYTES : 4 * RC_P16_WAVE_BYTES;
// K-split form: every wave stages its own chunks' 9 fragments, all of them up front (NS <= 4)
constexpr int RC_KS_MAX_NS = 4;
constexpr int RC_KS_BYTES = 4 * RC_KS_MAX_NS * 9 * 1024;
static_assert(RC_KS_BYTES >= 4 * RC_P16_WAVE_BYTES, "the P16 tile fits the K-split ring");

// the accumulators of one unit: acc[r][i] = y[co = cob*32 + 8(i>>2) + 4h + (i&3)][row b*R + r][col]
// Every wave of the workgroup runs this (an invalid unit reads zeros), so the barriers match.
//
// The kx taps are three loads of each input row at the lane's column ox - 1, ox, ox + 1 (a lane
// whose neighbour column leaves the image row reads zeros through the buffer range check): no
// cross-lane moves, no masks, no VALU in the loop.  S chunks are in flight: chunk c computes from
// registers while c + 1 .. c + S - 1 load (rows into registers, the 9 weight fragments by LDS-DMA
// into a ring shared by the workgroup's four waves).
// UNC (chunk count a multiple of the ring depth): every step waits, issues and reads
// unconditionally -- the last steps load chunks past the end (never consumed) -- so the loop body
// is straight-line code.  With the issue under a branch, hipcc's waitcnt pass takes the path that
// skipped it and waits for vmcnt(3) before the first tap shift: the whole ring, the chunk just
// issued included, drained every step.
template <int W, int R, bool UNC>
__device__ __forceinline__ void rowconv_compute(const RowConvArgs& a, const RowUnit<W, R>& U, int lane, int wid,
                                                int8_t* smem, v16i (&acc)[R]) {
    // W = 0: the row-segment form, its side a.hw at run time; halo lanes supply the kx neighbours,
    // so the DPP shifts need no row-end masks (as W = 16)
    constexpr int NR = R + 2, WS = W == 0 ? 16 : W;
    const int H = W == 0 ? a.hw : W, WR = W == 0 ? a.hw : W;
    // kx shifts: DPP row shifts of the centre column (zero fill at the 16-lane DPP row ends, a
    // mask where a narrower image row ends inside a DPP row) -- one load per row: each 16-byte
    // wave load costs the CU's texture addresser ~16 cycles, and three loads per row (the
    // shifted columns from memory) made the K loop address-bound (stamps: 8.5k of 23k cycles
    // issuing loads on conv4)
    constexpr bool DPPX = true;
    constexpr int KXL = DPPX ? 1 : 3;        // loads per row and chunk
    constexpr int S = 4;                     // ring stages: chunk c computes, c + 1 .. c + 3 in flight
    constexpr int L = KXL * NR + 3;          // vector-memory instructions per wave per chunk
    const int h = lane >> 5, c = lane & 31, ox = W == 0 ? U.x : c % WS;
    const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.x, a.xbytes);
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.wf, a.wbytes);
    const uint32_t xl = !(U.img_ok && U.x_ok) ? OOB
                        : W == 0 ? (uint32_t)U.img * a.xis + (uint32_t)ox * a.xps + 16u * h
                                 : (uint32_t)((((int64_t)U.img * a.CB * H) * WR + ox) * 32 + 16 * h);
    const uint32_t CHUNK = W == 0 ? a.xcs : (uint32_t)H * WR * 32;
    const uint32_t XROW = W == 0 ? a.xrs : (uint32_t)WR * 32;
    const int y0 = U.b * R - 1;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[r][i] = 0;
    // per row and kx: the lane's byte offset in chunk 0, OOB outside the image (rows) or the row (kx)
    uint32_t off[3][NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        const int iy = y0 + j;
        const bool row_ok = iy >= 0 && iy < H && xl != OOB;
        const uint32_t base = xl + (uint32_t)iy * XROW;
        off[0][j] = row_ok && ox > 0 ? base - 32u : OOB;  // (unused: DPPX)
        off[1][j] = row_ok ? base : OOB;
        off[2][j] = row_ok && ox < WR - 1 ? base + 32u : OOB;
    }
    // this wave's three DMA pieces of a chunk's 9 fragments (pieces 9..11 are dummies: OOB source)
    const uint32_t dv2 = wid == 0 ? (uint32_t)lane * 16u : OOB;
    const int cb = a.CB;
    const uint32_t wbase = (uint32_t)(U.cob * cb * 9) * 1024u;
    v4i X[S][KXL][NR];
    auto issue = [&](auto st_c, int cc) {
        constexpr int ST = decltype(st_c)::value;
        int8_t* lds = smem + ST * RC_STAGE_BYTES;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int piece = wid + 4 * k;  // 0..11
            dma16(rW, lds + piece * 1024, k < 2 ? (uint32_t)lane * 16u : dv2,
                  wbase + (uint32_t)cc * 9216u + (uint32_t)(piece < 9 ? piece : 0) * 1024u);
        }
#pragma unroll
        for (int j = 0; j < NR; ++j)
#pragma unroll
            for (int kx = 0; kx < KXL; ++kx)
                X[ST][kx][j] = buf_load16(rX, off[DPPX ? 1 : kx][j] + (uint32_t)cc * CHUNK);
    };
    const uint32_t lds_lane = lds_addr(smem) + (uint32_t)lane * 16u;
    unsigned long long t_wait = 0, t_read = 0, t_issue = 0;
    const bool stamp = a.stamps != nullptr;
    // Software pipeline, per step c: wait for chunk c + 1's own loads (c + 2 stays in flight) and
    // meet at the barrier (chunk c + 1's weights are in LDS, chunk c - 1's stage is free), refill
    // that stage with chunk c + 3, read chunk c + 1's weight fragments (landing while chunk c's MFMAs
    // run), shift chunk c's rows and run its 9 R MFMAs.
    v4i wreg[2][9];
    auto read_w = [&](auto st_c, v4i (&w)[9]) {
        constexpr int ST = decltype(st_c)::value;
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t] = lds_b128(lds_lane + (uint32_t)(ST * RC_STAGE_BYTES + t * 1024));
    };
    auto fence_w = [&](v4i (&w)[9]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int t = 0; t < 9; ++t) reg_fence(w[t]);
    };
    auto arrive = [&](int later) {
        if (later >= 1)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto step = [&](auto st_c, int cc) {
        constexpr int ST = decltype(st_c)::value, WB = ST & 1;
        const unsigned long long s0 = stamp ? __builtin_amdgcn_s_memtime() : 0ull;
        const bool more = UNC || cc + 1 < cb;
        if (more && !(RC_EXP & 2)) arrive(UNC || cc + 2 < cb ? 1 : 0);
        const unsigned long long s1 = stamp ? __builtin_amdgcn_s_memtime() : 0ull;
        if ((UNC || cc + 3 < cb) && !(RC_EXP & 8)) issue(std::integral_constant<int, (ST + 3) % S>(), cc + 3);
        if (stamp) {
            asm volatile("" ::: "memory");
            t_issue += __builtin_amdgcn_s_memtime() - s1;
        }
        if (more && !(RC_EXP & 4)) read_w(std::integral_constant<int, (ST + 1) % S>(), wreg[1 - WB]);
        const v4i (&w)[9] = wreg[(RC_EXP & 4) ? 0 : WB];
        if constexpr (DPPX) {
            v4i XL[NR], XR[NR];
#pragma unroll
            for (int j = 0; j < NR; ++j) {
                XL[j] = (RC_EXP & 1) ? X[ST][0][j] : shift_in_left<WS>(X[ST][0][j], ox == 0);
                XR[j] = (RC_EXP & 1) ? X[ST][0][j] : shift_in_right<WS>(X[ST][0][j], ox == WS - 1);
            }
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int ky = 0; ky < 3; ++ky) {
                    acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky], XL[r + ky], acc[r], 0, 0, 0);
                    acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky + 1], X[ST][0][r + ky], acc[r], 0, 0, 0);
                    acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky + 2], XR[r + ky], acc[r], 0, 0, 0);
                }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx)
                        acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky + kx], X[ST][kx][r + ky], acc[r], 0, 0, 0);
        }
        const unsigned long long s2 = stamp ? __builtin_amdgcn_s_memtime() : 0ull;
        if (more) fence_w(wreg[1 - WB]);
        if (stamp) {
            t_wait += s1 - s0;
            t_read += __builtin_amdgcn_s_memtime() - s2;
        }
    };
#pragma unroll
    for (int k = 0; k < S - 1; ++k)
        if (k < cb) {
            if (k == 0) issue(std::integral_constant<int, 0>(), 0);
            if (k == 1) issue(std::integral_constant<int, 1>(), 1);
            if (k == 2) issue(std::integral_constant<int, 2>(), 2);
        }
    arrive(cb > 1 ? 1 : 0);  // chunk 0 (chunk 1 / 2 may stay in flight: the wait keeps L per later chunk)
    read_w(std::integral_constant<int, 0>(), wreg[0]);
    fence_w(wreg[0]);
    if (stamp && lane == 0) a.stamps[(blockIdx.x * 4 + wid) * 16 + 1] = __builtin_amdgcn_s_memtime();
    if constexpr (UNC) {
        for (int cc = 0; cc < cb; cc += S) {
            step(std::integral_constant<int, 0>(), cc);
            step(std::integral_constant<int, 1>(), cc + 1);
            step(std::integral_constant<int, 2>(), cc + 2);
            step(std::integral_constant<int, 3>(), cc + 3);
        }
        // the past-the-end chunks' loads (LDS-DMA into the ring the epilogue reuses) land first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int cc = 0; cc < cb; cc += S) {
            step(std::integral_constant<int, 0>(), cc);
            if (cc + 1 < cb) step(std::integral_constant<int, 1>(), cc + 1);
            if (cc + 2 < cb) step(std::integral_constant<int, 2>(), cc + 2);
            if (cc + 3 < cb) step(std::integral_constant<int, 3>(), cc + 3);
        }
    }
    // the ring's LDS is reused by the next unit's prologue only after every wave's last reads
    __builtin_amdgcn_s_barrier();
    if (stamp && lane == 0) {
        unsigned long long* st = a.stamps + (blockIdx.x * 4 + wid) * 16;
        st[3] = __builtin_amdgcn_s_memtime();
        st[2] = t_issue;
        st[6] = t_wait;
        st[7] = t_read;
    }
}

// K-split form for whole-image units (R == H: W = 2) on layers with too few units to fill the chip
// (VGG-11's 2x2 layers: 256 units of 32 channels x 16 images, i.e. 64 workgroups of four): the
// workgroup owns ONE unit and wave w takes the channel chunks w, w + 4, ..., NS = CB / 4 of them,
// each wave staging its own chunks' weight fragments in its own LDS region (no barrier in the
// loop).  Every load is issued up front (NS <= 4) in straight-line code, so hipcc's counted
// waits are exact.  Rows 0 and R + 1 of the loaded band lie outside the image (y0 = -1, R == H):
// they are neither loaded nor multiplied -- 6 of the 9 (ky, row) products of a 2-row unit remain.
// The four partial tiles are summed through LDS into wave 0 (ks_reduce).
template <int W, int R, int NS>
__device__ __forceinline__ void rowconv_compute_ks(const RowConvArgs& a, const RowUnit<W, R>& U, int lane, int wid,
                                                   int8_t* smem, v16i (&acc)[R]) {
    static_assert(R == W && NS >= 1 && NS <= RC_KS_MAX_NS, "whole-image units, all chunks staged at once");
    constexpr int H = W;
    const int h = lane >> 5, c = lane & 31, ox = c % W;
    const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.x, a.xbytes);
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.wf, a.wbytes);
    const uint32_t xl = U.img_ok ? (uint32_t)((((int64_t)U.img * a.CB * H) * W + ox) * 32 + 16 * h) : OOB;
    constexpr uint32_t CHUNK = (uint32_t)H * W * 32;
    const uint32_t wbase = (uint32_t)(U.cob * a.CB * 9) * 1024u;
    int8_t* ring = smem + wid * (RC_KS_MAX_NS * 9 * 1024);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[r][i] = 0;
    v4i X[NS][R];  // the image's R rows of each of the wave's chunks
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const uint32_t cc = (uint32_t)(wid + 4 * k);
        // the counted waits below assume this issue order; the memory clobbers keep hipcc from
        // hoisting a later chunk's row loads above an earlier chunk's DMA
#pragma unroll
        for (int t = 0; t < 9; ++t)
            dma16(rW, ring + (k * 9 + t) * 1024, (uint32_t)lane * 16u, wbase + cc * 9216u + (uint32_t)t * 1024u);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int r = 0; r < R; ++r)
            X[k][r] = buf_load16(rX, xl == OOB ? OOB : xl + (uint32_t)r * W * 32 + cc * CHUNK);
        asm volatile("" ::: "memory");
    }
    const uint32_t lds_lane = lds_addr(ring) + (uint32_t)lane * 16u;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        // chunk k's DMA and rows are in once the later chunks' 9 + R loads are the only ones left
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1 - k) * (9 + R)) : "memory");
        v4i w[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t] = lds_b128(lds_lane + (uint32_t)((k * 9 + t) * 1024));
        v4i XL[R], XR[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            reg_fence(X[k][r]);
            XL[r] = shift_in_left<W>(X[k][r], ox == 0);
            XR[r] = shift_in_right<W>(X[k][r], ox == W - 1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int t = 0; t < 9; ++t) reg_fence(w[t]);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const int j = r + ky - 1;  // the image row this tap reads
                if (j < 0 || j >= R) continue;
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky], XL[j], acc[r], 0, 0, 0);
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky + 1], X[k][j], acc[r], 0, 0, 0);
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky + 2], XR[j], acc[r], 0, 0, 0);
            }
    }
}

// the four waves' partial tiles -> wave 0's acc (the other waves' acc stay partial); the ring is
// free again afterwards (three barriers)
template <int R>
__device__ __forceinline__ void ks_reduce(v16i (&acc)[R], int8_t* smem, int wid, int lane) {
    static_assert(3 * R * 16 * 64 * 4 <= RC_KS_BYTES, "partials fit the ring");
    int32_t* part = (int32_t*)smem;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (wid != 0) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) part[(((wid - 1) * R + r) * 16 + i) * 64 + lane] = acc[r][i];
    }
    __syncthreads();
    if (wid == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i)
                acc[r][i] += part[((0 * R + r) * 16 + i) * 64 + lane] + part[((1 * R + r) * 16 + i) * 64 + lane] +
                             part[((2 * R + r) * 16 + i) * 64 + lane];
    }
    __syncthreads();
}

// W = 1: a 1x1 map per image, 32 images per wave (the MFMA B columns), out channels cob*32 + 0..31
// as the A rows; K in 32-channel chunks straight from the row-major tensors (zero past K / rows / n)
template <int R>
__device__ __forceinline__ void fc_compute(const RowConvArgs& a, const RowUnit<1, R>& U, int lane, v16i (&acc)[R]) {
    static_assert(R == 1, "one row");
    const int h = lane >> 5, c = lane & 31;
    const int row = U.cob * 32 + c;
    const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.x, a.xbytes);
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.wf, a.wbytes);
    const uint32_t xo = U.img_ok ? (uint32_t)U.img * (uint32_t)a.xld : OOB;
    const uint32_t wo = row < a.rows ? (uint32_t)row * (uint32_t)a.wld : OOB;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[0][i] = 0;
    for (int k0 = 0; k0 < a.K; k0 += 32) {
        const int k = k0 + 16 * h;
        const bool kin = k < a.K;
        const v4i wv = buf_load16(rW, kin && wo != OOB ? wo + (uint32_t)k : OOB);
        const v4i xv = buf_load16(rX, kin && xo != OOB ? xo + (uint32_t)k : OOB);
        acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(wv, xv, acc[0], 0, 0, 0);
    }
}

__device__ __forceinline__ uint32_t pack4(const int8_t* v) {
    return (uint32_t)(uint8_t)v[0] | (uint32_t)(uint8_t)v[1] << 8 | (uint32_t)(uint8_t)v[2] << 16 |
           (uint32_t)(uint8_t)v[3] << 24;
}
// lane (col, half h) holds co 8j + 4h + 0..3 as byte quads q[4j..4j+3]; after the half-wave swaps
// the lower half-wave holds co 0..15 and the upper half co 16..31 of its column
__device__ __forceinline__ v4i pack_cols(const int8_t* q) {
    uint32_t d[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = pack4(q + 4 * j);
    const auto x02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
    const auto x13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
    return v4i{(int)x02[0], (int)x02[1], (int)x13[0], (int)x13[1]};
}

// The input-gradient epilogue's operands (the relu mask, or the pool's input window and output),
// loaded before the grid barrier and turned into byte masks while the barrier completes: the
// epilogue then only ANDs the requantised gradient with them
// PX false: no pool window (an input-gradient launch without a pool gradient -- 8 R fewer VGPRs)
template <int R, bool PX = true>
struct EpiIn {
    v4i x[PX ? R : 1][4];  // pool: the 2x2 window of pool_x per row, then its routing masks
    v4i y[R];     // pool: pool_y; relu: relu_mask, then its byte mask (one member for the tensors
                  // at the output's own pixels: hipcc merges the two branches' loads into one)
};

// (SWAR byte helpers sw_ge_hi / sw_pos_hi / sw_expand and the 2x2 pool codes: niti_device.hpp)

template <int R, bool PX = true>
__device__ __forceinline__ void epi_masks(const RowConvArgs& a, EpiIn<R, PX>& e) {
    if (PX && a.pool_dx != nullptr && a.pool_code != nullptr) {
        // the route the forward pass recorded: e.y holds the code bytes
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int t = 0; t < 4; ++t) e.x[PX ? r : 0][t][k] = (int)pool_code_mask((uint32_t)e.y[r][k], t);
    } else if (PX && a.pool_dx != nullptr) {
        // NITI_CPUPoolGrad_Int8's scan: the first window element >= the pool output takes it
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t m = (uint32_t)e.y[r][k];
                uint32_t done = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t x = (uint32_t)e.x[PX ? r : 0][t][k];
                    uint32_t take = sw_ge_hi(x, m) & ~done;
                    done |= take;
                    if (a.pool_relu) take &= sw_pos_hi(x);
                    e.x[PX ? r : 0][t][k] = (int)sw_expand(take);
                }
            }
    } else if (a.relu_mask != nullptr) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k) e.y[r][k] = (int)sw_expand(sw_pos_hi((uint32_t)e.y[r][k]));
    }
}

template <int W, int R>
__device__ __forceinline__ void epi_prefetch(const RowConvArgs& a, const RowUnit<W, R>& U, int lane, EpiIn<R>& e) {
    constexpr int H = W;
    const int h = lane >> 5, ox = (lane & 31) % W;
    const int64_t img = U.img_ok ? U.img : 0;
    const int cb16 = U.cob * 32 + 16 * h;
    // the offsets pass through an empty asm: the loads cannot be hoisted into the K loop, where
    // their registers would sit beside the operand ring
    uint32_t z = 0;
    asm volatile("" : "+s"(z));
    // the tensor at the output's own pixels (pool_y or relu_mask) in one branch-free load per row
    // (two branches writing e.y were merged by hipcc through a scratch array)
    const bool pool = a.pool_dx != nullptr;
    const bool code = pool && a.pool_code != nullptr;  // the recorded route: one load per row
    const int8_t* ps = (pool ? (code ? a.pool_code : a.pool_y) : a.relu_mask) + z;
    const int8_t* px = a.pool_x + z;
    if (!pool && a.relu_mask == nullptr) return;
#pragma unroll
    for (int r = 0; r < R; ++r)
        e.y[r] = *(const v4i*)(ps + ((img * H + U.b * R + r) * W + ox) * a.cop + cb16);
    if (pool && !code) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                e.x[r][t] = *(const v4i*)(px + ((img * 2 * H + 2 * (U.b * R + r) + (t >> 1)) * 2 * W + 2 * ox + (t & 1)) *
                                                   a.cop + cb16);
    }
}

// The wave's output tile, staged in LDS as rows of 32 channel bytes in pixel order (row =
// (image, row, column) of the wave's pixels), leaves in the weight gradient's P16 layout: per 16-lane
// group, two ds_read_b64_tr_b8 give lane j the 16 pixels of channel j (8 rows each), one 16-byte
// store.  A round covers two 16-pixel blocks x 32 channels (the four groups).  ROWS: the wave's
// band rows at the tile's resolution (R, or 2R through the pool), WD its image width.
template <int ROWS, int WD, int G>
__device__ __forceinline__ void p16_store(const RowConvArgs& a, int lane, const int8_t* tile, int img0, int y0, int hd,
                                          int cob) {
    constexpr int PPI = ROWS * WD;  // the tile's pixels per image (G images)
    constexpr int NROWS = G * PPI;
    static_assert(NROWS % 32 == 0 && NROWS * 32 <= RC_P16_WAVE_BYTES, "whole rounds in the wave's slot");
    const int gi = lane >> 4, j = lane & 15, chalf = gi & 1;
#pragma unroll
    for (int q = 0; q < NROWS / 32; ++q) {
        const int r0 = 16 * (2 * q + (gi >> 1));
        const int8_t* t = tile + (r0 + (j >> 1)) * 32 + 16 * chalf + 8 * (j & 1);
        const v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(t));
        const v2i hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(t + 8 * 32));
        const int g = r0 / PPI, rem = r0 % PPI;
        const int64_t P = ((int64_t)(img0 + g) * hd + y0 + rem / WD) * WD + rem % WD;
        if (P < a.p16_pixels)
            *(v4i*)(a.p16 + ((P >> 4) * a.cop + cob * 32 + 16 * chalf + j) * 16) = v4i{lo[0], lo[1], hi[0], hi[1]};
    }
}

template <int W, int R, bool DG>
__device__ __forceinline__ void rowconv_epilogue(const RowConvArgs& a, const RowUnit<W, R>& U, int lane,
                                                 const v16i (&acc)[R], uint32_t gmax, const EpiIn<DG ? R : 1>& e,
                                                 int8_t* tile) {
    constexpr int H = W;
    const int h = lane >> 5, c = lane & 31, ox = c % W;
    // NITI_Conv_Int8.cpp:266-307 with wave-uniform branches: shift <= 0 the raw int8 cast, else
    // PSTO(acc, max(shift, 2)); under relu a negative value is 0 whatever its rounding, so the
    // positive-only PSTO serves (ReLU after requantisation, NITI_Relu_Int8)
    const int shift = __builtin_amdgcn_readfirstlane(bitwidth_rc(gmax) - 7);
    int8_t q[R][16];
    if (shift <= 0) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int32_t v = (int32_t)(int8_t)acc[r][i];
                q[r][i] = (int8_t)(a.relu && v < 0 ? 0 : v);
            }
    } else {
        const uint32_t s = shift > 1 ? shift : 2, hh = s >> 1, odd = s & 1;
        auto pos = [&](uint32_t u) -> uint32_t {  // PSTO of u >= 0
            const uint32_t qv = u >> s;
            const uint32_t hi = __builtin_amdgcn_ubfe(u, hh, s - hh);
            const uint32_t lo = __builtin_amdgcn_ubfe(u, 0, hh) << odd;
            const uint32_t rr = qv + (hi > lo ? 1u : 0u);
            return rr < 127u ? rr : 127u;
        };
        if (a.relu) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int i = 0; i < 16; ++i) q[r][i] = (int8_t)pos((uint32_t)max(acc[r][i], 0));
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int32_t v = acc[r][i];
                    const int32_t p = (int32_t)pos(uabs32(v));
                    q[r][i] = (int8_t)(v < 0 ? -p : p);
                }
        }
    }
    const int64_t img = U.img;
    const int cb16 = U.cob * 32 + 16 * h;  // this lane's 16 channels after pack_cols
    if (DG && a.pool_dx != nullptr) {
        // through the previous layer's 2x2 max pool: the window scan of maxpool_grad_tiled_kernel
        constexpr int H2 = 2 * H, W2 = 2 * W;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const v4i v = pack_cols(q[r]);
            const int oy = U.b * R + r;
            if (!U.img_ok) continue;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int iy = 2 * oy + (t >> 1), ix = 2 * ox + (t & 1);
                const v4i d = v & e.x[DG ? r : 0][t];  // the routing mask (epi_masks)
                if (a.pool_dx_nhwc) *(v4i*)(a.pool_dx + ((img * H2 + iy) * W2 + ix) * a.cop + cb16) = d;
                if (a.pool_dx_next != nullptr)
                    *(v4i*)(a.pool_dx_next + (((img * a.COB + U.cob) * H2 + iy) * W2 + ix) * 32 + 16 * h) = d;
                if (a.p16 != nullptr)
                    *(v4i*)(tile + ((((c / W) * 2 * R + 2 * r + (t >> 1)) * W2) + ix) * 32 + 16 * h) = d;
            }
        }
        if constexpr (DG && R <= 4)
            if (a.p16 != nullptr) p16_store<2 * R, 2 * W, 32 / W>(a, lane, tile, U.img - c / W, 2 * U.b * R, H2, U.cob);
        return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v4i v = pack_cols(q[r]);
        const int oy = U.b * R + r;
        if (U.img_ok) {
            const int64_t po = ((img * H + oy) * W + ox) * a.cop + cb16;
            if (DG && a.relu_mask != nullptr) v &= e.y[DG ? r : 0];
            if (a.out != nullptr && (W > 1 || cb16 < a.cop)) *(v4i*)(a.out + po) = v;  // (a 1x1 head: 16 channels)
            if (a.next != nullptr && a.pool_out == nullptr)
                *(v4i*)(a.next + (((img * a.COB + U.cob) * H + oy) * W + ox) * 32 + 16 * h) = v;
            if (DG && a.p16 != nullptr) *(v4i*)(tile + (((c / W) * R + r) * W + ox) * 32 + 16 * h) = v;
        }
    }
    if constexpr (DG && (R * W >= 16 || W == 2))
        if (a.p16 != nullptr) p16_store<R, W, 32 / W>(a, lane, tile, U.img - c / W, U.b * R, H, U.cob);
    if (a.pool_out != nullptr) {
        constexpr int HO = H / 2, WO = W / 2;
#pragma unroll
        for (int r = 0; r + 1 < R; r += 2) {
            int8_t pm[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int v0 = q[r][i] > q[r + 1][i] ? q[r][i] : q[r + 1][i];
                const int v1 = __builtin_amdgcn_mov_dpp(v0, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]: lane ^ 1
                pm[i] = (int8_t)(v0 > v1 ? v0 : v1);
            }
            const v4i v = pack_cols(pm);
            v4i code{0, 0, 0, 0};
            if (a.pool_code_out != nullptr) {
                // the window's elements: this lane's (top, bottom) and the odd neighbour's
                const v4i t0 = pack_cols(q[r]), t2 = pack_cols(q[r + 1]);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t t1 = (uint32_t)__builtin_amdgcn_mov_dpp(t0[k], 0xB1, 0xF, 0xF, false);
                    const uint32_t t3 = (uint32_t)__builtin_amdgcn_mov_dpp(t2[k], 0xB1, 0xF, 0xF, false);
                    code[k] = (int)pool_code4((uint32_t)t0[k], t1, (uint32_t)t2[k], t3, (uint32_t)v[k], a.relu != 0);
                }
            }
            if (U.img_ok && (ox & 1) == 0) {
                const int py = (U.b * R + r) / 2, px = ox / 2;
                *(v4i*)(a.pool_out + ((img * HO + py) * WO + px) * a.cop + cb16) = v;
                if (a.pool_code_out != nullptr) *(v4i*)(a.pool_code_out + ((img * HO + py) * WO + px) * a.cop + cb16) = code;
                if (a.next != nullptr)
                    *(v4i*)(a.next + (((img * a.COB + U.cob) * HO + py) * WO + px) * 32 + 16 * h) = v;
            }
        }
    }
}

__device__ __forceinline__ uint32_t max_abs16(const v16i& v, uint32_t m) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t u = uabs32(v[i]);
        m = m > u ? m : u;
    }
    return m;
}

// ---- the row-segment form's epilogue (W = 0) ---------------------------------------------------
// Its MFMA columns are 14-px segments (or 7-px rows) with halo lanes, so a lane's output pixel is
// (U.img, row, U.x) where U.out_ok; the halo lanes' accumulators are partial sums and are neither
// ranged nor stored.  Same rule, relu / pool / pool-gradient epilogues and layouts as the W > 0 form.
template <int R, bool PX = true>
__device__ __forceinline__ void seg_prefetch(const RowConvArgs& a, const RowUnit<0, R>& U, int lane, EpiIn<R, PX>& e) {
    const int h = lane >> 5, W = a.hw, H = a.hw;
    const int64_t img = U.img_ok ? U.img : 0;
    const int xs = U.x < 0 ? 0 : (U.x >= W ? W - 1 : U.x);  // a halo lane reads a real pixel (unused)
    const int cb16 = U.cob * 32 + 16 * h;
    uint32_t z = 0;
    asm volatile("" : "+s"(z));
    const bool pool = PX && a.pool_dx != nullptr;
    const bool code = pool && a.pool_code != nullptr;  // the recorded route: one load per row
    const int8_t* ps = (pool ? (code ? a.pool_code : a.pool_y) : a.relu_mask) + z;
    const int8_t* px = a.pool_x + z;
    if (!pool && a.relu_mask == nullptr) return;
#pragma unroll
    for (int r = 0; r < R; ++r) e.y[r] = *(const v4i*)(ps + ((img * H + U.b * R + r) * W + xs) * a.cop + cb16);
    if constexpr (PX)
    if (pool && !code) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                e.x[r][t] = *(const v4i*)(px + ((img * 2 * H + 2 * (U.b * R + r) + (t >> 1)) * 2 * W + 2 * xs + (t & 1)) *
                                                   a.cop + cb16);
    }
}

template <int R, bool DG, bool PX = true>
__device__ __forceinline__ void seg_epilogue(const RowConvArgs& a, const RowUnit<0, R>& U, int lane,
                                             const v16i (&acc)[R], uint32_t gmax, const EpiIn<DG ? R : 1, PX>& e) {
    const int h = lane >> 5, W = a.hw, H = a.hw;
    const int shift = __builtin_amdgcn_readfirstlane(bitwidth_rc(gmax) - 7);
    int8_t q[R][16];
    if (shift <= 0) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int32_t v = (int32_t)(int8_t)acc[r][i];
                q[r][i] = (int8_t)(a.relu && v < 0 ? 0 : v);
            }
    } else {
        const uint32_t s = shift > 1 ? shift : 2, hh = s >> 1, odd = s & 1;
        auto pos = [&](uint32_t u) -> uint32_t {  // PSTO of u >= 0
            const uint32_t qv = u >> s;
            const uint32_t hi = __builtin_amdgcn_ubfe(u, hh, s - hh);
            const uint32_t lo = __builtin_amdgcn_ubfe(u, 0, hh) << odd;
            const uint32_t rr = qv + (hi > lo ? 1u : 0u);
            return rr < 127u ? rr : 127u;
        };
        if (a.relu) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int i = 0; i < 16; ++i) q[r][i] = (int8_t)pos((uint32_t)max(acc[r][i], 0));
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int32_t v = acc[r][i];
                    const int32_t p = (int32_t)pos(uabs32(v));
                    q[r][i] = (int8_t)(v < 0 ? -p : p);
                }
        }
    }
    const int64_t img = U.img;
    const int x = U.x;
    const int cb16 = U.cob * 32 + 16 * h;
    if (DG && PX && a.pool_dx != nullptr) {  // through the previous layer's 2x2 max pool
        const int H2 = 2 * H, W2 = 2 * W;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const v4i v = pack_cols(q[r]);
            const int oy = U.b * R + r;
            if (!U.out_ok) continue;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int iy = 2 * oy + (t >> 1), ix = 2 * x + (t & 1);
                const v4i d = v & e.x[DG && PX ? r : 0][t];
                if (a.pool_dx_nhwc) *(v4i*)(a.pool_dx + ((img * H2 + iy) * W2 + ix) * a.cop + cb16) = d;
                if (a.pool_dx_next != nullptr)
                    *(v4i*)(a.pool_dx_next + (((img * a.COB + U.cob) * H2 + iy) * W2 + ix) * 32 + 16 * h) = d;
            }
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v4i v = pack_cols(q[r]);
        const int oy = U.b * R + r;
        if (U.out_ok) {
            if (DG && a.relu_mask != nullptr) v &= e.y[DG ? r : 0];
            if (a.out != nullptr) *(v4i*)(a.out + ((img * H + oy) * W + x) * a.cop + cb16) = v;
            if (a.next != nullptr && a.pool_out == nullptr)
                *(v4i*)(a.next + (((img * a.COB + U.cob) * H + oy) * W + x) * 32 + 16 * h) = v;
        }
    }
    if (a.pool_out != nullptr) {  // pairs (x, x + 1), x even, never straddle a segment (14 even)
        const int HO = H / 2, WO = W / 2;
#pragma unroll
        for (int r = 0; r + 1 < R; r += 2) {
            int8_t pm[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int v0 = q[r][i] > q[r + 1][i] ? q[r][i] : q[r + 1][i];
                const int v1 = __builtin_amdgcn_update_dpp(0, v0, 0x101, 0xF, 0xF, true);  // row_shl:1: lane + 1
                pm[i] = (int8_t)(v0 > v1 ? v0 : v1);
            }
            const v4i v = pack_cols(pm);
            v4i code{0, 0, 0, 0};
            if (a.pool_code_out != nullptr) {  // the window: this lane's (top, bottom) and lane + 1's
                const v4i t0 = pack_cols(q[r]), t2 = pack_cols(q[r + 1]);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t t1 = (uint32_t)__builtin_amdgcn_update_dpp(0, t0[k], 0x101, 0xF, 0xF, true);
                    const uint32_t t3 = (uint32_t)__builtin_amdgcn_update_dpp(0, t2[k], 0x101, 0xF, 0xF, true);
                    code[k] = (int)pool_code4((uint32_t)t0[k], t1, (uint32_t)t2[k], t3, (uint32_t)v[k], a.relu != 0);
                }
            }
            if (U.out_ok && (x & 1) == 0) {
                const int py = (U.b * R + r) / 2, pxo = x / 2;
                *(v4i*)(a.pool_out + ((img * HO + py) * WO + pxo) * a.cop + cb16) = v;
                if (a.pool_code_out != nullptr)
                    *(v4i*)(a.pool_code_out + ((img * HO + py) * WO + pxo) * a.cop + cb16) = code;
                if (a.next != nullptr)
                    *(v4i*)(a.next + (((img * a.COB + U.cob) * HO + py) * WO + pxo) * 32 + 16 * h) = v;
            }
        }
    }
}

template <int W, int R>
__device__ __forceinline__ void unit_prefetch(const RowConvArgs& a, const RowUnit<W, R>& U, int lane, EpiIn<R>& e) {
    if constexpr (W == 0)
        seg_prefetch<R>(a, U, lane, e);
    else
        epi_prefetch<W, R>(a, U, lane, e);
}

template <int W, int R, bool DG>
__device__ __forceinline__ void unit_epilogue(const RowConvArgs& a, const RowUnit<W, R>& U, int lane,
                                              const v16i (&acc)[R], uint32_t gmax, const EpiIn<DG ? R : 1>& e,
                                              int8_t* tile) {
    if constexpr (W == 0)
        seg_epilogue<R, DG>(a, U, lane, acc, gmax, e);
    else
        rowconv_epilogue<W, R, DG>(a, U, lane, acc, gmax, e, tile);
}

// max |acc| over the unit's output columns (the row-segment form's halo lanes hold partial sums)
template <int W, int R>
__device__ __forceinline__ uint32_t unit_max(const RowUnit<W, R>& U, const v16i (&acc)[R], uint32_t m) {
    if (W == 0 && !U.out_ok) return m;
#pragma unroll
    for (int r = 0; r < R; ++r) m = max_abs16(acc[r], m);
    return m;
}

// a unit's accumulators in acc_store: [unit][r][i / 4][lane][4] -- one 1 KiB wave store / load per
// 4 registers (unit = workgroup tile x 4 + wave; a K-split workgroup's unit is its wave 0's)
template <int R>
__device__ __forceinline__ int32_t* acc_slot(const RowConvArgs& a, int wg, int wid, int lane) {
    return a.acc_store + ((int64_t)(wg * 4 + wid) * R) * 1024 + lane * 4;
}
template <int R>
__device__ __forceinline__ void acc_put(const RowConvArgs& a, int wg, int wid, int lane, const v16i (&acc)[R]) {
    int32_t* p = acc_slot<R>(a, wg, wid, lane);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *(v4i*)(p + r * 1024 + q * 256) = v4i{acc[r][4 * q], acc[r][4 * q + 1], acc[r][4 * q + 2], acc[r][4 * q + 3]};
}
template <int R>
__device__ __forceinline__ void acc_get(const RowConvArgs& a, int wg, int wid, int lane, v16i (&acc)[R]) {
    const int32_t* p = acc_slot<R>(a, wg, wid, lane);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4i v = *(const v4i*)(p + r * 1024 + q * 256);
            acc[r][4 * q] = v[0];
            acc[r][4 * q + 1] = v[1];
            acc[r][4 * q + 2] = v[2];
            acc[r][4 * q + 3] = v[3];
        }
}

__device__ __forceinline__ void write_exponent(const RowConvArgs& a, uint32_t gmax) {
    if (a.exp_out == nullptr) return;
    const int shift = bitwidth_rc(gmax) - 7;
    const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
    *a.exp_out = (int8_t)((a.exp_in ? (int)*a.exp_in : 0) + (a.wscale ? (int)*a.wscale : 0) + inc);
}

// The same speculation for the two-launch form (several devices, graph capture, and the
// row-segment maps, which have no fused form): launch A multiplies, requantises with the hint and
// publishes its max; launch B (after the all-reduce MAX, when there is one) compares the max's bit
// width with the guess A used and redoes the launch only when they differ -- otherwise every
// workgroup exits at once, so a hit costs one GEMM pass instead of two (or a pass plus an int32
// accumulator round trip).  A layer whose bit width has just changed may flip again (gradients
// near a power of two): after a change, where the caller gave an accumulator store (the W > 0
// forms), the next pairs store the accumulators in A instead of requantising and B requantises
// them -- the range + stored-requantise cost -- until SPEC_COOLDOWN pairs in a row see the bit
// width hold.  Slot words:
// [0] the hint (bw + 1, 0 none; written by B's block 0, read by A), [1] what A did (the hint it
// used, bit 31 set when it stored instead; written by A's block 0, read by B), [2] redone launches,
// [3] pairs left in store mode (read and written by B's thread 0, read by A), [4] stored pairs,
// [0], [5], [6], [8, 26) the predictor's state (spec_learn, written by B's bookkeeping wave), [7] /
// [26, 32) the diagnostic record of the last 6 pairs (niti_model_spec_slot).
// Every other reader of a word runs in the other launch, so no launch's blocks race on a word.
// The guess (spec_pick / spec_learn, niti_device.hpp): of three predictors -- the most frequent of
// the layer's last 8 bit widths, the same on its input's scale (forward slots), the bit width two
// pairs back -- the one that has been right most often lately.
// the input's scale for the hint (spec_pick): exponent in + weight scale, both settled before A;
// forward slots only -- an input gradient's bit width follows its own value better than dy's scale
// (tools/spec_trace.py, profiles/r06_spec_trace_resnet18.txt: K = bw + escale drifts down steadily
// over the steps while bw stays within 14-16)
__device__ __forceinline__ int spec_escale(const RowConvArgs& a) {
    if (!a.hint_scale) return 0;
    return __builtin_amdgcn_readfirstlane((a.exp_in ? (int)*a.exp_in : 0) + (a.wscale ? (int)*a.wscale : 0));
}
constexpr uint32_t SPEC_COOLDOWN = 8;  // the default of spec_cooldown() (NITI_SPEC_COOLDOWN overrides; profiles/r05_spec_cooldown_ab.txt)
__device__ __forceinline__ int spec_guess(const RowConvArgs& a, bool can_store, bool& store) {
    uint32_t f = 0;
    const uint32_t gh = spec_pick_e(a.hint, a.exp_in, a.wscale, a.hint_scale != 0, &f);  // the guess, bw + 1 (0: none)
    store = can_store && a.acc_store != nullptr && f != 0;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(a.hint + 1, gh | (store ? 0x80000000u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (int)gh - 1;
}

// launch B: g = the rule's max word; returns whether this launch has work (A stored the
// accumulators -- `stored` -- or guessed a different bit width), else every block returns.  The
// bookkeeping (exponent, the next guess, store flag, counts) is spec_book's, by one block, up front
// (after its work it delayed the launch's end by its memory round trips and stores).
struct SpecBook {
    uint32_t g, w1;
    int bw, esc, eiw;  // eiw: exponent in + weight scale (the exponent's base)
    bool stored, changed;
};
__device__ __forceinline__ bool spec_settle(const RowConvArgs& a, uint32_t& g, bool& stored, SpecBook& bk) {
    g = read_max(a.amax);
    bk.g = g;
    bk.bw = bitwidth_rc(g);
    bk.eiw = __builtin_amdgcn_readfirstlane((a.exp_in ? (int)*a.exp_in : 0) + (a.wscale ? (int)*a.wscale : 0));
    bk.esc = a.hint_scale ? bk.eiw : 0;  // read before the exponent write (exp_out may alias a later exp_in)
    bk.w1 = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(a.hint + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    stored = (bk.w1 >> 31) != 0;
    bk.stored = stored;
    bk.changed = bk.bw != (int)(bk.w1 & 0x7fffffffu) - 1;
    return stored || bk.changed;
}
// called by every thread of every block of launch B after spec_settle: the last block (a persistent
// grid's fewest units) writes the exponent, the next guess, the store flag and the counts
__device__ __forceinline__ void spec_book(const RowConvArgs& a, const SpecBook& bk) {
    if (blockIdx.x != gridDim.x - 1 || threadIdx.x >= 64) return;
    // (these loads issue with spec_learn's: one memory round trip for the whole bookkeeping)
    const uint32_t cd = __hip_atomic_load(a.hint + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t hn = __hip_atomic_load(a.hint + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    spec_learn(a.hint, bk.bw, bk.esc, threadIdx.x);  // the next guess (spec_pick)
    if (threadIdx.x == 0) {
        if (a.exp_out != nullptr) {  // write_exponent on the base read up front
            const int shift = bitwidth_rc(bk.g) - 7;
            *a.exp_out = (int8_t)(bk.eiw + (shift > 1 ? shift : (shift == 1 ? 2 : 0)));
        }
        // store mode for the next SPEC_COOLDOWN pairs after a change (a layer whose bit width flips
        // from step to step, gradients near a power of two, stays there; this block of B is the only
        // reader-writer of this word within a launch)
        __hip_atomic_store(a.hint + 3, bk.changed ? a.spec_cooldown : (cd > 0u ? cd - 1u : 0u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        // the last 6 pairs' record (niti_model_spec_slot): word 7 counts, 26 + (count mod 6) holds
        // bw | (escale + 256) << 8 | the guess A used (bw + 1) << 20
        __hip_atomic_store(a.hint + 26 + hn % 6u,
                           (uint32_t)bk.bw | ((uint32_t)(bk.esc + 256) << 8) | ((bk.w1 & 0xfffu) << 20),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.hint + 7, hn + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (bk.stored) __hip_atomic_fetch_add(a.hint + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (bk.changed) __hip_atomic_fetch_add(a.hint + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}


// KS = 0: four units per workgroup; KS = NS: one unit, K split over the waves (wave 0 holds the sum)
template <int W, int R, bool UNC, int KS>
__device__ __forceinline__ void compute_unit(const RowConvArgs& a, const RowUnit<W, R>& U, int lane, int wid,
                                             int8_t* smem, v16i (&acc)[R]) {
    if constexpr (W == 1) {
        fc_compute<R>(a, U, lane, acc);
    } else if constexpr (KS > 0) {
        rowconv_compute_ks<W, R, KS>(a, U, lane, wid, smem, acc);
        ks_reduce<R>(acc, smem, wid, lane);
    } else {
        rowconv_compute<W, R, UNC>(a, U, lane, wid, smem, acc);
    }
}

// s_waitcnt vmcnt(n) for a run-time, wave-uniform n in [LO, HI] (a binary search of scalar
// branches down to the immediate; n above HI waits for HI, which only waits longer)
template <int LO, int HI>
__device__ __forceinline__ void vm_wait_dyn(int n) {
    if constexpr (LO == HI) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LO) : "memory");
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (n <= MID)
            vm_wait_dyn<LO, MID>(n);
        else
            vm_wait_dyn<MID + 1, HI>(n);
    }
}

// VMEM stores a valid unit's seg_epilogue issues -- a lower bound (a store split in two only makes
// the counted waits below wait longer; a count above the real one would let them pass early)
template <int R, bool DG>
__device__ __forceinline__ int seg_epi_stores(const RowConvArgs& a) {
    if (DG && a.pool_dx != nullptr) return 4 * R * ((a.pool_dx_nhwc ? 1 : 0) + (a.pool_dx_next != nullptr ? 1 : 0));
    int e = R * ((a.out != nullptr ? 1 : 0) + (a.next != nullptr && a.pool_out == nullptr ? 1 : 0));
    if (a.pool_out != nullptr) e += (R / 2) * (1 + (a.next != nullptr ? 1 : 0) + (a.pool_code_out != nullptr ? 1 : 0));
    return e;
}

// The row-segment form's persistent modes (RANGE, REQUANT) as ONE software-pipelined stream of
// (tile, chunk) steps over the block's tiles t = blockIdx.x, + gridDim.x, ...: the next tile's first
// chunks load while this tile's last ones compute (the per-unit prologue of rowconv_compute left a
// shallow conv -- 2 to 4 chunks per unit -- waiting for memory once per unit).  Same ring as
// rowconv_compute: 4 stages, the R + 2 input rows of a chunk in registers, its 9 weight fragments
// LDS-DMA'd by the four waves; steps past the last tile load out of range (zeros) and feed nothing.
// A tile's epilogue (the max, or the requantised outputs) runs after its last chunk, with the next
// tile's loads in flight.  Its stores (and the input gradient's operand prefetch) are VMEM operations
// the ring's counted waits must allow for: a step waits for vmcnt(L + the extra operations issued
// after the stage it needs) instead of draining the queue after every tile (a full memory round trip
// per tile: ~30 % of a shallow layer's launch).
template <int R, int MODE, bool DG, bool PX = true>
__device__ __forceinline__ void seg_run(const RowConvArgs& a, int lane, int wid, int8_t* smem, uint32_t& m,
                                        uint32_t g) {
    constexpr int NR = R + 2, S = 4, L = NR + 3;
    const int H = a.hw, CB = a.CB;
    const int h = lane >> 5, c = lane & 31;
    const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.x, a.xbytes);
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.wf, a.wbytes);
    const uint32_t CHUNK = a.xcs;
    const int ntiles = (int)blockIdx.x < a.wgs ? (a.wgs - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const int total = ntiles * CB;
    const int steps = (total + S - 1) / S * S;  // whole ring turns: straight-line steps
    auto tile_wg = [&](int k) {
        const int b = (int)blockIdx.x + k * (int)gridDim.x;
        return a.wmajor && (int)gridDim.x == a.wgs ? xcd_remap(b, gridDim.x) : b;
    };
    // issue side: the tile whose chunks are being loaded, its rows' lane offsets and weight base
    int ik = 0, icc = 0;
    uint32_t ioff[NR], iwb = 0;
    auto set_issue = [&](int k) {
        if (k >= ntiles) {
#pragma unroll
            for (int j = 0; j < NR; ++j) ioff[j] = OOB;
            iwb = 0;
            return;
        }
        const RowUnit<0, R> U(a, tile_wg(k), wid, c, false);
        const uint32_t xl = U.img_ok && U.x_ok ? (uint32_t)U.img * a.xis + (uint32_t)U.x * a.xps + 16u * h : OOB;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int iy = U.b * R - 1 + j;
            ioff[j] = xl != OOB && iy >= 0 && iy < H ? xl + (uint32_t)iy * a.xrs : OOB;
        }
        iwb = (uint32_t)(U.cob * CB * 9) * 1024u;
    };
    const uint32_t dv2 = wid == 0 ? (uint32_t)lane * 16u : OOB;
    v4i X[S][NR];
    auto issue = [&](auto st_c) {
        constexpr int ST = decltype(st_c)::value;
        int8_t* lds = smem + ST * RC_STAGE_BYTES;
        const bool real = ik < ntiles;
        const uint32_t wo = iwb + (uint32_t)icc * 9216u;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int piece = wid + 4 * k;
            dma16(rW, lds + piece * 1024, real ? (k < 2 ? (uint32_t)lane * 16u : dv2) : OOB,
                  wo + (uint32_t)(piece < 9 ? piece : 0) * 1024u);
        }
#pragma unroll
        for (int j = 0; j < NR; ++j) X[ST][j] = buf_load16(rX, ioff[j] == OOB ? OOB : ioff[j] + (uint32_t)icc * CHUNK);
        if (++icc == CB) {  // the next tile
            icc = 0;
            set_issue(++ik);
        }
    };
    const uint32_t lds_lane = lds_addr(smem) + (uint32_t)lane * 16u;
    v4i wreg[2][9];
    auto read_w = [&](auto st_c, v4i (&w)[9]) {
        constexpr int ST = decltype(st_c)::value;
#pragma unroll
        for (int t = 0; t < 9; ++t) w[t] = lds_b128(lds_lane + (uint32_t)(ST * RC_STAGE_BYTES + t * 1024));
    };
    auto fence_w = [&](v4i (&w)[9]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int t = 0; t < 9; ++t) reg_fence(w[t]);
    };
    // compute side: the tile whose chunks are being multiplied
    int ck = 0, ccc = 0;
    // the input-gradient epilogue's operands (relu mask / pool window) load with the tile's first
    // chunk and land while its chunks multiply (loaded after the last one, they stalled every tile
    // for a memory round trip: the requantise launch ran 2-3x its range launch in the VGG-16 step);
    // the step after such a prefetch allows its pf loads in flight beside the ring's
    EpiIn<DG ? R : 1, PX> ein = {};
    // extra VMEM operations (outside the ring) of step s - 2 after its ring issue (xa2), and of step
    // s - 1 before / after it (xb1, xa1): everything issued after the stage step s waits for
    int xa2 = 0, xb1 = 0, xa1 = 0, xb = 0, xa = 0;
    const int pf_n = __builtin_amdgcn_readfirstlane(
        DG && MODE != RC_RANGE ? (PX && a.pool_dx != nullptr ? (a.pool_code != nullptr ? R : 5 * R)
                                                             : (a.relu_mask != nullptr ? R : 0))
                               : 0);
    const int st_n = __builtin_amdgcn_readfirstlane(MODE == RC_RANGE ? (a.acc_store != nullptr ? 4 * R : 0)
                                                                      : seg_epi_stores<R, DG>(a));
    v16i acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[r][i] = 0;
    auto finish = [&]() {  // tile ck's last chunk is in acc
        const RowUnit<0, R> U(a, tile_wg(ck), wid, c, false);
        if constexpr (MODE == RC_RANGE) {
            m = unit_max<0, R>(U, acc, m);
            if (a.acc_store != nullptr) acc_put<R>(a, tile_wg(ck), wid, lane, acc);
        } else {
            if (a.spec2 == 1) m = unit_max<0, R>(U, acc, m);  // speculative launch A publishes the max too
            if constexpr (DG) epi_masks<R, PX>(a, ein);
            if (U.valid) seg_epilogue<R, DG, PX>(a, U, lane, acc, g, ein);
            xa = __builtin_amdgcn_readfirstlane(U.valid ? st_n : 0);
        }
        if constexpr (MODE == RC_RANGE) xa = st_n;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[r][i] = 0;
    };
    auto step = [&](auto st_c, int s) {
        constexpr int ST = decltype(st_c)::value, WB = ST & 1;
        // chunk s + 1 has landed (s + 2 may still be in flight) and chunk s - 1's stage is free
        {
            const int ex = xa2 + xb1 + xa1;
            if (ex == 0)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
            else
                vm_wait_dyn<L, 63>(L + ex);
            xa2 = xa1;
            xb = xa = 0;
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if constexpr (DG && MODE != RC_RANGE) {
            if (s < total && ccc == 0) {
                const RowUnit<0, R> U(a, tile_wg(ck), wid, c, false);
                seg_prefetch<R, PX>(a, U, lane, ein);
                xb = pf_n;
            }
        }
        issue(std::integral_constant<int, (ST + 3) % S>());
        read_w(std::integral_constant<int, (ST + 1) % S>(), wreg[1 - WB]);
        const v4i (&w)[9] = wreg[WB];
        v4i XL[NR], XR[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            XL[j] = shift_in_left<16>(X[ST][j], false);
            XR[j] = shift_in_right<16>(X[ST][j], false);
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky], XL[r + ky], acc[r], 0, 0, 0);
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky + 1], X[ST][r + ky], acc[r], 0, 0, 0);
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(w[3 * ky + 2], XR[r + ky], acc[r], 0, 0, 0);
            }
        fence_w(wreg[1 - WB]);
        if (s < total && ++ccc == CB) {  // uniform: the tile's last chunk is in
            finish();
            ccc = 0;
            ++ck;
        }
        xb1 = xb;
        xa1 = xa;
    };
    set_issue(0);
    issue(std::integral_constant<int, 0>());
    issue(std::integral_constant<int, 1>());
    issue(std::integral_constant<int, 2>());
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");  // step 0 (and 1) landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read_w(std::integral_constant<int, 0>(), wreg[0]);
    fence_w(wreg[0]);
    for (int s = 0; s < steps; s += S) {
        step(std::integral_constant<int, 0>(), s);
        step(std::integral_constant<int, 1>(), s + 1);
        step(std::integral_constant<int, 2>(), s + 2);
        step(std::integral_constant<int, 3>(), s + 3);
    }
    // the look-ahead loads (LDS-DMA into the ring) land before the workgroup's LDS is reused
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// DG: the input-gradient epilogues (relu mask / pool gradient), their operands prefetched
template <int W, int R, int MODE, bool DG, bool UNC, int KS>
__global__ void __launch_bounds__(256, (RC_EXP & 16) ? 2 : 1) rowconv_fwd_kernel(RowConvArgs a) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: DMA bases stay scalar
    const int c = lane & 31;
    __shared__ __attribute__((aligned(16))) int8_t smem[KS > 0 ? RC_KS_BYTES : RC_SMEM_BYTES];
    __shared__ uint32_t red[4];
    __shared__ uint32_t gm;
    v16i acc[R];
    // the waves that own a unit's result: all four, or wave 0 of a K-split workgroup
    const bool owner = KS == 0 || wid == 0;
    RC_STAMP(0);
    if constexpr (MODE == RC_FUSED) {
        const RowUnit<W, R> U(a, a.wmajor ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x, wid, c, KS > 0);
        uint32_t* hint_p = a.hint;  // the host's slot choice (DG or the caller's dgrad_slot)
        // the guess: the previous launch's bit width (written by block 0 after its barrier; the launch
        // boundary orders it before this read)
        int guess = -1;
        if (a.spec != 0) {
            const uint32_t h = __hip_atomic_load(hint_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            guess = __builtin_amdgcn_readfirstlane((int)h) - 1;
            if (guess >= 0 && a.spec == 2) guess = guess < 31 ? guess + 1 : guess - 1;
        }
        const uint32_t g_guess = guess <= 0 ? 0u : 1u << guess;
        uint32_t m = 0;
        compute_unit<W, R, UNC, KS>(a, U, lane, wid, smem, acc);
        EpiIn<DG ? R : 1> ein = {};
        if constexpr (DG)
            if (owner) unit_prefetch<W, R>(a, U, lane, ein);
        if (owner) m = unit_max<W, R>(U, acc, m);
        m = wave_max(m);
        if (lane == 0) red[wid] = m;
        __syncthreads();
        if (wid == 0) {
            const uint32_t bm = max(max(red[0], red[1]), max(red[2], red[3]));
            if (a.stamps != nullptr && lane == 0) a.stamps[blockIdx.x * 64 + 8] = __builtin_amdgcn_s_memrealtime();
            grid_bw_arrive(a.bar, a.epoch, bitwidth_rc(bm), lane);
        }
        if constexpr (DG)
            if (owner) epi_masks<R>(a, ein);  // while the barrier completes
        int8_t* tile = smem + wid * RC_P16_WAVE_BYTES;
        // the speculative epilogue, while the barrier completes (the guess cannot be below this
        // workgroup's own bit width, so such a guess is not tried)
        const bool spec = guess >= 0 && guess >= bitwidth_rc(max(max(red[0], red[1]), max(red[2], red[3])));
        if (spec && U.valid && owner) unit_epilogue<W, R, DG>(a, U, lane, acc, g_guess, ein, tile);
        if (wid == 0) {
            const int gbw = grid_bw_wait(a.bar, a.epoch, a.err, a.spin_limit, a.expect_extra, lane);
            if (a.stamps != nullptr && lane == 0) a.stamps[blockIdx.x * 64 + 9] = __builtin_amdgcn_s_memrealtime();
            // the rule only needs bw: 2^bw stands for the max (bitwidth_rc(2^bw) == bw)
            const uint32_t g = gbw == 0 ? 0u : 1u << gbw;
            if (lane == 0) {
                gm = g;
                if (blockIdx.x == 0) {
                    write_exponent(a, g);
                    if (a.spec != 0) __hip_atomic_store(hint_p, (uint32_t)gbw + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        __syncthreads();
        RC_STAMP(4);
        if (U.valid && owner && (!spec || gm != g_guess)) unit_epilogue<W, R, DG>(a, U, lane, acc, gm, ein, tile);
        RC_STAMP(5);
    } else if constexpr (MODE == RC_RANGE && W == 0) {
        uint32_t m = 0;
        seg_run<R, RC_RANGE, false>(a, lane, wid, smem, m, 0u);
        m = wave_max(m);
        if (lane == 0) red[wid] = m;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(a.amax, max(max(red[0], red[1]), max(red[2], red[3])));
    } else if constexpr (MODE == RC_REQUANT && W == 0) {
        uint32_t g = 0;
        bool store = false;
        SpecBook bk{};
        if (a.spec2 == 1) {  // (the row-segment form stores no accumulators: always the guess)
            const int guess = spec_guess(a, false, store);
            g = guess <= 0 ? 0u : 1u << guess;
        } else if (a.spec2 == 2) {
            const bool work = spec_settle(a, g, store, bk);
            spec_book(a, bk);
            if (!work) return;
        } else {
            g = read_max(a.amax);
            if (blockIdx.x == 0 && threadIdx.x == 0) write_exponent(a, g);
        }
        uint32_t m = 0;
        // the row-segment form's KS: 1 = an input gradient through a pool (its window operands)
        seg_run<R, RC_REQUANT, DG, KS != 0>(a, lane, wid, smem, m, g);
        if (a.spec2 == 1) {
            m = wave_max(m);
            if (lane == 0) red[wid] = m;
            __syncthreads();
            if (threadIdx.x == 0) publish_max(a.amax, max(max(red[0], red[1]), max(red[2], red[3])));
        }
    } else if constexpr (MODE == RC_RANGE) {
        uint32_t m = 0;
        for (int b = blockIdx.x; b < a.wgs; b += gridDim.x) {
            const int wg = a.wmajor && (int)gridDim.x == a.wgs ? xcd_remap(b, gridDim.x) : b;
            const RowUnit<W, R> U(a, wg, wid, c, KS > 0);
            compute_unit<W, R, UNC, KS>(a, U, lane, wid, smem, acc);
            if (owner) {
                m = unit_max<W, R>(U, acc, m);
                if (a.acc_store != nullptr) acc_put<R>(a, wg, wid, lane, acc);
            }
        }
        m = wave_max(m);
        if (lane == 0) red[wid] = m;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(a.amax, max(max(red[0], red[1]), max(red[2], red[3])));
        RC_STAMP(5);
    } else {
        uint32_t g = 0, m = 0;
        // load: the accumulators come from acc_store (the range launch's, or a storing launch A's);
        // store: this launch A stores them instead of requantising (spec_guess)
        bool load = a.acc_store != nullptr, store = false;
        SpecBook bk{};
        if (a.spec2 == 1) {
            const int guess = spec_guess(a, true, store);
            g = guess <= 0 ? 0u : 1u << guess;
            load = false;
        } else if (a.spec2 == 2) {
            const bool work = spec_settle(a, g, load, bk);
            spec_book(a, bk);
            if (!work) return;
        } else {
            g = read_max(a.amax);
            if (blockIdx.x == 0 && threadIdx.x == 0) write_exponent(a, g);
        }
        for (int b = blockIdx.x; b < a.wgs; b += gridDim.x) {
            const int wg = a.wmajor && (int)gridDim.x == a.wgs ? xcd_remap(b, gridDim.x) : b;
            const RowUnit<W, R> U(a, wg, wid, c, KS > 0);
            if (load) {  // uniform branch
                if (owner) acc_get<R>(a, wg, wid, lane, acc);
            } else {
                compute_unit<W, R, UNC, KS>(a, U, lane, wid, smem, acc);
            }
            if (a.spec2 == 1 && owner) m = unit_max<W, R>(U, acc, m);
            if (store) {
                if (owner) acc_put<R>(a, wg, wid, lane, acc);
                continue;
            }
            EpiIn<DG ? R : 1> ein = {};
            if constexpr (DG) {
                if (owner) {
                    unit_prefetch<W, R>(a, U, lane, ein);
                    epi_masks<R>(a, ein);
                }
            }
            if (U.valid && owner) unit_epilogue<W, R, DG>(a, U, lane, acc, g, ein, smem + wid * RC_P16_WAVE_BYTES);
            if (DG && a.p16 != nullptr) __syncthreads();  // the P16 tiles sit in the next unit's ring
        }
        if (a.spec2 == 1) {
            m = wave_max(m);
            if (lane == 0) red[wid] = m;
            __syncthreads();
            if (threadIdx.x == 0) publish_max(a.amax, max(max(red[0], red[1]), max(red[2], red[3])));
        }
    }
}

// ---- layout conversions -----------------------------------------------------------------------
// NHWC16 [n][hw][cp] -> C32 [n][cb][hw][32], cb = ceil(c / 32) (channels >= cp read as zero)
struct Nhwc16ToC32 {
    const int8_t* in;
    int hw, cp, cb;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over 16-byte chunks of out
        const int half = (int)(i & 1);
        const int64_t q = i >> 1;                  // (img, cblk, p)
        const int p = (int)(q % hw);
        const int64_t r = q / hw;
        const int blk = (int)(r % cb);
        const int64_t img = r / cb;
        const int ch = blk * 32 + half * 16;
        v16c v = {};
        if (ch < cp) v = *(const v16c*)(in + (img * hw + p) * cp + ch);
        *(v16c*)(out + i * 16) = v;
    }
};

// OHWI16 [co][9][cip] -> WF [cob][cb][9][2][32][16]: fragment (cob, cb, tap) holds rows co
// cob*32 + r, k = ci cb*32 + 16 hh + e; dgrad (transpose): the input-gradient conv's weights,
// output channel = ci, input channel = co, tap t' reads w[co][8 - t'][ci] (rotate180)
struct WeightsToWF {
    const int8_t* w;
    int co, ci, cip, COB, CB;
    bool transpose;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over 16-byte rows of out
        const int r = (int)(i & 31);
        int64_t q = i >> 5;
        const int hh = (int)(q & 1);
        q >>= 1;
        const int t = (int)(q % 9);
        q /= 9;
        const int cb = (int)(q % CB);
        const int ob = (int)(q / CB);
        v16c v = {};
        if (!transpose) {
            const int o = ob * 32 + r;
            if (o < co) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int k = cb * 32 + 16 * hh + e;
                    v[e] = k < ci ? w[((int64_t)o * 9 + t) * cip + k] : (int8_t)0;
                }
            }
        } else {
            const int o = ob * 32 + r;  // the layer's input channel
            if (o < ci) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int k = cb * 32 + 16 * hh + e;  // the layer's output channel
                    v[e] = k < co ? w[((int64_t)k * 9 + (8 - t)) * cip + o] : (int8_t)0;
                }
            }
        }
        *(v16c*)(out + i * 16) = v;
    }
};

hipError_t nhwc16_to_c32(const int8_t* in, int n, int hw, int cp, int c, int8_t* out, hipStream_t st) {
    const int cb = (c + 31) / 32;
    return launch_map((int64_t)n * cb * hw * 2, Nhwc16ToC32{in, hw, cp, cb, out}, st);
}

// C32 [n][cb][hw][32] -> NHWC16 [n][hw][cp], one 16-byte chunk per thread
struct C32ToNhwc16 {
    const int8_t* in;
    int hw, cp, c, cb;
    int8_t* out;
    __device__ void operator()(int64_t i) const {  // i over 16-byte chunks of out
        const int cc = (int)(i % (cp / 16)) * 16;
        const int64_t q = i / (cp / 16);  // (img, p)
        const int p = (int)(q % hw);
        const int64_t img = q / hw;
        v16c v = {};
        if (cc < c) v = *(const v16c*)(in + (((img * cb + cc / 32) * hw + p) * 32 + (cc & 31)));
        *(v16c*)(out + i * 16) = v;
    }
};

hipError_t c32_to_nhwc16(const int8_t* in, int n, int hw, int cp, int c, int8_t* out, hipStream_t st) {
    const int cb = (c + 31) / 32;
    return launch_map((int64_t)n * hw * (cp / 16), C32ToNhwc16{in, hw, cp, c, cb, out}, st);
}

hipError_t weights_to_wf(const int8_t* w_ohwi16, int co, int ci, int cip, bool transpose, int8_t* out,
                         hipStream_t st) {
    const int COB = transpose ? (ci + 31) / 32 : (co + 31) / 32;
    const int CB = transpose ? (co + 31) / 32 : (ci + 31) / 32;
    return launch_map((int64_t)COB * CB * 9 * 2 * 32, WeightsToWF{w_ohwi16, co, ci, cip, COB, CB, transpose, out}, st);
}

size_t rowconv_wf_bytes(int co, int ci) { return (size_t)((co + 31) / 32) * ((ci + 31) / 32) * 9 * 1024; }

// ---- host side ---------------------------------------------------------------------------------
// the deepest conv (input channels) the row-segment form takes; NITI_SEG_MAX_CIN overrides (A/B)
static int seg_max_cin() {
    static const int v = getenv("NITI_SEG_MAX_CIN") ? atoi(getenv("NITI_SEG_MAX_CIN")) : 128;
    return v;
}

bool rowconv_ok(const ConvGeom& g) {
    if (g.kh != 3 || g.kw != 3 || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1) return false;
    if (g.pt != 1 || g.pl != 1 || g.pb != 1 || g.pr != 1) return false;
    if (g.h != g.w || g.oh != g.h || g.ow != g.w) return false;
    // W > 0 form: 2 / 4 / 8 / 16 px; the row-segment form (W = 0): 14-px segments of 224 / 112 / 56 /
    // 28 / 14 px maps, where it beats the implicit GEMM: shallow convs (c_in <= 128; per layer on
    // MI355X, tools/seg_bench.py, profiles/r04_seg_bench.txt)
    const bool seg = (g.w > 16 ? g.w % 28 == 0 : g.w == 14) && g.c_in <= seg_max_cin();
    if (!(g.w == 2 || g.w == 4 || g.w == 8 || g.w == 16 || seg)) return false;
    if (g.cop % 32 != 0) return false;
    return true;
}

bool rowconv_seg(const ConvGeom& g) { return g.w > 16 || g.w == 14; }

// the row-segment form can read its input as NHWC16 in place (RowConvOut::x_nhwc) ...
bool rowconv_nhwc_ok(const ConvGeom& g) { return rowconv_ok(g) && rowconv_seg(g) && g.cip % 32 == 0; }
// ... and the model does where that is not slower than a C32 copy: 64 channels (a wave load then
// spans whole 128-byte lines, half used per chunk; VGG-16 conv1_2 / conv2_1 as fast as from C32,
// conv0's C32 copy and a layout pass saved), and 128 channels on maps up to 28 px (ResNet-18's
// layer2: step 4.06 vs 4.12 ms), not on wider ones (VGG-16 conv2_2 @112 1.3-1.4x slower, conv3_1
// @56 1.2x; tools/gpu_r04k.sh, gpu_r04r.sh); NITI_SEG_NHWC_MAX_CIP sets one channel cap for every
// map (A/B)
bool rowconv_nhwc_pref(const ConvGeom& g) {
    if (!rowconv_nhwc_ok(g)) return false;
    if (const char* e = getenv("NITI_SEG_NHWC_MAX_CIP")) return g.cip <= atoi(e);
    return g.cip <= 64 || (g.cip <= 128 && g.w <= 28);
}

// the row-segment form's launch shape: 4 rows per band (2 at 14 px), units of 28 px (two 14-px
// segments of one row, or one 14-px row of two images), whole workgroups of 4 units per co block
struct SegPlan {
    int R, gw, nsp, nbands, ngb, upc4, wgs;
};
static SegPlan seg_plan(const ConvGeom& g) {
    SegPlan p{};
    // R = 2 (two blocks per CU: one wave's loads wait while the other's MFMAs run) measured faster
    // than R = 4 at every row-segment layer (profiles/r04_seg_bench.txt); NITI_SEG_R=4 for A/B
    static const int r_env = getenv("NITI_SEG_R") ? atoi(getenv("NITI_SEG_R")) : 2;
    p.R = g.h % 4 == 0 && r_env == 4 ? 4 : 2;
    p.gw = g.w == 14 ? 2 : 1;
    p.nsp = g.w >= 28 ? g.w / 28 : 1;
    p.nbands = g.h / p.R;
    p.ngb = ((g.n + p.gw - 1) / p.gw) * p.nbands;
    p.upc4 = (p.ngb * p.nsp + 3) / 4 * 4;
    p.wgs = (g.cop / 32) * p.upc4 / 4;
    return p;
}

// the row-segment form keeps its int32 accumulators between the range and requantise launches
// only where the GEMM is deep (K = 9 c_in >= 2304): recomputing 2 M N K ops costs more there than
// the 8 bytes per output of an int32 round trip; shallower layers recompute (no int32 tensor)
static int acc_min_cin() {  // NITI_RC_ACC_MIN_CIN overrides (A/B diagnostics)
    static const int v = getenv("NITI_RC_ACC_MIN_CIN") ? atoi(getenv("NITI_RC_ACC_MIN_CIN")) : 256;
    return v;
}
static bool seg_store_acc(const ConvGeom& g) { return g.c_in >= acc_min_cin(); }

bool rowconv_dgrad_geom(const ConvGeom& l, ConvGeom* d) {
    if (!rowconv_ok(l)) return false;
    ConvGeom g = l;
    g.c_in = l.c_out;
    g.c_out = l.c_in;
    if (!g.finalize() || g.cip != l.cop || g.cop != l.cip) return false;
    *d = g;
    return rowconv_ok(g);
}

// rows per band: the largest R (a power of two dividing H, at most 8: register budget) whose unit
// count fills the chip (>= 768 waves), else R = 2, the most units; FUSED needs one unit per wave
// and every workgroup resident (units <= 1024)
static int rowconv_rows(const ConvGeom& g, bool dg, int* units_out) {
    if (rowconv_seg(g)) {
        const SegPlan p = seg_plan(g);
        *units_out = p.wgs * 4;
        return p.R;
    }
    const int W = g.w, G = 32 / W;
    const int64_t groups = (g.n + G - 1) / G, cob = g.cop / 32;
    // register budget: 8 rows at W = 16 (DPP shifts), else 4; the input-gradient epilogue's
    // prefetched operands (5 x 16 bytes per row) cap it at 4
    int R = W == 16 && !dg ? 8 : (W < 4 ? W : 4);
    if (RC_EXP & 16) R = 2;
    while (R > 2 && groups * (W / R) * cob < 768) R /= 2;
    const int64_t ngb4 = (groups * (W / R) + 3) / 4 * 4;
    *units_out = (int)(ngb4 * cob);  // waves, whole workgroups of 4
    return R;
}

static int rowconv_ks(const ConvGeom& g, bool dg);

// the accumulator store of modes RANGE + REQUANT: every wave slot of the launch, R x 1 KiB x 4
size_t rowconv_acc_bytes(const ConvGeom& g, bool dg) {
    if (!rowconv_ok(g)) return 0;
    if (rowconv_seg(g)) {
        const SegPlan p = seg_plan(g);
        return seg_store_acc(g) ? (size_t)p.wgs * 4 * p.R * 1024 * sizeof(int32_t) : 0;
    }
    // the W > 0 forms (VGG-11's data-parallel path) store at every depth: recomputing VGG-11's
    // conv1 / conv2 (c_in 64 / 128) in the requantise launch measured no faster (--dp-path 0.578 vs
    // 0.575 ms per step); NITI_RC_ACC_MIN_CIN applies the row-segment rule here too (A/B)
    if (getenv("NITI_RC_ACC_MIN_CIN") != nullptr && g.c_in < acc_min_cin()) return 0;
    int u = 0;
    const int R = rowconv_rows(g, dg, &u);
    const int G = 32 / g.w, ngb = ((g.n + G - 1) / G) * (g.h / R), ngb4 = (ngb + 3) / 4 * 4, COB = g.cop / 32;
    const int64_t wgs = rowconv_ks(g, dg) > 0 ? (int64_t)COB * ngb : (int64_t)COB * ngb4 / 4;
    return (size_t)wgs * 4 * R * 1024 * sizeof(int32_t);
}

bool rowconv_p16_ok(const ConvGeom& d, bool pool) {
    if (!rowconv_ok(d) || rowconv_seg(d)) return false;
    int u = 0;
    const int R = rowconv_rows(d, true, &u), W = d.w;
    const int64_t px = (int64_t)d.n * d.h * d.w * (pool ? 4 : 1);
    if (px % 16 != 0) return false;
    return pool || R * W >= 16 || (W == 2 && R == 2);
}

// the K-split form (rowconv_compute_ks): chunks per wave, or 0.  Whole-image 2-row units whose
// one-unit-per-wave grid leaves the chip more than a quarter empty, and at most 4 chunks per wave
static int rowconv_ks(const ConvGeom& g, bool dg) {
    int u = 0;
    const int R = rowconv_rows(g, dg, &u);
    const int CB = (g.c_in + 31) / 32;
    if (g.w != 2 || R != 2 || CB % 4 != 0 || CB / 4 > RC_KS_MAX_NS || u >= 768) return 0;
    return CB / 4;
}

// waves of the launch (K-split: four per unit)
int rowconv_units(const ConvGeom& g, bool dg) {
    if (rowconv_seg(g)) return seg_plan(g).wgs * 4;
    int u = 0;
    (void)rowconv_rows(g, dg, &u);
    if (rowconv_ks(g, dg) > 0) {
        const int64_t units = (int64_t)(g.n + 15) / 16 * (g.cop / 32);  // W = 2: 16 images per unit
        return (int)(units * 4);
    }
    return u;
}

// the instantiation a launch runs (ks > 0: the K-split form, W = R = 2)
template <int MODE, bool DG>
static const void* rc_kernel(int W, int R, bool unc, int ks) {
    if constexpr (MODE == RC_REQUANT && DG) {  // row-segment input gradients: ks = 1 through a pool
        if (W == 0 && ks == 1 && R == 4) return reinterpret_cast<const void*>(&rowconv_fwd_kernel<0, 4, MODE, DG, false, 1>);
        if (W == 0 && ks == 1 && R == 2) return reinterpret_cast<const void*>(&rowconv_fwd_kernel<0, 2, MODE, DG, false, 1>);
    }
    if (W == 0 && ks != 0) return nullptr;
    if (ks > 0) {
        if (ks == 4) return reinterpret_cast<const void*>(&rowconv_fwd_kernel<2, 2, MODE, DG, false, 4>);
        if (ks == 2) return reinterpret_cast<const void*>(&rowconv_fwd_kernel<2, 2, MODE, DG, false, 2>);
        if (ks == 1) return reinterpret_cast<const void*>(&rowconv_fwd_kernel<2, 2, MODE, DG, false, 1>);
        return nullptr;
    }
#define RC_CASE(WW, RR)                                                                                  \
    if (W == WW && R == RR)                                                                              \
        return (WW != 1 && unc) ? reinterpret_cast<const void*>(&rowconv_fwd_kernel<WW, RR, MODE, DG, true, 0>) \
                                : reinterpret_cast<const void*>(&rowconv_fwd_kernel<WW, RR, MODE, DG, false, 0>);
    if constexpr (!DG) RC_CASE(16, 8)
    RC_CASE(16, 4)
    RC_CASE(16, 2)
    RC_CASE(8, 4)
    RC_CASE(8, 2)
    RC_CASE(4, 4)
    RC_CASE(4, 2)
    RC_CASE(2, 2)
    RC_CASE(1, 1)
    RC_CASE(0, 4)  // the row-segment form
    RC_CASE(0, 2)
#undef RC_CASE
    return nullptr;
}

template <int MODE, bool DG>
static hipError_t launch_rc(int W, int R, int grid, RowConvArgs a, hipStream_t st, int ks = 0) {
    const void* f = rc_kernel<MODE, DG>(W, R, W != 1 && a.CB % 4 == 0, ks);
    if (f == nullptr) return hipErrorInvalidValue;
    void* args[] = {&a};
    return hipLaunchKernel(f, dim3((unsigned)grid), dim3(256), args, 0, st);
}

// Workgroups of kernel f the current device holds at once: CUs x the kernel's occupancy per CU
// (hipOccupancyMaxActiveBlocksPerMultiprocessor over its LDS and registers), cached per (device,
// kernel); 0 without a device.  The fused mode's grid barrier needs the whole grid resident, so a
// smaller or partitioned device takes the two-launch form instead.
int resident_wgs(const void* f, int threads) {
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, int> cache;
    int dev = -1;
    if (f == nullptr || hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(dev, f);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 0, occ = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, f, threads, 0) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return cache[key] = cus * occ;
}

// workgroups of a launch (K-split: one unit each; else four units)
static int rowconv_wgs(const ConvGeom& g, bool dg, int* R_out, int* ks_out) {
    if (rowconv_seg(g)) {
        const SegPlan p = seg_plan(g);
        *R_out = p.R;
        *ks_out = 0;
        return p.wgs;
    }
    int u = 0;
    const int R = rowconv_rows(g, dg, &u);
    const int ks = rowconv_ks(g, dg);
    const int G = 32 / g.w, ngb = ((g.n + G - 1) / G) * (g.h / R), ngb4 = (ngb + 3) / 4 * 4, COB = g.cop / 32;
    *R_out = R;
    *ks_out = ks;
    return ks > 0 ? COB * ngb : COB * ngb4 / 4;
}

// FUSED needs every workgroup resident (one unit per wave, the grid barrier inside the kernel)
bool rowconv_fused_ok(const ConvGeom& g, bool dg) {
    if (!rowconv_ok(g)) return false;
    int R = 0, ks = 0;
    const int wgs = rowconv_wgs(g, dg, &R, &ks);
    const bool unc = (g.c_in + 31) / 32 % 4 == 0;
    const int W = rowconv_seg(g) ? 0 : g.w;
    const void* f = dg ? rc_kernel<RC_FUSED, true>(W, R, unc, ks) : rc_kernel<RC_FUSED, false>(W, R, unc, ks);
    return wgs <= resident_wgs(f);
}

static uint32_t g_rc_spin_limit = BAR_SPIN_LIMIT, g_rc_expect_extra = 0;
// the speculative epilogue is off by default: VGG-11 batch 256, 3 alternating runs each on one box,
// 0.4115 ms per step with it against 0.3988 without (profiles/r04_ab.txt) -- the early epilogues'
// stores compete with the slowest workgroups' K loops, which set the launch's end
static int g_rc_spec = 0;
void rowconv_barrier_diag(uint32_t spin_limit, uint32_t expect_extra) {
    g_rc_spin_limit = spin_limit ? spin_limit : BAR_SPIN_LIMIT;
    g_rc_expect_extra = expect_extra;
}
void rowconv_speculate(int mode) { g_rc_spec = mode; }
uint32_t* rowconv_spec_slot(uint32_t* bar, bool dg) { return bar + (16 + (dg ? 1 : 0)) * BAR_LINE; }
// pairs a layer stays in store mode after its bit width changed (A/B knob NITI_SPEC_COOLDOWN; 0 never
// stores: a miss then redoes the GEMM instead of reading back stored accumulators)
// NITI_SPEC_SCALE=0: the forward slots' guesses bare too (an A/B switch for the scaled form)
static bool spec_scale_on() {
    static const bool v = getenv("NITI_SPEC_SCALE") ? atoi(getenv("NITI_SPEC_SCALE")) != 0 : true;
    return v;
}
static uint32_t spec_cooldown() {
    static const int v = getenv("NITI_SPEC_COOLDOWN") ? atoi(getenv("NITI_SPEC_COOLDOWN")) : (int)SPEC_COOLDOWN;
    return v < 0 ? 0u : (uint32_t)v;
}

bool rowconv_spec2_on() {
    static const char* env = getenv("NITI_RC_SPEC2");
    return env == nullptr || env[0] != '0';
}

// Tile order over the XCDs: weight-major when the layer's weights outweigh its input (VGG-11's
// 4x4 / 2x2 layers: 16 image groups re-read each co block's 147 KiB panel), else dispatch order.
// NITI_RC_MAP=x / w forces one (A/B diagnostics).
static int rowconv_wmajor(int64_t xbytes, int64_t wbytes) {
    static const char* env = getenv("NITI_RC_MAP");
    if (env != nullptr && env[0] == 'x') return 0;
    if (env != nullptr && env[0] == 'w') return 1;
    return wbytes > xbytes ? 1 : 0;
}

static unsigned long long* g_rc_stamps = nullptr;
void rowconv_stamps_arm(unsigned long long* buf) { g_rc_stamps = buf; }

hipError_t rowconv_fwd(const ConvGeom& g, const int8_t* x_c32, const int8_t* wf, const RowConvOut& o, int mode,
                       uint32_t* amax, uint32_t* bar, uint32_t epoch, uint32_t* err, hipStream_t st) {
    if (!rowconv_ok(g) || x_c32 == nullptr || wf == nullptr || amax == nullptr) return hipErrorInvalidValue;
    // modes RC_SPEC_A / RC_SPEC_B: the requantise instantiation as a speculative pair (spec_guess)
    const bool spec = mode == RC_SPEC_A || mode == RC_SPEC_B;
    if (spec && bar == nullptr) return hipErrorInvalidValue;
    const int spec2 = spec ? mode - RC_SPEC_A + 1 : 0;
    if (spec) mode = RC_REQUANT;
    // an output: NHWC16 out, the pool gradient, or (input gradient) only the C32 / P16 copies
    if (mode != RC_RANGE && o.out == nullptr && o.pool_dx == nullptr && o.next == nullptr && o.p16 == nullptr &&
        o.pool_out == nullptr)
        return hipErrorInvalidValue;
    if (o.pool_dx != nullptr && ((o.pool_code == nullptr && (o.pool_x == nullptr || o.pool_y == nullptr)) ||
                                 o.out != nullptr || o.pool_out != nullptr || o.relu_mask != nullptr || o.next != nullptr))
        return hipErrorInvalidValue;
    // the recorded pool route (pool_code4)
    if ((o.pool_code != nullptr && o.pool_dx == nullptr) || (o.pool_code_out != nullptr && o.pool_out == nullptr))
        return hipErrorInvalidValue;
    RowConvArgs a{};
    const int CB = (g.c_in + 31) / 32, COB = g.cop / 32;
    // the row-segment form may read x as NHWC16 (o.x_nhwc; cip a multiple of 32)
    if (o.x_nhwc && (!rowconv_seg(g) || g.cip % 32 != 0)) return hipErrorInvalidValue;
    const int64_t xb = o.x_nhwc ? (int64_t)g.n * g.h * g.w * g.cip : (int64_t)g.n * CB * g.h * g.w * 32;
    const int64_t wb = (int64_t)COB * CB * 9 * 1024;
    if (xb > 0x7fffffff || wb > 0x7fffffff) return hipErrorInvalidValue;
    if (o.x_nhwc) {
        a.xps = (uint32_t)g.cip;
        a.xrs = (uint32_t)(g.w * g.cip);
        a.xis = (uint32_t)(g.h * g.w * g.cip);
        a.xcs = 32u;
    } else {
        a.xps = 32u;
        a.xrs = (uint32_t)(g.w * 32);
        a.xis = (uint32_t)(CB * g.h * g.w * 32);
        a.xcs = (uint32_t)(g.h * g.w * 32);
    }
    a.x = x_c32;
    a.wf = wf;
    a.xbytes = (uint32_t)xb;
    a.wbytes = (uint32_t)wb;
    a.n = g.n;
    a.CB = CB;
    a.COB = COB;
    const bool dg = o.relu_mask != nullptr || o.pool_dx != nullptr || o.p16 != nullptr;
    int units = 0;
    const int R = rowconv_rows(g, dg, &units);
    const bool seg = rowconv_seg(g);
    const int Wk = seg ? 0 : g.w;  // the kernel's W (0: the row-segment form)
    int ks = 0;
    if (seg) {
        const SegPlan p = seg_plan(g);
        a.hw = g.w;
        a.gw = p.gw;
        a.nsp = p.nsp;
        a.nbands = p.nbands;
        a.ngb = p.ngb;
        a.upc4 = p.upc4;
        a.wgs = p.wgs;
    } else {
        const int G = 32 / g.w;
        a.nbands = g.h / R;
        a.ngb = ((g.n + G - 1) / G) * a.nbands;
        a.ngb4 = (a.ngb + 3) / 4 * 4;
        ks = rowconv_ks(g, dg);
        a.wgs = ks > 0 ? COB * a.ngb : COB * a.ngb4 / 4;
    }
    a.wmajor = rowconv_wmajor(xb, wb);
    a.out = o.out;
    a.cop = g.cop;
    a.pool_out = o.pool_out;
    a.next = o.next;
    a.exp_in = o.exp_in;
    a.wscale = o.wscale;
    a.exp_out = o.exp_out;
    a.relu = o.relu;
    a.amax = amax;
    a.bar = bar;
    a.epoch = epoch;
    a.err = err;
    a.spin_limit = g_rc_spin_limit;
    a.expect_extra = g_rc_expect_extra;
    a.spec = g_rc_spec;
    a.stamps = g_rc_stamps;
    a.relu_mask = o.relu_mask;
    a.pool_x = o.pool_x;
    a.pool_y = o.pool_y;
    a.pool_dx = o.pool_dx;
    a.pool_dx_next = o.pool_dx_next;
    a.pool_relu = o.pool_relu;
    a.pool_code = o.pool_code;
    a.pool_code_out = o.pool_code_out;
    a.pool_dx_nhwc = o.pool_dx_nhwc;
    a.p16 = o.p16;
    a.p16_pixels = (int64_t)g.n * g.h * g.w * (o.pool_dx != nullptr ? 4 : 1);
    a.acc_store = mode == RC_FUSED ? nullptr : o.acc_store;
    a.spec2 = spec2;
    a.spec_cooldown = spec_cooldown();
    // the hint slot (the speculative pair's, and the fused mode's speculative epilogue): forward or
    // input gradient, by the operands or the caller's dgrad_slot, so the two directions never share it
    a.hint = (spec || mode == RC_FUSED) && bar != nullptr ? bar + (16 + (dg || o.dgrad_slot ? 1 : 0)) * BAR_LINE : nullptr;
    a.hint_scale = dg || o.dgrad_slot || !spec_scale_on() ? 0 : 1;
    if (o.p16 != nullptr && (!dg || !rowconv_p16_ok(g, o.pool_dx != nullptr))) return hipErrorInvalidValue;
    if (o.pool_out != nullptr && (R % 2 != 0 || g.h % 2 != 0)) return hipErrorInvalidValue;
    if (mode == RC_FUSED) {
        if (bar == nullptr || err == nullptr || epoch == 0 || !rowconv_fused_ok(g, dg)) return hipErrorInvalidValue;
        return dg ? launch_rc<RC_FUSED, true>(Wk, R, a.wgs, a, st, ks) : launch_rc<RC_FUSED, false>(Wk, R, a.wgs, a, st, ks);
    }
    int grid = a.wgs;
    grid = grid > 1024 ? 1024 : grid;
    if (seg) {  // one resident wave of blocks, each streaming its tiles through one pipeline (seg_run)
        // an input gradient without a pool gradient takes the instantiation without the pool window's
        // registers (252 VGPRs at R = 2: two blocks per CU instead of one)
        ks = mode == RC_REQUANT && dg && o.pool_dx != nullptr ? 1 : 0;
        const void* f = mode == RC_RANGE ? rc_kernel<RC_RANGE, false>(0, R, false, 0)
                                         : (dg ? rc_kernel<RC_REQUANT, true>(0, R, false, ks)
                                               : rc_kernel<RC_REQUANT, false>(0, R, false, 0));
        const int res = resident_wgs(f);
        if (res > 0 && grid > res) grid = res;
    }
    if (mode == RC_RANGE) return launch_rc<RC_RANGE, false>(Wk, R, grid, a, st, ks);
    return dg ? launch_rc<RC_REQUANT, true>(Wk, R, grid, a, st, ks) : launch_rc<RC_REQUANT, false>(Wk, R, grid, a, st, ks);
}

// ---- the classifier head's weight gradient ------------------------------------------------------
// dw[co][ci] = Σ_p dy[p][co] x[p][ci] (exact int32) for co < 32: one workgroup per 32-channel ci
// block, its four waves taking 32-pixel K chunks round robin.  A chunk's x [32 px][32 ci] and dy
// [32 px][32 co] tiles go through the wave's own LDS slot and come back K-major by
// ds_read_b64_tr_b8 (16-lane group g: channels 16 (g & 1) .. + 15, pixels 16 (g >> 1) .. + 15 = the
// MFMA fragment of lanes 16 g .. 16 g + 15); the waves' tiles are summed through LDS, written
// into dw (OHWI16 rows of cip) and their max published (NITI_RangeEstimate, single device).
__global__ void __launch_bounds__(256) head_wgrad_kernel(const int8_t* __restrict__ x, int xld,
                                                         const int8_t* __restrict__ dy, int dld, int n, int c_out,
                                                         int cip, int32_t* __restrict__ dw, uint32_t* amax) {
    __shared__ __attribute__((aligned(16))) int8_t tile[4][2][32 * 32];
    __shared__ int32_t part[4][16][64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int ci0 = blockIdx.x * 32;
    const __amdgpu_buffer_rsrc_t rX = make_rsrc(x, (uint32_t)((int64_t)n * xld));
    const __amdgpu_buffer_rsrc_t rD = make_rsrc(dy, (uint32_t)((int64_t)n * dld));
    const int lp = lane >> 1, lh = (lane & 1) * 16;  // staging: pixel, 16-byte half
    const int g = lane >> 4, j = lane & 15;
    v16i acc = {};
    for (int p0 = wid * 32; p0 < n; p0 += 128) {
        const int p = p0 + lp;
        const v4i xv = buf_load16(rX, p < n && ci0 + lh < xld ? (uint32_t)(p * xld + ci0 + lh) : OOB);
        const v4i dv = buf_load16(rD, p < n && lh < dld ? (uint32_t)(p * dld + lh) : OOB);
        *(v4i*)(&tile[wid][0][lp * 32 + lh]) = xv;
        *(v4i*)(&tile[wid][1][lp * 32 + lh]) = dv;
        v4i fr[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int8_t* b = &tile[wid][t][(16 * (g >> 1) + (j >> 1)) * 32 + 16 * (g & 1) + 8 * (j & 1)];
            const v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(b));
            const v2i hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(b + 8 * 32));
            fr[t] = v4i{lo[0], lo[1], hi[0], hi[1]};
        }
        // lane 16 g + j now holds channel 16 (g & 1) + j = lane & 31 and pixels 16 (g >> 1) + 0..15 =
        // 16 (lane >> 5) + 0..15: the MFMA fragment as it is; A = dy (rows co), B = x (columns ci)
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(fr[1], fr[0], acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) part[wid][i][lane] = acc[i];
    __syncthreads();
    if (wid != 0) return;
    uint32_t m = 0;
    const int ci = ci0 + (lane & 31), h = lane >> 5;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int32_t v = part[0][i][lane] + part[1][i][lane] + part[2][i][lane] + part[3][i][lane];
        const int co = 8 * (i >> 2) + 4 * h + (i & 3);
        if (co < c_out && ci < cip) {
            dw[(int64_t)co * cip + ci] = v;
            m = max(m, uabs32(v));
        }
    }
    m = wave_max(m);
    if (lane == 0 && amax != nullptr) publish_max(amax, m);
}

hipError_t head_wgrad(int n, int c_out, int cip, const int8_t* x, int xld, const int8_t* dy, int dld, int32_t* dw,
                      uint32_t* amax, hipStream_t st) {
    if (n <= 0 || c_out <= 0 || c_out > 32 || cip % 32 != 0 || xld < cip || dld < c_out || dld > 32) return hipErrorInvalidValue;
    if (xld % 16 != 0 || dld % 16 != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(head_wgrad_kernel, dim3((unsigned)(cip / 32)), dim3(256), 0, st, x, xld, dy, dld, n, c_out, cip,
                       dw, amax);
    return hipGetLastError();
}

// A 1x1 layer over 1x1 maps (the classifier head) on the same kernel with W = 1: out[n][cop] (or
// the input gradient's epilogues) = requant(Σ_k x[n][k] w[row][k]) for rows = cop channels.
bool rowconv_fc_ok(int n, int K, int rows, bool fused) {
    if (n <= 0 || K <= 0 || rows <= 0) return false;
    const int64_t wgs = (int64_t)((n + 31) / 32 + 3) / 4 * ((rows + 31) / 32);
    if (!fused) return true;
    // either epilogue form: the resident limit of the smaller-occupancy instantiation
    const int cap = std::min(resident_wgs(rc_kernel<RC_FUSED, false>(1, 1, false, 0)),
                             resident_wgs(rc_kernel<RC_FUSED, true>(1, 1, false, 0)));
    return wgs <= cap;
}

hipError_t rowconv_fc(int n, int K, int rows, const int8_t* x, int xld, const int8_t* w, int wld,
                      const RowConvOut& o, int mode, uint32_t* amax, uint32_t* bar, uint32_t epoch, uint32_t* err,
                      hipStream_t st) {
    if (!rowconv_fc_ok(n, K, rows, mode == RC_FUSED) || x == nullptr || w == nullptr || amax == nullptr)
        return hipErrorInvalidValue;
    const bool spec = mode == RC_SPEC_A || mode == RC_SPEC_B;
    if (spec && bar == nullptr) return hipErrorInvalidValue;
    const int spec2 = spec ? mode - RC_SPEC_A + 1 : 0;
    if (spec) mode = RC_REQUANT;
    if (xld % 16 != 0 || wld % 16 != 0 || xld < K || wld < K) return hipErrorInvalidValue;
    // an output: NHWC16 out, the pool gradient, or (input gradient) only the C32 / P16 copies
    if (mode != RC_RANGE && o.out == nullptr && o.pool_dx == nullptr && o.next == nullptr && o.p16 == nullptr)
        return hipErrorInvalidValue;
    if (o.pool_out != nullptr || o.pool_code_out != nullptr || (o.pool_code != nullptr && o.pool_dx == nullptr) ||
        (o.pool_dx != nullptr && o.pool_code == nullptr && (o.pool_x == nullptr || o.pool_y == nullptr)))
        return hipErrorInvalidValue;
    const int64_t xb = (int64_t)n * xld, wb = (int64_t)rows * wld;
    if (xb > 0x7fffffff || wb > 0x7fffffff) return hipErrorInvalidValue;
    RowConvArgs a{};
    a.x = x;
    a.wf = w;
    a.xbytes = (uint32_t)xb;
    a.wbytes = (uint32_t)wb;
    a.xld = xld;
    a.wld = wld;
    a.K = K;
    a.rows = rows;
    a.n = n;
    a.CB = 0;
    a.COB = (rows + 31) / 32;
    a.nbands = 1;
    a.ngb = (n + 31) / 32;
    a.ngb4 = (a.ngb + 3) / 4 * 4;
    a.wgs = a.COB * a.ngb4 / 4;
    a.out = o.out;
    a.cop = (rows + 15) / 16 * 16;
    a.next = o.next;
    a.exp_in = o.exp_in;
    a.wscale = o.wscale;
    a.exp_out = o.exp_out;
    a.relu = o.relu;
    a.amax = amax;
    a.bar = bar;
    a.epoch = epoch;
    a.err = err;
    a.spin_limit = g_rc_spin_limit;
    a.expect_extra = g_rc_expect_extra;
    a.spec = g_rc_spec;
    a.stamps = nullptr;
    a.relu_mask = o.relu_mask;
    a.pool_x = o.pool_x;
    a.pool_y = o.pool_y;
    a.pool_dx = o.pool_dx;
    a.pool_dx_next = o.pool_dx_next;
    a.pool_relu = o.pool_relu;
    a.pool_code = o.pool_code;
    a.pool_dx_nhwc = o.pool_dx_nhwc;
    a.p16 = o.p16;
    a.p16_pixels = (int64_t)n * (o.pool_dx != nullptr ? 4 : 1);
    const bool dg = o.relu_mask != nullptr || o.pool_dx != nullptr || o.p16 != nullptr;
    a.spec2 = spec2;
    a.spec_cooldown = spec_cooldown();
    // the hint slot (the speculative pair's, and the fused mode's speculative epilogue): forward or
    // input gradient, by the operands or the caller's dgrad_slot, so the two directions never share it
    a.hint = (spec || mode == RC_FUSED) && bar != nullptr ? bar + (16 + (dg || o.dgrad_slot ? 1 : 0)) * BAR_LINE : nullptr;
    a.hint_scale = dg || o.dgrad_slot || !spec_scale_on() ? 0 : 1;
    if (o.p16 != nullptr && (o.pool_dx == nullptr || a.p16_pixels % 16 != 0)) return hipErrorInvalidValue;
    if (o.next != nullptr && a.cop % 32 != 0) return hipErrorInvalidValue;
    if (mode == RC_FUSED) {
        if (bar == nullptr || err == nullptr || epoch == 0) return hipErrorInvalidValue;
        return dg ? launch_rc<RC_FUSED, true>(1, 1, a.wgs, a, st) : launch_rc<RC_FUSED, false>(1, 1, a.wgs, a, st);
    }
    const int grid = a.wgs > 1024 ? 1024 : a.wgs;
    if (mode == RC_RANGE) return launch_rc<RC_RANGE, false>(1, 1, grid, a, st);
    return dg ? launch_rc<RC_REQUANT, true>(1, 1, grid, a, st) : launch_rc<RC_REQUANT, false>(1, 1, grid, a, st);
}

}  // namespace niti
