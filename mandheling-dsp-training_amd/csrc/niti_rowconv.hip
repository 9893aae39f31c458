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

#include <algorithm>

#include "niti_device.hpp"
#include "niti_kernels.hpp"
#include "niti_map.hpp"

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

// ---- grid barrier with the max folded in (mode FUSED) -----------------------------------------
// State per parity (launch epoch & 1), every word on a 128-byte line of its own:
//   cnt[8] arrivals per shard (workgroup b joins shard b & 7), mx[8] the shard's max,
//   top_cnt shards complete, top_mx their max, gran the released {epoch, max} granule.
// Every access is an agent-scope atomic or an sc1 (agent relaxed) access, the protocol measured
// coherent across XCDs on gfx950 (MI355X_MICROARCH.md, inter-workgroup visibility): a workgroup
// max-es its shard word and only then (its atomic has returned) counts itself in; the shard's last
// arriver carries the shard max to the top, the top's last arriver releases the granule, every
// workgroup polls the granule (one lane, s_sleep, bounded).  Launch e zeroes parity (e + 1) & 1
// for the next launch: the previous launch that used it has completed (same stream).
constexpr int BAR_LINE = 32;                         // words per 128-byte line
constexpr int BAR_WORDS = (8 + 8 + 3) * BAR_LINE;    // one parity
static_assert(2 * BAR_WORDS == ROWCONV_BAR_WORDS, "barrier state size");
constexpr uint32_t BAR_SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ uint32_t* bar_word(uint32_t* base, int line) { return base + line * BAR_LINE; }

__device__ uint32_t grid_max_barrier(uint32_t* state, uint32_t epoch, uint32_t m, uint32_t* err) {
    uint32_t* S = state + (epoch & 1) * BAR_WORDS;
    const int nwg = gridDim.x;
    const int b = blockIdx.x;
    if (b == 0) {  // reset the other parity for the next launch
        uint32_t* T = state + ((epoch + 1) & 1) * BAR_WORDS;
        for (int l = 0; l < 19; ++l) __hip_atomic_store(bar_word(T, l), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long* tg = (unsigned long long*)bar_word(T, 18);
        __hip_atomic_store(tg, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int nsh = nwg < 8 ? nwg : 8;
    const int sh = b % nsh;
    const uint32_t expect = (uint32_t)((nwg - sh + nsh - 1) / nsh);  // workgroups b' < nwg with b' % nsh == sh
    (void)__hip_atomic_fetch_max(bar_word(S, 8 + sh), m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(bar_word(S, sh), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long* gran = (unsigned long long*)bar_word(S, 18);
    if (old == expect - 1) {  // this shard is complete: its max to the top
        const uint32_t smax = __hip_atomic_fetch_max(bar_word(S, 8 + sh), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        (void)__hip_atomic_fetch_max(bar_word(S, 17), smax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t t = __hip_atomic_fetch_add(bar_word(S, 16), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t == (uint32_t)nsh - 1) {  // every shard is in: release
            const uint32_t g = __hip_atomic_fetch_max(bar_word(S, 17), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(gran, ((unsigned long long)epoch << 32) | g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    uint32_t spins = 0;
    for (;;) {
        const unsigned long long v = __hip_atomic_load(gran, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(v >> 32) == epoch) return (uint32_t)v;
        if (++spins > BAR_SPIN_LIMIT) {  // never hang the GPU: flag it and go on (results invalid)
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return 0xffffffffu;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

struct RowConvArgs {
    const int8_t* x;  // C32 [n][CB][H][W][32]
    const int8_t* wf; // WF [COB][CB][9][2][32][16]
    uint32_t xbytes, wbytes;
    int n, CB, COB;
    int units, nbands;
    int8_t* out;      // NHWC16 [n][H][W][cop]
    int cop;
    int8_t* pool_out; // NHWC16 [n][H/2][W/2][cop] or null
    int8_t* next;     // C32 [n][COB][Ho][Wo][32] of the (pooled) output, or null
    const int8_t* exp_in;
    const int8_t* wscale;
    int8_t* exp_out;
    int relu;
    uint32_t* amax;   // RANGE: published; REQUANT: read
    uint32_t* bar;    // FUSED: barrier state
    uint32_t epoch;
    uint32_t* err;
};

enum RowMode { RC_FUSED = 0, RC_RANGE = 1, RC_REQUANT = 2 };

template <int W, int R>
struct RowUnit {
    static constexpr int G = 32 / W, H = W, NR = R + 2;
    int cob, b, img;
    bool img_ok;
    __device__ RowUnit(const RowConvArgs& a, int u, int c) {
        cob = u % a.COB;
        const int rest = u / a.COB;
        b = rest % a.nbands;
        img = (rest / a.nbands) * G + c / W;
        img_ok = img < a.n;
    }
};

// the accumulators of one unit: acc[r][i] = y[co = cob*32 + 8(i>>2) + 4h + (i&3)][row b*R + r][col]
template <int W, int R>
__device__ __forceinline__ void rowconv_compute(const RowConvArgs& a, const RowUnit<W, R>& U, int lane, v16i (&acc)[R]) {
    constexpr int H = W, NR = R + 2;
    const int h = lane >> 5, c = lane & 31, ox = c % W;
    const bool row_start = ox == 0, row_end = ox == W - 1;
    const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.x, a.xbytes);
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.wf, a.wbytes);
    const uint32_t xl = U.img_ok ? (uint32_t)((((int64_t)U.img * a.CB * H) * W + ox) * 32 + 16 * h) : OOB;
    const uint32_t wl = (uint32_t)(h * 512 + c * 16);
    constexpr uint32_t CHUNK = (uint32_t)H * W * 32;
    const int y0 = U.b * R - 1;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[r][i] = 0;
    v4i X[2][NR], Wt[2][9];
    auto load = [&](int buf, int cc) {
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int iy = y0 + j;
            if (iy >= 0 && iy < H)
                X[buf][j] = buf_load16(rX, xl + (uint32_t)cc * CHUNK + (uint32_t)iy * W * 32);
            else
                X[buf][j] = v4i{0, 0, 0, 0};
        }
        const uint32_t wo = (uint32_t)((U.cob * a.CB + cc) * 9) * 1024u;
#pragma unroll
        for (int t = 0; t < 9; ++t) Wt[buf][t] = buf_load16(rW, wl + wo + (uint32_t)t * 1024u);
    };
    auto compute = [&](int buf) {
        v4i XL[NR], XR[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            XL[j] = shift_in_left<W>(X[buf][j], row_start);
            XR[j] = shift_in_right<W>(X[buf][j], row_end);
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Wt[buf][3 * ky], XL[r + ky], acc[r], 0, 0, 0);
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Wt[buf][3 * ky + 1], X[buf][r + ky], acc[r], 0, 0, 0);
                acc[r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(Wt[buf][3 * ky + 2], XR[r + ky], acc[r], 0, 0, 0);
            }
    };
    load(0, 0);
    int cc = 0;
    for (; cc + 2 <= a.CB; cc += 2) {
        if (cc + 1 < a.CB) load(1, cc + 1);
        compute(0);
        if (cc + 2 < a.CB) load(0, cc + 2);
        compute(1);
    }
    if (cc < a.CB) compute(0);
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

template <int W, int R>
__device__ __forceinline__ void rowconv_epilogue(const RowConvArgs& a, const RowUnit<W, R>& U, int lane,
                                                 const v16i (&acc)[R], uint32_t gmax) {
    constexpr int H = W;
    const int h = lane >> 5, c = lane & 31, ox = c % W;
    const int shift = bitwidth_rc(gmax) - 7;
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    int8_t q[R][16];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            int32_t v = raw ? (int32_t)(int8_t)acc[r][i] : psto_rc(acc[r][i], s);
            if (a.relu && v < 0) v = 0;
            q[r][i] = (int8_t)v;
        }
    const int64_t img = U.img;
    const int cb16 = U.cob * 32 + 16 * h;  // this lane's 16 channels after pack_cols
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const v4i v = pack_cols(q[r]);
        const int oy = U.b * R + r;
        if (U.img_ok) {
            *(v4i*)(a.out + ((img * H + oy) * W + ox) * a.cop + cb16) = v;
            if (a.next != nullptr && a.pool_out == nullptr)
                *(v4i*)(a.next + (((img * a.COB + U.cob) * H + oy) * W + ox) * 32 + 16 * h) = v;
        }
    }
    if (a.pool_out != nullptr) {
        constexpr int HO = H / 2, WO = W / 2;
#pragma unroll
        for (int r = 0; r + 1 < R; r += 2) {
            int8_t pm[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int v0 = q[r][i] > q[r + 1][i] ? q[r][i] : q[r + 1][i];
                const int v1 = __shfl_xor(v0, 1, 64);
                pm[i] = (int8_t)(v0 > v1 ? v0 : v1);
            }
            const v4i v = pack_cols(pm);
            if (U.img_ok && (ox & 1) == 0) {
                const int py = (U.b * R + r) / 2, px = ox / 2;
                *(v4i*)(a.pool_out + ((img * HO + py) * WO + px) * a.cop + cb16) = v;
                if (a.next != nullptr)
                    *(v4i*)(a.next + (((img * a.COB + U.cob) * HO + py) * WO + px) * 32 + 16 * h) = v;
            }
        }
    }
}

__device__ __forceinline__ void write_exponent(const RowConvArgs& a, uint32_t gmax) {
    if (a.exp_out == nullptr) return;
    const int shift = bitwidth_rc(gmax) - 7;
    const int inc = shift > 1 ? shift : (shift == 1 ? 2 : 0);
    *a.exp_out = (int8_t)((a.exp_in ? (int)*a.exp_in : 0) + (a.wscale ? (int)*a.wscale : 0) + inc);
}

__device__ __forceinline__ uint32_t max_abs16(const v16i& v, uint32_t m) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t u = uabs32(v[i]);
        m = m > u ? m : u;
    }
    return m;
}

template <int W, int R, int MODE>
__global__ void __launch_bounds__(256) rowconv_fwd_kernel(RowConvArgs a) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int c = lane & 31;
    __shared__ uint32_t red[4];
    __shared__ uint32_t gm;
    v16i acc[R];
    if constexpr (MODE == RC_FUSED) {
        const int u = blockIdx.x * 4 + wid;
        uint32_t m = 0;
        const RowUnit<W, R> U(a, u < a.units ? u : 0, c);
        if (u < a.units) {
            rowconv_compute<W, R>(a, U, lane, acc);
#pragma unroll
            for (int r = 0; r < R; ++r) m = max_abs16(acc[r], m);
        }
        m = wave_max(m);
        if (lane == 0) red[wid] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t bm = max(max(red[0], red[1]), max(red[2], red[3]));
            const uint32_t g = grid_max_barrier(a.bar, a.epoch, bm, a.err);
            gm = g;
            if (blockIdx.x == 0) {
                publish_max(a.amax, g);  // the layer's range, for the record
                write_exponent(a, g);
            }
        }
        __syncthreads();
        if (u < a.units) rowconv_epilogue<W, R>(a, U, lane, acc, gm);
    } else if constexpr (MODE == RC_RANGE) {
        uint32_t m = 0;
        for (int u = blockIdx.x * 4 + wid; u < a.units; u += gridDim.x * 4) {
            const RowUnit<W, R> U(a, u, c);
            rowconv_compute<W, R>(a, U, lane, acc);
#pragma unroll
            for (int r = 0; r < R; ++r) m = max_abs16(acc[r], m);
        }
        m = wave_max(m);
        if (lane == 0) red[wid] = m;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(a.amax, max(max(red[0], red[1]), max(red[2], red[3])));
    } else {
        const uint32_t g = read_max(a.amax);
        if (blockIdx.x == 0 && threadIdx.x == 0) write_exponent(a, g);
        for (int u = blockIdx.x * 4 + wid; u < a.units; u += gridDim.x * 4) {
            const RowUnit<W, R> U(a, u, c);
            rowconv_compute<W, R>(a, U, lane, acc);
            rowconv_epilogue<W, R>(a, U, lane, acc, g);
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

hipError_t weights_to_wf(const int8_t* w_ohwi16, int co, int ci, int cip, bool transpose, int8_t* out,
                         hipStream_t st) {
    const int COB = transpose ? (ci + 31) / 32 : (co + 31) / 32;
    const int CB = transpose ? (co + 31) / 32 : (ci + 31) / 32;
    return launch_map((int64_t)COB * CB * 9 * 2 * 32, WeightsToWF{w_ohwi16, co, ci, cip, COB, CB, transpose, out}, st);
}

size_t rowconv_wf_bytes(int co, int ci) { return (size_t)((co + 31) / 32) * ((ci + 31) / 32) * 9 * 1024; }

// ---- host side ---------------------------------------------------------------------------------
bool rowconv_ok(const ConvGeom& g) {
    if (g.kh != 3 || g.kw != 3 || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1) return false;
    if (g.pt != 1 || g.pl != 1 || g.pb != 1 || g.pr != 1) return false;
    if (g.h != g.w || g.oh != g.h || g.ow != g.w) return false;
    if (!(g.w == 2 || g.w == 4 || g.w == 8 || g.w == 16)) return false;
    if (g.cop % 32 != 0) return false;
    return true;
}

// rows per band: the largest R (a power of two dividing H, at most 8: register budget) whose unit
// count fills the chip (>= 768 waves), else R = 2, the most units; FUSED needs one unit per wave
// and every workgroup resident (units <= 1024)
static int rowconv_rows(const ConvGeom& g, int* units_out) {
    const int W = g.w, G = 32 / W;
    const int64_t groups = (g.n + G - 1) / G, cob = g.cop / 32;
    int R = W < 8 ? W : 8;
    while (R > 2 && groups * (W / R) * cob < 768) R /= 2;
    *units_out = (int)(groups * (W / R) * cob);
    return R;
}

int rowconv_units(const ConvGeom& g) {
    int u = 0;
    (void)rowconv_rows(g, &u);
    return u;
}

bool rowconv_fused_ok(const ConvGeom& g) { return rowconv_ok(g) && rowconv_units(g) <= 4 * 256; }

template <int MODE>
static hipError_t launch_rc(int W, int R, int grid, const RowConvArgs& a, hipStream_t st) {
#define RC_CASE(WW, RR)                                                                                       \
    if (W == WW && R == RR) {                                                                                 \
        hipLaunchKernelGGL((rowconv_fwd_kernel<WW, RR, MODE>), dim3((unsigned)grid), dim3(256), 0, st, a);    \
        return hipGetLastError();                                                                             \
    }
    RC_CASE(16, 8)
    RC_CASE(16, 4)
    RC_CASE(16, 2)
    RC_CASE(8, 8)
    RC_CASE(8, 4)
    RC_CASE(8, 2)
    RC_CASE(4, 4)
    RC_CASE(4, 2)
    RC_CASE(2, 2)
#undef RC_CASE
    return hipErrorInvalidValue;
}

hipError_t rowconv_fwd(const ConvGeom& g, const int8_t* x_c32, const int8_t* wf, const RowConvOut& o, int mode,
                       uint32_t* amax, uint32_t* bar, uint32_t epoch, uint32_t* err, hipStream_t st) {
    if (!rowconv_ok(g) || x_c32 == nullptr || wf == nullptr || amax == nullptr) return hipErrorInvalidValue;
    if (mode != RC_RANGE && o.out == nullptr) return hipErrorInvalidValue;
    RowConvArgs a{};
    const int CB = (g.c_in + 31) / 32, COB = g.cop / 32;
    const int64_t xb = (int64_t)g.n * CB * g.h * g.w * 32;
    const int64_t wb = (int64_t)COB * CB * 9 * 1024;
    if (xb > 0x7fffffff || wb > 0x7fffffff) return hipErrorInvalidValue;
    a.x = x_c32;
    a.wf = wf;
    a.xbytes = (uint32_t)xb;
    a.wbytes = (uint32_t)wb;
    a.n = g.n;
    a.CB = CB;
    a.COB = COB;
    int units = 0;
    const int R = rowconv_rows(g, &units);
    a.units = units;
    a.nbands = g.h / R;
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
    if (o.pool_out != nullptr && (R % 2 != 0 || g.h % 2 != 0)) return hipErrorInvalidValue;
    if (mode == RC_FUSED) {
        if (bar == nullptr || err == nullptr || epoch == 0 || units > 4 * 256) return hipErrorInvalidValue;
        return launch_rc<RC_FUSED>(g.w, R, (units + 3) / 4, a, st);
    }
    int grid = (units + 3) / 4;
    grid = grid > 1024 ? 1024 : grid;
    if (mode == RC_RANGE) return launch_rc<RC_RANGE>(g.w, R, grid, a, st);
    return launch_rc<RC_REQUANT>(g.w, R, grid, a, st);
}

}  // namespace niti
