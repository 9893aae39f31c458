// niti_sgd.hpp -- the range / PSTO helpers and one NITI_SGD tile, shared by the GEMM epilogues,
// the update launch (niti_kernels.hip) and the fused row kernels' side updates (niti_rowconv.hip).
#pragma once

#include "niti_device.hpp"
#include "niti_kernels.hpp"

#ifndef NITI_SGD_NT
#define NITI_SGD_NT 0  // diagnostics: nontemporal loads of the int32 gradient in the update
#endif
#ifndef NITI_SGD_PREFETCH
#define NITI_SGD_PREFETCH 0  // diagnostics: the update loads the next tile before finishing this one
#endif

namespace niti {

// NITI_RangeEstimate on the max word: ceil(log2(m)), 0 for m <= 1.
__device__ __forceinline__ int bitwidth_of(uint32_t m) { return m <= 1u ? 0 : 32 - __clz((int)(m - 1u)); }

__device__ __forceinline__ int32_t clip127(int32_t a) { return a > 127 ? 127 : (a < -127 ? -127 : a); }

// (1 << s) as the reference's x86 build executes it for a run-time s (count & 31).
__device__ __forceinline__ int32_t pow2_x86(int s) { return (int32_t)(1u << ((unsigned)s & 31u)); }

// NITI_MNNPstoShiftInt32 (CommonOptFunction.cpp:1595-1627), exact for any shift the
// reference can produce; the fast path covers 0 <= s <= 30.
__device__ __forceinline__ int32_t psto_fast(int32_t a, int s) {
    const uint32_t ua = a < 0 ? 0u - (uint32_t)a : (uint32_t)a;
    const uint32_t q = ua >> s;
    const uint32_t prob = ua & ((1u << s) - 1u);
    const int h = s >> 1;
    const uint32_t qp = prob >> h;
    uint32_t pr = prob & ((1u << h) - 1u);
    if (s & 1) pr <<= 1;
    const int32_t r = (int32_t)q + (qp > pr ? 1 : 0);
    return clip127(a < 0 ? -r : r);
}

__device__ inline int32_t psto_generic(int32_t a, int s) {
    const int32_t p = pow2_x86(s);
    const int32_t q = a / p;
    int32_t prob = (int32_t)((uint32_t)a - (uint32_t)q * (uint32_t)p);
    prob = prob < 0 ? -prob : prob;
    const int32_t hp = pow2_x86(s / 2);
    const int32_t qp = prob / hp;
    int32_t pr = (int32_t)((uint32_t)prob - (uint32_t)qp * (uint32_t)hp);
    if (s % 2 == 1) pr = (int32_t)((uint32_t)pr * 2u);
    const int32_t sg = a > 0 ? 1 : (a < 0 ? -1 : 0);
    return clip127((int32_t)((uint32_t)q + (uint32_t)((qp > pr) * sg)));
}

__device__ __forceinline__ int32_t psto_any(int32_t a, int s) {
    return (s >= 0 && s <= 30) ? psto_fast(a, s) : psto_generic(a, s);
}

// One 64 (co) x 64 (ci) tile of tap k of a layer's NITI_SGD step (NITI_SGD.hpp:20-54,
// CPUBinary.cpp:424-426): g = PSTO(acc, bw - rule) (NITI_GradientConv_Int8.cpp:274-296), w <- clip(w - g,
// +-127), and the weight copies the next step's kernels read.  256 threads; T: 64 x 68 bytes of LDS.
// Split in two so a caller can have a tile's operands in flight while it works on another (or
// while it reads the gradient's range): sgd_tile_load issues the loads, sgd_tile_finish the rest.
struct SgdTileIn {
    v4i a[4];  // this thread's 16 gradient words
    v16c w;    // and its 16 weights
};
__device__ __forceinline__ void sgd_tile_load(const SgdJob& J, int ci0, int co0, int k, SgdTileIn& in) {
    const int t = threadIdx.x;
    const int r = t >> 2, c = (t & 3) * 16;
    if (co0 + r < J.co && ci0 + c < J.cip) {
        const int64_t idx = ((int64_t)(co0 + r) * J.kk + k) * J.cip + ci0 + c;
        const v4i* a4 = (const v4i*)(J.acc + idx);
#pragma unroll
        for (int q = 0; q < 4; ++q) in.a[q] = NITI_SGD_NT ? __builtin_nontemporal_load(a4 + q) : a4[q];
        in.w = *(const v16c*)(J.w + idx);
    }
}
__device__ __forceinline__ void sgd_tile_finish(const SgdJob& J, int bw, int ci0, int co0, int k, const SgdTileIn& in,
                                                int8_t (*T)[64 + 4]) {
    const int t = threadIdx.x;
    const int sh = bw - J.rule;
    {
        const int r = t >> 2, c = (t & 3) * 16;
        v16c wn;
#pragma unroll
        for (int j = 0; j < 16; ++j) wn[j] = 0;
        if (co0 + r < J.co && ci0 + c < J.cip) {
            const int64_t idx = ((int64_t)(co0 + r) * J.kk + k) * J.cip + ci0 + c;
            v16c g;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const v4i v = in.a[q];
#pragma unroll
                for (int e = 0; e < 4; ++e) g[q * 4 + e] = (signed char)(bw == 0 ? 0 : psto_any(v[e], sh));
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) wn[j] = (signed char)clip127((int32_t)in.w[j] - (int32_t)g[j]);
            *(v16c*)(J.w + idx) = wn;
            if (J.g_out != nullptr) *(v16c*)(J.g_out + idx) = g;
            if (J.wf != nullptr) {  // WF [co/32][ci/32][9][2][32][16]: this row's 16 ci of one co
                const int o = co0 + r, i0 = ci0 + c, cb = (J.ci + 31) / 32;
                *(v16c*)(J.wf + (((((int64_t)(o >> 5) * cb + (i0 >> 5)) * 9 + k) * 2 + ((i0 >> 4) & 1)) * 32 + (o & 31)) * 16) = wn;
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) T[r][c + j] = wn[j];
    }
    __syncthreads();
    if (J.wT != nullptr || J.wft != nullptr || J.subw != nullptr) {
        const int r = t >> 2, c = (t & 3) * 16;  // r: ci within the tile, c: co offset
        if (ci0 + r < J.ci && co0 + c < J.cop) {
            v16c o;
#pragma unroll
            for (int j = 0; j < 16; ++j) o[j] = T[c + j][r];
            if (J.wT != nullptr) *(v16c*)(J.wT + ((int64_t)(ci0 + r) * J.kk + k) * J.cop + co0 + c) = o;
            if (J.subw != nullptr) {  // the sub-pixel class copy: class of the tap, then [ci][jy][jx][cop]
                const int ky = k / J.sub_kw, kx = k - ky * J.sub_kw;
                const int py = (ky - J.sub_pt) & 1, px = (kx - J.sub_pl) & 1;
                auto taps = [](int kn, int pad, int par) {
                    const int k0 = (par + pad) & 1;
                    return k0 < kn ? (kn - k0 + 1) / 2 : 0;
                };
                int64_t off = 0;
                for (int cl = 0; cl < py * 2 + px; ++cl)
                    off += (int64_t)taps(J.sub_kh, J.sub_pt, cl >> 1) * taps(J.sub_kw, J.sub_pl, cl & 1) * J.ci * J.cop;
                const int ny = taps(J.sub_kh, J.sub_pt, py), nx = taps(J.sub_kw, J.sub_pl, px);
                *(v16c*)(J.subw + off + (((int64_t)(ci0 + r) * ny + (ky >> 1)) * nx + (kx >> 1)) * J.cop + co0 + c) = o;
            }
            if (J.wft != nullptr) {  // the input gradient's WF: output channel ci, k = 16 co, tap 8 - k
                const int i = ci0 + r, o0 = co0 + c, ob = (J.co + 31) / 32;
                *(v16c*)(J.wft + (((((int64_t)(i >> 5) * ob + (o0 >> 5)) * 9 + (8 - k)) * 2 + ((o0 >> 4) & 1)) * 32 + (i & 31)) * 16) = o;
            }
        }
    }
}
__device__ __forceinline__ void sgd_tile(const SgdJob& J, int bw, int ci0, int co0, int k, int8_t (*T)[64 + 4]) {
    SgdTileIn in;
    sgd_tile_load(J, ci0, co0, k, in);
    sgd_tile_finish(J, bw, ci0, co0, k, in, T);
}

// NITI_LOSS_Grad rows (niti_kernels.hip loss_grad*, niti_head.hip): see loss_grad in niti_kernels.hpp
__device__ __forceinline__ int64_t ipow2_64(int64_t t) { return (int64_t)pow2_x86((int)(t & 31)); }
// v / ipow2_64(k) (C division, truncation toward zero) by shifts: the divisor is 2^(k & 31) as an
// int32, so -2^31 when k & 31 == 31 (no 64-bit division)
__device__ __forceinline__ int64_t div_pow2_x86(int64_t v, int64_t k) {
    const int e = (int)(k & 31);
    const int64_t q = v >= 0 ? (v >> e) : -((-v) >> e);
    return e == 31 ? -q : q;
}

// NITI_CPULossGrad_Int8.cpp:81-200 for rows of at most 16 classes: a 16-lane group per sample,
// one lane per class, the row's max and sums reduced across the group (int64, exact).  (The
// first form ran a thread per sample with the class row in registers: 16 sequential 64-bit
// divisions per thread on 4 waves, 12 us for batch 256.)
constexpr int LOSS_MAXC = 16;
// max / sum over each 16-lane group, every lane receiving it, with DPP moves (no LDS round trips):
// lane ^ 1 and lane ^ 2 inside each quad, then rotations of the 16-lane row by 4 and 8
template <int CTRL>
__device__ __forceinline__ int64_t dpp64(int64_t v) {
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)((uint64_t)v >> 32), CTRL, 0xF, 0xF, false);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ int64_t group16_reduce(int64_t v, bool is_max) {
    auto op = [&](int64_t w) { v = is_max ? (v > w ? v : w) : v + w; };
    op(dpp64<0xB1>(v));   // quad_perm [1,0,3,2]
    op(dpp64<0x4E>(v));   // quad_perm [2,3,0,1]
    op(dpp64<0x124>(v));  // row_ror:4
    op(dpp64<0x128>(v));  // row_ror:8
    return v;
}
// a / b with C semantics (truncation toward zero) for |a|, |b| < 2^52, b != 0: the correctly rounded
// double quotient is within one of the integer one; the remainder's sign and size fix it (no 64-bit
// integer division)
__device__ __forceinline__ int64_t div_trunc52(int64_t a, int64_t b) {
    int64_t q = (int64_t)__builtin_trunc((double)a / (double)b);
    const int64_t r = a - q * b;
    const bool same = (a >= 0) == (b > 0);
    if (r != 0 && (r > 0) != (a > 0))
        q += same ? -1 : 1;
    else if ((r >= 0 ? r : -r) >= (b >= 0 ? b : -b))
        q += same ? 1 : -1;
    return q;
}
__device__ __forceinline__ void loss_rows16(const int8_t* __restrict__ logits, int batch, int classes, int ld,
                                            const int8_t* __restrict__ ascale_p, const int32_t* __restrict__ labels,
                                            int8_t* __restrict__ out, int t) {
    const int i = t >> 4, j = t & 15;
    const bool row = i < batch;  // whole groups stay in the shuffles
    const bool cls = row && j < classes;
    const int as = (int)*ascale_p;
    const int8_t* L = logits + (int64_t)(row ? i : 0) * ld;
    int64_t o = 0;
    if (as > -7) {
        int64_t sv = INT64_MIN;
        if (cls) {
            int64_t v = (int64_t)L[j] * 47274;
            v = v / (1 << 15);
            sv = as >= 0 ? v * ipow2_64(as) : div_pow2_x86(v, -as);
        }
        const int64_t mx = group16_reduce(sv, true) - 10;
        int64_t d = cls ? sv - mx : 0;
        d = d > 0 ? d : 0;
        o = cls ? ipow2_64(d) - 1 : 0;
    } else {
        const int64_t base = ipow2_64(1 - 2 * (int64_t)as);
        const int64_t sb = ipow2_64(1 - (int64_t)as);
        const int64_t v = cls ? L[j] : 0;
        o = cls ? base + v * sb + v * v : 0;
    }
    const int64_t sum = group16_reduce(o, false);
    // |o| < 2^39 and |sum| < 2^43 (o = 2^d - 1 with d <= 31, or base + v sb + v^2 with base, sb <=
    // 2^31 and |v| <= 128), so o * 2^11 and sum stay inside div_trunc52's range
    o = cls ? (sum != 0 ? div_trunc52(o * (1 << 11), sum) : 0) : 0;
    const int64_t gs = group16_reduce(o, false);
    if (!row) return;
    const int32_t gf = (int32_t)(j == labels[i] ? o - gs : o);
    int8_t* O = out + (int64_t)i * ld;
    if (j < ld) O[j] = cls ? (int8_t)psto_any(gf, 4) : (int8_t)0;
    for (int jj = j + 16; jj < ld; jj += 16) O[jj] = 0;
}
// The same row with one thread per sample (the head chain: one workgroup takes every row, so a
// 16-lane group per row would take n / 16 dependent passes): the classes in a loop, the one division
// per class on the double path (div_trunc52).  Identical results to loss_rows16.
__device__ __forceinline__ void loss_row_serial(const int8_t* __restrict__ L, int classes, int as, int label,
                                                int8_t* __restrict__ out, int ld) {
    int64_t o[LOSS_MAXC];
    if (as > -7) {
        int64_t sv[LOSS_MAXC];
        int64_t mx = INT64_MIN;
#pragma unroll
        for (int j = 0; j < LOSS_MAXC; ++j) {
            sv[j] = INT64_MIN;
            if (j < classes) {
                int64_t v = (int64_t)L[j] * 47274;
                v = v / (1 << 15);
                sv[j] = as >= 0 ? v * ipow2_64(as) : div_pow2_x86(v, -as);
                mx = mx > sv[j] ? mx : sv[j];
            }
        }
        mx -= 10;
#pragma unroll
        for (int j = 0; j < LOSS_MAXC; ++j) {
            int64_t d = j < classes ? sv[j] - mx : 0;
            d = d > 0 ? d : 0;
            o[j] = j < classes ? ipow2_64(d) - 1 : 0;
        }
    } else {
        const int64_t base = ipow2_64(1 - 2 * (int64_t)as);
        const int64_t sb = ipow2_64(1 - (int64_t)as);
#pragma unroll
        for (int j = 0; j < LOSS_MAXC; ++j) {
            const int64_t v = j < classes ? L[j] : 0;
            o[j] = j < classes ? base + v * sb + v * v : 0;
        }
    }
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < LOSS_MAXC; ++j) sum += o[j];
    int64_t gs = 0;
#pragma unroll
    for (int j = 0; j < LOSS_MAXC; ++j) {
        o[j] = j < classes ? (sum != 0 ? div_trunc52(o[j] * (1 << 11), sum) : 0) : 0;
        gs += o[j];
    }
#pragma unroll
    for (int j = 0; j < LOSS_MAXC; ++j) {
        const int32_t gf = (int32_t)(j == label ? o[j] - gs : o[j]);
        if (j < ld) out[j] = j < classes ? (int8_t)psto_any(gf, 4) : (int8_t)0;
    }
    for (int j = LOSS_MAXC; j < ld; ++j) out[j] = 0;
}
}  // namespace niti
