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

}  // namespace niti
