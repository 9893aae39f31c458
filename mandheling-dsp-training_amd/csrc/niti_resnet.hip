// niti_resnet.hip -- the element-wise pieces a ResNet step adds to the NITI ops: the residual add
// (and the gradient sum at a block input) with power-of-two exponent alignment, and the global
// sum pool with its gradient.
//
// The reference defines no residual rule: NITI_Eltwise_Int8 is an empty stub
// (execution-engine/source/backend/cpu/NITI_Eltwise_Int8.cpp:20-28).  The rule here keeps NITI's
// integer-only arithmetic and its one requantisation per tensor:
//   z = hi * 2^d + (lo >> r)        d = min(|ea - eb|, 23), r = |ea - eb| - d  (arithmetic shift)
// where hi is the operand with the larger exponent (a on ties) and lo the other one; z is exact in
// int32 (128 * 2^23 + 128 < 2^31) with exponent e_hi - d.  z then takes the forward path's range
// estimate and PSTO requantisation (requant_act: shift = bitwidth(max|z|) - 7, exponent
// e_z + inc), relu included for a block output.  The global pool is the sum over the pixels
// (int32, the exponent unchanged) followed by the same requantisation; its gradient hands dy to
// every pixel of the image.  oracle/niti_resnet_ref.py restates all three.  The fused form
// (residual_requant in niti_kernels.hip) takes the range in a pass without z and recomputes z
// from the int8 operands while requantising: 2 x 2 int8 reads instead of an int32 write + read.
#include "niti_device.hpp"
#include "niti_gridbar.hpp"
#include "niti_kernels.hpp"
#include "niti_sgd.hpp"

namespace niti {

__global__ void __launch_bounds__(256) residual_add_kernel(const int8_t* __restrict__ a, const int8_t* __restrict__ ea,
                                                           const int8_t* __restrict__ b, const int8_t* __restrict__ eb,
                                                           int64_t n16, int32_t* __restrict__ z,
                                                           int8_t* __restrict__ ez, uint32_t* __restrict__ amax) {
    const int xa = *ea, xb = *eb;
    const bool a_hi = xa >= xb;
    const int diff = a_hi ? xa - xb : xb - xa;
    const int d = diff < 23 ? diff : 23, r = diff - d;
    if (blockIdx.x == 0 && threadIdx.x == 0 && ez != nullptr) *ez = (int8_t)((a_hi ? xa : xb) - d);
    uint32_t m = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const v16c va = ((const v16c*)a)[i], vb = ((const v16c*)b)[i];
        v4i out[4];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int32_t hi = a_hi ? va[e] : vb[e], lo = a_hi ? vb[e] : va[e];
            const int32_t s = residual_z(hi, lo, d, r);
            out[e >> 2][e & 3] = s;
            const uint32_t u = uabs32(s);
            m = m > u ? m : u;
        }
        if (z != nullptr)  // else the range pass of the fused form (residual_requant)
#pragma unroll
            for (int q = 0; q < 4; ++q) ((v4i*)z)[4 * i + q] = out[q];
    }
    if (amax != nullptr) {
        m = wave_max(m);
        __shared__ uint32_t red[4];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(amax, max(max(red[0], red[1]), max(red[2], red[3])));
    }
}

hipError_t residual_add(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n,
                        int32_t* z, int8_t* ez, uint32_t* amax, hipStream_t st) {
    if (n < 0 || n % 16 != 0 || !a || !b || !ea || !eb || (!z && !amax)) return hipErrorInvalidValue;
    const int64_t n16 = n / 16;
    int64_t blocks = (n16 + 255) / 256;
    blocks = blocks < 1 ? 1 : blocks > 2048 ? 2048 : blocks;
    hipLaunchKernelGGL(residual_add_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, ea, b, eb, n16, z, ez, amax);
    return hipGetLastError();
}

// The single-launch form of residual_add + residual_requant (single device): every thread keeps
// its VPT 16-byte chunks of both operands in registers, the grid barrier of the fused row kernels
// (niti_gridbar.hpp) folds the tensor's range into its arrival, and z is recomputed from the
// registers and requantised -- one read of a and b, one write of the output, one launch.  Measured
// slower than the two launches on MI355X (ResNet-18 batch 128: 17.5 vs 14.0 us at 401 K chunks,
// 11-13 vs 9.9 us at 200 K; a kernel boundary costs ~1 us here, the grid barrier and the
// register-bound occupancy more), so ResNetModel runs it only with NITI_RES_FUSED=1.
struct ResFused {
    const int8_t *a, *ea, *b, *eb;
    int64_t n16;
    int8_t *ez, *exp_out;
    int relu;
    const int8_t* relu_mask;
    int8_t* out;
    uint32_t* bar;
    uint32_t epoch;
    uint32_t* err;
};

// byte k of a packed word, sign-extended
__device__ __forceinline__ int32_t sbyte(uint32_t w, int k) { return (int32_t)(w << (24 - 8 * k)) >> 24; }

template <int VPT, bool MASK>
__global__ void __launch_bounds__(256) residual_fused_kernel(ResFused p) {
    const int xa = *p.ea, xb = *p.eb;
    const bool a_hi = xa >= xb;
    const int diff = a_hi ? xa - xb : xb - xa;
    const int d = diff < 23 ? diff : 23, r = diff - d;
    const int64_t stride = (int64_t)gridDim.x * 256, i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    // the operands stay packed (4 words per 16 bytes: 12 VGPRs per chunk with the mask), so the grid
    // that holds a ResNet-18 block output at batch 128 fits the GPU at once
    v4i hi[VPT], lo[VPT], mk[MASK ? VPT : 1];
    uint32_t m = 0;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const int64_t i = i0 + v * stride;
        if (i < p.n16) {
            const v4i va = ((const v4i*)p.a)[i], vb = ((const v4i*)p.b)[i];
            hi[v] = a_hi ? va : vb;
            lo[v] = a_hi ? vb : va;
            if (MASK) mk[MASK ? v : 0] = ((const v4i*)p.relu_mask)[i];  // lands during the barrier
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t u = uabs32(residual_z(sbyte(hi[v][q], k), sbyte(lo[v][q], k), d, r));
                    m = m > u ? m : u;
                }
        }
    }
    __shared__ uint32_t red[4];
    __shared__ int gbw;
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const uint32_t bm = max(max(red[0], red[1]), max(red[2], red[3]));
        grid_bw_arrive(p.bar, p.epoch, bitwidth_of(bm), lane);
        const int g = grid_bw_wait(p.bar, p.epoch, p.err, BAR_SPIN_LIMIT, 0u, lane);
        if (lane == 0) gbw = g;
    }
    __syncthreads();
    const int shift = gbw - 7;  // as residual_requant_kernel (niti_kernels.hip)
    const int s = shift > 1 ? shift : 2;
    const bool raw = shift <= 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int e_z = (a_hi ? xa : xb) - d;
        if (p.ez != nullptr) *p.ez = (int8_t)e_z;
        if (p.exp_out != nullptr) *p.exp_out = (int8_t)(e_z + (shift > 1 ? shift : (shift == 1 ? 2 : 0)));
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const int64_t i = i0 + v * stride;
        if (i < p.n16) {
            v4i q;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t word = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int32_t z = residual_z(sbyte(hi[v][w], k), sbyte(lo[v][w], k), d, r);
                    int32_t o = raw ? (int32_t)(int8_t)z : psto_fast(z, s);
                    if (p.relu && o < 0) o = 0;
                    if (MASK && sbyte(mk[MASK ? v : 0][w], k) <= 0) o = 0;
                    word |= ((uint32_t)o & 0xffu) << (8 * k);
                }
                q[w] = (int)word;
            }
            ((v4i*)p.out)[i] = q;
        }
    }
}

hipError_t residual_fused(const int8_t* a, const int8_t* ea, const int8_t* b, const int8_t* eb, int64_t n, int8_t* ez,
                          int8_t* exp_out, int relu, int8_t* out, uint32_t* bar, uint32_t epoch, uint32_t* err,
                          hipStream_t st, const int8_t* relu_mask) {
    if (n < 0 || n % 16 != 0 || !a || !b || !ea || !eb || !out || !bar || !err || epoch == 0) return hipErrorInvalidValue;
    const int64_t n16 = n / 16;
    ResFused p{a, ea, b, eb, n16, ez, exp_out, relu, relu_mask, out, bar, epoch, err};
    // the smallest per-thread depth whose grid is resident at once (the barrier needs every block)
    auto try_vpt = [&](auto vc, auto mc) -> hipError_t {
        constexpr int V = decltype(vc)::value;
        constexpr bool MK = decltype(mc)::value;
        const void* f = (const void*)residual_fused_kernel<V, MK>;
        const int64_t blocks = std::max<int64_t>(1, (n16 + 256 * V - 1) / (256 * V));
        if (blocks > resident_wgs(f)) return hipErrorNotSupported;
        hipLaunchKernelGGL((residual_fused_kernel<V, MK>), dim3((unsigned)blocks), dim3(256), 0, st, p);
        return hipGetLastError();
    };
    auto over = [&](auto mc) -> hipError_t {
        hipError_t r = try_vpt(std::integral_constant<int, 4>(), mc);
        if (r == hipErrorNotSupported) r = try_vpt(std::integral_constant<int, 5>(), mc);
        if (r == hipErrorNotSupported) r = try_vpt(std::integral_constant<int, 6>(), mc);
        if (r == hipErrorNotSupported) r = try_vpt(std::integral_constant<int, 8>(), mc);
        return r;
    };
    return relu_mask != nullptr ? over(std::true_type()) : over(std::false_type());
}

// acc[img][c] = sum over the image's hw pixels of x[img][p][c] (NHWC16, cp % 16 == 0): one thread
// per (image, channel), consecutive threads consecutive channels
__global__ void __launch_bounds__(256) sum_pool_kernel(const int8_t* __restrict__ x, int n, int hw, int cp,
                                                       int32_t* __restrict__ acc, uint32_t* __restrict__ amax) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t m = 0;
    if (t < (int64_t)n * cp) {
        const int64_t img = t / cp;
        const int c = (int)(t - img * cp);
        const int8_t* p = x + img * hw * cp + c;
        int32_t s = 0;
        for (int i = 0; i < hw; ++i) s += p[(int64_t)i * cp];
        acc[t] = s;
        m = uabs32(s);
    }
    if (amax != nullptr) {
        m = wave_max(m);
        __shared__ uint32_t red[4];
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(amax, max(max(red[0], red[1]), max(red[2], red[3])));
    }
}

hipError_t sum_pool(const int8_t* x, int n, int hw, int cp, int32_t* acc, uint32_t* amax, hipStream_t st) {
    if (n <= 0 || hw <= 0 || cp <= 0 || cp % 16 != 0 || (int64_t)hw * 127 * 2 > 0x7fffffff) return hipErrorInvalidValue;
    const int64_t t = (int64_t)n * cp;
    hipLaunchKernelGGL(sum_pool_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, x, n, hw, cp, acc, amax);
    return hipGetLastError();
}

// dx[img][p][c] = dy[img][c] for every pixel p (16-byte chunks); with relu_mask (NHWC16, the pooled
// map -- the last block's output) the relu gradient too: dx = mask > 0 ? dy : 0
__global__ void __launch_bounds__(256) sum_pool_grad_kernel(const int8_t* __restrict__ dy, int64_t total16, int hw,
                                                            int c16, const int8_t* __restrict__ relu_mask,
                                                            int8_t* __restrict__ dx) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total16; i += (int64_t)gridDim.x * 256) {
        const int64_t img = i / ((int64_t)hw * c16);
        const int ch = (int)(i % c16);
        v16c v = ((const v16c*)dy)[img * c16 + ch];
        if (relu_mask != nullptr) {
            const v16c m = ((const v16c*)relu_mask)[i];
#pragma unroll
            for (int e = 0; e < 16; ++e) v[e] = m[e] > 0 ? v[e] : (int8_t)0;
        }
        ((v16c*)dx)[i] = v;
    }
}

hipError_t sum_pool_grad(const int8_t* dy, int n, int hw, int cp, int8_t* dx, hipStream_t st, const int8_t* relu_mask) {
    if (n <= 0 || hw <= 0 || cp <= 0 || cp % 16 != 0) return hipErrorInvalidValue;
    const int64_t total16 = (int64_t)n * hw * (cp / 16);
    int64_t blocks = (total16 + 255) / 256;
    blocks = blocks > 4096 ? 4096 : blocks;
    hipLaunchKernelGGL(sum_pool_grad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dy, total16, hw, cp / 16,
                       relu_mask, dx);
    return hipGetLastError();
}

// im2col of a shallow input (NHWC16, c_in <= 4: the ResNet stem's 3 channels) for a conv that
// then runs as a 1x1 conv over kp columns: xcol[p][k], k = (ky * KW + kx) * c_in + c for
// k < KH * KW * c_in, zero beyond and outside the image.  One workgroup per output row: the KH
// input rows it reads are staged once in LDS as packed c_in-byte pixels (a dword load per input
// pixel: 4 of its 16 bytes), then every thread builds 16-byte output chunks from LDS bytes (a
// byte gather straight from HBM / L2 per output byte ran ~9x slower).  KH, KW, C as template
// arguments (the stem's 7, 7, 3) make the byte -> (tap, channel) map compile-time; 0 = run time.
constexpr int IM2COL_LDS = 16384;
// NCHW: x is int8 NCHW [n][c_in][h][w] (the input quantiser's planar output): each input row of
// each channel is a contiguous run, loaded bytewise (coalesced) -- a 16-byte NHWC16 pixel carries
// 3 useful bytes, so the NCHW source reads ~5x fewer lines.
template <int KH_, int KW_, int C_, bool NCHW>
__global__ void __launch_bounds__(256) im2col_small_kernel(const int8_t* __restrict__ x, ConvGeom g, int kp,
                                                           int8_t* __restrict__ xcol) {
    __shared__ int8_t tile[IM2COL_LDS];
    const int KH = KH_ ? KH_ : g.kh, KW = KW_ ? KW_ : g.kw, C = C_ ? C_ : g.c_in;
    const int row = blockIdx.x;  // n * oh + oy
    const int n = row / g.oh, oy = row - n * g.oh;
    const int cols = (g.ow - 1) * g.sw + (KW - 1) * g.dw + 1;  // input columns the row reads
    if constexpr (NCHW) {
        // dword loads over each (ky, c) input row's span [ix0, ix0 + cols), aligned down to 4 bytes
        // when the plane rows are (w % 4 == 0; else bytewise), 4 bytes scattered into the tile
        const int ix0 = -g.pl;
        const bool al = (g.w & 3) == 0;
        const int lead = al ? (ix0 & 3) : 0;  // bytes of the first dword before ix0
        const int nd = al ? (lead + cols + 3) / 4 : cols;
        for (int e = threadIdx.x; e < KH * C * nd; e += 256) {
            const int kc = e / nd, d = e - kc * nd;
            const int ky = kc / C, c = kc - ky * C;
            const int iy = oy * g.sh + ky * g.dh - g.pt;
            const bool row_ok = (unsigned)iy < (unsigned)g.h;
            const int8_t* rowp = x + (((int64_t)n * g.c_in + c) * g.h + (row_ok ? iy : 0)) * g.w;
            if (al) {
                const int ixa = ix0 - lead + 4 * d;  // first input column of this dword
                uint32_t v = 0;
                if (row_ok && ixa >= 0 && ixa + 3 < g.w) {
                    v = *(const uint32_t*)(rowp + ixa);
                } else if (row_ok) {
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        if ((unsigned)(ixa + b) < (unsigned)g.w) v |= (uint32_t)(uint8_t)rowp[ixa + b] << (8 * b);
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int cx = ixa + b - ix0;
                    if (cx >= 0 && cx < cols) tile[(ky * cols + cx) * C + c] = (int8_t)(v >> (8 * b));
                }
            } else {
                const int ix = ix0 + d;
                tile[(ky * cols + d) * C + c] = row_ok && (unsigned)ix < (unsigned)g.w ? rowp[ix] : (int8_t)0;
            }
        }
    } else {
        for (int e = threadIdx.x; e < KH * cols; e += 256) {
            const int ky = e / cols, cx = e - ky * cols;
            const int iy = oy * g.sh + ky * g.dh - g.pt, ix = cx - g.pl;
            uint32_t v = 0;
            if ((unsigned)iy < (unsigned)g.h && (unsigned)ix < (unsigned)g.w)
                v = *(const uint32_t*)(x + (((int64_t)n * g.h + iy) * g.w + ix) * g.cip);
#pragma unroll
            for (int c = 0; c < (C_ ? C_ : 4); ++c)
                if (C_ || c < C) tile[e * C + c] = (int8_t)(v >> (8 * c));
        }
    }
    __syncthreads();
    const int kc = kp / 16, kt = KH * KW * C;
    int8_t* out = xcol + (int64_t)row * g.ow * kp;
    // a thread keeps one 16-byte column chunk j of every output pixel it writes (ox steps by
    // 256 / kc), so the chunk's 16 tile offsets (tap and channel, without the pixel's column) are
    // computed once into registers; -1: a padding column k >= KH KW C
    const int per = 256 / kc;  // pixels per pass
    if ((int)threadIdx.x >= per * kc) return;
    const int j = threadIdx.x % kc;
    int koff[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        const int k = 16 * j + b;
        const int tap = k / C, c = k - tap * C;
        const int ky = tap / KW, kx = tap - ky * KW;
        koff[b] = k < kt ? (ky * cols + kx * g.dw) * C + c : -1;
    }
    for (int ox = threadIdx.x / kc; ox < g.ow; ox += per) {
        const int xo = ox * g.sw * C;
        v16c o;
#pragma unroll
        for (int b = 0; b < 16; ++b) o[b] = koff[b] >= 0 ? tile[xo + koff[b]] : (int8_t)0;
        *(v16c*)(out + (int64_t)ox * kp + 16 * j) = o;
    }
}

hipError_t im2col_small(const ConvGeom& g, const int8_t* x, int kp, int8_t* xcol, hipStream_t st, bool nchw) {
    // kp <= 4096: a thread keeps one 16-byte column chunk, so 256 threads cover at most 256 chunks
    if (kp % 16 != 0 || kp > 4096 || kp < g.kh * g.kw * g.c_in || g.c_in > 4 || g.cip > 16) return hipErrorInvalidValue;
    const int cols = (g.ow - 1) * g.sw + (g.kw - 1) * g.dw + 1;
    if ((int64_t)g.kh * cols * g.c_in > IM2COL_LDS) return hipErrorInvalidValue;
    const int64_t rows = (int64_t)g.n * g.oh;
    if (rows == 0) return hipSuccess;
    if (rows > 0x7fffffff) return hipErrorInvalidValue;
    const dim3 grid((unsigned)rows);
    if (g.kh == 7 && g.kw == 7 && g.c_in == 3) {
        if (nchw)
            hipLaunchKernelGGL((im2col_small_kernel<7, 7, 3, true>), grid, dim3(256), 0, st, x, g, kp, xcol);
        else
            hipLaunchKernelGGL((im2col_small_kernel<7, 7, 3, false>), grid, dim3(256), 0, st, x, g, kp, xcol);
    } else if (nchw) {
        hipLaunchKernelGGL((im2col_small_kernel<0, 0, 0, true>), grid, dim3(256), 0, st, x, g, kp, xcol);
    } else {
        hipLaunchKernelGGL((im2col_small_kernel<0, 0, 0, false>), grid, dim3(256), 0, st, x, g, kp, xcol);
    }
    return hipGetLastError();
}

}  // namespace niti
