// niti_quant.hip -- the NITIInt8Train input quantiser on device.
//
// Reference (execution-engine/tools/train/source/demo/MnistUtils.cpp:83-93), per batch:
//     cast  = float(images)                      uint8 pixels
//     mean  = ReduceMean(cast)
//     std   = sqrt(ReduceSum((cast - mean)^2) / (batchSize * 28 * 28))   (:86, literally)
//     Y     = (cast - mean) / std
//     range = ReduceMax(|Y|)
//     ascale = int8(ceil(ln(range)) - 7)          (natural log, as written)
//     x     = int8(round(Y / range * 127))
// The reference leaves the float summation order to MNN's reduction kernels, so the only
// order-independent statement of it is in terms of exact integer statistics of the pixels:
//     S1 = sum x, S2 = sum x^2 (int64, exact), xmin, xmax
//     mean  = float(S1) / float(count)                       (= the float sequential sum while
//                                                              S1 < 2^24, e.g. LeNet batch 64)
//     ss    = double(S2) - 2 mean S1 + count mean^2           (double, no contraction)
//     std   = sqrtf(float(ss / var_count))   var_count = images x 784, the reference's literal
//                                              divisor for any image size (= count for MNIST)
//     range = max(|float(xmax - mean)|, |float(xmin - mean)|) / std   (the max of |Y| sits at
//             an extreme pixel: fl(x - mean) and fl(./std) are monotonic in x)
// and the per-pixel formula is evaluated in float in the reference's operation order.  The
// oracle (oracle/niti_oracle.c niti_ref_image_quantize) states the same contract.  This is an
// EXACT-STATISTICS CONTRACT, not a float-order match: the reference's float sums have no fixed
// order under -ffast-math (CMakeLists.txt:429-430; sequential in the C source, vector lanes when
// compiled), and its float readings (niti_ref_quantize_input_lanes, 1 / 4 / 8 / 16 lanes) move
// 0-4 of the 256 pixel-value codes by one at the per-GPU BASELINE shapes and agree on ascale
// (DESIGN.md "Input quantiser", profiles/r04_quant_parity.txt, tests/test_quant.py).  Because the statistics are integers, data-parallel ranks all-reduce them (SUM S1, S2;
// MAX xmax, 255 - xmin) and quantise their shard exactly as one device would the global batch.
// ascale is computed in float as the graph does (_Ceil(_Log(range)) on float tensors, :89-91),
// logf taken as the correctly rounded float natural log, (float)log((double)range), so host and
// device agree bit for bit.  A constant batch (std = 0) is undefined in the reference (0/0); here
// it quantises to zeros with ascale = -7.
#include "niti_device.hpp"
#include "niti_kernels.hpp"
#include "niti_map.hpp"

namespace niti {

namespace {

typedef signed char v16c __attribute__((ext_vector_type(16)));
typedef int v4i_q __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t = __shfl_xor(v, o, 64);
        v = v > t ? v : t;
    }
    return v;
}

// block b's partial statistics into slots[4 b .. 4 b + 3] = {S1, S2, xmax, 255 - xmin}: plain
// stores, no atomics (device-scope u64 atomics of many blocks on one line serialise at the memory
// side); the consumers sum the slots (stats_from_slots).  ATOMIC (the standalone op, no slot
// workspace): every block adds / maxes its partials into slots[0..3] (zeroed by the caller) -- a
// few dozen blocks' atomics, where one block over a 224x224 batch took 2.6 ms
template <bool ATOMIC>
__global__ void __launch_bounds__(256) image_stats_kernel(const uint8_t* __restrict__ img, int64_t n,
                                                          unsigned long long* __restrict__ slots,
                                                          uint4* __restrict__ zero = nullptr, int64_t zero16 = 0) {
    // a side job: the step's range words zeroed here, the step's first launch (a memset of its own
    // was a ~5 us blit launch)
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < zero16; i += (int64_t)gridDim.x * blockDim.x)
        zero[i] = uint4{0u, 0u, 0u, 0u};
    unsigned long long s1 = 0, s2 = 0;
    uint32_t mx = 0, mn = 0;  // mn holds 255 - min
    const int64_t nv = n / 16;
    const uint4* v = reinterpret_cast<const uint4*>(img);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
        const uint4 q = v[i];
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
        uint32_t a1 = 0, a2 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t p = (w[j] >> (8 * b)) & 255u;
                a1 += p;
                a2 += p * p;
                mx = p > mx ? p : mx;
                mn = 255u - p > mn ? 255u - p : mn;
            }
        s1 += a1;
        s2 += a2;
    }
    for (int64_t i = nv * 16 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t p = img[i];
        s1 += p;
        s2 += p * p;
        mx = p > mx ? p : mx;
        mn = 255u - p > mn ? 255u - p : mn;
    }
    s1 = wave_sum_u64(s1);
    s2 = wave_sum_u64(s2);
    mx = wave_max_u32(mx);
    mn = wave_max_u32(mn);
    __shared__ unsigned long long r[4][4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        r[wv][0] = s1;
        r[wv][1] = s2;
        r[wv][2] = mx;
        r[wv][3] = mn;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int k = threadIdx.x;
        unsigned long long t = 0;
        for (int w = 0; w < 4; ++w) t = k < 2 ? t + r[w][k] : (r[w][k] > t ? r[w][k] : t);
        if constexpr (ATOMIC) {
            if (k < 2)
                atomicAdd(slots + k, t);
            else
                atomicMax(slots + k, t);
        } else {
            slots[4 * blockIdx.x + k] = t;
        }
    }
}

// the whole block sums nslots partials (S1, S2 added, the maxima max-ed) into out[4] (shared)
__device__ void stats_from_slots(const unsigned long long* __restrict__ slots, int nslots, unsigned long long* out) {
    __shared__ unsigned long long r[4][4];
    unsigned long long s1 = 0, s2 = 0;
    uint32_t mx = 0, mn = 0;
    for (int b = threadIdx.x; b < nslots; b += blockDim.x) {
        s1 += slots[4 * b];
        s2 += slots[4 * b + 1];
        mx = max(mx, (uint32_t)slots[4 * b + 2]);
        mn = max(mn, (uint32_t)slots[4 * b + 3]);
    }
    s1 = wave_sum_u64(s1);
    s2 = wave_sum_u64(s2);
    mx = wave_max_u32(mx);
    mn = wave_max_u32(mn);
    const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        r[wv][0] = s1;
        r[wv][1] = s2;
        r[wv][2] = mx;
        r[wv][3] = mn;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int k = threadIdx.x;
        unsigned long long t = 0;
        for (int w = 0; w < nw; ++w) t = k < 2 ? t + r[w][k] : (r[w][k] > t ? r[w][k] : t);
        out[k] = t;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(256) stats_finalize_kernel(const unsigned long long* __restrict__ slots, int nslots,
                                                             unsigned long long* __restrict__ stats) {
    __shared__ unsigned long long t[4];
    stats_from_slots(slots, nslots, t);
    if (threadIdx.x < 4) stats[threadIdx.x] = t[threadIdx.x];
}

struct QuantParams {
    float mean, sd, range;
    int ascale;
    int ok;
};

// The contract in the file header, evaluated without floating-point contraction so the host
// oracle (gcc, x86-64: no FMA) computes the identical values.
__device__ QuantParams quant_params(const unsigned long long* stats, int64_t count, int64_t var_count) {
#pragma clang fp contract(off)
    QuantParams q;
    const double s1 = (double)stats[0], s2 = (double)stats[1];
    const float xmax = (float)stats[2], xmin = (float)(255ull - stats[3]);
    q.mean = (float)stats[0] / (float)count;
    const double m = (double)q.mean;
    const double ss = s2 - 2.0 * m * s1 + (double)count * m * m;
    const float var = (float)(ss / (double)var_count);
    q.sd = sqrtf(var > 0.f ? var : 0.f);
    q.ok = q.sd > 0.f;
    if (!q.ok) {
        q.range = 0.f;
        q.ascale = -7;
        return q;
    }
    const float hi = fabsf(xmax - q.mean) / q.sd, lo = fabsf(xmin - q.mean) / q.sd;
    q.range = hi > lo ? hi : lo;
    q.ascale = (int)(int8_t)(int)(ceilf((float)log((double)q.range)) - 7.0f);
    return q;
}

__device__ __forceinline__ int8_t quant_pixel(uint32_t p, const QuantParams& q) {
#pragma clang fp contract(off)
    if (!q.ok) return 0;
    const float y = ((float)p - q.mean) / q.sd;
    return (int8_t)(int)roundf(y / q.range * 127.0f);
}

// A pixel is a uint8, so the whole map is 256 entries: each block evaluates quant_pixel once per
// value into LDS (the same float sequence, so the same bytes) and the per-pixel work is a lookup
// instead of two float divisions.  Call with all threads of a 256-thread block after q is set.
__device__ __forceinline__ void quant_lut_fill(int8_t* lut, const QuantParams& q) {
    if (threadIdx.x < 256) lut[threadIdx.x] = quant_pixel(threadIdx.x, q);
    __syncthreads();
}

// out: NHWC16 [n][hw][cp] (nhwc = true, the step's layer-0 input: one thread per pixel, its c
// channels packed into 16-byte stores) or NCHW [n][c][hw] (one thread per element).  Thread 0 of
// each block derives the parameters (double log / sqrt), so the grid is kept to a few blocks per
// CU and each thread loops.
template <bool NHWC>
__global__ void __launch_bounds__(256) image_quant_kernel(const uint8_t* __restrict__ img, int n, int c, int hw,
                                                          int cp, const unsigned long long* __restrict__ stats,
                                                          int64_t count, int64_t var_count,
                                                          int8_t* __restrict__ out, int8_t* __restrict__ ascale) {
    __shared__ QuantParams sq;
    __shared__ int8_t lut[256];
    if (threadIdx.x == 0) {
        sq = quant_params(stats, count, var_count);
        if (blockIdx.x == 0 && ascale != nullptr) *ascale = (int8_t)sq.ascale;
    }
    __syncthreads();
    quant_lut_fill(lut, sq);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (NHWC) {
        const int64_t pixels = (int64_t)n * hw;
        const int c16 = cp / 16;
        for (int64_t pxl = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; pxl < pixels; pxl += stride) {
            const int64_t b = pxl / hw, px = pxl - b * hw;
            const uint8_t* src = img + b * c * hw + px;
            int8_t* dst = out + pxl * cp;
            for (int k = 0; k < c16; ++k) {
                v16c v;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int ch = 16 * k + j;
                    v[j] = ch < c ? lut[src[(int64_t)ch * hw]] : (int8_t)0;
                }
                *(v16c*)(dst + 16 * k) = v;
            }
        }
    } else {
        // 16 pixels per thread and step (16-byte loads and stores), the tail one by one
        const int64_t total = (int64_t)n * c * hw, n16 = total / 16;
        const uint4* in16 = reinterpret_cast<const uint4*>(img);
        uint4* out16 = reinterpret_cast<uint4*>(out);
        for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
            const uint4 v = in16[i];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t r = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) r |= (uint32_t)(uint8_t)lut[(w[j] >> (8 * b)) & 255u] << (8 * b);
                o[j] = r;
            }
            out16[i] = uint4{o[0], o[1], o[2], o[3]};
        }
        for (int64_t i = n16 * 16 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride)
            out[i] = lut[img[i]];
    }
}

// The first layer's input straight from the batch: quantise (or take the int8 pixels as they
// are) and write the im2col copy the K = 32 first-layer conv reads, xcol[p][(ky KW + kx) C + c]
// (32 bytes per output pixel, zero outside the image and for k >= C KH KW), in one pass.  A
// workgroup takes one image's band of BAND output rows: it stages the band's input rows (halo
// included) once in LDS as 4-byte pixels (C <= 4 channels), writes its own rows' int8 pixels
// (NCHW, the input tap), then builds each output pixel's 32 bytes from the 4-byte pixels of its
// taps.  The quantisation parameters come from the statistics slots (stats_from_slots).
template <int C, int KH, int KW, bool QUANT>
__global__ void __launch_bounds__(256) input_im2col_kernel(const void* __restrict__ in, int n, int h, int w, int oh,
                                                           int ow, int pt, int pl, int band,
                                                           const unsigned long long* __restrict__ slots, int nslots,
                                                           int64_t count, int64_t var_count,
                                                           int8_t* __restrict__ x_nchw, int8_t* __restrict__ xcol,
                                                           int8_t* __restrict__ ascale, Conv0Range r0) {
    static_assert(C <= 4 && C * KH * KW <= 32, "one 32-byte im2col row");
    extern __shared__ __attribute__((aligned(16))) uint32_t px[];  // [rows][w + KW - 1] 4-byte pixels
    __shared__ QuantParams sq;
    const int bands = (oh + band - 1) / band;
    const int img = blockIdx.x / bands, oy0 = (blockIdx.x % bands) * band;
    const int oy1 = min(oh, oy0 + band);
    const int iy0 = oy0 - pt, rows = oy1 - oy0 + KH - 1, wp = w + KW - 1;
    if constexpr (QUANT) {
        __shared__ unsigned long long st[4];
        stats_from_slots(slots, nslots, st);
        if (threadIdx.x == 0) {
            sq = quant_params(st, count, var_count);
            if (blockIdx.x == 0 && ascale != nullptr) *ascale = (int8_t)sq.ascale;
        }
        __syncthreads();
    }
    __shared__ int8_t lut[256];
    if constexpr (QUANT) quant_lut_fill(lut, sq);
    // input rows this band writes to the tap: [oy0, oy0 + band), the last band through h
    const bool last = blockIdx.x % bands == bands - 1;
    const int own0 = oy0, own1 = last ? h : oy0 + band;
    // the band's input rows (zero halo): one thread per (row, column) of the padded band
    for (int t = threadIdx.x; t < rows * wp; t += blockDim.x) {
        const int r = t / wp, xx = t - r * wp;
        const int iy = iy0 + r, ix = xx - pl;
        uint32_t v = 0;
        if (iy >= 0 && iy < h && ix >= 0 && ix < w) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int64_t e = (((int64_t)img * C + c) * h + iy) * w + ix;
                int8_t qv;
                if constexpr (QUANT)
                    qv = lut[((const uint8_t*)in)[e]];
                else
                    qv = ((const int8_t*)in)[e];
                v |= (uint32_t)(uint8_t)qv << (8 * c);
                if (x_nchw != nullptr && iy >= own0 && iy < own1) x_nchw[e] = qv;
            }
        }
        px[t] = v;
    }
    __syncthreads();
    const int npx = (oy1 - oy0) * ow;
    // the first conv's range (r0.w set): its GEMM over the rows just built, K = 32, one
    // v_mfma_i32_32x32x32_i8 per 32 pixels x 32 output channels -- the wave's 64 pixels are two
    // B tiles after one half-wave swap (lane l holds pixel l's 32 bytes; a tile wants lane l and
    // l + 32 to hold the two 16-byte halves of pixel l), the weights' A fragments loaded once
    const int lane = threadIdx.x & 63, hh = lane >> 5;
    v4i wa[2] = {};
    if (r0.w != nullptr) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int co = t * 32 + (lane & 31);
            if (t * 32 < r0.cop && co < r0.co) wa[t] = *(const v4i*)(r0.w + co * 32 + 16 * hh);
        }
    }
    uint32_t m0 = 0;
    const int npx_r = r0.w != nullptr ? (npx + blockDim.x - 1) / blockDim.x * blockDim.x : npx;
    for (int t = threadIdx.x; t < npx_r; t += blockDim.x) {
        const int oy = t / ow, ox = t - oy * ow;
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // t >= npx (a whole-wave MFMA pass): a zero column
        const int ld = t < npx ? (oy * wp + ox) : 0;  // (past the band: any staged pixel, masked below)
        const uint32_t keep = t < npx ? 0xffffffffu : 0u;
#pragma unroll
        for (int ky = 0; ky < KH; ++ky)
#pragma unroll
            for (int kx = 0; kx < KW; ++kx) {
                const uint32_t v = px[ld + ky * wp + kx] & keep;
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int k = (ky * KW + kx) * C + c;
                    d[k >> 2] |= ((v >> (8 * c)) & 0xffu) << (8 * (k & 3));
                }
            }
        if (t < npx) {
            int8_t* o = xcol + (((int64_t)img * oh + oy0 + oy) * ow + ox) * 32;
            *(v4i_q*)o = v4i_q{(int)d[0], (int)d[1], (int)d[2], (int)d[3]};
            *(v4i_q*)(o + 16) = v4i_q{(int)d[4], (int)d[5], (int)d[6], (int)d[7]};
        }
        if (r0.w != nullptr) {
            // lanes < 32: own bytes 0..15 (tile 0) and, from lane + 32, its bytes 0..15 (tile 1);
            // lanes >= 32: from lane - 32, its bytes 16..31 (tile 0) and own bytes 16..31 (tile 1)
            // v_permlane32_swap(x, y) swaps the lower half-wave's y with the upper half-wave's x:
            // lanes >= 32 get y of lane - 32 as the first result, lanes < 32 get x of lane + 32 as
            // the second (conv0_kernel's pack() relies on the same)
            v4i b0, b1;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const auto sw = __builtin_amdgcn_permlane32_swap(d[j], d[4 + j], false, false);
                b0[j] = hh == 0 ? (int)d[j] : (int)sw[0];
                b1[j] = hh == 0 ? (int)sw[1] : (int)d[4 + j];
            }
#pragma unroll
            for (int tc = 0; tc < 2; ++tc) {
                if (tc * 32 >= r0.cop) break;
#pragma unroll
                for (int tp = 0; tp < 2; ++tp) {
                    const v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(wa[tc], tp ? b1 : b0, v16i{}, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const uint32_t u = uabs32(acc[i]);
                        m0 = m0 > u ? m0 : u;
                    }
                }
            }
        }
    }
    if (r0.w != nullptr) {  // output channels >= co have zero weights: their sums are 0
        m0 = wave_max_u32(m0);
        __shared__ uint32_t red0[4];
        if (lane == 0) red0[threadIdx.x >> 6] = m0;
        __syncthreads();
        if (threadIdx.x == 0) publish_max(r0.amax, max(max(red0[0], red0[1]), max(red0[2], red0[3])));
    }
}

}  // namespace

// slots: IMAGE_STATS_SLOTS x 4 u64 of per-block partials
hipError_t image_stats_slots(const uint8_t* img, int64_t n, unsigned long long* slots, int* nslots, hipStream_t st,
                             void* zero, size_t zero_bytes) {
    if (n <= 0 || zero_bytes % 16 != 0 || (zero_bytes != 0 && zero == nullptr)) return hipErrorInvalidValue;
    int64_t blocks = (n / 16 + 255) / 256;
    blocks = blocks < 1 ? 1 : blocks > IMAGE_STATS_SLOTS ? IMAGE_STATS_SLOTS : blocks;
    hipLaunchKernelGGL(image_stats_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, img, n, slots, (uint4*)zero,
                       (int64_t)(zero_bytes / 16));
    *nslots = (int)blocks;
    return hipGetLastError();
}

hipError_t stats_finalize(const unsigned long long* slots, int nslots, unsigned long long* stats, hipStream_t st) {
    hipLaunchKernelGGL(stats_finalize_kernel, dim3(1), dim3(256), 0, st, slots, nslots, stats);
    return hipGetLastError();
}

bool input_im2col_ok(int c, int kh, int kw) { return (c == 3 && kh == 3 && kw == 3) || (c == 1 && kh == 5 && kw == 5); }

hipError_t input_im2col(const void* in, bool quant, int n, int c, int h, int w, int kh, int kw, int pt, int pl,
                        const unsigned long long* slots, int nslots, int64_t count, int8_t* x_nchw, int8_t* xcol,
                        int8_t* ascale, hipStream_t st, const Conv0Range& r0) {
    if (!input_im2col_ok(c, kh, kw) || n <= 0 || (quant && (count <= 0 || slots == nullptr))) return hipErrorInvalidValue;
    if (r0.w != nullptr && (r0.amax == nullptr || r0.cop > 64 || r0.cop % 32 != 0 || r0.co > r0.cop)) return hipErrorInvalidValue;
    const int oh = h + 2 * pt - kh + 1, ow = w + 2 * pl - kw + 1;
    if (oh <= 0 || ow <= 0) return hipErrorInvalidValue;
    // bands of output rows: ~16 KiB of staged pixels, at least 2 workgroups per image at 32x32
    int band = oh;
    while (band > 1 && (int64_t)(band + kh - 1) * (w + kw - 1) * 4 > 16384) band = (band + 1) / 2;
    if (oh >= 32 && band > oh / 2) band = (oh + 1) / 2;
    const int bands = (oh + band - 1) / band;
    const size_t lds = (size_t)(band + kh - 1) * (w + kw - 1) * 4;
    const int64_t var_count = count / ((int64_t)c * h * w) * 784;  // MnistUtils.cpp:86 (see image_quantize)
    const dim3 grid((unsigned)((int64_t)n * bands));
#define IIC(CC, KK, Q)                                                                                            \
    hipLaunchKernelGGL((input_im2col_kernel<CC, KK, KK, Q>), grid, dim3(256), lds, st, in, n, h, w, oh, ow, pt, pl, \
                       band, slots, nslots, count, var_count, x_nchw, xcol, ascale, r0)
    if (c == 3 && quant)
        IIC(3, 3, true);
    else if (c == 3)
        IIC(3, 3, false);
    else if (quant)
        IIC(1, 5, true);
    else
        IIC(1, 5, false);
#undef IIC
    return hipGetLastError();
}

hipError_t image_stats(const uint8_t* img, int64_t n, unsigned long long* stats, hipStream_t st) {
    // the standalone op: up to 512 blocks' atomics into the zeroed stats (the step spreads the
    // pixels over IMAGE_STATS_SLOTS blocks and sums their slots where it uses them).  64 blocks
    // (one wave per CU) took 43 us over a 128 x 224 x 224 batch: latency-bound loads, not the
    // atomics
    if (n <= 0) return hipErrorInvalidValue;
    int64_t blocks = (n / 16 + 255) / 256;
    blocks = blocks < 1 ? 1 : blocks > 512 ? 512 : blocks;
    const hipError_t e = hipMemsetAsync(stats, 0, 4 * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(image_stats_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, img, n, stats);
    return hipGetLastError();
}

hipError_t image_quantize(const uint8_t* img, int n, int c, int hw, int cp, const unsigned long long* stats,
                          int64_t count, int8_t* out, int8_t* ascale, bool nhwc16, hipStream_t st) {
    if (n <= 0 || c <= 0 || hw <= 0 || count <= 0 || (nhwc16 && cp < c)) return hipErrorInvalidValue;
    if (nhwc16 && cp % 16 != 0) return hipErrorInvalidValue;
    const int64_t total = nhwc16 ? (int64_t)n * hw : (int64_t)n * c * hw;
    // MnistUtils.cpp:86: the variance over batchSize * 28 * 28, batchSize = the images `count` covers
    const int64_t var_count = count / ((int64_t)c * hw) * 784;
    const int64_t work = nhwc16 ? total : total / 16 + 1;  // NCHW: 16 pixels per thread
    int64_t blocks = (work + 255) / 256;
    blocks = blocks > 2048 ? 2048 : blocks;
    if (nhwc16)
        hipLaunchKernelGGL(image_quant_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, img, n, c, hw, cp,
                           stats, count, var_count, out, ascale);
    else
        hipLaunchKernelGGL(image_quant_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, img, n, c, hw, cp,
                           stats, count, var_count, out, ascale);
    return hipGetLastError();
}

}  // namespace niti
