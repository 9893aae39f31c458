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
// oracle (oracle/niti_oracle.c niti_ref_quantize_images) states the same contract; its
// float-sequential restatement (niti_ref_quantize_input) agrees wherever the float sums are
// exact.  Because the statistics are integers, data-parallel ranks all-reduce them (SUM S1, S2;
// MAX xmax, 255 - xmin) and quantise their shard exactly as one device would the global batch.
// ascale is computed in float as the graph does (_Ceil(_Log(range)) on float tensors, :89-91),
// logf taken as the correctly rounded float natural log, (float)log((double)range), so host and
// device agree bit for bit.  A constant batch (std = 0) is undefined in the reference (0/0); here
// it quantises to zeros with ascale = -7.
#include "niti_kernels.hpp"
#include "niti_map.hpp"

namespace niti {

namespace {

typedef signed char v16c __attribute__((ext_vector_type(16)));

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

// stats[0] += S1, stats[1] += S2, stats[2] max= xmax, stats[3] max= 255 - xmin
__global__ void __launch_bounds__(256) image_stats_kernel(const uint8_t* __restrict__ img, int64_t n,
                                                          unsigned long long* __restrict__ stats) {
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
    if (threadIdx.x == 0) {
        unsigned long long t[4] = {0, 0, 0, 0};
        for (int k = 0; k < 4; ++k) {
            t[0] += r[k][0];
            t[1] += r[k][1];
            t[2] = r[k][2] > t[2] ? r[k][2] : t[2];
            t[3] = r[k][3] > t[3] ? r[k][3] : t[3];
        }
        atomicAdd(&stats[0], t[0]);
        atomicAdd(&stats[1], t[1]);
        atomicMax(&stats[2], t[2]);
        atomicMax(&stats[3], t[3]);
    }
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
    if (threadIdx.x == 0) {
        sq = quant_params(stats, count, var_count);
        if (blockIdx.x == 0 && ascale != nullptr) *ascale = (int8_t)sq.ascale;
    }
    __syncthreads();
    const QuantParams q = sq;
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
                    v[j] = ch < c ? quant_pixel(src[(int64_t)ch * hw], q) : (int8_t)0;
                }
                *(v16c*)(dst + 16 * k) = v;
            }
        }
    } else {
        const int64_t total = (int64_t)n * c * hw;
        for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride)
            out[i] = quant_pixel(img[i], q);
    }
}

}  // namespace

hipError_t image_stats(const uint8_t* img, int64_t n, unsigned long long* stats, hipStream_t st) {
    if (n <= 0) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(stats, 0, 4 * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    // a few blocks, each thread looping over 16-byte loads: every block ends in 4 device-scope
    // atomics on one cache line, and 192 blocks of them serialised into ~8 us
    int64_t blocks = (n / 16 + 2047) / 2048;
    blocks = blocks < 1 ? 1 : blocks > 32 ? 32 : blocks;
    hipLaunchKernelGGL(image_stats_kernel, dim3((unsigned)blocks), dim3(256), 0, st, img, n, stats);
    return hipGetLastError();
}

hipError_t image_quantize(const uint8_t* img, int n, int c, int hw, int cp, const unsigned long long* stats,
                          int64_t count, int8_t* out, int8_t* ascale, bool nhwc16, hipStream_t st) {
    if (n <= 0 || c <= 0 || hw <= 0 || count <= 0 || (nhwc16 && cp < c)) return hipErrorInvalidValue;
    if (nhwc16 && cp % 16 != 0) return hipErrorInvalidValue;
    const int64_t total = nhwc16 ? (int64_t)n * hw : (int64_t)n * c * hw;
    // MnistUtils.cpp:86: the variance over batchSize * 28 * 28, batchSize = the images `count` covers
    const int64_t var_count = count / ((int64_t)c * hw) * 784;
    int64_t blocks = (total + 255) / 256;
    blocks = blocks > 512 ? 512 : blocks;
    if (nhwc16)
        hipLaunchKernelGGL(image_quant_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, img, n, c, hw, cp,
                           stats, count, var_count, out, ascale);
    else
        hipLaunchKernelGGL(image_quant_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, img, n, c, hw, cp,
                           stats, count, var_count, out, ascale);
    return hipGetLastError();
}

}  // namespace niti
