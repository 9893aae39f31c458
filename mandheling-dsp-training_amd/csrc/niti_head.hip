// niti_head.hip -- the classifier head's whole training-step chain in ONE launch (VGG-11's 512 -> 10
// head after the last 2x2 pool):
//
//   forward      logits = NITI_Conv_Int8 (1x1 over 1x1 maps) of the pooled input, the rescale rule
//                over the whole batch (NITI_Conv_Int8.cpp:260-307)
//   loss         NITI_LOSS_Grad (the rows of loss_rows16, niti_kernels.hip)
//   weight grad  dw = dy^T x, int32, its range published (NITI_GradientConv_Int8.cpp:274-296; the
//                update launch requantises it with NITI_SGD)
//   input grad   dx = dy w, rescaled (NITI_DeConv_Int8.cpp:294-329), routed through the previous
//                layer's 2x2 max pool by the codes its forward recorded (pool_code4; relu included)
//
// Every one of these is a few million multiply-adds, so the four launches they took (the row kernel
// at W = 1 twice with its grid barrier, the loss launch, the head weight gradient: ~25 us of launch
// and barrier latency per VGG-11 step) become one: each of the G = K / 32 head workgroups recomputes
// the forward, the loss and the whole input gradient's range by itself (128 MFMAs each, no grid
// barrier) and then writes its own 32 input channels -- the routed input gradient (NHWC16, C32 and
// P16 copies) and that slice of the weight gradient.  Workgroup 0 also writes the logits, their
// exponent and dy.  (The backward pass's P16 input copies, which loss_grad_p16 converts beside the
// loss rows, take a launch of their own: in this launch their workgroups would carry its LDS and
// registers -- two per CU instead of nine -- and the launch ran 54 us.)
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdio.h>
#include <stdlib.h>

#include "niti_device.hpp"
#include "niti_kernels.hpp"
#include "niti_sgd.hpp"

namespace niti {

constexpr int HEAD_MAXN = 512;  // batch rows held in LDS
constexpr int HEAD_MAXK = 512;  // input channels (the weights staged in LDS)

// requantisation of one accumulator under the forward rule (raw cast for shift <= 0)
__device__ __forceinline__ int8_t head_rq(int32_t v, int shift, int relu) {
    int32_t q = shift <= 0 ? (int32_t)(int8_t)v : psto_any(v, shift > 1 ? shift : 2);
    if (relu && q < 0) q = 0;
    return (int8_t)q;
}

constexpr int HEAD_THREADS = 1024;  // 16 waves: four per SIMD, so each SIMD hides one wave's latency behind
                                    // the others' (one wave per SIMD ran every phase as a dependent chain)
constexpr int HEAD_WAVES = HEAD_THREADS / 64;

__device__ __forceinline__ uint32_t head_block_max(uint32_t m, uint32_t* red) {
    m = wave_max(m);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    uint32_t r = red[0];
#pragma unroll
    for (int w = 1; w < HEAD_WAVES; ++w) r = max(r, red[w]);
    return r;
}

// diagnostics (NITI_HEAD_STAMPS=1): workgroup 0's s_memtime at each phase boundary
__device__ unsigned long long g_head_stamps[16];
#define HEAD_STAMP(k)                                                                          \
    do {                                                                                       \
        if (h.stamps && blockIdx.x == 0 && threadIdx.x == 0) g_head_stamps[k] = __builtin_amdgcn_s_memtime(); \
    } while (0)

__global__ void __launch_bounds__(HEAD_THREADS) head_chain_kernel(HeadChain h) {
    __shared__ __attribute__((aligned(16))) int8_t ws_[16 * HEAD_MAXK];   // w [class][k] (rows >= c_out zero)
    __shared__ __attribute__((aligned(16))) int8_t wts[HEAD_MAXK * 16];   // wT [k][class]
    __shared__ __attribute__((aligned(16))) int8_t lg[HEAD_MAXN * 16];    // logits [row][16]
    __shared__ __attribute__((aligned(16))) int8_t dys[HEAD_MAXN * 16];   // dy [row][16]
    __shared__ __attribute__((aligned(16))) int8_t dyT[16 * HEAD_MAXN];   // dy [class][row]
    __shared__ __attribute__((aligned(16))) int8_t dxs[HEAD_MAXN * 32];   // this slice's input gradient
    __shared__ __attribute__((aligned(16))) int8_t xsT[32 * HEAD_MAXN];   // this slice's input columns [ch][row]
    __shared__ __attribute__((aligned(16))) int8_t cds[HEAD_MAXN * 32];   // this slice's pool codes
    __shared__ int32_t part[4][16][64];
    __shared__ int32_t labs[HEAD_MAXN];
    __shared__ uint32_t red[HEAD_WAVES];
    __shared__ int8_t ascale;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int hf = lane >> 5, c = lane & 31;
    const int n = h.n, K = h.K;
    const int n32 = (n + 31) / 32 * 32;
    const int ci0 = blockIdx.x * 32;
    HEAD_STAMP(0);
    // ---- the forward's batch rows first (wave w: row tile w; its K steps all in flight while the
    // workgroup stages the rest)
    const int row = wid * 32 + c;
    const bool tile_on = wid * 32 < n;  // (wave-uniform)
    v4i xv[HEAD_MAXK / 32];
    {
        const int8_t* xr = h.x + (int64_t)(row < n ? row : 0) * h.xld + 16 * hf;
#pragma unroll
        for (int u = 0; u < HEAD_MAXK / 32; ++u)
            xv[u] = tile_on && row < n && 32 * u < K ? *(const v4i*)(xr + 32 * u) : v4i{0, 0, 0, 0};
    }
    // ---- stage the small operands in LDS: the weights both ways, this slice's input columns
    // (transposed) and pool codes, the labels; rows past n read as zero
    for (int t = tid; t < 16 * K / 16; t += HEAD_THREADS) {  // w: 16-byte chunks of [class][k]
        const int cls = t / (K / 16), k16 = t - cls * (K / 16);
        *(v4i*)(ws_ + cls * HEAD_MAXK + 16 * k16) = cls < h.c_out ? *(const v4i*)(h.w + (int64_t)cls * K + 16 * k16)
                                                                 : v4i{0, 0, 0, 0};
    }
    for (int t = tid; t < K; t += HEAD_THREADS) *(v4i*)(wts + t * 16) = *(const v4i*)(h.wT + (int64_t)t * h.cop);
    for (int t = tid; t < n32 * 2; t += HEAD_THREADS) {
        const int r = t >> 1, o = 16 * (t & 1);
        const bool ok = r < n;
        const v4i xv = ok ? *(const v4i*)(h.x + (int64_t)r * h.xld + ci0 + o) : v4i{0, 0, 0, 0};
        *(v4i*)(cds + t * 16) = ok ? *(const v4i*)(h.code + (int64_t)r * K + ci0 + o) : v4i{0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 16; ++e) xsT[(o + e) * HEAD_MAXN + r] = (int8_t)(xv[e >> 2] >> (8 * (e & 3)));
    }
    for (int t = tid; t < n; t += HEAD_THREADS) labs[t] = h.labels[t];
    __syncthreads();
    HEAD_STAMP(1);

    // ---- forward: logits (MFMA rows = classes, columns = the batch)
    v16i facc = {};
    uint32_t m = 0;
    if (tile_on) {
#pragma unroll
        for (int u = 0; u < HEAD_MAXK / 32; ++u) {
            if (32 * u < K) {
                const v4i wv = c < 16 ? *(const v4i*)(ws_ + c * HEAD_MAXK + 32 * u + 16 * hf) : v4i{0, 0, 0, 0};
                facc = __builtin_amdgcn_mfma_i32_32x32x32_i8(wv, xv[u], facc, 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int cls = (i & 3) + 8 * (i >> 2) + 4 * hf;
            if (row < n && cls < h.c_out) m = max(m, uabs32(facc[i]));
        }
    }
    const int fshift = bitwidth_of(head_block_max(m, red)) - 7;
    if (tile_on && row < n) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int cls = (i & 3) + 8 * (i >> 2) + 4 * hf;
            if (cls < 16) lg[row * 16 + cls] = cls < h.c_out ? head_rq(facc[i], fshift, h.relu) : (int8_t)0;
        }
    }
    if (tid == 0) {
        const int inc = fshift > 1 ? fshift : (fshift == 1 ? 2 : 0);
        ascale = (int8_t)((h.exp_in ? (int)*h.exp_in : 0) + (h.wscale ? (int)*h.wscale : 0) + inc);
        if (blockIdx.x == 0 && h.exp_out != nullptr) *h.exp_out = ascale;
    }
    __syncthreads();
    HEAD_STAMP(2);

    // ---- the loss gradient: 16 lanes per row (DPP reductions), 64 rows per pass
    for (int t0 = 0; t0 < n * 16; t0 += 2 * HEAD_THREADS) {  // two independent passes interleave
        loss_rows16(lg, n, h.c_out, 16, &ascale, labs, dys, t0 + tid);
        loss_rows16(lg, n, h.c_out, 16, &ascale, labs, dys, t0 + HEAD_THREADS + tid);  // (rows past n: no-op)
    }
    __syncthreads();
    for (int t = tid; t < n32 * 16; t += HEAD_THREADS) {  // transposed for the weight gradient
        const int r = t >> 4, j = t & 15;
        dyT[j * HEAD_MAXN + r] = r < n ? dys[r * 16 + j] : (int8_t)0;
    }
    HEAD_STAMP(3);
    if (blockIdx.x == 0) {  // logits and dy as the model keeps them ([n][cop], cop = 16)
        for (int t = tid; t < n; t += HEAD_THREADS) {
            *(v4i*)(h.logits + (int64_t)t * h.cop) = *(const v4i*)(lg + t * 16);
            *(v4i*)(h.dy + (int64_t)t * h.cop) = *(const v4i*)(dys + t * 16);
        }
    }

    // ---- input gradient: dx[row][k] = sum_c dy[row][c] wT[k][c] (MFMA rows = k, columns = the
    // batch, K = the 16 classes, its upper half zero).  Wave w: row tile w, every column tile for the
    // range; this workgroup's own column tile is kept.
    const int ct_n = K / 32;
    v16i own = {};
    m = 0;
    if (tile_on) {
        // (rows past n have a zero dy row, so their products are zero and need no mask)
        const v4i a = row < n && hf == 0 ? *(const v4i*)(dys + row * 16) : v4i{0, 0, 0, 0};
#pragma unroll
        for (int ct = 0; ct < HEAD_MAXK / 32; ++ct) {
            if (ct < ct_n) {
                const v4i b = hf == 0 ? *(const v4i*)(wts + (ct * 32 + c) * 16) : v4i{0, 0, 0, 0};
                const v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, v16i{}, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 16; ++i) m = max(m, uabs32(acc[i]));
            }
        }
        const v4i b = hf == 0 ? *(const v4i*)(wts + (blockIdx.x * 32 + c) * 16) : v4i{0, 0, 0, 0};
        own = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, v16i{}, 0, 0, 0);  // this workgroup's tile again
    }
    HEAD_STAMP(4);
    const int dshift = bitwidth_of(head_block_max(m, red)) - 7;
    if (tile_on && row < n) {
#pragma unroll
        for (int i = 0; i < 16; ++i) dxs[row * 32 + (i & 3) + 8 * (i >> 2) + 4 * hf] = head_rq(own[i], dshift, 0);
    }
    __syncthreads();
    HEAD_STAMP(5);

    // ---- the input gradient through the previous layer's 2x2 max pool: window element t of
    // (image, channel) takes dx where the recorded code has bit t
    for (int t = tid; t < n * 2; t += HEAD_THREADS) {
        const int img = t >> 1, c16 = 16 * (t & 1);
        const v4i v = *(const v4i*)(dxs + img * 32 + c16);
        const v4i cd = *(const v4i*)(cds + img * 32 + c16);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            v4i d;
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] = v[q] & (int)pool_code_mask((uint32_t)cd[q], w);
            if (h.pool_dx != nullptr) *(v4i*)(h.pool_dx + ((int64_t)img * 4 + w) * K + ci0 + c16) = d;
            if (h.pool_dx_c32 != nullptr)
                *(v4i*)(h.pool_dx_c32 + (((int64_t)img * (K / 32) + blockIdx.x) * 4 + w) * 32 + c16) = d;
        }
    }
    if (h.p16 != nullptr) {  // [pixel / 16][K][16]: 16 pixels = 4 images x 4 window positions
        for (int t = tid; t < (n / 4) * 32; t += HEAD_THREADS) {
            const int q4 = t >> 5, ch = t & 31;
            v4i o;
#pragma unroll
            for (int im = 0; im < 4; ++im) {
                const int img = 4 * q4 + im;
                const uint32_t v = (uint32_t)(uint8_t)dxs[img * 32 + ch];
                const uint32_t cd = (uint32_t)(uint8_t)cds[img * 32 + ch];
                uint32_t wv4 = 0;
#pragma unroll
                for (int w = 0; w < 4; ++w) wv4 |= ((cd >> w) & 1u ? v : 0u) << (8 * w);
                o[im] = (int)wv4;
            }
            *(v4i*)(h.p16 + ((int64_t)q4 * K + ci0 + ch) * 16) = o;
        }
    }
    __syncthreads();  // (dyT complete)
    HEAD_STAMP(6);

    // ---- weight gradient of this slice: dw[cls][ci0 + j] = sum_row dy[row][cls] x[row][ci0 + j]
    // (MFMA rows = classes, columns = the slice's channels, K = the batch: 16 consecutive rows of
    // one class / channel are one 16-byte read of the transposed copies; waves 0-3 split the rows)
    if (wid < 4) {
        v16i acc = {};
        for (int r0 = wid * 32; r0 < n; r0 += 128) {
            const int rr = r0 + 16 * hf;
            const v4i a = c < 16 ? *(const v4i*)(dyT + c * HEAD_MAXN + rr) : v4i{0, 0, 0, 0};
            const v4i b = *(const v4i*)(xsT + c * HEAD_MAXN + rr);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) part[wid][i][lane] = acc[i];
    }
    __syncthreads();
    if (wid == 0) {
        uint32_t wm = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int32_t v = part[0][i][lane] + part[1][i][lane] + part[2][i][lane] + part[3][i][lane];
            const int cls = (i & 3) + 8 * (i >> 2) + 4 * hf;
            if (cls < h.c_out) {
                h.dw[(int64_t)cls * K + ci0 + c] = v;
                wm = max(wm, uabs32(v));
            }
        }
        wm = wave_max(wm);
        if (lane == 0 && h.dw_amax != nullptr) publish_max(h.dw_amax, wm);
    }
    HEAD_STAMP(7);
}

bool head_chain_ok(int n, int K, int c_out, int cop) {
    return n > 0 && n <= HEAD_MAXN && n % 4 == 0 && K % 32 == 0 && K >= 32 && K <= HEAD_MAXK && c_out >= 1 &&
           c_out <= 16 && cop == 16;
}

static std::atomic<unsigned long long> g_head_chain_launches{0};
unsigned long long head_chain_launches() { return g_head_chain_launches.load(); }
// Off by default: on MI355X the one-workgroup-per-slice chain ran 24-25 us against ~20 us for the
// launches it replaces (every phase a dependent latency chain inside one workgroup).
// NITI_HEAD_CHAIN=1 or niti_diag_head_chain(1) turns it on.
static std::atomic<int> g_head_chain_on{-1};
bool head_chain_enabled() {
    int v = g_head_chain_on.load();
    if (v < 0) {
        const char* e = getenv("NITI_HEAD_CHAIN");
        v = e != nullptr && atoi(e) != 0;
        g_head_chain_on.store(v);
    }
    return v != 0;
}
void head_chain_enable(int on) { g_head_chain_on.store(on ? 1 : 0); }

hipError_t head_chain(const HeadChain& a, hipStream_t st) {
    if (!head_chain_ok(a.n, a.K, a.c_out, a.cop) || a.x == nullptr || a.w == nullptr || a.wT == nullptr ||
        a.logits == nullptr || a.labels == nullptr || a.dy == nullptr || a.dw == nullptr || a.code == nullptr ||
        a.xld < a.K || a.xld % 16 != 0)
        return hipErrorInvalidValue;
    HeadChain h = a;
    h.G = a.K / 32;
    static const bool stamps = getenv("NITI_HEAD_STAMPS") != nullptr;
    h.stamps = stamps ? 1 : 0;
    g_head_chain_launches.fetch_add(1);
    hipLaunchKernelGGL(head_chain_kernel, dim3((unsigned)h.G), dim3(HEAD_THREADS), 0, st, h);
    if (stamps) {  // diagnostics: cycles per phase of workgroup 0
        unsigned long long t[16] = {};
        if (hipStreamSynchronize(st) == hipSuccess && hipMemcpyFromSymbol(t, HIP_SYMBOL(g_head_stamps), sizeof(t)) == hipSuccess)
            fprintf(stderr, "head_chain cycles: fwd %llu range+rq %llu loss %llu dgrad %llu rq %llu route %llu wgrad %llu\n",
                    t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], t[5] - t[4], t[6] - t[5], t[7] - t[6]);
    }
    return hipGetLastError();
}

}  // namespace niti
