// niti_device.hpp -- gfx950 device helpers shared by the kernel translation units
// (niti_kernels.hip, niti_wgrad.hip): buffer resources and LDS-DMA, counted waits,
// transposed LDS reads, multiply-shift division, the range-estimate max words and the
// XCD-aware block remap.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "niti_kernels.hpp"

namespace niti {

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef signed char v16c __attribute__((ext_vector_type(16)));

// byte offset that reads zeros through the buffer range check
constexpr uint32_t OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ v4i buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

// multiply-shift division for 0 <= n < 2^31 (Granlund-Montgomery, round-up variant)
struct FastDiv {
    uint32_t m = 1, s = 0, d = 1;
};
static inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    f.s = 0;
    while ((1ull << f.s) < d) ++f.s;
    f.m = (uint32_t)((((uint64_t)1 << 32) * ((1ull << f.s) - d)) / d + 1);
    return f;
}
__device__ __forceinline__ uint32_t fdiv(const FastDiv& f, uint32_t n) { return (__umulhi(n, f.m) + n) >> f.s; }

__device__ __forceinline__ uint32_t uabs32(int v) { return v < 0 ? 0u - (uint32_t)v : (uint32_t)v; }

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t = __shfl_xor(v, o, 64);
        v = v > t ? v : t;
    }
    return v;
}

// One atomic per workgroup, skipped when the word already holds a larger value (the
// single max word is otherwise a serialisation point for thousands of workgroups).
// A range is MAX_SLOTS words on separate 128-byte lines: each block publishes into one slot
// (spread by block id), so no line sees more than grid/MAX_SLOTS atomics.  With one word,
// every block of a launch whose blocks all finish together (2048 reduce blocks) read 0 and
// queued its atomic on the same line: ~25 us of serialised atomics per launch.
__device__ __forceinline__ void publish_max(uint32_t* amax, uint32_t m) {
    if (m == 0u) return;
    const uint32_t slot = (blockIdx.x + blockIdx.y * 13u + blockIdx.z * 7u) & (MAX_SLOTS - 1);
    uint32_t* w = amax + slot * MAX_SLOT_STRIDE;
    if (m > __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(w, m);
}
// max|acc| of a range: the max over its slots, one slot per lane (call with the whole wave
// active; read after a kernel boundary or collective)
__device__ __forceinline__ uint32_t read_max(const uint32_t* amax) {
    static_assert(MAX_SLOTS == 64, "one slot per lane");
    return wave_max(amax[(threadIdx.x & 63) * MAX_SLOT_STRIDE]);
}

// SWAR on 4 int8 lanes of a dword; a "hi" result is meaningful in bit 7 of each byte only
constexpr uint32_t SW_H = 0x80808080u, SW_L = 0x7F7F7F7Fu;
__device__ __forceinline__ uint32_t sw_ge_hi(uint32_t x, uint32_t m) {  // signed x >= m
    const uint32_t ax = x ^ SW_H, bm = m ^ SW_H;  // as unsigned
    const uint32_t t = (ax | SW_H) - (bm & SW_L);  // bit 7: low 7 bits of ax >= those of bm
    const uint32_t d = ax ^ bm;                    // bit 7: the top bits differ -> ax's top bit decides
    return ((d & ax) | (~d & t)) & SW_H;
}
__device__ __forceinline__ uint32_t sw_pos_hi(uint32_t x) {  // signed x > 0
    const uint32_t nz = (((x & SW_L) + SW_L) | x) & SW_H;
    return nz & ~x;
}
__device__ __forceinline__ uint32_t sw_expand(uint32_t hb) { return hb | (hb - (hb >> 7)); }

// The 2x2 max pool's gradient route, decided by the forward pass that pools (NITI_CPUPoolGrad_Int8.cpp:
// 21-77: the first window element -- (0,0), (0,1), (1,0), (1,1) -- that is >= the pooled value takes
// the gradient): one code byte per pooled element and channel, bit t set when window element t
// takes it and, for a relu layer, the pooled value (the routed element's own value) is > 0 -- the
// relu gradient of NITI_ReluGrad_Int8 at that element.  4 channels per dword: t0..t3 the window's
// elements, m their max.  The input-gradient pass reads one byte per pooled element instead of the
// 4 window elements and the pooled value.
__device__ __forceinline__ uint32_t pool_code4(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, uint32_t m,
                                               bool relu) {
    const uint32_t h0 = sw_ge_hi(t0, m);
    const uint32_t h1 = sw_ge_hi(t1, m) & ~h0;
    const uint32_t d1 = h0 | h1;
    const uint32_t h2 = sw_ge_hi(t2, m) & ~d1;
    const uint32_t h3 = SW_H & ~(d1 | h2);
    uint32_t code = (h0 >> 7) | (h1 >> 6) | (h2 >> 5) | (h3 >> 4);
    if (relu) code &= sw_expand(sw_pos_hi(m));
    return code;
}
// the byte mask (0xff where it takes the gradient) of window element t from 4 code bytes
__device__ __forceinline__ uint32_t pool_code_mask(uint32_t code, int t) {
    return sw_expand(((code >> t) & 0x01010101u) << 7);
}

// The residual rule, 4 sums per operand dword with bit-field extracts: the compiler's form of
// residual_z + psto_fast ran ~18.5 VALU per element and the pass VALU-bound (15.7 us against 12 us
// of memory for layer1's 77 MB, tools/probes/exit_probe.hip).  Per byte e: hi = sbfe(hw, 8e, 8),
// lo >> r = sbfe(lw, 8e + min(r, 7), 8 - min(r, 7)) (lo's sign once r >= 7), z = (hi << d) + that
// (d <= 23), then PSTO (psto_fast): q = u >> s, qp = ubfe(u, h, s - h) (= (u mod 2^s) >> h),
// pr = ubfe(u, 0, h) << (s & 1), q + (qp > pr), clip 127, the sign restored; relu: u = max(z, 0).
// The range (launch A) as a running max and min of z.  Not used for the raw cast (shift <= 0).
// (Packed 16-bit VALU, two sums per lane, measured 2.4x slower on gfx950: 37 vs 15.7 us.)
struct ResRule {
    uint32_t d, loff, lw, s, h, hs, odd;
};
__device__ __forceinline__ ResRule res_rule(int d, int r, int s) {
    const int rr = r < 7 ? r : 7;
    return ResRule{(uint32_t)d, (uint32_t)rr, (uint32_t)(8 - rr), (uint32_t)s, (uint32_t)(s >> 1),
                   (uint32_t)(s - (s >> 1)), (uint32_t)(s & 1)};
}
template <bool RELU>
__device__ __forceinline__ uint32_t res_rule4(uint32_t hw, uint32_t lw, const ResRule& k, int& mx, int& mn, bool range) {
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int hi = __builtin_amdgcn_sbfe((int)hw, 8 * e, 8);
        const int lo = __builtin_amdgcn_sbfe((int)lw, 8 * e + (int)k.loff, (int)k.lw);
        const int z = (int)(((uint32_t)hi << k.d) + (uint32_t)lo);
        if (range) {
            mx = max(mx, z);
            mn = min(mn, z);
        }
        const uint32_t u = RELU ? (uint32_t)max(z, 0) : (uint32_t)max(z, -z);
        const uint32_t q = u >> k.s;
        const uint32_t qp = __builtin_amdgcn_ubfe(u, k.h, k.hs);
        const uint32_t pr = __builtin_amdgcn_ubfe(u, 0, k.h) << k.odd;
        uint32_t v = min(q + (qp > pr ? 1u : 0u), 127u);
        if (!RELU) v = z < 0 ? 0u - v : v;
        o[e] = v & 0xffu;
    }
    return o[0] | (o[1] << 8) | (o[2] << 16) | (o[3] << 24);
}

// A speculative pair's guess and its update.  Slot words: [0] / [24] / [25] the next pair's guess
// by three predictors (below), [5] their hit counters (3 x 4 bits), [6] bit widths recorded,
// [8, 16) / [16, 24) the last SPEC_HIST bit widths in two forms (rings): on the scale of the layer's
// input, K = bw + escale with escale = the input's exponent + the weight's, and bare; every value
// stored as value + 1 + SPEC_K0 (0: none).  The predictors:
// - mode (bare, [0]): the most frequent of the last 8 bit widths, ties to the most recent.  On the
//   bench's steps many layers' bit widths scatter over two or three values at random rather than
//   hold, and "the last value" then hits less often than the mode;
// - mode on the input's scale ([24]): the int8 rule keeps every tensor's maximum in [64, 127], so
//   when an upstream layer's bit width crosses a power of two its output exponent moves by one and
//   its int8 values halve or double; a layer whose accumulators follow its input keeps K while its bw
//   moves (ResNet-18 layer1.1.a's forward; the input gradients' K drifts instead: the input-gradient
//   slots record escale 0, profiles/r06_spec_trace_resnet18.txt);
// - alternation ([25]): the bit width two pairs back, for a layer that flips back and forth.
// Each predictor's counter moves +1 / -1 (0..7) on its hit / miss; pick follows the highest (ties:
// bare mode, alternation, scaled mode).  learn (one wave of the pair's second launch, with the true
// bw) keeps the rings and leaves the three guesses in their words, so pick (every wave of launch A)
// reads four words in one memory round trip.  The guess is bw + 1, 0 none.
constexpr int SPEC_K0 = 512;
constexpr int SPEC_HIST = 8;
// a recorded value back to a guess (bw + 1) at this pair's input scale
__device__ __forceinline__ uint32_t spec_unscale(uint32_t v, int escale) {
    if (v == 0u) return 0u;
    const int g = (int)v - SPEC_K0 - escale;
    return (uint32_t)(g < 1 ? 1 : g > 32 ? 32 : g);
}
__device__ __forceinline__ uint32_t spec_ld(const uint32_t* p) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ uint32_t spec_choose(uint32_t cnt, uint32_t gb, uint32_t gs, uint32_t ga) {
    const uint32_t cb = cnt & 15u, cs = (cnt >> 4) & 15u, ca = (cnt >> 8) & 15u;
    if (cb >= cs && cb >= ca) return gb;
    return ca >= cs ? ga : gs;
}
__device__ __forceinline__ uint32_t spec_pick(const uint32_t* hint, int escale) {
    const uint32_t cnt = spec_ld(hint + 5), vb = spec_ld(hint), vs = spec_ld(hint + 24), va = spec_ld(hint + 25);
    return spec_choose(cnt, spec_unscale(vb, 0), spec_unscale(vs, escale), spec_unscale(va, 0));
}
// the same with the input's scale read here (exponent in + weight scale, when on): every load is
// issued before any is used -- one memory round trip at the head of launch A, not two; *f gets
// slot word [3] (the row kernels' store flag) from the same trip
__device__ __forceinline__ uint32_t spec_pick_e(const uint32_t* hint, const int8_t* e_in, const int8_t* ws, bool on,
                                                uint32_t* f) {
    const uint32_t cnt = __hip_atomic_load(hint + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t vb = __hip_atomic_load(hint, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t vs = __hip_atomic_load(hint + 24, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t va = __hip_atomic_load(hint + 25, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t w3 = __hip_atomic_load(hint + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int8_t zero = 0;
    const int ei = *(on && e_in ? e_in : &zero), wv = *(on && ws ? ws : &zero);
    *f = (uint32_t)__builtin_amdgcn_readfirstlane((int)w3);
    const int esc = __builtin_amdgcn_readfirstlane(ei + wv);
    return spec_choose((uint32_t)__builtin_amdgcn_readfirstlane((int)cnt),
                       spec_unscale((uint32_t)__builtin_amdgcn_readfirstlane((int)vb), 0),
                       spec_unscale((uint32_t)__builtin_amdgcn_readfirstlane((int)vs), esc),
                       spec_unscale((uint32_t)__builtin_amdgcn_readfirstlane((int)va), 0));
}
// learn, by one whole wave (the second launch's bookkeeping block): lane j < SPEC_HIST takes ring
// entry j, the counts and the mode's pick are lane-parallel (a thread-serial form counted 64 pairs
// per ring on the launch's path)
__device__ __forceinline__ uint32_t spec_mode_wave(uint32_t v, uint32_t n, int lane) {
    uint32_t c = 0u;
#pragma unroll
    for (int k = 0; k < SPEC_HIST; ++k) c += (uint32_t)__builtin_amdgcn_readlane((int)v, k) == v ? 1u : 0u;
    const uint32_t age = (n - 1u - (uint32_t)lane) % (uint32_t)SPEC_HIST;  // 0: the most recent
    const uint32_t score = lane < SPEC_HIST && v != 0u ? ((c * 16u + (15u - age)) << 16) | (v & 0xffffu) : 0u;
    return wave_max(score) & 0xffffu;
}
__device__ __forceinline__ uint32_t spec_count(uint32_t c, bool hit) {
    return hit ? (c < 7u ? c + 1u : 7u) : (c > 0u ? c - 1u : 0u);
}
__device__ __forceinline__ void spec_learn(uint32_t* hint, int bw, int escale, int lane) {
    const uint32_t n = spec_ld(hint + 6), vb = spec_ld(hint), vs = spec_ld(hint + 24), va = spec_ld(hint + 25);
    const uint32_t cnt = spec_ld(hint + 5);
    const bool in = lane < SPEC_HIST;
    uint32_t rs = in ? __hip_atomic_load(hint + 8 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    uint32_t rb = in ? __hip_atomic_load(hint + 16 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const uint32_t t = (uint32_t)bw + 1u;
    const uint32_t cnt2 = spec_count(cnt & 15u, spec_unscale(vb, 0) == t) |
                          (spec_count((cnt >> 4) & 15u, spec_unscale(vs, escale) == t) << 4) |
                          (spec_count((cnt >> 8) & 15u, spec_unscale(va, 0) == t) << 8);
    const uint32_t kb = (uint32_t)(bw + 1 + SPEC_K0), ks = kb + (uint32_t)escale;
    const uint32_t slot = n % (uint32_t)SPEC_HIST;
    // the alternation guess for the next pair: this pair's predecessor (two pairs back from it)
    const uint32_t prev = n > 0u ? (uint32_t)__builtin_amdgcn_readlane((int)rb, (int)((n - 1u) % (uint32_t)SPEC_HIST)) : 0u;
    if ((uint32_t)lane == slot) {
        rs = ks;
        rb = kb;
    }
    const uint32_t ms = spec_mode_wave(rs, n + 1u, lane), mb = spec_mode_wave(rb, n + 1u, lane);
    if (lane == 0) {
        __hip_atomic_store(hint + 8 + slot, ks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hint + 16 + slot, kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hint + 5, cnt2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hint + 6, n + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hint, mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hint + 24, ms, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hint + 25, prev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The residual rule (niti_resnet.hip): z = hi * 2^d + (lo >> r), arithmetic shift
__device__ __forceinline__ int32_t residual_z(int32_t hi, int32_t lo, int d, int r) {
    return hi * (1 << d) + (r >= 31 ? (lo < 0 ? -1 : 0) : lo >> r);
}

// kernel-span probe: every block writes its own {start, end} on the device wall clock into its
// slot pair (plain stores, host takes min start / max end).  The first form max-ed every block's
// start into one word with an atomic at block entry: 256 atomics on one address serialise at the
// memory side, and the block's first counted vmcnt wait held until its atomic had completed.
__device__ __forceinline__ unsigned long long span_begin(unsigned long long* span) {
    return span != nullptr ? __builtin_amdgcn_s_memrealtime() : 0ull;
}
__device__ __forceinline__ void span_end(unsigned long long* span, unsigned long long t0) {
    if (span != nullptr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const unsigned b = blockIdx.x + blockIdx.y * gridDim.x;
        if (threadIdx.x == 0 && b < (unsigned)SPAN_MAX_BLOCKS) {
            span[2 * b] = t0;
            span[2 * b + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// bijective XCD remap: blocks b, b+8, b+16, ... (one XCD under round-robin dispatch) get
// consecutive tile ids.  Speed only; any placement is correct.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `later` steps of this wave's loads (L each) are outstanding
template <int L, int MAXL>
__device__ __forceinline__ void wait_steps(int later) {
    if (MAXL >= 6 && later >= 6)
        wait_vmcnt<6 * L>();
    else if (MAXL >= 5 && later == 5)
        wait_vmcnt<5 * L>();
    else if (MAXL >= 4 && later == 4)
        wait_vmcnt<4 * L>();
    else if (MAXL >= 3 && later == 3)
        wait_vmcnt<3 * L>();
    else if (MAXL >= 2 && later == 2)
        wait_vmcnt<2 * L>();
    else if (MAXL >= 1 && later == 1)
        wait_vmcnt<L>();
    else
        wait_vmcnt<0>();
}

// 4 x 4 byte transpose inside a lane quad (j = lane & 3): byte r of lane k -> byte k of lane r.
// Every lane of the wave must execute it (DPP reads the quad partners' registers).
__device__ __forceinline__ uint32_t quad_transpose(uint32_t d, int j) {
    const uint32_t y1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, 0xB1, 0xF, 0xF, false);  // lane ^ 1
    d = __builtin_amdgcn_perm(y1, d, (j & 1) ? 0x03070105u : 0x06020400u);
    const uint32_t y2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, 0x4E, 0xF, 0xF, false);  // lane ^ 2
    return __builtin_amdgcn_perm(y2, d, (j & 2) ? 0x03020706u : 0x05040100u);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ v4i lds_b128(uint32_t a) {
    v4i r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
    return r;
}
// two transposed 8x8-byte reads, rows r and r+8 (ROW8 = 8 rows of the image in bytes)
__device__ __forceinline__ v4i lds_tr8x2(uint32_t a, int row8) {
    v2i x0, x1;
    asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(x0) : "v"(a));
    asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(x1) : "v"(a + row8));
    return v4i{x0[0], x0[1], x1[0], x1[1]};
}
// one transposed read at a compile-time immediate offset
template <int IMM>
__device__ __forceinline__ v2i tr8_at(uint32_t a) {
    v2i r;
    asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(IMM));
    return r;
}
template <int N>
__device__ __forceinline__ void lgkm_wait() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N < 15 ? N : 15));
}
// orders a use of v after the preceding (volatile) wait
__device__ __forceinline__ void reg_fence(v4i& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void reg_fence(v2i& v) { asm volatile("" : "+v"(v)); }

// LDS-DMA: 16 bytes per lane from the buffer into the wave's 1 KiB LDS block (lane-linear)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, int8_t* lds_wave_base, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff,
                                             soff, 0, 0);
}

// P16 conversion jobs (niti_wgrad.hip: nhwc16_to_p16_many; niti_kernels.hip: loss_grad_p16)
struct P16Job {
    const int8_t* in;
    int8_t* out;
    int64_t blocks;
    int lg;       // log2 CP
    uint32_t wg0; // first workgroup
};
struct P16Jobs {
    P16Job j[P16_MAX_JOBS];
    int n;
};

// one workgroup's share of a P16Jobs launch (256 threads; tile: 16 KiB of LDS, 16-byte aligned)
__device__ __forceinline__ void p16_convert_block(const P16Jobs& J, uint32_t wg, int8_t* tile) {
    int k = 0;
    while (k + 1 < J.n && wg >= J.j[k + 1].wg0) ++k;
    const P16Job jb = J.j[k];
    const int lg = jb.lg, cp = 1 << lg;
    const int bpw = lg < 8 ? 1 << (8 - lg) : 1;
    const int64_t b0 = (int64_t)(wg - jb.wg0) * bpw;
    const int nb = (int)(jb.blocks - b0 < bpw ? jb.blocks - b0 : bpw);
    const int bytes = nb * 16 * cp;
    const int8_t* src = jb.in + b0 * 16 * cp;
    for (int o = threadIdx.x * 16; o < bytes; o += 256 * 16) *(v4i*)(tile + o) = *(const v4i*)(src + o);
    __syncthreads();
    int8_t* dst = jb.out + b0 * 16 * cp;
    for (int t = threadIdx.x; t < (nb << lg); t += 256) {
        const int bl = t >> lg, c = t & (cp - 1);
        const uint8_t* s = (const uint8_t*)tile + (bl << (lg + 4)) + c;
        v4i o;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t w = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) w |= (uint32_t)s[(4 * q + e) << lg] << (8 * e);
            o[q] = (int)w;
        }
        *(v4i*)(dst + (int64_t)t * 16) = o;
    }
}

}  // namespace niti
