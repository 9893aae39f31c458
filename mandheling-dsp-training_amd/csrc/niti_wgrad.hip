// niti_wgrad.hip -- weight gradient of NITI_GradientConv_Int8 (NITI_GradientConv_Int8.cpp:165-298;
// graph grad/NITI_Conv_Int8_Grad.cpp:124-191) for stride-1, pad-1 3x3 convolutions.
//
//   C[co][tap][ci] = sum over output pixels p of dy[p][co] * x[p + tap][ci]      (exact int32)
//
// Operand layout P16 ("pixel blocks"): an activation of P pixels (n, y, x) and Cp channels
// (Cp % 32 == 0, P % 16 == 0) is stored as [P/16][Cp][16]: 16 consecutive pixels of one channel
// are 16 contiguous bytes, and consecutive channels follow each other.  That is exactly the
// operand fragment of v_mfma_i32_32x32x32_i8 (lane l: column l & 31, k = 16 (l >> 5) + 0..15),
// so every lane loads its fragment straight from memory -- 16 bytes, 32 lanes reading 512
// contiguous bytes -- with no LDS staging, no transposed reads and no barrier in the K loop.
// (The NHWC16 kernels in niti_kernels.hip stage 32-byte channel segments of pixel rows through
// LDS; at 256 channels each 1 KiB LDS-DMA touched 32 cache lines and the loop ran at ~36 % of
// the MFMA rate.)
//
// A 16-pixel block is whole output rows (OW = 8: 2 rows, OW = 16: 1 row) or whole images
// (OW = 4: one 4x4 image, OW = 2: four 2x2 images).  The taps' B fragments come from the lane's
// window -- its block plus the rows above and below (OW 8 / 16, zero outside the image) -- by
// byte shifts in registers: a kx shift moves bytes inside a row (v_alignbit, zero filled at the
// row ends), a ky shift selects rows.
//
// Block: 32 output channels x 9 taps x 32 input channels (9 accumulator tiles, 36 KiB of int32).
// Its NW waves (one per SIMD) split the block's K range into contiguous runs of 32-pixel K groups
// (two blocks, one per half-wave) that cover whole images.  Loads -- dy, the x block and the x
// rows above / below it -- run D K groups ahead in registers (inline-asm loads with counted
// waits); every address moves through the uniform soffset, out-of-range reads return zeros, so
// the loop has no per-iteration branch and almost no address arithmetic.  The waves meet through LDS once
// at the end: each adds its tile into one row-major LDS tile, which leaves as 16-byte row chunks.
//
// Split K: the blocks of a split tile store their partial tiles (plain stores, C's layout) into
// per-split slabs, which splitk_reduce_linear sums into C with the max|C| of NITI_RangeEstimate.
// (An in-launch combine -- write-through partials, an arrival ticket, the last block summing --
// was measured: the publish and the latency-bound combine took ~15 us of a 26 us launch.  Round 3
// measured it again on the current kernel -- plain slab stores, agent-scope fences around a
// per-tile arrival word, the last split summing the others' slabs with 36 loads in flight: an 8x8 layer
// 26.1 us against 10.3 us + a 4.8 us reduce launch, and the autotuner then preferred the taps
// kernel for conv4; step 0.423 ms against 0.403 ms.)
#include <hip/hip_ext.h>

#include <algorithm>
#include <type_traits>

#include "niti_device.hpp"
#include "niti_kernels.hpp"

namespace niti {

struct WgP16 {
    const int8_t* x;   // P16 [N*H*W/16][CIP][16]
    const int8_t* dy;  // P16 [N*OH*OW/16][COP][16]
    uint32_t xbytes, dybytes;
    int CIP, COP, c_out;
    int64_t ldc;       // C row pitch (elements): 9 * CIP
    int bpi;           // 16-pixel blocks per image (OW 8: 4, OW 16: 16)
    int kg_total, kg_per_split, kg_per_wave, splits;
    int tiles_ci, tiles;
    FastDiv fTiles, fTci;
    int32_t* C;
    uint32_t* amax;
    int32_t* slab;     // splits > 1: one C-shaped partial per split, slab_stride elements apart
    int64_t slab_stride;
    unsigned long long* span;
    unsigned long long* stamps;  // diagnostic builds
};

constexpr int P16_TILE = 9 * 32 * 32;  // int32 outputs per block tile
constexpr int P16_WAVES = 4;           // one wave per SIMD

// Diagnostic builds only (tools/wg_diag.sh): NITI_WG_STAMPS = 1 writes per-block s_memtime marks
// {start, loop entered, loop done, partials in LDS, output start, end, wall start, wall end} to the buffer armed by
// niti_diag_wgrad_stamps; NITI_WG_ABLATE skips a part (results wrong by design):
// 1 operand loads, 2 MFMA, 3 fragment shifts, 5 the output stores.
#ifndef NITI_WG_STAMPS
#define NITI_WG_STAMPS 0
#endif
#ifndef NITI_WG_ABLATE
#define NITI_WG_ABLATE 0
#endif
// NITI_WG_ATOMIC_OUT = 1 (diagnostic timing): split partials atomically added into C instead of slabs
// ring depth (K groups in flight) of the 8x8-image kernel; diagnostic builds vary it (the K loop
// ran the same 358 cycles per K group at depth 4, 6 and 8 on conv4; deeper rings only lengthen
// the prologue)
#ifndef NITI_WG_D8
#define NITI_WG_D8 4
#endif
#ifndef NITI_WG_D4  // ... and of the 4x4 / 2x2-image kernels
#define NITI_WG_D4 4
#endif
// merge of the 4 waves' partial tiles: 1 = register-owned quarters exchanged through LDS,
// 0 = ds_add into one LDS tile (diagnostic builds A/B them)
#ifndef NITI_WG_MERGE
#define NITI_WG_MERGE 1
#endif
#ifndef NITI_WG_NT_OUT
#define NITI_WG_NT_OUT 1
#endif
// NITI_WG_SWAP = 1: the MFMAs compute the transposed tile (x taps as A, dy taps as B), so after the
// merge a lane holds 4 consecutive ci of one co and the slab stores are 16 bytes wide
#ifndef NITI_WG_SWAP
#define NITI_WG_SWAP 1
#endif
#ifndef NITI_WG_ATOMIC_OUT
#define NITI_WG_ATOMIC_OUT 0
#endif
// (Measured and dropped, round 2: zeroing the accumulators ahead of the first ring wait, and a
// sched_group_barrier interleave of one MFMA with 2-3 VALU per K group -- 321 vs 342 cycles per K
// group, but the block end moved < 1 %: the merge and the output dominate the tail.)
// per-wave stamps (diagnostic): wave start and K-loop end after the 8 block stamps
#define WG_WSTAMP(k)                                                                                       \
    do {                                                                                                   \
        if (NITI_WG_STAMPS && g.stamps != nullptr && (threadIdx.x & 63) == 0)                              \
            g.stamps[gridDim.x * 8 + (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define WG_STAMP(k)                                                                            \
    do {                                                                                       \
        if (NITI_WG_STAMPS && g.stamps != nullptr && threadIdx.x == 0) {                        \
            g.stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime();                     \
            if ((k) == 0 || (k) == 5)                                                          \
                g.stamps[blockIdx.x * 8 + 6 + ((k) == 5)] = __builtin_amdgcn_s_memrealtime();  \
        }                                                                                      \
    } while (0)

__device__ __forceinline__ int ab(int hi, int lo, int s) {
    return (int)__builtin_amdgcn_alignbit((uint32_t)hi, (uint32_t)lo, (uint32_t)s);
}

// v_perm_b32 byte selectors for a 2x2 image in one dword (byte 2 oy + ox); 0x0c reads a zero byte
template <int DY, int DX>
constexpr uint32_t perm2x2() {  // out(oy, ox) = in(oy + DY, ox + DX)
    uint32_t s = 0;
    for (int i = 0; i < 4; ++i) {
        const int iy = (i >> 1) + DY, ix = (i & 1) + DX;
        const uint32_t b = (iy >= 0 && iy < 2 && ix >= 0 && ix < 2) ? (uint32_t)(2 * iy + ix) : 0x0cu;
        s |= b << (8 * i);
    }
    return s;
}

// The taps.  C[co][ky][kx][ci] = sum over (oy, ox) of dy[oy][ox - kx + 1][co] * x[oy + ky - 1][ox][ci]
// (substituting ox -> ox - kx + 1; dy and x read as zero outside the image): the kx shift moves
// along dy's rows, the ky shift selects x's rows.  A lane's dy fragment is 16 pixels (OW 8: two
// rows, OW 16: one row, OW 4: one 4x4 image, OW 2: four 2x2 images, one dword each); its x
// window adds the row above and below (OW 8 / 16).
//
// A operand for tap column kx: dy shifted by kx - 1 pixels inside each row, zero filled.
template <int OW, int KX>
__device__ __forceinline__ v4i dy_tap(v4i d) {
    if constexpr (KX == 1) {
        return d;
    } else if constexpr (OW == 8) {  // two 8-byte rows
        if constexpr (KX == 0)
            return v4i{ab(d[1], d[0], 8), (int)((uint32_t)d[1] >> 8), ab(d[3], d[2], 8), (int)((uint32_t)d[3] >> 8)};
        else
            return v4i{(int)((uint32_t)d[0] << 8), ab(d[1], d[0], 24), (int)((uint32_t)d[2] << 8), ab(d[3], d[2], 24)};
    } else if constexpr (OW == 16) {  // one 16-byte row
        if constexpr (KX == 0)
            return v4i{ab(d[1], d[0], 8), ab(d[2], d[1], 8), ab(d[3], d[2], 8), (int)((uint32_t)d[3] >> 8)};
        else
            return v4i{(int)((uint32_t)d[0] << 8), ab(d[1], d[0], 24), ab(d[2], d[1], 24), ab(d[3], d[2], 24)};
    } else if constexpr (OW == 4) {  // four 4-byte rows
        v4i r;
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = KX == 0 ? (int)((uint32_t)d[i] >> 8) : (int)((uint32_t)d[i] << 8);
        return r;
    } else {  // four 2x2 images
        constexpr uint32_t sel = perm2x2<0, 1 - KX>();
        v4i r;
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = (int)__builtin_amdgcn_perm((uint32_t)d[i], (uint32_t)d[i], sel);
        return r;
    }
}

// B operand for tap row ky from the lane's block and the rows above / below it (OW 8: 8-byte
// rows in .xy, OW 16: whole 16-byte rows; OW 4 / 2: the block is whole images)
template <int OW, int KY>
__device__ __forceinline__ v4i x_tap(const v4i& up, const v4i& x, const v4i& dn) {
    if constexpr (KY == 1) {
        return x;
    } else if constexpr (OW == 8) {
        return KY == 0 ? v4i{up[0], up[1], x[0], x[1]} : v4i{x[2], x[3], dn[0], dn[1]};
    } else if constexpr (OW == 16) {
        return KY == 0 ? up : dn;
    } else if constexpr (OW == 4) {
        return KY == 0 ? v4i{0, x[0], x[1], x[2]} : v4i{x[1], x[2], x[3], 0};
    } else {
        constexpr uint32_t sel = perm2x2<KY - 1, 0>();
        v4i r;
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = (int)__builtin_amdgcn_perm((uint32_t)x[i], (uint32_t)x[i], sel);
        return r;
    }
}

__device__ __forceinline__ v2i asm_load8(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    v2i v;
    asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(r), "s"(soff));
    return v;
}
__device__ __forceinline__ v4i asm_load16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    v4i v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(r), "s"(soff));
    return v;
}

template <int OW, int NW, int D>
__global__ void __launch_bounds__(NW * 64) wgrad_p16_kernel(WgP16 g) {
    static_assert(D >= 2 && D % 2 == 0, "the next K group's window must be resident; operand buffers alternate");
    // the block's tile, row-major [co 32][tap 9][ci 32] int32 (every wave adds its partial into it),
    // plus the block-max scratch
    // merge 0: one row-major LDS tile every wave ds_adds into; merge 1: quarter slots
    // [src wave][dst wave][tap][lane] (16 x 9 KiB, the 4 diagonal slots unused)
    constexpr int SMEM = (NITI_WG_MERGE ? 4 * P16_TILE * 4 : P16_TILE * 4) + 64;
    // typed as 16-byte vectors: the exchange stores / loads go through lds4 itself (byte-array
    // storage accessed as v4i is an aliasing violation the optimiser is free to act on)
    __shared__ v4i lds4[SMEM / 16];
    int8_t* smem = (int8_t*)lds4;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const unsigned long long span_t0 = span_begin(g.span);
    WG_STAMP(0);
    WG_WSTAMP(0);
    const int logical = xcd_remap(blockIdx.x, gridDim.x);
    const int split = (int)fdiv(g.fTiles, (uint32_t)logical);
    const int tile = logical - split * g.tiles;
    const int tco = (int)fdiv(g.fTci, (uint32_t)tile), tci = tile - tco * g.tiles_ci;
    const int co0 = tco * 32, ci0 = tci * 32;
    // the wave's K groups: a contiguous run [kb, kb + n_w) of the block's split, whole images
    // (kg_per_split and kg_per_wave are multiples of the K groups per image)
    const int kg_begin = split * g.kg_per_split;
    const int kg_end = min(g.kg_total, kg_begin + g.kg_per_split);
    const int kb = kg_begin + wid * g.kg_per_wave;
    const int n_w = max(0, min(kg_end, kb + g.kg_per_wave) - kb);

    const __amdgpu_buffer_rsrc_t rX = make_rsrc(g.x, g.xbytes);
    const __amdgpu_buffer_rsrc_t rD = make_rsrc(g.dy, g.dybytes);
    const int h = lane >> 5, c = lane & 31;
    // byte offsets of the lane's fragment in K group kg: block b = 2 kg + h
    const uint32_t xrow = (uint32_t)g.CIP * 16u, drow = (uint32_t)g.COP * 16u;
    const uint32_t lx = (uint32_t)h * xrow + (uint32_t)(ci0 + c) * 16u;
    const uint32_t ld = (uint32_t)h * drow + (uint32_t)(co0 + c) * 16u;
    // The ring loads are inline asm, so their vmcnt is ours (hipcc's waitcnt insertion drained the
    // ring at the loop head).  A lane's voffset is fixed (channel, half-wave, image position of
    // the K group); the K group moves the uniform soffset.  The range check covers voffset +
    // soffset (measured, tools/probes/soffset_probe.hip), so look-ahead past the tensor reads
    // zeros, and dy past the wave's run is pushed out of range through its soffset.
    constexpr uint32_t OOBS = 0x80000000u;
    const uint32_t ci16 = (uint32_t)(ci0 + c) * 16u;

    v16i acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0;
    int32_t* tile_lds = (int32_t*)smem;
    if (!NITI_WG_MERGE)
        for (int e = tid; e < P16_TILE / 4; e += NW * 64) ((v4i*)tile_lds)[e] = v4i{0, 0, 0, 0};

    // OW 8 / 16: the rows above / below the lane's block are loaded as well (OW 8: the 8-byte row
    // of the block before / after, OW 16: the whole block).  Runs are whole images (KPI K groups
    // each), so the image position of every unrolled step is known: the first K group of an image
    // has no row above its first block, the last none below its second block.
    //   above, first K group of an image: half 1 <- block 2 kg (its own K group), half 0 zero
    //   above, otherwise: block 2 kg + h - 1 (soffset one block back)
    //   below: block 2 kg + h + 1; the last K group's half 1 zero
    constexpr bool NB = OW == 8 || OW == 16;
    constexpr int KPI = OW == 8 ? 2 : OW == 16 ? 8 : 1;  // K groups per image
    constexpr uint32_t UPOFF = OW == 8 ? 8u : 0u;       // the block above's last row
    constexpr int L = NB ? 4 : 2;                        // loads per K group
    static_assert(D % KPI == 0, "unrolled steps cover whole images");
    const uint32_t vup_first = h ? ci16 + UPOFF : OOB, vup = lx + UPOFF;
    const uint32_t vdn = lx + xrow, vdn_last = h ? OOB : lx + xrow;
    // ring slot: dy, the x block, the rows above / below (OW 8: one 8-byte row each)
    typedef typename std::conditional<OW == 8, v2i, v4i>::type Row;
    struct Ring {
        v4i d, x;
        Row up, dn;
    };
    Ring ring[D];
    auto issue = [&](Ring& r, auto u_c, int j) {
        constexpr int U = decltype(u_c)::value;
        const uint32_t sx = (uint32_t)(kb + j) * 2u * xrow;
        const uint32_t sd = j < n_w ? (uint32_t)(kb + j) * 2u * drow : OOBS;
        if (NITI_WG_ABLATE == 1) return;
        r.d = asm_load16(rD, ld, sd);
        r.x = asm_load16(rX, lx, sx);
        if constexpr (NB) {
            constexpr bool first = U % KPI == 0, last = U % KPI == KPI - 1;
            if constexpr (OW == 8) {
                r.up = first ? asm_load8(rX, vup_first, sx) : asm_load8(rX, vup, sx - xrow);
                r.dn = asm_load8(rX, last ? vdn_last : vdn, sx);
            } else {
                r.up = first ? asm_load16(rX, vup_first, sx) : asm_load16(rX, vup, sx - xrow);
                r.dn = asm_load16(rX, last ? vdn_last : vdn, sx);
            }
        }
    };
    [&]<int... U>(std::integer_sequence<int, U...>) {
        ((ring[U] = Ring{}, issue(ring[U], std::integral_constant<int, U>(), U)), ...);
    }(std::make_integer_sequence<int, D>());
    WG_STAMP(1);
    // Software pipeline: the tap operands of K group j + 1 (dy shifted for kx = 0 / 2, x rows for
    // ky = 0 / 2; kx = ky = 1 are the ring registers themselves) are built while K group j's nine
    // MFMAs run, so the VALU work fills MFMA gaps instead of stalling the pipe at every K group.
    struct Ops {
        v4i a0, a2, b0, b2;
    };
    Ops ops[2];
    auto prep = [&](Ring& r, Ops& o) {
        reg_fence(r.d);
        reg_fence(r.x);
        if constexpr (NB) {
            reg_fence(r.up);
            reg_fence(r.dn);
        }
        v4i up{0, 0, 0, 0}, dn{0, 0, 0, 0};
        if constexpr (OW == 8) {
            up = v4i{r.up[0], r.up[1], 0, 0};
            dn = v4i{r.dn[0], r.dn[1], 0, 0};
        } else if constexpr (OW == 16) {
            up = r.up;
            dn = r.dn;
        }
        if constexpr (NITI_WG_ABLATE == 3) {
            o.a0 = o.a2 = r.d;
            o.b0 = o.b2 = r.x;
        } else {
            o.a0 = dy_tap<OW, 0>(r.d);
            o.a2 = dy_tap<OW, 2>(r.d);
            o.b0 = x_tap<OW, 0>(up, r.x, dn);
            o.b2 = x_tap<OW, 2>(up, r.x, dn);
        }
    };
    wait_vmcnt<L * (D - 1)>();  // K group 0 has landed
    prep(ring[0], ops[0]);
    auto step = [&](auto u_c, int j0) {
        constexpr int u = decltype(u_c)::value, un = (u + 1) % D;
        // K group j + 1 has landed (j + 2 .. j + D - 1 may still be in flight): its operands
        wait_vmcnt<L * (D - 2)>();
        prep(ring[un], ops[(u + 1) & 1]);
        const Ops& o = ops[u & 1];
        const v4i A[3] = {o.a0, ring[u].d, o.a2};
        const v4i B[3] = {o.b0, ring[u].x, o.b2};
        [&]<int... T>(std::integer_sequence<int, T...>) {
            (([&] {
                 constexpr int KY = T / 3, KX = T % 3;
                 if constexpr (NITI_WG_ABLATE == 2)
                     acc[T][0] += A[KX][0] ^ B[KY][1];
                 else if constexpr (NITI_WG_MERGE && NITI_WG_SWAP)  // C^T: a lane holds one co, rows = ci
                     acc[T] = __builtin_amdgcn_mfma_i32_32x32x32_i8(B[KY], A[KX], acc[T], 0, 0, 0);
                 else
                     acc[T] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[KX], B[KY], acc[T], 0, 0, 0);
             }()),
             ...);
        }(std::make_integer_sequence<int, 9>());
        // slot u is free again: K group j + D
        issue(ring[u], u_c, j0 + u + D);
    };
    for (int j0 = 0; j0 < n_w; j0 += D) {
        [&]<int... U>(std::integer_sequence<int, U...>) {
            (step(std::integral_constant<int, U>(), j0), ...);
        }(std::make_integer_sequence<int, D>());
    }
    // The last D look-ahead loads (and all of them for a wave without K groups) are never consumed:
    // to hipcc their destination registers are dead at once, and it may hand them to other values
    // while the loads are still in flight.  Drain, then touch every ring register, so none of them
    // is reused before its data has landed.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < D; ++u) {
        reg_fence(ring[u].d);
        reg_fence(ring[u].x);
        if constexpr (NB) {
            reg_fence(ring[u].up);
            reg_fence(ring[u].dn);
        }
    }
    WG_STAMP(2);
    WG_WSTAMP(1);

    constexpr int THREADS = NW * 64;
    const bool partial = g.splits > 1;
    int32_t* dst = partial ? g.slab + (int64_t)split * g.slab_stride : g.C;
    uint32_t lmax = 0;
    uint32_t* red = (uint32_t*)(smem + SMEM - 64);
    if constexpr (NITI_WG_MERGE) {
        static_assert(NW == 4, "one accumulator row quarter per wave");
        if constexpr (NITI_WG_SWAP) {
            // The tile is C^T: lane (co = lane & 31, h = lane >> 5) holds, in accumulator registers
            // 4q..4q+3, the 16 bytes ci 8q + 4h + 0..3 of row co.  Wave w owns rows co 8w..8w+7:
            // every wave writes its whole partial tile to LDS, slot [src wave][q][tap], and wave w's
            // lane (r = lane >> 3, c = lane & 7) sums the four waves' 16 bytes ci 4c..4c+3 of row
            // 8w + r -- so each store instruction covers 8 rows x 128 contiguous bytes (9 16-byte
            // stores per wave; the tail is store-issue bound, 36 dword stores took 3x as long).
            // The lane position inside a slot is XOR-swizzled by s = (2q + h) + 8 (q & 1): a
            // ds_write_b128 group (8 consecutive lanes, fixed q and h) stays a permutation of one
            // 128-byte run, and the 16 lanes of each ds_read_b128 group ({0-3,12-15,20-27}, ...)
            // land on 16 different 16-byte bank slots (XOR by 2q + h alone leaves them 2-way).
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int t = 0; t < 9; ++t)
                    lds4[((wid * 4 + q) * 9 + t) * 64 + (lane ^ (2 * q + (lane >> 5) + 8 * (q & 1)))] =
                        v4i{acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
            __syncthreads();  // every partial tile is in LDS (waits for the slowest wave's K loop)
            WG_STAMP(3);
            const int r = lane >> 3, c = lane & 7, co = 8 * wid + r;
            const int pos = (co + 32 * (c & 1)) ^ (c + 8 * ((c >> 1) & 1)), q = c >> 1;
            v4i sum[9];
#pragma unroll
            for (int t = 0; t < 9; ++t) sum[t] = lds4[((0 * 4 + q) * 9 + t) * 64 + pos];
#pragma unroll
            for (int w = 1; w < 4; ++w)
#pragma unroll
                for (int t = 0; t < 9; ++t) sum[t] += lds4[((w * 4 + q) * 9 + t) * 64 + pos];
            WG_STAMP(4);
            if (co0 + co < g.c_out && NITI_WG_ABLATE != 5) {
                int32_t* o = dst + (int64_t)(co0 + co) * g.ldc + ci0 + 4 * c;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    __builtin_nontemporal_store(sum[t], (v4i*)(o + t * g.CIP));
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t u = uabs32(sum[t][j]);
                        lmax = lmax > u ? lmax : u;
                    }
                }
            }
        } else {
        // The waves meet through 16-byte lane-linear LDS writes: quarter q of a wave's partial tile
        // is accumulator registers 4q..4q+3 (rows 8q + 0..3 + 4h); wave w owns quarter w, sends
        // the other three to their owners, adds the three it receives to its own and stores those
        // rows straight from registers -- no atomics, no row-major staging tile.
        // slot [src wave][dst wave][tap][lane]: a wave writes only the three quarters it does
        // not own and keeps its own quarter in registers
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q != wid) {
#pragma unroll
                for (int t = 0; t < 9; ++t)
                    lds4[((wid * 4 + q) * 9 + t) * 64 + lane] =
                        v4i{acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
            }
        v4i sum[9];
        switch (wid) {  // the own quarter, registers 4w..4w+3 (static indices per case)
#define NITI_OWN(W)                                                                                          \
    case W:                                                                                                  \
        for (int t = 0; t < 9; ++t) sum[t] = v4i{acc[t][4 * W], acc[t][4 * W + 1], acc[t][4 * W + 2], acc[t][4 * W + 3]}; \
        break;
            NITI_OWN(0)
            NITI_OWN(1)
            NITI_OWN(2)
            default:
                NITI_OWN(3)
#undef NITI_OWN
        }
        __syncthreads();  // every quarter is in LDS (waits for the slowest wave's K loop)
        WG_STAMP(3);
#pragma unroll
        for (int k = 1; k < 4; ++k) {  // the other three waves, no branches: all 27 reads in flight
            const int w = (wid + k) & 3;
#pragma unroll
            for (int t = 0; t < 9; ++t) sum[t] += lds4[((w * 4 + wid) * 9 + t) * 64 + lane];
        }
        WG_STAMP(4);
        // rows 8w + j + 4h, column lane & 31: 128-byte runs per half-wave and register
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 8 * wid + j + 4 * (lane >> 5);
            if (co0 + row < g.c_out && NITI_WG_ABLATE != 5) {
                int32_t* o = dst + (int64_t)(co0 + row) * g.ldc + ci0 + (lane & 31);
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int32_t v = sum[t][j];
                    __builtin_nontemporal_store(v, o + t * g.CIP);
                    const uint32_t u = uabs32(v);
                    lmax = lmax > u ? lmax : u;
                }
            }
        }
        }
    } else {
    // the waves meet: each adds its partial tile into the zeroed LDS tile (ds_add, the two
    // half-waves on separate 128-byte rows); then every thread stores 16-byte row chunks
    __syncthreads();  // the zeroed tile (the K loop has no barrier; this one waits for the slowest wave)
    WG_STAMP(3);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
            __hip_atomic_fetch_add(tile_lds + (row * 9 + t) * 32 + (lane & 31), acc[t][i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    __syncthreads();
    WG_STAMP(4);

    // ---- output: C[co][tap][ci] (S = 1), or this split's C-shaped partial (reduced by
    // splitk_reduce_linear); chunk c = (row, tap, 4 columns)
    for (int c = tid; c < P16_TILE / 4; c += THREADS) {
        const int row = c / 72, rem = c - row * 72, t = rem >> 3, c4 = rem & 7;
        const v4i v = ((const v4i*)tile_lds)[c];
        if (co0 + row < g.c_out && NITI_WG_ABLATE != 5) {
            if (NITI_WG_ATOMIC_OUT && partial) {  // diagnostic: split-K partials added into C
                int32_t* q = g.C + (int64_t)(co0 + row) * g.ldc + t * g.CIP + ci0 + 4 * c4;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    __hip_atomic_fetch_add(q + e, v[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (NITI_WG_NT_OUT) {  // streaming stores: the partials leave L2 during the kernel
                __builtin_nontemporal_store(v, (v4i*)(dst + (int64_t)(co0 + row) * g.ldc + t * g.CIP + ci0 + 4 * c4));
            } else {
                *(v4i*)(dst + (int64_t)(co0 + row) * g.ldc + t * g.CIP + ci0 + 4 * c4) = v;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t u = uabs32(v[e]);
                lmax = lmax > u ? lmax : u;
            }
        }
    }
    }
    if (!partial && g.amax != nullptr) {
        lmax = wave_max(lmax);
        if (lane == 0) red[wid] = lmax;
        __syncthreads();
        if (tid == 0) {
            uint32_t m = red[0];
            for (int w = 1; w < NW; ++w) m = m > red[w] ? m : red[w];
            publish_max(g.amax, m);
        }
    }
    if (NITI_WG_STAMPS) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        WG_STAMP(5);
    }
    span_end(g.span, span_t0);
}

// NHWC16 [P][CP] -> P16 [P/16][CP][16].  A 16-pixel block is 16 * CP contiguous bytes on both
// sides (16 rows of CP channels in, CP rows of 16 pixels out), so each workgroup copies whole
// blocks into LDS with 16-byte coalesced loads and writes them back transposed: a lane gathers one
// channel's 16 pixels with byte reads (4 lanes share each LDS dword, no bank conflicts) and stores
// one 16-byte chunk, consecutive lanes consecutive chunks.  CP is a power of two from 32 to 1024:
// a workgroup takes 256 / CP blocks (CP <= 256) or one block (CP > 256).  One launch serves up to
// P16_MAX_JOBS tensors, each owning a contiguous range of workgroups.
__global__ void __launch_bounds__(256) nhwc16_to_p16_kernel(P16Jobs J) {
    __shared__ __attribute__((aligned(16))) int8_t tile[16 * 1024];
    p16_convert_block(J, blockIdx.x, tile);
}

// any CP % 16 == 0: one thread per (16-pixel block, 16-channel chunk), a 16 x 16 byte transpose
// in registers
__global__ void nhwc16_to_p16_any_kernel(const int8_t* __restrict__ in, int64_t blocks, int cp,
                                         int8_t* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int cc = cp / 16;
    if (e >= blocks * cc) return;
    const int64_t b = e / cc;
    const int c16 = (int)(e - b * cc);
    v16c px[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) px[p] = *(const v16c*)(in + ((b * 16 + p) * cp + c16 * 16));
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        v16c o;
#pragma unroll
        for (int p = 0; p < 16; ++p) o[p] = px[p][k];
        *(v16c*)(out + (b * cp + c16 * 16 + k) * 16) = o;
    }
}

// the power-of-two-CP jobs as one P16Jobs launch of *wgs workgroups; any other CP runs its own
// generic launch here
hipError_t p16_jobs_build(const P16Conv* jobs, int n, hipStream_t st, P16Jobs* out, uint32_t* wgs_out) {
    if (n < 0 || n > P16_MAX_JOBS) return hipErrorInvalidValue;
    P16Jobs& J = *out;
    J = P16Jobs{};
    uint32_t wg = 0;
    for (int i = 0; i < n; ++i) {
        const P16Conv& c = jobs[i];
        if (c.cp <= 0 || c.cp % 16 != 0 || c.pixels < 0 || c.pixels % 16 != 0) return hipErrorInvalidValue;
        if (c.pixels == 0) continue;
        const int64_t blocks = c.pixels / 16;
        if ((c.cp & (c.cp - 1)) != 0 || c.cp < 32 || c.cp > 1024) {  // not a power of two: generic kernel
            const int64_t t = blocks * (c.cp / 16);
            hipLaunchKernelGGL(nhwc16_to_p16_any_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, c.in,
                               blocks, c.cp, c.out);
            continue;
        }
        int lg = 0;
        while ((1 << lg) < c.cp) ++lg;
        const int bpw = lg < 8 ? 1 << (8 - lg) : 1;
        const int64_t wgs = (blocks + bpw - 1) / bpw;
        if ((int64_t)wg + wgs > 0x7fffffff) return hipErrorInvalidValue;
        J.j[J.n++] = P16Job{c.in, c.out, blocks, lg, wg};
        wg += (uint32_t)wgs;
    }
    *wgs_out = wg;
    return hipGetLastError();
}

hipError_t nhwc16_to_p16_many(const P16Conv* jobs, int n, hipStream_t st) {
    P16Jobs J;
    uint32_t wg = 0;
    hipError_t e = p16_jobs_build(jobs, n, st, &J, &wg);
    if (e != hipSuccess) return e;
    if (J.n > 0) hipLaunchKernelGGL(nhwc16_to_p16_kernel, dim3(wg), dim3(256), 0, st, J);
    return hipGetLastError();
}

hipError_t nhwc16_to_p16(const int8_t* in, int64_t pixels, int cp, int8_t* out, hipStream_t st) {
    const P16Conv c{in, pixels, cp, out};
    return nhwc16_to_p16_many(&c, 1, st);
}

// ---- host side --------------------------------------------------------------------------------
static unsigned long long* g_wg_stamps = nullptr;  // diagnostic builds: armed by niti_diag_wgrad_stamps
void wgrad_stamps_arm(unsigned long long* buf) { g_wg_stamps = buf; }

static bool p16_geom(const ConvGeom& g, WgP16* t) {
    if (g.kh != 3 || g.kw != 3 || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1) return false;
    if (g.pt != 1 || g.pl != 1 || g.pb != 1 || g.pr != 1) return false;
    if (g.cip % 32 != 0 || g.cop % 32 != 0) return false;
    // a 16-pixel block is whole rows (OW 8 / 16) or whole images (OW 4 / 2)
    const int ow = g.ow, oh = g.oh;
    // square images (the block-in-image masks use a power-of-two block count: 4 for 8x8, 16 for 16x16)
    if (oh != ow || !(ow == 8 || ow == 16 || ow == 4 || ow == 2)) return false;
    const int64_t po = (int64_t)g.n * oh * ow;
    if (po % 32 != 0) return false;  // whole K groups (two blocks)
    if (po * g.cip > 0x7fffffff || po * g.cop > 0x7fffffff) return false;
    WgP16 w{};
    w.CIP = g.cip;
    w.COP = g.cop;
    w.c_out = g.c_out;
    w.ldc = (int64_t)9 * g.cip;
    w.bpi = ow == 8 ? oh / 2 : ow == 16 ? oh : 1;
    w.xbytes = (uint32_t)(po * g.cip);
    w.dybytes = (uint32_t)(po * g.cop);
    w.kg_total = (int)(po / 32);
    w.tiles_ci = g.cip / 32;
    w.tiles = (g.cop / 32) * w.tiles_ci;
    w.fTci = make_fastdiv((uint32_t)w.tiles_ci);
    *t = w;
    return true;
}

bool conv_wgrad_p16_ok(const ConvGeom& g) {
    WgP16 t;
    return p16_geom(g, &t);
}

// default split count: one block per CU, at most 8 partial tiles per combine
int conv_wgrad_p16_splits(const ConvGeom& g) {
    WgP16 t;
    if (!p16_geom(g, &t)) return 0;
    const int kpi = g.ow == 8 ? 2 : g.ow == 16 ? 8 : 1;
    int s = std::max(1, 256 / t.tiles);
    s = std::min(s, 8);
    s = std::min(s, std::max(1, t.kg_total / kpi));
    return s;
}

static int64_t p16_slab_stride(const ConvGeom& g) {
    // an odd number of 4 KiB pages between slabs: the S reads of one element hit different channels
    const int64_t bytes = (int64_t)g.c_out * 9 * g.cip * 4;
    return ((bytes + 4095) / 4096 | 1) * 1024;
}

size_t conv_wgrad_p16_workspace(const ConvGeom& g, int splits) {
    WgP16 t;
    if (!p16_geom(g, &t)) return 0;
    if (splits <= 0) splits = conv_wgrad_p16_splits(g);
    return splits > 1 ? (size_t)splits * p16_slab_stride(g) * 4 : 0;
}

hipError_t conv_wgrad_p16(const ConvGeom& g, const int8_t* x_p16, const int8_t* dy_p16, int32_t* acc,
                          uint32_t* amax, void* ws, size_t ws_bytes, int splits, hipStream_t st, hipEvent_t ev_b,
                          hipEvent_t ev_e, unsigned long long* span, SgdJob* defer) {
    WgP16 t;
    if (!p16_geom(g, &t)) return hipErrorInvalidValue;
    if (splits <= 0) splits = conv_wgrad_p16_splits(g);
    if (splits < 1 || splits > 64) return hipErrorInvalidValue;
    t.x = x_p16;
    t.dy = dy_p16;
    // splits and wave runs cover whole images (K groups per image: 2 for 8x8, 8 for 16x16)
    const int kpi = g.ow == 8 ? 2 : g.ow == 16 ? 8 : 1;
    auto round_kpi = [&](int v) { return (v + kpi - 1) / kpi * kpi; };
    t.kg_per_split = round_kpi((t.kg_total + splits - 1) / splits);
    t.splits = (t.kg_total + t.kg_per_split - 1) / t.kg_per_split;  // no empty split
    t.kg_per_wave = round_kpi((t.kg_per_split + P16_WAVES - 1) / P16_WAVES);
    if (t.splits > 1 && (ws == nullptr || ws_bytes < (size_t)t.splits * p16_slab_stride(g) * 4))
        return hipErrorInvalidValue;
    t.fTiles = make_fastdiv((uint32_t)t.tiles);
    t.C = acc;
    t.amax = amax;
    t.slab = (int32_t*)ws;
    t.slab_stride = p16_slab_stride(g);
    t.span = span;
    t.stamps = g_wg_stamps;
    constexpr int NW = P16_WAVES;
    const dim3 grid((unsigned)(t.tiles * t.splits));
    auto launch = [&](auto k) {
        if (ev_b != nullptr && ev_e != nullptr)
            hipExtLaunchKernelGGL(k, grid, dim3(NW * 64), 0, st, ev_b, ev_e, 0, t);
        else
            hipLaunchKernelGGL(k, grid, dim3(NW * 64), 0, st, t);
    };
    switch (g.ow) {
        case 8: launch(wgrad_p16_kernel<8, NW, NITI_WG_D8>); break;
        case 16: launch(wgrad_p16_kernel<16, NW, 8>); break;
        case 4: launch(wgrad_p16_kernel<4, NW, NITI_WG_D4>); break;
        default: launch(wgrad_p16_kernel<2, NW, NITI_WG_D4>); break;
    }
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && t.splits > 1) {
        const int64_t n = (int64_t)g.c_out * 9 * g.cip;
        if (defer != nullptr) {  // the NITI_SGD launch combines the slabs (sgd_update_many)
            defer->slab = t.slab;
            defer->splits = t.splits;
            defer->slab_stride = t.slab_stride;
            defer->slab_n = n;
        } else {
            e = splitk_reduce_linear(t.slab, t.splits, n, t.slab_stride, acc, amax, st);
        }
    }
    return e;
}

}  // namespace niti
