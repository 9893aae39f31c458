// niti_gridbar.hpp -- the in-kernel grid barrier with the range folded in, shared by the fused row
// kernels (niti_rowconv.hip) and the fused residual launch (niti_resnet.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "niti_kernels.hpp"

namespace niti {

// ---- grid barrier with the range folded in (mode FUSED) ---------------------------------------
// The requantisation needs only the tensor's bit width bw = ceil(log2 max|y|) (NITI_RangeEstimate),
// and the bit width of a max is the max of the bit widths.  Each workgroup ORs (1 << its bw) into
// its shard word and then adds (1 << 32) to the same 64-bit word -- two no-return atomics on ONE
// address, so they are performed in order and no wait sits between them: once a shard's count is
// complete, every OR of that shard is in.  One wave per workgroup polls the 8 shard words (lane s
// reads shard s with agent-scope loads, s_sleep between polls, bounded) until every count is
// complete; the global bw is the highest bit of the ORed words.  (The first form -- max words
// carried up a two-level tree by returning atomics and a released granule -- took ~3 us from the
// last arrival to the last release.)  Parity: launch e uses word set e & 1 and zeroes the other set
// for launch e + 1 (the launch that used it last has completed: same stream).
constexpr int BAR_LINE = 32;                         // words per 128-byte line
constexpr int BAR_WORDS = 19 * BAR_LINE;             // one parity (8 shard lines used)
static_assert(2 * BAR_WORDS == ROWCONV_BAR_WORDS, "barrier state size");
constexpr uint32_t BAR_SPIN_LIMIT = 1u << 22;  // ~seconds of polling: only a non-resident grid reaches it

__device__ __forceinline__ unsigned long long* bar_shard(uint32_t* base, int s) {
    return (unsigned long long*)(base + s * BAR_LINE);
}

// Called by one whole wave of each workgroup (lane 0's bw): the arrival, then -- after whatever
// work the workgroup can do meanwhile -- the wait, which returns the grid's bw to every lane.
__device__ inline void grid_bw_arrive(uint32_t* state, uint32_t epoch, int bw, int lane) {
    uint32_t* S = state + (epoch & 1) * BAR_WORDS;
    const int nwg = gridDim.x, b = blockIdx.x;
    const int nsh = nwg < 8 ? nwg : 8;
    if (b == 0 && lane < 8)  // reset the other parity for the next launch
        __hip_atomic_store(bar_shard(state + ((epoch + 1) & 1) * BAR_WORDS, lane), 0ull, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
        unsigned long long* w = bar_shard(S, b % nsh);
        __hip_atomic_fetch_or(w, 1ull << bw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(w, 1ull << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// A workgroup that is not resident never arrives: after spin_limit polls the waiters set *err
// (the Executions return NITI_NO_EXECUTION, the model step reports it: niti_model_rowconv_error)
// and go on with bw = 31 instead of hanging the GPU.
__device__ inline int grid_bw_wait(uint32_t* state, uint32_t epoch, uint32_t* err, uint32_t spin_limit, uint32_t extra,
                            int lane) {
    uint32_t* S = state + (epoch & 1) * BAR_WORDS;
    const int nwg = gridDim.x;
    const int nsh = nwg < 8 ? nwg : 8;
    // lane s < nsh polls shard s until its count is complete
    const uint32_t expect = lane < nsh ? (uint32_t)((nwg - lane + nsh - 1) / nsh) + (lane == 0 ? extra : 0u) : 0u;
    uint32_t spins = 0;
    unsigned long long v = 0;
    for (;;) {
        v = lane < nsh ? __hip_atomic_load(bar_shard(S, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const bool done = (uint32_t)(v >> 32) >= expect;
        if (__all(done)) break;
        if (++spins > spin_limit) {  // never hang the GPU: flag it and go on (results invalid)
            if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return 31;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    uint32_t bits = (uint32_t)v;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) bits |= __shfl_xor(bits, o, 64);
    return bits == 0u ? 0 : 31 - __clz((int)bits);
}

}  // namespace niti
