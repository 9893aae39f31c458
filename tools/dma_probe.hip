// LDS-DMA pipeline probe (diagnostic, GPU box): cycles per K step of a GEMM-like staging loop
// with no compute -- NB blocks of 8 waves, each step every wave issues LPW 1 KiB
// buffer_load_dwordx4 ... lds into a STAGES-deep ring, waits for the step STAGES-2 back with a
// counted vmcnt and passes a barrier.  Source: SRC_MB of memory read as rows of ROWB bytes at a
// row pitch of PITCH bytes (the VGG weight-gradient operands: 128 B runs at a 256 B pitch).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dma_probe.hip -o tools/bin/dma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int STAGES, int LPW, bool BARRIER>
__global__ void __launch_bounds__(512) probe_kernel(const int8_t* src, uint32_t bytes, int steps, int rowb, int pitch,
                                                    int* sink) {
    __shared__ __attribute__((aligned(16))) int8_t smem[STAGES * 8 * LPW * 1024];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(src, bytes);
    // lane's 16-byte chunk inside a 1 KiB instruction: rows of rowb bytes at pitch
    const int cpr = rowb / 16;
    const uint32_t lane_off = (uint32_t)((lane / cpr) * pitch + (lane % cpr) * 16);
    const uint32_t step_bytes = (uint32_t)(8 * LPW * (64 / cpr) * pitch);
    const uint32_t base = (uint32_t)(blockIdx.x * 7919u * 4096u) % (bytes / 2);
    auto issue = [&](int s) {
        int8_t* st = smem + (s % STAGES) * 8 * LPW * 1024;
#pragma unroll
        for (int i = 0; i < LPW; ++i) {
            const uint32_t off = (base + (uint32_t)s * step_bytes + (uint32_t)((wid * LPW + i) * (64 / cpr) * pitch)) %
                                 (bytes - 4096u);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(st + (wid * LPW + i) * 1024),
                                                     16, lane_off, off, 0, 0);
        }
    };
    for (int s = 0; s < STAGES - 1; ++s) issue(s);
    int acc = 0;
    for (int s = 0; s < steps; ++s) {
        wait_vmcnt<(STAGES - 2) * LPW>();
        if (BARRIER) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        issue(s + STAGES - 1);
        acc += smem[(s % STAGES) * 8 * LPW * 1024 + threadIdx.x];
    }
    wait_vmcnt<0>();
    if (acc == 0x7fffffff) sink[0] = acc;
}

// the same staging by plain 16-byte loads into VGPRs and ds_write_b128 (register ring of
// DEPTH steps: load step s+DEPTH while writing step s)
template <int STAGES, int LPW, int DEPTH>
__global__ void __launch_bounds__(512) reg_kernel(const int8_t* src, uint32_t bytes, int steps, int rowb, int pitch,
                                                  int* sink) {
    __shared__ __attribute__((aligned(16))) int8_t smem[STAGES * 8 * LPW * 1024];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t r = make_rsrc(src, bytes);
    const int cpr = rowb / 16;
    const uint32_t lane_off = (uint32_t)((lane / cpr) * pitch + (lane % cpr) * 16);
    const uint32_t step_bytes = (uint32_t)(8 * LPW * (64 / cpr) * pitch);
    const uint32_t base = (uint32_t)(blockIdx.x * 7919u * 4096u) % (bytes / 2);
    v4i ring[DEPTH][LPW];
    auto load = [&](int s, v4i (&dst)[LPW]) {
#pragma unroll
        for (int i = 0; i < LPW; ++i) {
            const uint32_t off = (base + (uint32_t)s * step_bytes + (uint32_t)((wid * LPW + i) * (64 / cpr) * pitch)) %
                                 (bytes - 4096u);
            dst[i] = __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, off, 0);
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) load(d, ring[d]);
    int acc = 0;
    for (int s = 0; s < steps; s += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            int8_t* st = smem + ((s + d) % STAGES) * 8 * LPW * 1024;
#pragma unroll
            for (int i = 0; i < LPW; ++i) *(v4i*)(st + (wid * LPW + i) * 1024 + lane * 16) = ring[d][i];
            load(s + d + DEPTH, ring[d]);
            __syncthreads();
            acc += smem[((s + d) % STAGES) * 8 * LPW * 1024 + threadIdx.x];
        }
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

#define CK(x)                                                     \
    do {                                                          \
        hipError_t e_ = (x);                                      \
        if (e_ != hipSuccess) {                                   \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                             \
        }                                                         \
    } while (0)

template <int STAGES, int LPW, bool BARRIER, int REG = 0>
static int run(const int8_t* src, uint32_t bytes, int nb, int rowb, int pitch, int* sink, const char* tag) {
    const int steps = 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(a, 0));
        if constexpr (REG > 0)
            hipLaunchKernelGGL((reg_kernel<STAGES, LPW, REG>), dim3(nb), dim3(512), 0, 0, src, bytes, steps, rowb, pitch,
                               sink);
        else
            hipLaunchKernelGGL((probe_kernel<STAGES, LPW, BARRIER>), dim3(nb), dim3(512), 0, 0, src, bytes, steps, rowb,
                               pitch, sink);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
    }
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double step_us = ms * 1e3 / steps;
    const double kb = 8.0 * LPW;
    printf("%-10s blocks %3d stages %d lpw %d barrier %d rowb %3d pitch %4d src %5u MB: %6.3f us/step  %7.1f cyc@2.4  %6.1f B/clk/CU\n",
           tag, nb, STAGES, LPW, (int)BARRIER, rowb, pitch, bytes >> 20, step_us, step_us * 2400,
           kb * 1024 / (step_us * 2400));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    int8_t* src;
    const size_t big = (size_t)1 << 30;
    CK(hipMalloc(&src, big));
    CK(hipMemset(src, 1, big));
    int* sink;
    CK(hipMalloc(&sink, 64));
    for (uint32_t mb : {4u, 512u}) {
        const uint32_t bytes = mb << 20;
        for (int nb : {36, 256}) {
            run<4, 2, true>(src, bytes, nb, 128, 256, sink, "base");
            run<4, 2, false>(src, bytes, nb, 128, 256, sink, "nobar");
            run<4, 4, true>(src, bytes, nb, 128, 256, sink, "lpw4");
            run<2, 2, true, 2>(src, bytes, nb, 128, 256, sink, "reg d2");
            run<2, 2, true, 4>(src, bytes, nb, 128, 256, sink, "reg d4");
            run<2, 4, true, 2>(src, bytes, nb, 128, 256, sink, "reg4 d2");
            run<2, 2, true, 4>(src, bytes, nb, 1024, 1024, sink, "reg d4 ctg");
        }
    }
    return 0;
}
