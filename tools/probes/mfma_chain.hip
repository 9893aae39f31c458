// Probe: cycles per v_mfma_i32_32x32x32_i8 on one SIMD (one wave per SIMD) with NACC independent
// accumulators, and with a VALU-produced B operand (v_mov_b32_dpp + v_cndmask) written right
// before each MFMA, as the register-fed conv's kx taps are.  Prints cycles per MFMA (s_memtime).
//   hipcc --offload-arch=gfx950 -O3 -o mfma_chain mfma_chain.hip && ./mfma_chain
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int NACC, int MODE>
__global__ void __launch_bounds__(256, 1) chain(const v4i* in, int* out, unsigned long long* cyc, int iters) {
    const int lane = threadIdx.x & 63;
    v4i a = in[lane], b = in[64 + lane];
    v16i acc[NACC];
#pragma unroll
    for (int k = 0; k < NACC; ++k)
        for (int i = 0; i < 16; ++i) acc[k][i] = 0;
    const bool edge = (lane & 7) == 0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 36; ++j) {
            v4i bb = b;
            if constexpr (MODE == 1) {  // DPP row shift + edge mask per MFMA operand
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    int t = __builtin_amdgcn_update_dpp(0, b[q] + j, 0x111, 0xF, 0xF, true);
                    bb[q] = edge ? 0 : t;
                }
            }
            acc[j % NACC] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bb, acc[j % NACC], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int s = 0;
#pragma unroll
    for (int k = 0; k < NACC; ++k)
        for (int i = 0; i < 16; ++i) s += acc[k][i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC, int MODE>
static void run(v4i* in, int* out, unsigned long long* cyc) {
    const int iters = 64;
    hipLaunchKernelGGL((chain<NACC, MODE>), dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
    hipLaunchKernelGGL((chain<NACC, MODE>), dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256; ++i) s += (double)h[i];
    printf("accumulators %d, %s: %.1f cycles per MFMA\n", NACC, MODE ? "dpp+mask B operand" : "register B operand",
           s / 256 / (iters * 36.0));
}

int main() {
    v4i* in;
    int* out;
    unsigned long long* cyc;
    hipMalloc(&in, 128 * sizeof(v4i));
    hipMemset(in, 1, 128 * sizeof(v4i));
    hipMalloc(&out, 256 * 256 * sizeof(int));
    hipMalloc(&cyc, 256 * sizeof(unsigned long long));
    run<1, 0>(in, out, cyc);
    run<2, 0>(in, out, cyc);
    run<4, 0>(in, out, cyc);
    run<9, 0>(in, out, cyc);
    run<1, 1>(in, out, cyc);
    run<2, 1>(in, out, cyc);
    run<4, 1>(in, out, cyc);
    return 0;
}
