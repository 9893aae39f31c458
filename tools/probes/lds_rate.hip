// LDS read-rate probe (diagnostic, not product code): cycles per wave-instruction of
// ds_read_b64_tr_b8 vs ds_read_b64 for the tap-sharing weight-gradient fragment pattern
// (8 consecutive 32-byte rows per half-wave) and for a linear pattern, 4 waves per CU,
// every CU busy.  Build: hipcc --offload-arch=gfx950 -O3 lds_rate.hip -o lds_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
typedef int v2i __attribute__((ext_vector_type(2)));

template <int MODE, int PAT>
__global__ void __launch_bounds__(256) k(unsigned long long* out, int iters, int* sink) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[16384];
    for (int i = threadIdx.x; i < 16384 / 4; i += 256) ((int*)lds)[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t a;
    if (PAT == 0) {  // wgrad-taps x fragment: row (lane&15)>>1 (+16 for the upper half), 8-byte col
        const int p = 16 * (lane >> 5) + ((lane & 15) >> 1);
        a = p * 32 + 16 * ((lane >> 4) & 1) + 8 * (lane & 1);
    } else {  // linear
        a = lane * 8;
    }
    a += (threadIdx.x >> 6) * 2048;
    a += (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds;
    v2i acc = {0, 0};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        v2i r[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (MODE == 0)
                asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(r[j]) : "v"(a), "n"(j * 64));
            else
                asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[j]) : "v"(a), "n"(j * 64));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += r[j];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (acc[0] == 0x12345 && acc[1] == 0x54321) sink[0] = 1;
}

template <int MODE, int PAT>
static void run(const char* name, int iters) {
    unsigned long long* d;
    int* sink;
    hipMalloc(&d, 256 * 8);
    hipMalloc(&sink, 4);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k<MODE, PAT>), dim3(256), dim3(256), 0, 0, d, iters, sink);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(256);
    hipMemcpy(h.data(), d, 256 * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double cyc = (double)h[128] / iters / 16;  // per wave-instruction, 4 waves per CU issuing
    printf("%-28s %6.2f cycles per wave-instruction per wave (%.2f per CU-instruction)\n", name, cyc, cyc / 4);
    hipFree(d);
    hipFree(sink);
}

int main() {
    run<0, 0>("tr_b8  taps pattern", 2000);
    run<1, 0>("b64    taps pattern", 2000);
    run<0, 1>("tr_b8  linear", 2000);
    run<1, 1>("b64    linear", 2000);
    return 0;
}
