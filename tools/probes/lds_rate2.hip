// LDS read-rate probe 2 (diagnostic): cycles per CU-instruction of ds_read_b64_tr_b8 / ds_read_b64 /
// ds_read_b64_tr_b16 at 4 or 8 waves per CU with R reads in flight per wave between drains.
// hipcc --offload-arch=gfx950 -O3 -std=c++20 lds_rate2.hip -o lds_rate2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
typedef int v2i __attribute__((ext_vector_type(2)));

template <int MODE, int R>
__global__ void k(unsigned long long* out, int iters, int* sink) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[32768];
    for (int i = threadIdx.x; i < 32768 / 4; i += blockDim.x) ((int*)lds)[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int p = 16 * (lane >> 5) + ((lane & 15) >> 1);  // wgrad-taps fragment pattern
    uint32_t a = p * 32 + 16 * ((lane >> 4) & 1) + 8 * (lane & 1);
    a += ((threadIdx.x >> 6) & 7) * 1024;
    a += (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds;
    v2i acc = {0, 0};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        v2i r[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            if (MODE == 0)
                asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(r[j]) : "v"(a), "n"((j % 16) * 64));
            else if (MODE == 1)
                asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r[j]) : "v"(a), "n"((j % 16) * 64));
            else
                asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r[j]) : "v"(a), "n"((j % 16) * 64));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < R; ++j) acc += r[j];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (acc[0] == 0x12345 && acc[1] == 0x54321) sink[0] = 1;
}

template <int MODE, int R>
static void run(const char* name, int threads, int iters) {
    unsigned long long* d;
    int* sink;
    hipMalloc(&d, 256 * 8);
    hipMalloc(&sink, 4);
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k<MODE, R>), dim3(256), dim3(threads), 0, 0, d, iters, sink);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(256);
    hipMemcpy(h.data(), d, 256 * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double per_wave = (double)h[128] / iters / R;
    printf("%-10s waves/CU %2d reads/drain %2d: %6.2f cycles per CU-instruction\n", name, threads / 64, R,
           per_wave / (threads / 64));
    hipFree(d);
    hipFree(sink);
}

int main() {
    run<0, 16>("tr_b8", 256, 1000);
    run<0, 32>("tr_b8", 256, 1000);
    run<0, 16>("tr_b8", 512, 1000);
    run<0, 32>("tr_b8", 512, 1000);
    run<0, 32>("tr_b8", 1024, 1000);
    run<1, 32>("b64", 512, 1000);
    run<2, 32>("tr_b16", 512, 1000);
    return 0;
}
