// Probe the lane mapping of ds_read_b64_tr_b8 on gfx950 (diagnostic, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(unsigned char* out, int mode) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = (unsigned char)(i & 255);
    __syncthreads();
    int addr = mode == 0 ? threadIdx.x * 8 : (threadIdx.x & 15) * 16 + (threadIdx.x >> 4) * 8;
    v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(lds + addr));
    unsigned char* b = (unsigned char*)&v;
    for (int j = 0; j < 8; ++j) out[threadIdx.x * 8 + j] = b[j];
}
int main() {
    unsigned char* d;
    unsigned char h[512];
    hipMalloc(&d, 512);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
        printf("mode %d (lane: address -> 8 bytes)\n", mode);
        for (int l = 0; l < 64; ++l) {
            int addr = mode == 0 ? l * 8 : (l & 15) * 16 + (l >> 4) * 8;
            printf("lane %2d addr %3d:", l, addr);
            for (int j = 0; j < 8; ++j) printf(" %3d", h[l * 8 + j]);
            printf("\n");
        }
    }
    return 0;
}
