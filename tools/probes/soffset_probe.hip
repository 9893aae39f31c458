// Does the raw-buffer range check include soffset?  Loads at voffset 0 with soffset past
// num_records: 0 if soffset is range-checked, the data there otherwise.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const int* p, int* o) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 256, 0x00020000);  // 256 valid bytes
    v4i a, b, c;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(a) : "v"(0u), "s"(r), "s"(512u));
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(b) : "v"(512u), "s"(r), "s"(0u));
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(c) : "v"(240u), "s"(r), "s"(16u));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) { o[0] = a[0]; o[1] = b[0]; o[2] = c[0]; }
}
int main() {
    int h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = i + 1;
    int *d, *o;
    hipMalloc(&d, 4096); hipMalloc(&o, 64);
    hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
    int r[3];
    hipMemcpy(r, o, 12, hipMemcpyDeviceToHost);
    printf("soffset past range: %d (data there: %d); voffset past range: %d; voffset in + soffset past: %d (data %d)\n",
           r[0], h[128], r[1], r[2], h[64]);
    return 0;
}
