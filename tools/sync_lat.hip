// Cross-stream dependency cost (diagnostic, GPU box): a main stream of ~4 us kernels that
// releases a side stream after each one, by event record, by an event attached to the kernel
// dispatch (hipExtLaunchKernelGGL stop event) and by stream write/wait value.
// hipcc --offload-arch=gfx950 -O3 tools/sync_lat.hip -o tools/bin/sync_lat
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void work_kernel(int* p, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] += 1;
}
__global__ void small_kernel(int* p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

#define CK(x)                                                     \
    do {                                                          \
        hipError_t e_ = (x);                                      \
        if (e_ != hipSuccess) {                                   \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                             \
        }                                                         \
    } while (0)

int main() {
    hipStream_t ms, ss;
    CK(hipStreamCreateWithFlags(&ms, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
    const int N = 200, n = 2 << 20;  // 8 MB per work kernel
    int *buf, *sbuf;
    CK(hipMalloc(&buf, (size_t)n * 4));
    CK(hipMalloc(&sbuf, 1 << 20));
    uint32_t* flags;
    CK(hipMalloc((void**)&flags, N * 128));
    CK(hipMemset(flags, 0, N * 128));
    hipEvent_t ev[N], evt[N];
    for (int i = 0; i < N; ++i) {
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
        CK(hipEventCreate(&evt[i]));
    }
    hipEvent_t a, b, c;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    for (int mode = 0; mode < 6; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(flags, 0, N * 128));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, ms));
            CK(hipStreamWaitEvent(ss, a, 0));
            for (int i = 0; i < N; ++i) {
                if (mode == 3)
                    hipExtLaunchKernelGGL(work_kernel, dim3(1024), dim3(256), 0, ms, nullptr, evt[i], 0, buf, n);
                else
                    hipLaunchKernelGGL(work_kernel, dim3(1024), dim3(256), 0, ms, buf, n);
                if (mode == 1 || mode == 2) CK(hipEventRecord(mode == 1 ? ev[i] : evt[i], ms));
                if (mode == 4) CK(hipStreamWriteValue32(ms, flags + i * 32, 1, 0));
                if (mode == 5) {
                    // side kernels only every 4th kernel
                    if (i % 4 == 3) CK(hipEventRecord(ev[i], ms));
                }
                if (mode >= 1 && mode <= 3) {
                    CK(hipStreamWaitEvent(ss, mode == 1 ? ev[i] : evt[i], 0));
                    hipLaunchKernelGGL(small_kernel, dim3(64), dim3(64), 0, ss, sbuf);
                } else if (mode == 4) {
                    CK(hipStreamWaitValue32(ss, flags + i * 32, 1, hipStreamWaitValueEq, 0xffffffffu));
                    hipLaunchKernelGGL(small_kernel, dim3(64), dim3(64), 0, ss, sbuf);
                } else if (mode == 5 && i % 4 == 3) {
                    CK(hipStreamWaitEvent(ss, ev[i], 0));
                    hipLaunchKernelGGL(small_kernel, dim3(64), dim3(64), 0, ss, sbuf);
                }
            }
            CK(hipEventRecord(b, ms));
            CK(hipEventRecord(c, ss));
            CK(hipEventSynchronize(b));
            CK(hipEventSynchronize(c));
            float t_main, t_side;
            CK(hipEventElapsedTime(&t_main, a, b));
            CK(hipEventElapsedTime(&t_side, a, c));
            const char* name[] = {"no sync", "event record (no timing)", "event record (timing)",
                                  "ext launch stop event", "stream write/wait value", "event every 4th"};
            if (rep)
                printf("%-28s main %6.2f us/kernel   side done %+7.2f us after main\n", name[mode], t_main * 1e3 / N,
                       (t_side - t_main) * 1e3);
        }
    }
    return 0;
}
