// Launch-latency microbenchmark (diagnostic, GPU box): time per kernel for back-to-back
// dependent launches on one stream, by grid size and work, plus a grid-barrier kernel.
// hipcc --offload-arch=gfx950 -O3 tools/launch_lat.hip -o gpurun_out/launch_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void empty_kernel() {}

__global__ void touch_kernel(int* p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1;
}

// software grid barrier: every block arrives once on a counter and spins until all arrived
__global__ void barrier_kernel(unsigned* ctr, unsigned target, int rounds) {
    for (int r = 0; r < rounds; ++r) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            atomicAdd(ctr, 1u);
            const unsigned goal = target * (r + 1);
            while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < goal) __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();
    }
}

#define CK(x)                                                            \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                    \
        }                                                                \
    } while (0)

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int* buf;
    CK(hipMalloc(&buf, 64 << 20));
    CK(hipMemset(buf, 0, 64 << 20));
    unsigned* ctr;
    CK(hipMalloc(&ctr, 256));
    const int N = 2000;
    struct Cfg {
        int blocks, threads, work;
    } cfgs[] = {{1, 64, 0}, {256, 256, 0}, {2048, 512, 0}, {256, 256, 1}, {1024, 256, 1}, {16384, 256, 1}};
    for (auto c : cfgs) {
        const int n = c.blocks * c.threads;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(a, st));
            for (int i = 0; i < N; ++i) {
                if (c.work)
                    hipLaunchKernelGGL(touch_kernel, dim3(c.blocks), dim3(c.threads), 0, st, buf, n);
                else
                    hipLaunchKernelGGL(empty_kernel, dim3(c.blocks), dim3(c.threads), 0, st);
            }
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep) printf("launch %6d x %4d %s: %7.2f us per kernel\n", c.blocks, c.threads, c.work ? "touch" : "empty",
                            ms * 1e3 / N);
        }
    }
    // grid barrier cost: 256 blocks (one per CU), R rounds in one launch
    for (int rounds : {1, 10, 100}) {
        for (int blocks : {256, 512}) {
            CK(hipMemsetAsync(ctr, 0, 4, st));
            CK(hipEventRecord(a, st));
            hipLaunchKernelGGL(barrier_kernel, dim3(blocks), dim3(256), 0, st, ctr, (unsigned)blocks, rounds);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("grid barrier %4d blocks x %3d rounds: %8.2f us total, %6.2f us per round\n", blocks, rounds, ms * 1e3,
                   ms * 1e3 / rounds);
        }
    }
    return 0;
}
