// niti_map.hpp -- grid-stride elementwise launcher used by the layout converters.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace niti {

template <class F>
__global__ void map_kernel(int64_t total, F f) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        f(i);
}

template <class F>
inline hipError_t launch_map(int64_t total, F f, hipStream_t st) {
    if (total <= 0) return hipSuccess;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(map_kernel<F>, dim3((unsigned)blocks), dim3(256), 0, st, total, f);
    return hipGetLastError();
}

}  // namespace niti
