// Launch-cost probe for the speculative pairs' second launch and the residual pass (ResNet-18 at
// 224 px, batch 128: 25.7 M elements in layer1).  Times, per launch over 100 back-to-back launches
// on one stream: an empty kernel, a kernel whose blocks read the 64 range slots + the hint word and
// exit (the "hit" path of launch B), and memory passes of the residual's shape (two int8 inputs, one
// int8 output) with a trivial op and with the residual rule (residual_z + psto_fast per byte).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I../../mandheling-dsp-training_amd/csrc exit_probe.hip -o /tmp/exit_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "niti_device.hpp"
#include "niti_sgd.hpp"

using namespace niti;


__global__ void k_empty() {}

__global__ void k_exit(const uint32_t* amax, const uint32_t* hint, int* sink) {
    const int bw = bitwidth_of(read_max(amax));
    const int used = __builtin_amdgcn_readfirstlane(
                         (int)__hip_atomic_load(hint + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - 1;
    if (bw == used) return;
    sink[blockIdx.x] = bw;
}

// the exit test by one block's first wave only through a plain load (no agent-scope atomic)
__global__ void k_exit_plain(const uint32_t* amax, const uint32_t* hint, int* sink) {
    const int bw = bitwidth_of(read_max(amax));
    const int used = __builtin_amdgcn_readfirstlane((int)hint[1]) - 1;
    if (bw == used) return;
    sink[blockIdx.x] = bw;
}

template <int OP>
__global__ void __launch_bounds__(256) k_res(const int8_t* __restrict__ a, const int8_t* __restrict__ b, int64_t n16,
                                             int d, int r, int s, int8_t* __restrict__ out, uint32_t* amax) {
    uint32_t m = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const v16c va = ((const v16c*)a)[i], vb = ((const v16c*)b)[i];
        v16c q;
        if constexpr (OP == 0) {
            q = va + vb;
        } else {
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int32_t z = residual_z(va[e], vb[e], d, r);
                if (OP == 2) {
                    const uint32_t u = uabs32(z);
                    m = m > u ? m : u;
                }
                int32_t o = psto_fast(z, s);
                if (o < 0) o = 0;
                q[e] = (signed char)o;
            }
        }
        ((v16c*)out)[i] = q;
    }
    if (OP == 2) {
        m = wave_max(m);
        if ((threadIdx.x & 63) == 0 && m == 0xffffffffu) amax[0] = m;
    }
}

// the bit-field form (res_rule4, niti_device.hpp): PK 1 relu + range (launch A forward), 2 relu
// only, 3 signed + relu mask (backward)
template <int PK>
__global__ void __launch_bounds__(256) k_res_pk(const int8_t* __restrict__ a, const int8_t* __restrict__ b, int64_t n16,
                                                int d, int r, int s, int8_t* __restrict__ out, uint32_t* amax,
                                                const int8_t* __restrict__ mask) {
    const ResRule k = res_rule(d, r, s);
    int mx = 0, mn = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const v4i vh = ((const v4i*)a)[i], vl = ((const v4i*)b)[i];
        v4i mk;
        if (PK == 3) mk = ((const v4i*)mask)[i];
        v4i q;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            uint32_t o = PK == 3 ? res_rule4<false>((uint32_t)vh[w], (uint32_t)vl[w], k, mx, mn, false)
                                 : res_rule4<true>((uint32_t)vh[w], (uint32_t)vl[w], k, mx, mn, PK == 1);
            if (PK == 3) o &= sw_expand(sw_pos_hi((uint32_t)mk[w]));
            q[w] = (int)o;
        }
        ((v4i*)out)[i] = q;
    }
    if (PK == 1) {
        const uint32_t m = wave_max(max(uabs32(mx), uabs32(mn)));
        if ((threadIdx.x & 63) == 0 && m == 0xffffffffu) amax[0] = m;
    }
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <class F>
static float time_us(F f, int reps, hipEvent_t e0, hipEvent_t e1) {
    for (int i = 0; i < 5; ++i) f();
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return 1000.f * ms / reps;
}

int main() {
    const int64_t n = 128LL * 56 * 56 * 64;  // ResNet-18 layer1 at 224 px, batch 128
    int8_t *a, *b, *o;
    uint32_t *amax, *hint;
    int* sink;
    CK(hipMalloc(&a, n));
    CK(hipMalloc(&b, n));
    CK(hipMalloc(&o, n));
    CK(hipMalloc(&amax, 64 * MAX_SLOT_STRIDE * 4));
    CK(hipMalloc(&hint, 64));
    CK(hipMalloc(&sink, 65536 * 4));
    CK(hipMemset(a, 3, n));
    CK(hipMemset(b, 5, n));
    CK(hipMemset(amax, 0, 64 * MAX_SLOT_STRIDE * 4));
    std::vector<uint32_t> hh(16, 0);
    hh[1] = 1;  // used = 0 = bitwidth_of(0): the exit path
    CK(hipMemcpy(hint, hh.data(), 64, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int g : {1, 64, 256, 512, 1024, 2048}) {
        const float te = time_us([&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0); }, 100, e0, e1);
        const float tx = time_us([&] { hipLaunchKernelGGL(k_exit, dim3(g), dim3(256), 0, 0, amax, hint, sink); }, 100, e0, e1);
        const float tp =
            time_us([&] { hipLaunchKernelGGL(k_exit_plain, dim3(g), dim3(256), 0, 0, amax, hint, sink); }, 100, e0, e1);
        printf("grid %5d: empty %.2f us  exit(agent hint) %.2f us  exit(plain hint) %.2f us\n", g, te, tx, tp);
    }
    const int64_t n16 = n / 16;
    for (int g : {512, 1024, 2048, 4096, 8192}) {
        const float t0 = time_us([&] { hipLaunchKernelGGL((k_res<0>), dim3(g), dim3(256), 0, 0, a, b, n16, 1, 0, 8, o, amax); }, 50, e0, e1);
        const float t1 = time_us([&] { hipLaunchKernelGGL((k_res<1>), dim3(g), dim3(256), 0, 0, a, b, n16, 1, 0, 8, o, amax); }, 50, e0, e1);
        const float t2 = time_us([&] { hipLaunchKernelGGL((k_res<2>), dim3(g), dim3(256), 0, 0, a, b, n16, 1, 0, 8, o, amax); }, 50, e0, e1);
        const float p1 = time_us([&] { hipLaunchKernelGGL((k_res_pk<1>), dim3(g), dim3(256), 0, 0, a, b, n16, 1, 0, 8, o, amax, a); }, 50, e0, e1);
        const float p2 = time_us([&] { hipLaunchKernelGGL((k_res_pk<2>), dim3(g), dim3(256), 0, 0, a, b, n16, 1, 0, 8, o, amax, a); }, 50, e0, e1);
        const float p3 = time_us([&] { hipLaunchKernelGGL((k_res_pk<3>), dim3(g), dim3(256), 0, 0, a, b, n16, 1, 0, 8, o, amax, a); }, 50, e0, e1);
        printf("residual pass, grid %5d: add %.2f us (%.2f TB/s)  rule %.2f us  rule+range %.2f us | bit-field: "
               "relu+range %.2f  relu %.2f  signed+mask %.2f us\n", g, t0, 3.0 * n / t0 * 1e-6, t1, t2, p1, p2, p3);
    }
    return 0;
}
