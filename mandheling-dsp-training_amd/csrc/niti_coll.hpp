// niti_coll.hpp -- the data-parallel transports shared by the step drivers (niti_model.hip: LeNet /
// VGG, niti_resnet_model.hip: ResNet-18).
#pragma once

#include <rccl/rccl.h>
#include <stdlib.h>

#include <condition_variable>
#include <memory>
#include <mutex>

#include "niti_kernels.hpp"

namespace niti {

// ---------------------------------------------------------------------------- collectives
// The data-parallel step's collectives run on two communicators, each used in one fixed program
// order on every rank:
//   ranges (`coll`, the step stream): the input quantiser's statistics and every forward /
//     input-gradient range (MAX), each needed by the very next launch on the step stream;
//   gradients (`coll_grad`, the comm stream `cst`): one SUM per gradient bucket (consecutive
//     layers in backward order, ~8 MB or more), issued as soon as the bucket's weight gradients
//     are in and followed on cst by those layers' ranges, so the SUMs overlap the rest of the
//     backward pass.
// RCCL serialises the operations of ONE communicator in issue order whatever stream they are on
// (each launch waits for the communicator's previous one), so a range MAX on the same
// communicator as a large SUM would wait for that SUM and stall the input-gradient chain behind
// it.  With two communicators the step stream's MAXes never wait for a SUM; no operation of one
// communicator waits for an operation of the other (the SUMs wait only for weight-gradient
// kernels, the step stream for the SUMs only at the NITI_SGD join), and each communicator's
// operations are issued in the same order on every rank, so the two cannot deadlock.
// Gradient buckets close once they hold this many int32 gradient bytes (backward order).  Each
// bucket costs one event record on the step stream (a ~6.5 us bubble before the next launch), so
// fewer, larger buckets; NITI_BUCKET_MB overrides (A/B).
inline size_t grad_bucket_bytes() {
    static const long mb = getenv("NITI_BUCKET_MB") ? atol(getenv("NITI_BUCKET_MB")) : 8;
    return (size_t)(mb > 0 ? mb : 1) << 20;
}

enum CollOp { COLL_MAX_U32 = 0, COLL_SUM_I32 = 1, COLL_SUM_U64 = 2, COLL_MAX_U64 = 3 };

struct Collective {
    virtual ~Collective() = default;
    virtual int size() const = 0;
    // in place, on stream st, asynchronous where the transport allows
    virtual hipError_t allreduce(void* p, size_t n, CollOp op, hipStream_t st) = 0;
};

struct RcclCollective final : Collective {
    ncclComm_t comm = nullptr;
    int world = 1;
    bool owns = true;  // false: another RcclCollective's communicator (the no-split fallback)
    ~RcclCollective() override {
        if (comm && owns) (void)ncclCommDestroy(comm);
    }
    int size() const override { return world; }
    hipError_t allreduce(void* p, size_t n, CollOp op, hipStream_t st) override {
        static const ncclDataType_t ty[4] = {ncclUint32, ncclInt32, ncclUint64, ncclUint64};
        static const ncclRedOp_t ro[4] = {ncclMax, ncclSum, ncclSum, ncclMax};
        return ncclAllReduce(p, p, n, ty[op], ro[op], comm, st) == ncclSuccess ? hipSuccess : hipErrorUnknown;
    }
};

// In-process group of `world` ranks on ONE device, one host thread per rank (tests): each
// collective synchronises the caller's stream, the last rank to arrive reduces every rank's
// buffer on the device and writes the result back to all of them.  It runs the model's exact
// data-parallel protocol -- the same calls, in the same order, on the same streams -- with a
// transport that needs no second GPU.  A group has one channel per communicator (ranges,
// gradients), each its own rendezvous.
struct LocalChannel {
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    unsigned long long gen = 0;
    void* ptr[16] = {};
    size_t n = 0;
    int op = -1;
    bool mismatch = false;
    hipError_t err = hipSuccess;
    // the result of generation g, published before the waiters are released: a waiter reads
    // its own generation's slot, which a faster rank entering generation g + 1 cannot reset
    // (generation g + 2 needs this waiter's arrival first)
    hipError_t result[2] = {hipSuccess, hipSuccess};
};

struct LocalGroup {
    static constexpr int MAX_RANKS = 16;
    int world = 1;
    LocalChannel ch[2];
    hipStream_t rst = nullptr;
    ~LocalGroup() {
        if (rst) (void)hipStreamDestroy(rst);
    }
};

struct RankPtrs {
    void* p[LocalGroup::MAX_RANKS];
    int world;
};
template <class T, bool MAX>
__global__ void local_reduce_kernel(RankPtrs r, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v = static_cast<T*>(r.p[0])[i];
        for (int k = 1; k < r.world; ++k) {
            const T t = static_cast<T*>(r.p[k])[i];
            v = MAX ? (t > v ? t : v) : (T)(v + t);
        }
        for (int k = 0; k < r.world; ++k) static_cast<T*>(r.p[k])[i] = v;
    }
}

struct LocalCollective final : Collective {
    std::shared_ptr<LocalGroup> g;
    int rank = 0, chan = 0;
    int size() const override { return g->world; }
    hipError_t allreduce(void* p, size_t n, CollOp op, hipStream_t st) override {
        if (g->world == 1) return hipSuccess;  // one rank: the all-reduce is the identity
        LocalChannel& c = g->ch[chan];
        hipError_t e = hipStreamSynchronize(st);
        std::unique_lock<std::mutex> lk(c.mu);
        const unsigned long long my_gen = c.gen;
        if (c.arrived == 0) {
            c.n = n;
            c.op = op;
            c.mismatch = false;
            c.err = hipSuccess;
        } else if (c.n != n || c.op != op) {
            c.mismatch = true;  // ranks disagree on the sequence: a protocol bug
        }
        c.ptr[rank] = p;
        if (e != hipSuccess) c.err = e;
        if (++c.arrived == g->world) {
            if (!c.mismatch && c.err == hipSuccess) {
                RankPtrs r{};
                for (int k = 0; k < g->world; ++k) r.p[k] = c.ptr[k];
                r.world = g->world;
                const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 1024);
                if (blocks > 0) {
                    if (op == COLL_MAX_U32)
                        hipLaunchKernelGGL((local_reduce_kernel<uint32_t, true>), dim3(blocks), dim3(256), 0, g->rst, r, n);
                    else if (op == COLL_SUM_I32)
                        hipLaunchKernelGGL((local_reduce_kernel<int32_t, false>), dim3(blocks), dim3(256), 0, g->rst, r, n);
                    else if (op == COLL_SUM_U64)
                        hipLaunchKernelGGL((local_reduce_kernel<unsigned long long, false>), dim3(blocks), dim3(256), 0,
                                           g->rst, r, n);
                    else
                        hipLaunchKernelGGL((local_reduce_kernel<unsigned long long, true>), dim3(blocks), dim3(256), 0,
                                           g->rst, r, n);
                    c.err = hipGetLastError();
                    if (c.err == hipSuccess) c.err = hipStreamSynchronize(g->rst);
                }
            }
            if (c.mismatch) c.err = hipErrorInvalidValue;
            c.result[my_gen & 1] = c.err;
            c.arrived = 0;
            ++c.gen;
            c.cv.notify_all();
        } else {
            c.cv.wait(lk, [&] { return c.gen != my_gen; });
        }
        return c.result[my_gen & 1];
    }
};

}  // namespace niti
