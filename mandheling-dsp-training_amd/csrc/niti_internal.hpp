// niti_internal.hpp -- host-side classes shared by the C ABI translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

#include <vector>

#include "../../include/niti_hip.h"
#include "niti_kernels.hpp"

namespace niti {

// Device memory owned by a handle; acquired in onResize, freed on re-resize / destroy
// (the reference acquires DYNAMIC buffers in onResize, NITI_Conv_Int8.cpp:119-157).
struct Workspace {
    std::vector<void*> ptrs;
    size_t total = 0;
    void* alloc(size_t bytes);
    // free `old` (one of ours, or null) and allocate `bytes` in its place
    void* replace(void* old, size_t bytes);
    void release();
    ~Workspace() { release(); }
};

// Execution (execution-engine/source/core/Execution.hpp:24-82) over niti_tensor views.
class Execution {
   public:
    virtual ~Execution() = default;
    virtual int onResize(const niti_tensor* inputs, int nin, const niti_tensor* outputs, int nout) = 0;
    virtual int onExecute(const niti_tensor* inputs, int nin, const niti_tensor* outputs, int nout,
                          hipStream_t st) = 0;
    size_t workspaceBytes() const { return ws_.total; }
    // a device word a launch of this Execution sets when it could not complete (the fused row
    // kernel's grid barrier timed out: results invalid), or null.  niti_execution_execute checks it
    // before a synchronous (host-tensor) call returns, niti_execution_status for device tensors.
    virtual uint32_t* errorFlag() { return nullptr; }

   protected:
    Workspace ws_;
};

Execution* create_execution(int op_type, const niti_conv2d_common* common, int* err);
// CPUTensorConverter::convert for int8 NCHW / NHWC / NC4HW4 (returns an ErrorCode value)
int convert_tensor(const niti_tensor& src, const niti_tensor& dst, hipStream_t st);
bool geom_from_common(const niti_conv2d_common& c, int n, int ci, int h, int w, int co, int kh, int kw,
                      ConvGeom* g);

}  // namespace niti
