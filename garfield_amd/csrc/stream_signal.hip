// Signal word writer for waits on a point inside a captured HIP graph (see
// bindings.cpp: signal_* and garfield_amd/parallel/grouped.py GraphSignal).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "gar_gpu.hpp"

namespace garfield {
namespace gpu {

namespace {
// one lane: a system-scope release store (a vector memory store) of the signal value;
// every earlier kernel of the stream has completed when this one starts
__global__ void k_signal_set(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

const void* signal_kernel() { return reinterpret_cast<const void*>(&k_signal_set); }

void signal_set(void* p, uint64_t value, hipStream_t stream) {
  hipLaunchKernelGGL(k_signal_set, dim3(1), dim3(1), 0, stream, static_cast<unsigned long long*>(p),
                     static_cast<unsigned long long>(value));
}

}  // namespace gpu
}  // namespace garfield
