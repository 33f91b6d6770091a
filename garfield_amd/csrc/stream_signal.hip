// Device-side signals between streams, for points inside a captured HIP graph (see
// bindings.cpp: signal_* / wait_geq and garfield_amd/parallel/grouped.py GraphSignal).
//
// Why device-side: on ROCm 7 / MI355X a HIP-level cross-stream dependency ON the main
// stream (another stream's hipStreamWaitEvent on an event recorded there) slows every
// later kernel of a graph replayed on the main stream by ~1-1.5 us, and the slowdown
// persists over several replays (scripts/probe_cross_stream.py,
// profiles/r3/probe_cross_stream.log: a 400-kernel graph 0.88 -> 1.34-1.47 ms). A
// counter written by a 1-lane kernel in the graph and waited for by a 1-lane kernel
// on the other stream is invisible to the runtime's dependency tracking.
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

// one lane: advance the counter by one (a vector-memory atomic, system scope, release):
// captured into a graph it signals "this point was passed" once per replay
__global__ void k_signal_add(unsigned long long* p) {
  __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one lane: wait until the counter reaches `target` (relaxed polls with s_sleep, then an
// acquire load), or until `timeout_us` of wall clock passed: then record the miss in
// err[0] and return (a lost signal must not hang the queue)
__global__ void k_wait_geq(const unsigned long long* p, unsigned long long target, unsigned long long timeout_us,
                           unsigned long long* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz constant clock
  const unsigned long long limit = timeout_us * 100ull;
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
      __hip_atomic_fetch_add(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  (void)__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

const void* signal_kernel() { return reinterpret_cast<const void*>(&k_signal_set); }
const void* signal_add_kernel() { return reinterpret_cast<const void*>(&k_signal_add); }

void signal_set(void* p, uint64_t value, hipStream_t stream) {
  hipLaunchKernelGGL(k_signal_set, dim3(1), dim3(1), 0, stream, static_cast<unsigned long long*>(p),
                     static_cast<unsigned long long>(value));
}

void signal_add(void* p, hipStream_t stream) {
  hipLaunchKernelGGL(k_signal_add, dim3(1), dim3(1), 0, stream, static_cast<unsigned long long*>(p));
}

void wait_geq(const void* p, uint64_t target, uint64_t timeout_us, void* err, hipStream_t stream) {
  hipLaunchKernelGGL(k_wait_geq, dim3(1), dim3(1), 0, stream, static_cast<const unsigned long long*>(p),
                     static_cast<unsigned long long>(target), static_cast<unsigned long long>(timeout_us),
                     static_cast<unsigned long long*>(err));
}

}  // namespace gpu
}  // namespace garfield
