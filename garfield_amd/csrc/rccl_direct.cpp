// Direct RCCL collectives on a caller-chosen HIP stream, on torch's own communicator.
//
// torch.distributed's ProcessGroupNCCL runs every collective on an internal stream that
// first waits (hipStreamWaitEvent) on the caller's current stream. On ROCm 7 / MI355X a
// pending cross-stream event wait ANYWHERE on the device while the step's HIP graph
// replays slows that graph by ~1-1.5 us per kernel (scripts/probe_cross_stream.py:
// a 400-kernel graph 0.88 -> 1.3-1.4 ms, also when the waiting stream is a third one).
// The exchange therefore enqueues RCCL's kernels straight onto the comm stream, which
// follows the main stream through device-side counters only (parallel/signals.py):
// nothing but in-order stream work and 1-lane polls while the graph runs.
//
// The library is torch's bundled librccl (the communicator handle comes from
// ProcessGroupNCCL._comm_ptr(), so the same library instance must drive it): it is
// already loaded by torch; dlopen(RTLD_NOLOAD) returns that instance.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>

namespace garfield {
namespace rccl {

namespace {
using Res = int;
using Comm = void*;
struct Api {
  void* handle = nullptr;
  Res (*group_start)() = nullptr;
  Res (*group_end)() = nullptr;
  Res (*all_to_all)(const void*, void*, size_t, int, Comm, hipStream_t) = nullptr;
  Res (*all_gather)(const void*, void*, size_t, int, Comm, hipStream_t) = nullptr;
  Res (*all_reduce)(const void*, void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  Res (*send)(const void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  Res (*recv)(void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  const char* (*error_string)(Res) = nullptr;
};
Api g_api;
std::mutex g_mu;

template <class F>
void sym(void* h, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(h, name));
  if (!out) throw std::runtime_error(std::string("garfield rccl: missing symbol ") + name);
}

void check(Res r, const char* what) {
  if (r != 0) {
    const char* msg = g_api.error_string ? g_api.error_string(r) : "?";
    throw std::runtime_error(std::string("garfield rccl: ") + what + " failed: " + msg);
  }
}

const Api& api() {
  if (!g_api.handle) throw std::runtime_error("garfield rccl: library not loaded (rccl_load)");
  return g_api;
}
}  // namespace

bool load(const std::string& path) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_api.handle) return true;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);   // torch's instance, already mapped
  if (!h) h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) return false;
  Api a;
  a.handle = h;
  sym(h, "ncclGroupStart", a.group_start);
  sym(h, "ncclGroupEnd", a.group_end);
  sym(h, "ncclAllToAll", a.all_to_all);
  sym(h, "ncclAllGather", a.all_gather);
  sym(h, "ncclAllReduce", a.all_reduce);
  sym(h, "ncclSend", a.send);
  sym(h, "ncclRecv", a.recv);
  sym(h, "ncclGetErrorString", a.error_string);
  g_api = a;
  return true;
}

void all_to_all(int64_t comm, const void* send, void* recv, size_t count, int dtype, hipStream_t stream) {
  check(api().all_to_all(send, recv, count, dtype, reinterpret_cast<Comm>(comm), stream), "ncclAllToAll");
}

// One group of point-to-point transfers: ops[i] = (ptr, count, peer), the first nsend are
// sends. Sends to one peer are matched with that peer's receives in issue order, so a
// bucket's rows leave straight from the exchange rows (one contiguous shard per worker
// row and destination) with no packing copy, and this rank's own shard never moves.
void exchange(int64_t comm, const int64_t* ptr, const int64_t* count, const int64_t* peer, int64_t nsend,
              int64_t nops, int dtype, hipStream_t stream) {
  const Api& a = api();
  Comm c = reinterpret_cast<Comm>(comm);
  check(a.group_start(), "ncclGroupStart");
  for (int64_t i = 0; i < nops; ++i) {
    Res r = i < nsend
        ? a.send(reinterpret_cast<const void*>(ptr[i]), static_cast<size_t>(count[i]), dtype,
                 static_cast<int>(peer[i]), c, stream)
        : a.recv(reinterpret_cast<void*>(ptr[i]), static_cast<size_t>(count[i]), dtype,
                 static_cast<int>(peer[i]), c, stream);
    if (r != 0) {
      a.group_end();
      check(r, i < nsend ? "ncclSend" : "ncclRecv");
    }
  }
  check(a.group_end(), "ncclGroupEnd");
}

void all_gather(int64_t comm, const void* send, void* recv, size_t count, int dtype, hipStream_t stream) {
  check(api().all_gather(send, recv, count, dtype, reinterpret_cast<Comm>(comm), stream), "ncclAllGather");
}

void all_reduce_sum(int64_t comm, const void* send, void* recv, size_t count, int dtype, hipStream_t stream) {
  check(api().all_reduce(send, recv, count, dtype, /*ncclSum*/ 0, reinterpret_cast<Comm>(comm), stream),
        "ncclAllReduce");
}

}  // namespace rccl
}  // namespace garfield
