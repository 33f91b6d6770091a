// Pinned multi-slot mailbox: the MI355X-side analogue of the reference's
// MultiRegister / multibuffer (tensorflow_impl/rsrcs/native/include/multiregister.hpp:
// 70-79, 232-420; op_multibuffer/op.cpp:40-173), which is a single-writer /
// multi-reader register with empty / writing / written / reading states.
//
// Here each slot is one sender's (gradient or model) vector, tagged with the
// iteration it belongs to. Producers (RPC handler threads, gRPC servicers, the
// async-quorum path) copy into a slot without holding the GIL; the consumer
// blocks on a condition variable until k slots carry the wanted tag (the
// reference's "wait for the fastest n - f" done by 10 ms sleep-polling in
// garfieldpp/server.py:134-155) or a timeout expires. Slot memory is page-locked
// with hipHostMalloc so the consumer's H2D copy is a DMA, not a staged copy.
#pragma once
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <vector>

namespace pybind11 { class module_; }

namespace garfield {
namespace mailbox {

class Mailbox {
 public:
  Mailbox(size_t nslots, size_t slot_bytes, bool pinned);
  ~Mailbox();
  Mailbox(const Mailbox&) = delete;
  Mailbox& operator=(const Mailbox&) = delete;

  size_t nslots() const { return nslots_; }
  size_t slot_bytes() const { return slot_bytes_; }
  bool pinned() const { return pinned_; }
  void* slot(size_t i) const { return static_cast<char*>(base_) + i * stride_; }

  // Copy `bytes` bytes into slot i and publish it with `tag` (overwrites any older tag).
  void write(size_t i, int64_t tag, const void* src, size_t bytes);
  // Mark slot i written with `tag` after the caller filled slot(i) itself.
  void publish(size_t i, int64_t tag);
  // Block until >= k slots carry `tag` or timeout_s elapses (< 0: forever).
  // Returns the slot ids carrying `tag`, in order of arrival.
  std::vector<size_t> wait(int64_t tag, size_t k, double timeout_s);
  // Slots currently carrying `tag` (arrival order), non-blocking.
  std::vector<size_t> ready(int64_t tag);
  int64_t tag_of(size_t i);
  void clear();

 private:
  size_t nslots_, slot_bytes_, stride_;
  bool pinned_;
  void* base_ = nullptr;
  std::vector<int64_t> tags_;
  std::vector<uint64_t> stamp_;  // arrival sequence numbers
  uint64_t seq_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
};

void bind(pybind11::module_& m);

}  // namespace mailbox
}  // namespace garfield
