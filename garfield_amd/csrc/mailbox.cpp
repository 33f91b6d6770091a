#include "mailbox.hpp"

#ifndef GARFIELD_NO_HIP
#include <hip/hip_runtime.h>
#endif
#ifndef GARFIELD_NO_TORCH
#include <torch/extension.h>
#endif

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>

namespace garfield {
namespace mailbox {

Mailbox::Mailbox(size_t nslots, size_t slot_bytes, bool pinned)
    : nslots_(nslots), slot_bytes_(slot_bytes), stride_(((slot_bytes + 255) / 256) * 256), pinned_(pinned),
      tags_(nslots, -1), stamp_(nslots, 0) {
  if (nslots == 0) throw std::invalid_argument("mailbox: nslots must be > 0");
  const size_t total = stride_ * nslots_ + 256;
#ifndef GARFIELD_NO_HIP
  if (pinned_) {
    if (hipHostMalloc(&base_, total, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      base_ = nullptr;
      pinned_ = false;  // no device / no driver: fall back to pageable memory
    }
  }
#else
  pinned_ = false;
#endif
  if (!base_) {
    base_ = std::aligned_alloc(256, ((total + 255) / 256) * 256);
    if (!base_) throw std::bad_alloc();
  }
}

Mailbox::~Mailbox() {
#ifndef GARFIELD_NO_HIP
  if (pinned_) {
    (void)hipHostFree(base_);
    return;
  }
#endif
  std::free(base_);
}

void Mailbox::write(size_t i, int64_t tag, const void* src, size_t bytes) {
  if (i >= nslots_) throw std::out_of_range("mailbox: slot out of range");
  if (bytes > slot_bytes_) throw std::invalid_argument("mailbox: payload larger than the slot");
  {
    std::lock_guard<std::mutex> g(mu_);
    tags_[i] = -1;  // "writing": never observed half-written by a reader
  }
  std::memcpy(slot(i), src, bytes);
  publish(i, tag);
}

void Mailbox::publish(size_t i, int64_t tag) {
  if (i >= nslots_) throw std::out_of_range("mailbox: slot out of range");
  {
    std::lock_guard<std::mutex> g(mu_);
    tags_[i] = tag;
    stamp_[i] = ++seq_;
  }
  cv_.notify_all();
}

std::vector<size_t> Mailbox::ready(int64_t tag) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<size_t> ids;
  for (size_t i = 0; i < nslots_; ++i)
    if (tags_[i] == tag) ids.push_back(i);
  std::sort(ids.begin(), ids.end(), [&](size_t a, size_t b) { return stamp_[a] < stamp_[b]; });
  return ids;
}

std::vector<size_t> Mailbox::wait(int64_t tag, size_t k, double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  auto count = [&] {
    size_t c = 0;
    for (size_t i = 0; i < nslots_; ++i) c += tags_[i] == tag;
    return c;
  };
  if (timeout_s < 0) {
    cv_.wait(lk, [&] { return count() >= k; });
  } else {
    cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), [&] { return count() >= k; });
  }
  std::vector<size_t> ids;
  for (size_t i = 0; i < nslots_; ++i)
    if (tags_[i] == tag) ids.push_back(i);
  std::sort(ids.begin(), ids.end(), [&](size_t a, size_t b) { return stamp_[a] < stamp_[b]; });
  return ids;
}

int64_t Mailbox::tag_of(size_t i) {
  std::lock_guard<std::mutex> g(mu_);
  return i < nslots_ ? tags_[i] : -1;
}

void Mailbox::clear() {
  std::lock_guard<std::mutex> g(mu_);
  std::fill(tags_.begin(), tags_.end(), -1);
}

#ifndef GARFIELD_NO_TORCH
void bind(pybind11::module_& m) {
  namespace py = pybind11;
  py::class_<Mailbox, std::shared_ptr<Mailbox>>(m, "Mailbox",
                                                 "Pinned multi-slot tagged mailbox (async quorum / gradient inbox)")
      .def(py::init<size_t, size_t, bool>(), py::arg("nslots"), py::arg("slot_bytes"), py::arg("pinned") = true)
      .def_property_readonly("nslots", &Mailbox::nslots)
      .def_property_readonly("slot_bytes", &Mailbox::slot_bytes)
      .def_property_readonly("pinned", &Mailbox::pinned)
      .def("write",
           [](Mailbox& self, size_t i, int64_t tag, const at::Tensor& t) {
             auto c = t.contiguous();
             TORCH_CHECK(c.device().is_cpu(), "mailbox: write expects a host tensor");
             const size_t bytes = static_cast<size_t>(c.numel()) * c.element_size();
             py::gil_scoped_release nogil;
             self.write(i, tag, c.data_ptr(), bytes);
           },
           py::arg("slot"), py::arg("tag"), py::arg("tensor"))
      .def("publish", &Mailbox::publish, py::arg("slot"), py::arg("tag"))
      .def("wait",
           [](Mailbox& self, int64_t tag, size_t k, double timeout) {
             py::gil_scoped_release nogil;
             return self.wait(tag, k, timeout);
           },
           py::arg("tag"), py::arg("k"), py::arg("timeout") = -1.0)
      .def("ready", &Mailbox::ready, py::arg("tag"))
      .def("tag_of", &Mailbox::tag_of)
      .def("clear", &Mailbox::clear)
      .def("tensor",
           [](std::shared_ptr<Mailbox> self, size_t i, int64_t numel, py::object dtype) {
             TORCH_CHECK(i < self->nslots(), "mailbox: slot out of range");
             const auto st = torch::python::detail::py_object_to_dtype(dtype);
             TORCH_CHECK(static_cast<size_t>(numel) * c10::elementSize(st) <= self->slot_bytes(),
                         "mailbox: view larger than the slot");
             auto keep = self;  // the view keeps the mailbox alive
             return torch::from_blob(self->slot(i), {numel}, [keep](void*) {},
                                     torch::TensorOptions().dtype(st));
           },
           py::arg("slot"), py::arg("numel"), py::arg("dtype"),
           "Zero-copy host view of slot i (valid while the mailbox lives)");
}

#endif  // GARFIELD_NO_TORCH

}  // namespace mailbox
}  // namespace garfield
