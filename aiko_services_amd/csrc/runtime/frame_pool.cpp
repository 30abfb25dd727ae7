// HBM frame-buffer pool: fixed-size slots carved out of ONE device allocation.
//
// Pipeline stages exchange frames by slot id (a small integer that travels in the MQTT
// process_frame metadata or an RCCL header) instead of allocating per frame; the pool is the
// stable receive buffer for RCCL P2P and the credit mechanism of the in-flight window: a
// producer that finds no free slot blocks (acquire with timeout) until a consumer releases
// one, which is the pipeline's back-pressure.  Sized for 288 GB of HBM per MI355X — even a
// deep window of 4096 x 640x640x3 bf16 frames is ~10 GB — the point is zero allocator churn
// and stable addresses, not saving memory.
//
// Exposed as the TorchScript custom class torch.classes.aiko.FramePool.
#include <ATen/ATen.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <vector>

namespace {

class FramePool : public torch::CustomClassHolder {
 public:
  FramePool(int64_t num_slots, int64_t slot_bytes, int64_t device_index)
      : num_slots_(num_slots), slot_bytes_((slot_bytes + 255) / 256 * 256) {
    TORCH_CHECK(num_slots > 0 && slot_bytes > 0, "FramePool: num_slots and slot_bytes must be > 0");
    auto opts = at::TensorOptions().dtype(at::kByte);
    if (device_index >= 0) {
      opts = opts.device(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device_index)));
    }
    storage_ = at::empty({num_slots_ * slot_bytes_}, opts);
    for (int64_t i = 0; i < num_slots_; ++i) free_.push_back(i);   // FIFO: slots rotate
    in_use_.assign(num_slots_, 0);
  }

  // Returns a slot id, or -1 when none became free within timeout_ms (<0: wait forever).
  int64_t acquire(int64_t timeout_ms) {
    std::unique_lock<std::mutex> lk(mu_);
    auto ready = [&] { return !free_.empty() || closed_; };
    if (timeout_ms < 0) {
      cv_.wait(lk, ready);
    } else if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready)) {
      ++exhausted_;
      return -1;
    }
    if (closed_ || free_.empty()) return -1;
    const int64_t slot = free_.front();
    free_.pop_front();
    in_use_[slot] = 1;
    const int64_t used = num_slots_ - static_cast<int64_t>(free_.size());
    if (used > high_water_) high_water_ = used;
    ++acquired_;
    return slot;
  }

  void release(int64_t slot) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      TORCH_CHECK(slot >= 0 && slot < num_slots_, "FramePool.release: bad slot ", slot);
      TORCH_CHECK(in_use_[slot], "FramePool.release: slot ", slot, " is not in use (double release)");
      in_use_[slot] = 0;
      free_.push_back(slot);
    }
    cv_.notify_one();
  }

  // A typed view of `slot` with the given shape (must fit in slot_bytes).
  at::Tensor view(int64_t slot, std::vector<int64_t> sizes, int64_t dtype_code) {
    TORCH_CHECK(slot >= 0 && slot < num_slots_, "FramePool.view: bad slot ", slot);
    const auto dtype = static_cast<at::ScalarType>(dtype_code);
    int64_t numel = 1;
    for (auto s : sizes) numel *= s;
    const int64_t nbytes = numel * static_cast<int64_t>(c10::elementSize(dtype));
    TORCH_CHECK(nbytes <= slot_bytes_, "FramePool.view: ", nbytes, " bytes exceed slot size ", slot_bytes_);
    return storage_.narrow(0, slot * slot_bytes_, nbytes).view(dtype).view(sizes);
  }

  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      closed_ = true;
    }
    cv_.notify_all();
  }

  int64_t capacity() const { return num_slots_; }
  int64_t slot_bytes() const { return slot_bytes_; }
  int64_t free_count() {
    std::lock_guard<std::mutex> lk(mu_);
    return static_cast<int64_t>(free_.size());
  }
  std::vector<int64_t> stats() {
    std::lock_guard<std::mutex> lk(mu_);
    return {num_slots_, num_slots_ - static_cast<int64_t>(free_.size()), high_water_, acquired_, exhausted_};
  }
  at::Tensor storage() const { return storage_; }

 private:
  int64_t num_slots_;
  int64_t slot_bytes_;
  at::Tensor storage_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<int64_t> free_;
  std::vector<uint8_t> in_use_;
  bool closed_ = false;
  int64_t high_water_ = 0, acquired_ = 0, exhausted_ = 0;
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(aiko, m) {
  m.class_<FramePool>("FramePool")
      .def(torch::init<int64_t, int64_t, int64_t>())
      .def("acquire", &FramePool::acquire)
      .def("release", &FramePool::release)
      .def("view", &FramePool::view)
      .def("close", &FramePool::close)
      .def("capacity", &FramePool::capacity)
      .def("slot_bytes", &FramePool::slot_bytes)
      .def("free_count", &FramePool::free_count)
      .def("stats", &FramePool::stats)
      .def("storage", &FramePool::storage);
}
