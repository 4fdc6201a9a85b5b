// Tensor of the C++ host API: logical shape + layout + dtype + device, shared storage.
//
// CPU tensors are fp32 NCHW (the reference's CPU form). GPU activations are bf16 NHWC — the
// layout the MFMA kernels read — and GPU parameters fp32 masters with bf16 operand shadows (see
// nn.hpp). Storage is shared (copies of a Tensor alias it); `ensure` is the reference's grow-only
// reallocation; `save` / `load` are the reference's .bin tensor format (uint64 shape[4] + fp32
// data in logical NCHW order), shared with the Python front end (nn/sequential.py).
// Reference parity: include/tensor/tensor.hpp:53-654 (to_device :424, resize :478, ensure :511,
// save/load :625), include/device/device_ptr.hpp:80-285.
#pragma once
#include <cstdint>
#include <cstring>
#include <iosfwd>
#include <memory>
#include <string>
#include <vector>

#include "layout.hpp"

namespace dcnn {

enum class DeviceType { CPU, GPU };

struct Device {
  DeviceType type = DeviceType::CPU;
  int index = 0;
  static Device cpu() { return {DeviceType::CPU, 0}; }
  static Device gpu(int i = 0) { return {DeviceType::GPU, i}; }
  static Device parse(const std::string& s);  // "CPU", "GPU", "GPU:1"
  bool is_gpu() const { return type == DeviceType::GPU; }
  std::string str() const;
  bool operator==(const Device& o) const { return type == o.type && index == o.index; }
  bool operator!=(const Device& o) const { return !(*this == o); }
};

enum class DType { F32, BF16, I32, I64, U8 };
size_t dtype_size(DType t);
const char* dtype_name(DType t);

// host bf16 <-> fp32 (round to nearest even)
uint16_t f32_to_bf16(float f);
float bf16_to_f32(uint16_t b);

// device memory entry points (implemented by the GPU backend, ops_gpu.hip)
namespace gpu {
int device_count();
void set_device(int dev);
// caching allocator: freed blocks are reused by later allocations of the same size class (the
// host API enqueues a thread's work on one flow in order, so reuse is ordered after the last
// reader); blocks allocated while a Graph captures belong to that graph (below)
void* alloc(size_t nbytes);
void free(void* p);
size_t cached_bytes();  // bytes held in the free lists
void empty_cache();     // synchronise and return every cached block to the driver
void copy(void* dst, const void* src, size_t nbytes, int kind);  // 0 h2d, 1 d2h (host waits), 2 d2d (async)
// two device-to-device copies in one kernel launch (stream-ordered, capturable)
void copy2_d2d(void* d0, const void* s0, size_t n0, void* d1, const void* s1, size_t n1);
void zero(void* p, size_t nbytes);                                // stream-ordered memset
void synchronize();

// Flows (reference include/device/flow.hpp:11-64): the HIP stream the calling thread's host API
// work is enqueued on. Default: the thread's own blocking stream on the current device (created on
// first use); set_flow() redirects the thread's work (nullptr: back to the default). Events order
// work across flows without a host wait.
using Flow = void*;   // hipStream_t
using Event = void*;  // hipEvent_t
Flow flow();
void set_flow(Flow f);
Flow flow_create();
void flow_destroy(Flow f);
void flow_synchronize(Flow f = nullptr);  // nullptr: the current flow
Event event_create();
void event_destroy(Event e);
void event_record(Event e, Flow f = nullptr);
void flow_wait(Flow f, Event e);  // f waits for e (device side)
void event_synchronize(Event e);

// Graph: captures the host API work the calling thread enqueues on its current flow between
// begin() and end() into one hipGraph and replays it with one launch (the reference runs every
// op eagerly; the Python front end captures its steps the same way, runtime/step.py). Every
// device block allocated during the capture belongs to the graph — freed blocks return to the
// graph's private free list, never to other users — so a replay finds the same addresses; the
// blocks return to the shared cache when the graph is destroyed. Inside a capture no host copy or
// host wait may run (the host API's loss readback is deferred: see gpu_ops::loss_device()).
class Graph {
 public:
  Graph() = default;
  ~Graph();
  Graph(const Graph&) = delete;
  Graph& operator=(const Graph&) = delete;
  void begin();
  void end();
  void replay();  // on the current flow
  bool ready() const { return exec_ != nullptr; }
  static bool capturing();  // the calling thread is inside begin() / end()

 private:
  void* graph_ = nullptr;  // hipGraph_t
  void* exec_ = nullptr;   // hipGraphExec_t
  void* pool_ = nullptr;   // the graph's private blocks
  Flow flow_ = nullptr;
};
// inter-process device buffers (same node): a dedicated allocation + its 64-byte IPC handle
constexpr size_t kIpcHandleBytes = 64;
void* ipc_alloc(size_t nbytes, void* handle_out);
void ipc_free(void* p);
void* ipc_open(const void* handle);  // map a peer process's buffer into this one
void ipc_close(void* p);
// stream-ordered 32-bit flag operations on device memory (also a peer's IPC mapping): the IPC
// transport's hand-off without a host wait. write: *p = v after the current flow's work so far;
// wait: the current flow's later work starts once *p >= v. false: the device lacks them.
bool stream_values_supported();
// inter-process events: an event another process can wait on (its 64-byte handle; nullptr when the
// runtime cannot export one), and a peer's event opened here
Event ipc_event_create(void* handle_out);
Event ipc_event_open(const void* handle);
void flow_write_u32(void* p, uint32_t v);
void flow_wait_u32_geq(void* p, uint32_t v);
}  // namespace gpu

class Storage {
 public:
  Storage(Device d, size_t nbytes);
  ~Storage();
  Storage(const Storage&) = delete;
  Storage& operator=(const Storage&) = delete;
  void* data() const { return p_; }
  size_t nbytes() const { return n_; }
  Device device() const { return dev_; }

 private:
  Device dev_;
  void* p_ = nullptr;
  size_t n_ = 0;
};

class Tensor {
 public:
  Tensor() = default;
  static Tensor empty(const std::vector<int64_t>& shape, DType dt, Device dev, Layout layout = Layout::NCHW);
  static Tensor zeros(const std::vector<int64_t>& shape, DType dt, Device dev, Layout layout = Layout::NCHW);
  // fp32 host values in LOGICAL (row-major NCHW) order -> tensor of the given dtype / device / layout
  static Tensor from_host(const std::vector<float>& v, const std::vector<int64_t>& shape, Device dev,
                          DType dt = DType::F32, Layout layout = Layout::NCHW);
  static Tensor from_host_i64(const std::vector<int64_t>& v, Device dev);

  bool defined() const { return (bool)st_; }
  const std::vector<int64_t>& shape() const { return shape_; }
  int64_t dim(int k) const { return shape_.at(k); }
  int rank() const { return (int)shape_.size(); }
  int64_t numel() const;
  size_t nbytes() const { return (size_t)numel() * dtype_size(dt_); }
  DType dtype() const { return dt_; }
  Device device() const { return st_ ? st_->device() : Device::cpu(); }
  Layout layout() const { return layout_; }
  void* data() const { return st_ ? static_cast<char*>(st_->data()) + off_ : nullptr; }
  template <typename T>
  T* ptr() const { return static_cast<T*>(data()); }

  // same storage, new logical shape / layout (element count must match)
  Tensor view(const std::vector<int64_t>& shape, Layout layout = Layout::NCHW) const;
  // a tensor over this one's storage from byte offset `byte_off` (parameter arenas)
  Tensor slice(size_t byte_off, const std::vector<int64_t>& shape, DType dt, Layout layout = Layout::NCHW) const;
  // grow-only: reallocate only when the new shape needs more bytes than the storage holds
  void ensure(const std::vector<int64_t>& shape, DType dt, Device dev, Layout layout = Layout::NCHW);
  Tensor clone() const;
  // copy to another device (same dtype / layout)
  Tensor to(Device dev) const;
  // fp32 values in LOGICAL row-major (NCHW) order, from any dtype / layout / device
  std::vector<float> to_host_f32() const;
  std::vector<int64_t> to_host_i64() const;
  void zero_();

  // reference .bin tensor record
  void save(std::ostream& os) const;
  static Tensor load(std::istream& is, Device dev = Device::cpu());

 private:
  std::shared_ptr<Storage> st_;
  size_t off_ = 0;  // byte offset into st_
  std::vector<int64_t> shape_;
  DType dt_ = DType::F32;
  Layout layout_ = Layout::NCHW;
};

std::string shape_str(const std::vector<int64_t>& s);

}  // namespace dcnn
