// Native device runtime: Device / Flow / Task and a stream-ordered caching allocator on HIP.
//
// Reference (what, not how): include/device/device.hpp:12-41 (Device: type, id, memory queries,
// allocate / free / copy), include/device/flow.hpp + include/device/task.hpp:26-209 (named
// execution queues and completion handles), include/device/device_ptr.hpp:80-285 (owning device
// pointers), src/device/cuda/cuda_context.cpp (cudaMalloc per allocation, one default stream).
//
// MI355X-first design:
// * a Flow is a HIP stream — created non-blocking (with an optional priority), or wrapping a
//   stream someone else owns (PyTorch's current stream, a capture stream) so work from both
//   runtimes orders on the same queue;
// * a Task is a HIP event recorded on a flow (timing disabled unless asked): sync() waits for that
//   event only, never the device;
// * memory comes from a per-device hipMemPool used through hipMallocAsync / hipFreeAsync on the
//   caller's flow. The pool's release threshold is raised to "keep everything", so memory freed on
//   a stream is reused by later allocations in stream order without going back to the driver: a
//   training step that allocates the same sizes every iteration reaches a steady state with no
//   new reservations (Allocator::stats() exposes the pool's reserved/used counters and the number
//   of allocations that had to grow the reservation);
// * buffers can be handed to PyTorch zero-copy through DLPack (kDLROCM), which is how the
//   framework's flat parameter/gradient/optimizer arenas live in this allocator.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace dcnn {
namespace rt {

#define RT_CHECK(expr)                                                                               \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess)                                                                            \
      throw std::runtime_error(std::string("HIP runtime error ") + hipGetErrorString(_e) + " in " + \
                               #expr);                                                               \
  } while (0)

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    RT_CHECK(hipGetDevice(&prev));
    if (prev != dev) RT_CHECK(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

// ------------------------------------------------------------------ Device
py::dict device_properties(int dev) {
  hipDeviceProp_t p;
  RT_CHECK(hipGetDeviceProperties(&p, dev));
  py::dict d;
  d["name"] = std::string(p.name);
  d["arch"] = std::string(p.gcnArchName);
  d["total_memory"] = (uint64_t)p.totalGlobalMem;
  d["multiprocessors"] = p.multiProcessorCount;
  d["max_threads_per_block"] = p.maxThreadsPerBlock;
  d["warp_size"] = p.warpSize;
  d["lds_per_block"] = (uint64_t)p.sharedMemPerBlock;
  d["l2_cache"] = p.l2CacheSize;
  d["clock_khz"] = p.clockRate;
  d["memory_pools"] = p.memoryPoolsSupported;
  d["pci_bus_id"] = p.pciBusID;
  return d;
}

std::pair<uint64_t, uint64_t> mem_info(int dev) {
  DeviceGuard g(dev);
  size_t f = 0, t = 0;
  RT_CHECK(hipMemGetInfo(&f, &t));
  return {(uint64_t)f, (uint64_t)t};
}

void device_synchronize(int dev) {
  DeviceGuard g(dev);
  RT_CHECK(hipDeviceSynchronize());
}

bool can_access_peer(int dev, int peer) {
  int ok = 0;
  RT_CHECK(hipDeviceCanAccessPeer(&ok, dev, peer));
  return ok != 0;
}

// ------------------------------------------------------------------ Flow / Task
class Flow {
 public:
  Flow(int dev, int priority) : dev_(dev), owned_(true) {
    DeviceGuard g(dev);
    RT_CHECK(hipStreamCreateWithPriority(&s_, hipStreamNonBlocking, priority));
  }
  Flow(int dev, uintptr_t external) : dev_(dev), s_(reinterpret_cast<hipStream_t>(external)), owned_(false) {}
  ~Flow() {
    if (owned_ && s_) {
      (void)hipStreamSynchronize(s_);
      (void)hipStreamDestroy(s_);
    }
  }
  Flow(const Flow&) = delete;
  Flow& operator=(const Flow&) = delete;

  uintptr_t handle() const { return reinterpret_cast<uintptr_t>(s_); }
  int device() const { return dev_; }
  bool owned() const { return owned_; }
  void synchronize() const {
    py::gil_scoped_release nogil;
    RT_CHECK(hipStreamSynchronize(s_));
  }
  bool query() const {
    const hipError_t e = hipStreamQuery(s_);
    if (e == hipErrorNotReady) return false;
    RT_CHECK(e);
    return true;
  }
  hipStream_t stream() const { return s_; }

 private:
  int dev_;
  hipStream_t s_ = nullptr;
  bool owned_;
};

class Task {
 public:
  Task(int dev, bool timing) : dev_(dev) {
    DeviceGuard g(dev);
    RT_CHECK(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming));
  }
  ~Task() {
    if (e_) (void)hipEventDestroy(e_);
  }
  Task(const Task&) = delete;
  Task& operator=(const Task&) = delete;

  void record(const Flow& f) {
    RT_CHECK(hipEventRecord(e_, f.stream()));
    recorded_ = true;
  }
  void sync() const {
    if (!recorded_) return;
    py::gil_scoped_release nogil;
    RT_CHECK(hipEventSynchronize(e_));
  }
  bool is_ready() const {
    if (!recorded_) return true;
    const hipError_t e = hipEventQuery(e_);
    if (e == hipErrorNotReady) return false;
    RT_CHECK(e);
    return true;
  }
  float elapsed_ms(const Task& end) const {
    float ms = 0.f;
    RT_CHECK(hipEventElapsedTime(&ms, e_, end.e_));
    return ms;
  }
  hipEvent_t event() const { return e_; }

 private:
  int dev_;
  hipEvent_t e_ = nullptr;
  bool recorded_ = false;
};

void flow_wait(const Flow& f, const Task& t) { RT_CHECK(hipStreamWaitEvent(f.stream(), t.event(), 0)); }

// ------------------------------------------------------------------ Allocator
class Allocator {
 public:
  static Allocator& get(int dev) {
    static std::mutex mu;
    static std::vector<std::unique_ptr<Allocator>> all;
    std::lock_guard<std::mutex> g(mu);
    if ((int)all.size() <= dev) all.resize(dev + 1);
    if (!all[dev]) all[dev].reset(new Allocator(dev));
    return *all[dev];
  }

  uintptr_t allocate(uint64_t nbytes, const Flow& f) {
    if (nbytes == 0) nbytes = 1;
    // dropped DLPack exports are reclaimed only when that can serve this request from the pool
    // (the queue holds at least nbytes) or the queue is large (>= 256 MiB / 256 buffers): the
    // reclaim synchronises the device, so small allocations next to a few small pending frees do
    // not drain every stream (other pipeline stages mid-step keep running)
    bool reclaim;
    {
      std::lock_guard<std::mutex> l(mu_);  // defer_free runs on any thread (DLPack deleters)
      reclaim = deferred_bytes_ >= std::max<uint64_t>(nbytes, 1) || deferred_bytes_ >= (256ull << 20) ||
                deferred_.size() >= 256;
    }
    if (reclaim) release_deferred();
    DeviceGuard g(dev_);
    const uint64_t before = reserved();
    void* p = nullptr;
    RT_CHECK(hipMallocFromPoolAsync(&p, nbytes, pool_, f.stream()));
    std::lock_guard<std::mutex> l(mu_);
    ++allocs_;
    if (reserved() > before) ++grows_;
    in_use_ += nbytes;
    peak_ = std::max(peak_, in_use_);
    return reinterpret_cast<uintptr_t>(p);
  }
  void free(uintptr_t p, uint64_t nbytes, const Flow& f) {
    DeviceGuard g(dev_);
    RT_CHECK(hipFreeAsync(reinterpret_cast<void*>(p), f.stream()));
    std::lock_guard<std::mutex> l(mu_);
    ++frees_;
    in_use_ -= std::min(in_use_, nbytes);
  }
  // Buffers whose last user is unknown (DLPack exports, freed by whoever drops the last tensor
  // reference — possibly Python's GC inside another thread's graph capture, where no HIP call may
  // run): only queued here, released by release_deferred() at the next allocation or an explicit
  // device synchronize.
  void defer_free(uintptr_t p, uint64_t nbytes) {
    std::lock_guard<std::mutex> l(mu_);
    deferred_.push_back({p, nbytes});
    deferred_bytes_ += nbytes;
  }
  void release_deferred() {
    std::vector<std::pair<uintptr_t, uint64_t>> todo;
    {
      std::lock_guard<std::mutex> l(mu_);
      todo.swap(deferred_);
      deferred_bytes_ = 0;
    }
    if (todo.empty()) return;
    DeviceGuard g(dev_);
    auto drain = [&] {  // every stream done with them
      RT_CHECK(hipDeviceSynchronize());
      for (auto& d : todo) RT_CHECK(hipFreeAsync(reinterpret_cast<void*>(d.first), nullptr));
      RT_CHECK(hipStreamSynchronize(nullptr));
    };
    if (PyGILState_Check()) {  // other Python threads (pipeline stages) keep running meanwhile
      py::gil_scoped_release nogil;
      drain();
    } else {
      drain();
    }
    std::lock_guard<std::mutex> l(mu_);
    for (auto& d : todo) {
      ++frees_;
      in_use_ -= std::min(in_use_, d.second);
    }
  }
  uint64_t reserved() const {
    uint64_t v = 0;
    RT_CHECK(hipMemPoolGetAttribute(pool_, hipMemPoolAttrReservedMemCurrent, &v));
    return v;
  }
  py::dict stats() const {
    py::dict d;
    uint64_t v = 0;
    RT_CHECK(hipMemPoolGetAttribute(pool_, hipMemPoolAttrReservedMemCurrent, &v));
    d["reserved_bytes"] = v;
    RT_CHECK(hipMemPoolGetAttribute(pool_, hipMemPoolAttrReservedMemHigh, &v));
    d["reserved_peak_bytes"] = v;
    RT_CHECK(hipMemPoolGetAttribute(pool_, hipMemPoolAttrUsedMemCurrent, &v));
    d["used_bytes"] = v;
    std::lock_guard<std::mutex> l(mu_);
    d["allocations"] = allocs_;
    d["frees"] = frees_;
    d["reservation_grows"] = grows_;
    d["in_use_bytes"] = in_use_;
    d["deferred_frees"] = (uint64_t)deferred_.size();
    d["peak_in_use_bytes"] = peak_;
    return d;
  }
  void trim(uint64_t keep) {
    DeviceGuard g(dev_);
    RT_CHECK(hipDeviceSynchronize());
    RT_CHECK(hipMemPoolTrimTo(pool_, keep));
  }
  int device() const { return dev_; }

 private:
  explicit Allocator(int dev) : dev_(dev) {
    DeviceGuard g(dev);
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    RT_CHECK(hipMemPoolCreate(&pool_, &props));
    uint64_t keep_all = ~0ull;  // never hand cached memory back to the driver at sync points
    RT_CHECK(hipMemPoolSetAttribute(pool_, hipMemPoolAttrReleaseThreshold, &keep_all));
  }
  int dev_;
  hipMemPool_t pool_ = nullptr;
  mutable std::mutex mu_;
  uint64_t allocs_ = 0, frees_ = 0, grows_ = 0, in_use_ = 0, peak_ = 0;
  std::vector<std::pair<uintptr_t, uint64_t>> deferred_;
  uint64_t deferred_bytes_ = 0;
};

// ------------------------------------------------------------------ DLPack export (zero copy)
// Minimal DLPack v0.x ABI (the legacy "dltensor" capsule every PyTorch accepts).
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
  void* data; DLDevice device; int32_t ndim; DLDataType dtype; int64_t* shape; int64_t* strides; uint64_t byte_offset;
};
struct DLManagedTensor { DLTensor dl_tensor; void* manager_ctx; void (*deleter)(DLManagedTensor*); };
constexpr int32_t kDLROCM = 10;

struct Export {
  DLManagedTensor m{};
  std::vector<int64_t> shape;
  int dev = 0;
  uintptr_t ptr = 0;
  uint64_t nbytes = 0;
};

void export_deleter(DLManagedTensor* m) {  // no HIP call here (see Allocator::defer_free)
  Export* e = static_cast<Export*>(m->manager_ctx);
  Allocator::get(e->dev).defer_free(e->ptr, e->nbytes);
  delete e;
}

// dtype codes: (DLPack code, bits): float 2, int 0, uint 1, bfloat 4
py::capsule alloc_dlpack(int dev, std::vector<int64_t> shape, int code, int bits, const Flow& f, bool zero) {
  int64_t numel = 1;
  for (auto s : shape) numel *= s;
  const uint64_t nbytes = (uint64_t)numel * (bits / 8);
  Export* e = new Export();
  e->dev = dev;
  e->nbytes = nbytes;
  e->shape = shape;
  try {
    e->ptr = Allocator::get(dev).allocate(nbytes, f);
    if (zero) {
      DeviceGuard g(dev);
      RT_CHECK(hipMemsetAsync(reinterpret_cast<void*>(e->ptr), 0, nbytes, f.stream()));
    }
  } catch (...) {
    delete e;
    throw;
  }
  DLTensor& t = e->m.dl_tensor;
  t.data = reinterpret_cast<void*>(e->ptr);
  t.device = DLDevice{kDLROCM, dev};
  t.ndim = (int32_t)e->shape.size();
  t.dtype = DLDataType{(uint8_t)code, (uint8_t)bits, 1};
  t.shape = e->shape.data();
  t.strides = nullptr;  // compact row-major
  t.byte_offset = 0;
  e->m.manager_ctx = e;
  e->m.deleter = export_deleter;
  return py::capsule(&e->m, "dltensor", [](PyObject* cap) {
    // called when the capsule dies: only if nobody consumed it (consumers rename it)
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* m = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
      if (m && m->deleter) m->deleter(m);
    }
  });
}

// ------------------------------------------------------------------ ActArena
// Per-step activation arena: every activation, statistics slab and split-K workspace of one
// training step is bump-allocated from device chunks owned here (drawn from the native pool), and
// the bump pointer is reset at the next step — no allocator call per tensor, identical addresses
// every step (so a hipGraph captured from a step sees the same buffers eager steps use), and no
// activation on PyTorch's caching allocator.
//
// Growth only on first use: a step that overruns the chunks appends a chunk (at least the current
// capacity: doubling); the next reset() coalesces every chunk into one of the high-water size, so
// from the second step on the arena neither grows nor allocates. Chunks are exported to PyTorch
// once each (DLPack, shared ownership): a tensor that outlives its step keeps its chunk alive, and
// the memory returns to the pool (Allocator::defer_free) only when the last view is gone.
// Reference parity: include/nn/mem_pool.hpp:11-101, include/device/device_ptr.hpp:184-217
// (grow-only ensure), include/tensor/tensor.hpp:424-511.
struct ArenaChunk {
  int dev = 0;
  uintptr_t ptr = 0;
  uint64_t nbytes = 0;
  int64_t id = 0;
  ~ArenaChunk() {
    if (ptr) Allocator::get(dev).defer_free(ptr, nbytes);  // no HIP call: any thread, any time
  }
};

struct ChunkExport {
  DLManagedTensor m{};
  std::shared_ptr<ArenaChunk> chunk;
  int64_t shape[1] = {0};
};

void chunk_export_deleter(DLManagedTensor* m) { delete static_cast<ChunkExport*>(m->manager_ctx); }

class ActArena {
 public:
  static constexpr uint64_t kAlign = 256;
  ActArena(int dev, uint64_t initial_bytes) : dev_(dev), initial_(std::max<uint64_t>(initial_bytes, 1u << 20)) {}

  // (chunk id, byte offset) of nbytes in the current step; (-1, 0) when it does not fit and the
  // arena is frozen (graph capture: no allocation may be recorded into the graph)
  std::pair<int64_t, uint64_t> alloc(uint64_t nbytes) {
    nbytes = (std::max<uint64_t>(nbytes, 1) + kAlign - 1) & ~(kAlign - 1);
    while (cur_ < chunks_.size()) {
      ArenaChunk& c = *chunks_[cur_];
      if (off_ + nbytes <= c.nbytes) {
        const uint64_t o = off_;
        off_ += nbytes;
        used_ += nbytes;
        high_ = std::max(high_, used_);
        ++allocs_;
        return {c.id, o};
      }
      ++cur_;  // the rest of this chunk stays unused this step (counted by the coalesce)
      used_ += c.nbytes - off_;
      off_ = 0;
    }
    if (frozen_) {
      ++refused_;
      return {-1, 0};
    }
    add_chunk(std::max<uint64_t>(nbytes, chunks_.empty() ? initial_ : capacity()));
    return alloc(nbytes);
  }

  // start of a step: rewind; merge a multi-chunk arena into one chunk of the high-water size
  // (allocated on `stream`, ordered after everything already queued there)
  bool reset(uintptr_t stream) {
    stream_ = stream;
    bool rebuilt = false;
    if (chunks_.size() > 1 && !frozen_) {
      const uint64_t want = (std::max(high_, capacity()) + (2u << 20) - 1) & ~((uint64_t)(2u << 20) - 1);
      chunks_.clear();
      add_chunk(want);
      ++coalesces_;
      rebuilt = true;
    }
    cur_ = 0;
    off_ = 0;
    used_ = 0;
    ++steps_;
    return rebuilt;
  }
  void set_frozen(bool f) { frozen_ = f; }
  bool frozen() const { return frozen_; }

  // the chunk as a flat uint8 DLPack tensor sharing ownership of its memory
  py::capsule chunk_capsule(int64_t id) {
    for (auto& c : chunks_) {
      if (c->id != id) continue;
      auto* e = new ChunkExport();
      e->chunk = c;
      e->shape[0] = (int64_t)c->nbytes;
      DLTensor& t = e->m.dl_tensor;
      t.data = reinterpret_cast<void*>(c->ptr);
      t.device = DLDevice{kDLROCM, dev_};
      t.ndim = 1;
      t.dtype = DLDataType{1, 8, 1};
      t.shape = e->shape;
      t.strides = nullptr;
      t.byte_offset = 0;
      e->m.manager_ctx = e;
      e->m.deleter = chunk_export_deleter;
      return py::capsule(&e->m, "dltensor", [](PyObject* cap) {
        if (PyCapsule_IsValid(cap, "dltensor")) {
          auto* m = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
          if (m && m->deleter) m->deleter(m);
        }
      });
    }
    throw std::out_of_range("ActArena: no live chunk with this id");
  }

  uint64_t capacity() const {
    uint64_t v = 0;
    for (auto& c : chunks_) v += c->nbytes;
    return v;
  }
  py::dict stats() const {
    py::dict d;
    d["capacity_bytes"] = capacity();
    d["chunks"] = (uint64_t)chunks_.size();
    d["used_bytes"] = used_;
    d["high_water_bytes"] = high_;
    d["allocations"] = allocs_;
    d["grows"] = grows_;
    d["coalesces"] = coalesces_;
    d["steps"] = steps_;
    d["refused"] = refused_;
    return d;
  }
  int device() const { return dev_; }

 private:
  void add_chunk(uint64_t nbytes) {
    auto c = std::make_shared<ArenaChunk>();
    c->dev = dev_;
    c->nbytes = nbytes;
    c->id = next_id_++;
    Flow f(dev_, stream_);
    c->ptr = Allocator::get(dev_).allocate(nbytes, f);
    chunks_.push_back(std::move(c));
    ++grows_;
  }
  int dev_;
  uint64_t initial_;
  uintptr_t stream_ = 0;
  std::vector<std::shared_ptr<ArenaChunk>> chunks_;
  size_t cur_ = 0;
  uint64_t off_ = 0, used_ = 0, high_ = 0;
  uint64_t allocs_ = 0, grows_ = 0, coalesces_ = 0, steps_ = 0, refused_ = 0;
  int64_t next_id_ = 0;
  bool frozen_ = false;
};

// ------------------------------------------------------------------ copies
// kind: 0 host->device, 1 device->host, 2 device->device, 3 default (unified addressing)
void memcpy_async(uintptr_t dst, uintptr_t src, uint64_t nbytes, int kind, const Flow& f) {
  static const hipMemcpyKind kinds[] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice,
                                        hipMemcpyDefault};
  if (kind < 0 || kind > 3) throw std::invalid_argument("memcpy_async: bad kind");
  RT_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), nbytes, kinds[kind],
                          f.stream()));
}

void memset_async(uintptr_t dst, int value, uint64_t nbytes, const Flow& f) {
  RT_CHECK(hipMemsetAsync(reinterpret_cast<void*>(dst), value, nbytes, f.stream()));
}

uintptr_t host_alloc_pinned(uint64_t nbytes) {
  void* p = nullptr;
  RT_CHECK(hipHostMalloc(&p, nbytes ? nbytes : 1, hipHostMallocDefault));
  return reinterpret_cast<uintptr_t>(p);
}
void host_free_pinned(uintptr_t p) { RT_CHECK(hipHostFree(reinterpret_cast<void*>(p))); }

}  // namespace rt
}  // namespace dcnn

void bind_runtime(py::module_& parent) {
  using namespace dcnn::rt;
  py::module_ m = parent.def_submodule("rt", "native HIP device runtime: Device / Flow / Task / Allocator");
  m.def("device_count", &device_count);
  m.def("device_properties", &device_properties);
  m.def("mem_info", &mem_info);
  m.def("device_synchronize", &device_synchronize, py::call_guard<py::gil_scoped_release>());
  m.def("can_access_peer", &can_access_peer);
  py::class_<Flow>(m, "Flow")
      .def(py::init<int, int>(), py::arg("device"), py::arg("priority") = 0)
      // (a separate factory, not an overloaded constructor: the null stream's handle is 0, which
      // an (int, int) overload would take as a priority and silently create a NEW stream)
      .def_static("wrap", [](int dev, uintptr_t handle) { return std::make_unique<Flow>(dev, handle); },
                  py::arg("device"), py::arg("external_stream"))
      .def_property_readonly("handle", &Flow::handle)
      .def_property_readonly("device", &Flow::device)
      .def_property_readonly("owned", &Flow::owned)
      .def("synchronize", &Flow::synchronize)
      .def("query", &Flow::query)
      .def("wait", &flow_wait);
  py::class_<Task>(m, "Task")
      .def(py::init<int, bool>(), py::arg("device"), py::arg("timing") = false)
      .def("record", &Task::record)
      .def("sync", &Task::sync)
      .def("is_ready", &Task::is_ready)
      .def("elapsed_ms", &Task::elapsed_ms);
  py::class_<Allocator, std::unique_ptr<Allocator, py::nodelete>>(m, "Allocator")
      .def_static("get", &Allocator::get, py::return_value_policy::reference)
      .def("allocate", &Allocator::allocate)
      .def("free", &Allocator::free)
      .def("stats", &Allocator::stats)
      .def("trim", &Allocator::trim, py::arg("keep_bytes") = 0)
      .def("release_deferred", &Allocator::release_deferred, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("device", &Allocator::device);
  py::class_<ActArena>(m, "ActArena")
      .def(py::init<int, uint64_t>(), py::arg("device"), py::arg("initial_bytes") = (uint64_t)256 << 20)
      .def("alloc", &ActArena::alloc)
      .def("reset", &ActArena::reset, py::arg("stream"))
      .def("set_frozen", &ActArena::set_frozen)
      .def_property_readonly("frozen", &ActArena::frozen)
      .def("chunk", &ActArena::chunk_capsule)
      .def("capacity", &ActArena::capacity)
      .def("stats", &ActArena::stats)
      .def_property_readonly("device", &ActArena::device);
  m.def("alloc_dlpack", &alloc_dlpack, py::arg("device"), py::arg("shape"), py::arg("code"), py::arg("bits"),
        py::arg("flow"), py::arg("zero") = false);
  m.def("memcpy_async", &memcpy_async);
  m.def("memset_async", &memset_async);
  m.def("host_alloc_pinned", &host_alloc_pinned);
  m.def("host_free_pinned", &host_free_pinned);
}
