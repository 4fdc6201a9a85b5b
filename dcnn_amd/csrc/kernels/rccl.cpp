// In-tree RCCL communicator: the MI355X collective data plane owned by the framework.
//
// librccl.so (ROCm's NCCL-API library, xGMI / PCIe transports) is dlopen'ed on first use, so the
// extension still builds and imports on hosts without it; nothing links against it at build time.
// The 128-byte ncclUniqueId is created on rank 0 and exchanged over the framework's own TCP
// control plane (csrc/native/comm.cpp, parallel/rccl.py) — no torch.distributed store involved.
// Every collective is enqueued on the caller's HIP stream, so it is captured into a hipGraph like
// any other kernel of the step (RCCL kernels are stream-capturable).
//
// Reference parity: the reference has no collective library at all; its only data plane is host
// fp32 over TCP (include/pipeline/tcp_communicator.hpp:190,455). SURVEY §5.8 / §2.13 map that
// plane to RCCL send/recv + all-reduce on MI355X.
#include <dlfcn.h>

#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include <pybind11/pybind11.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

namespace py = pybind11;

namespace dcnn {
namespace {

struct RcclLib {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGetVersion) get_version = nullptr;
  std::string error;
};

RcclLib& lib() {
  static RcclLib L;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"};
    for (const char* n : names) {
      L.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (L.h) break;
    }
    if (!L.h) {
      L.error = std::string("dlopen(librccl.so) failed: ") + (dlerror() ? dlerror() : "?");
      return;
    }
    auto sym = [&](const char* s) {
      void* p = dlsym(L.h, s);
      if (!p && L.error.empty()) L.error = std::string("librccl.so lacks ") + s;
      return p;
    };
    L.get_unique_id = reinterpret_cast<decltype(L.get_unique_id)>(sym("ncclGetUniqueId"));
    L.comm_init_rank = reinterpret_cast<decltype(L.comm_init_rank)>(sym("ncclCommInitRank"));
    L.comm_destroy = reinterpret_cast<decltype(L.comm_destroy)>(sym("ncclCommDestroy"));
    L.all_reduce = reinterpret_cast<decltype(L.all_reduce)>(sym("ncclAllReduce"));
    L.broadcast = reinterpret_cast<decltype(L.broadcast)>(sym("ncclBroadcast"));
    L.all_gather = reinterpret_cast<decltype(L.all_gather)>(sym("ncclAllGather"));
    L.reduce_scatter = reinterpret_cast<decltype(L.reduce_scatter)>(sym("ncclReduceScatter"));
    L.send = reinterpret_cast<decltype(L.send)>(sym("ncclSend"));
    L.recv = reinterpret_cast<decltype(L.recv)>(sym("ncclRecv"));
    L.group_start = reinterpret_cast<decltype(L.group_start)>(sym("ncclGroupStart"));
    L.group_end = reinterpret_cast<decltype(L.group_end)>(sym("ncclGroupEnd"));
    L.error_string = reinterpret_cast<decltype(L.error_string)>(sym("ncclGetErrorString"));
    L.get_version = reinterpret_cast<decltype(L.get_version)>(sym("ncclGetVersion"));
  });
  return L;
}

RcclLib& need() {
  RcclLib& L = lib();
  if (!L.error.empty()) throw std::runtime_error("rccl: " + L.error);
  return L;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    RcclLib& L = lib();
    throw std::runtime_error(std::string("rccl: ") + what + " failed: " +
                             (L.error_string ? L.error_string(r) : std::to_string((int)r)));
  }
}

// dtype codes shared with parallel/rccl.py: 0 float32, 1 bfloat16, 2 float16, 3 int32, 4 int8/uint8
ncclDataType_t dtype_of(int code) {
  switch (code) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclUint8;
  }
  throw std::runtime_error("rccl: unknown dtype code");
}
ncclRedOp_t op_of(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
  }
  throw std::runtime_error("rccl: unknown reduction op");
}

// One communicator: a handle over ncclComm_t. Collectives take raw device pointers and the
// caller's hipStream_t (uintptr_t), exactly like the compute kernels of this library.
class RcclComm {
 public:
  RcclComm(py::bytes uid, int world, int rank, int device) : world_(world), rank_(rank) {
    std::string s = uid;
    if (s.size() != sizeof(ncclUniqueId)) throw std::runtime_error("rccl: unique id must be 128 bytes");
    ncclUniqueId id;
    memcpy(&id, s.data(), sizeof(id));
    RcclLib& L = need();
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl: hipSetDevice failed");
    ncclResult_t r;
    {
      py::gil_scoped_release nogil;  // blocks until every rank has joined
      r = L.comm_init_rank(&comm_, world, id, rank);
    }
    check(r, "ncclCommInitRank");
  }
  ~RcclComm() { destroy(); }
  void destroy() {
    if (comm_) {
      lib().comm_destroy(comm_);
      comm_ = nullptr;
    }
  }
  int world() const { return world_; }
  int rank() const { return rank_; }
  void all_reduce(uintptr_t send, uintptr_t recv, size_t count, int dt, int op, uintptr_t stream) {
    check(need().all_reduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype_of(dt),
                            op_of(op), live(), reinterpret_cast<hipStream_t>(stream)),
          "ncclAllReduce");
  }
  void broadcast(uintptr_t send, uintptr_t recv, size_t count, int dt, int root, uintptr_t stream) {
    check(need().broadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype_of(dt),
                           root, live(), reinterpret_cast<hipStream_t>(stream)),
          "ncclBroadcast");
  }
  void all_gather(uintptr_t send, uintptr_t recv, size_t count, int dt, uintptr_t stream) {
    check(need().all_gather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count, dtype_of(dt),
                            live(), reinterpret_cast<hipStream_t>(stream)),
          "ncclAllGather");
  }
  void reduce_scatter(uintptr_t send, uintptr_t recv, size_t count, int dt, int op, uintptr_t stream) {
    check(need().reduce_scatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                                dtype_of(dt), op_of(op), live(), reinterpret_cast<hipStream_t>(stream)),
          "ncclReduceScatter");
  }
  void send(uintptr_t buf, size_t count, int dt, int peer, uintptr_t stream) {
    check(need().send(reinterpret_cast<const void*>(buf), count, dtype_of(dt), peer, live(),
                      reinterpret_cast<hipStream_t>(stream)),
          "ncclSend");
  }
  void recv(uintptr_t buf, size_t count, int dt, int peer, uintptr_t stream) {
    check(need().recv(reinterpret_cast<void*>(buf), count, dtype_of(dt), peer, live(),
                      reinterpret_cast<hipStream_t>(stream)),
          "ncclRecv");
  }

 private:
  ncclComm_t live() const {
    if (!comm_) throw std::runtime_error("rccl: communicator destroyed");
    return comm_;
  }
  ncclComm_t comm_ = nullptr;
  int world_, rank_;
};

}  // namespace
}  // namespace dcnn

void bind_rccl(py::module_& m) {
  using namespace dcnn;
  auto r = m.def_submodule("rccl", "in-tree RCCL communicator (librccl.so, dlopen'ed)");
  r.def("available", [] { return lib().error.empty(); });
  r.def("load_error", [] { return lib().error; });
  r.def("version", [] {
    int v = 0;
    check(need().get_version(&v), "ncclGetVersion");
    return v;
  });
  r.def("unique_id", [] {
    ncclUniqueId id;
    check(need().get_unique_id(&id), "ncclGetUniqueId");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  r.def("group_start", [] { check(need().group_start(), "ncclGroupStart"); });
  r.def("group_end", [] { check(need().group_end(), "ncclGroupEnd"); });
  py::class_<RcclComm>(r, "Comm")
      .def(py::init<py::bytes, int, int, int>(), py::arg("unique_id"), py::arg("world"), py::arg("rank"),
           py::arg("device"))
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("rank", &RcclComm::rank)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"),
           py::arg("op"), py::arg("stream"))
      .def("broadcast", &RcclComm::broadcast)
      .def("all_gather", &RcclComm::all_gather)
      .def("reduce_scatter", &RcclComm::reduce_scatter)
      .def("send", &RcclComm::send)
      .def("recv", &RcclComm::recv)
      .def("destroy", &RcclComm::destroy);
}
