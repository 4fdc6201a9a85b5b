// In-tree RCCL communicator core (collective.h).
#include "collective.h"

#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

namespace dcnn {
namespace coll {
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

}  // namespace

bool available() { return lib().error.empty(); }
std::string load_error() { return lib().error; }
int version() {
  int v = 0;
  check(need().get_version(&v), "ncclGetVersion");
  return v;
}
std::string unique_id() {
  ncclUniqueId id;
  check(need().get_unique_id(&id), "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}
namespace {
thread_local int t_group_depth = 0;
thread_local std::vector<std::function<void()>> t_after_group;
}  // namespace

void group_start() {
  check(need().group_start(), "ncclGroupStart");
  ++t_group_depth;
}
void group_end() {
  if (t_group_depth > 0) --t_group_depth;
  check(need().group_end(), "ncclGroupEnd");
  if (t_group_depth == 0 && !t_after_group.empty()) {
    std::vector<std::function<void()>> fs;
    fs.swap(t_after_group);
    for (auto& f : fs) f();
  }
}
bool in_group() { return t_group_depth > 0; }
void after_group(std::function<void()> f) {
  if (t_group_depth > 0)
    t_after_group.push_back(std::move(f));
  else
    f();
}

Comm::Comm(const std::string& uid, int world, int rank, int device) : world_(world), rank_(rank) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("rccl: unique id must be 128 bytes");
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  RcclLib& L = need();
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl: hipSetDevice failed");
  ncclComm_t c = nullptr;
  check(L.comm_init_rank(&c, world, id, rank), "ncclCommInitRank");
  comm_ = c;
}
Comm::~Comm() { destroy(); }
void Comm::destroy() {
  if (comm_) {
    lib().comm_destroy(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
  }
}
void* Comm::live() const {
  if (!comm_) throw std::runtime_error("rccl: communicator destroyed");
  return comm_;
}
#define DCNN_COMM static_cast<ncclComm_t>(live())
#define DCNN_STREAM(s) static_cast<hipStream_t>(s)
void Comm::all_reduce(const void* send, void* recv, size_t count, int dt, int op, void* stream) {
  check(need().all_reduce(send, recv, count, dtype_of(dt), op_of(op), DCNN_COMM, DCNN_STREAM(stream)), "ncclAllReduce");
}
void Comm::broadcast(const void* send, void* recv, size_t count, int dt, int root, void* stream) {
  check(need().broadcast(send, recv, count, dtype_of(dt), root, DCNN_COMM, DCNN_STREAM(stream)), "ncclBroadcast");
}
void Comm::all_gather(const void* send, void* recv, size_t count, int dt, void* stream) {
  check(need().all_gather(send, recv, count, dtype_of(dt), DCNN_COMM, DCNN_STREAM(stream)), "ncclAllGather");
}
void Comm::reduce_scatter(const void* send, void* recv, size_t count, int dt, int op, void* stream) {
  check(need().reduce_scatter(send, recv, count, dtype_of(dt), op_of(op), DCNN_COMM, DCNN_STREAM(stream)),
        "ncclReduceScatter");
}
void Comm::send(const void* buf, size_t count, int dt, int peer, void* stream) {
  check(need().send(buf, count, dtype_of(dt), peer, DCNN_COMM, DCNN_STREAM(stream)), "ncclSend");
}
void Comm::recv(void* buf, size_t count, int dt, int peer, void* stream) {
  check(need().recv(buf, count, dtype_of(dt), peer, DCNN_COMM, DCNN_STREAM(stream)), "ncclRecv");
}
#undef DCNN_COMM
#undef DCNN_STREAM

}  // namespace coll
}  // namespace dcnn
