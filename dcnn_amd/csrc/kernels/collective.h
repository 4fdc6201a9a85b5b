// In-tree RCCL communicator core, plain C++ (no Python, no HIP types in the interface): the
// collective data plane of both front ends — ops/parallel's `parallel/rccl.py` (through the pybind
// wrapper in rccl.cpp) and the C++ host API's data parallelism / pipeline (csrc/host/dist.cpp).
//
// librccl.so (ROCm's NCCL-API library, xGMI / PCIe transports) is dlopen'ed on first use, so the
// libraries still build and load on hosts without it; nothing links against it at build time.
// Every collective is enqueued on the caller's HIP stream (passed as void*), so it is captured
// into a hipGraph like any other kernel of the step (RCCL kernels are stream-capturable).
//
// Reference parity: the reference has no collective library; its only data plane is host fp32
// over TCP (include/pipeline/tcp_communicator.hpp:190,455). SURVEY §5.8 / §2.13 map that plane to
// RCCL send/recv + all-reduce on MI355X.
#pragma once
#include <cstddef>
#include <functional>
#include <string>

namespace dcnn {
namespace coll {

bool available();
std::string load_error();
int version();
std::string unique_id();  // a fresh 128-byte ncclUniqueId (rank 0 creates it, every rank joins with it)
// (nestable; the calling thread's group) RCCL enqueues a group's operations at its outermost end
void group_start();
void group_end();
bool in_group();  // the calling thread is inside group_start() / group_end()
// f after the calling thread's outermost group_end() (at once outside a group): work that must
// follow a grouped operation on its stream, e.g. an event record
void after_group(std::function<void()> f);

// dtype codes (shared with parallel/rccl.py): 0 float32, 1 bfloat16, 2 float16, 3 int32, 4 uint8;
// reduction ops: 0 sum, 1 prod, 2 max, 3 min, 4 avg
class Comm {
 public:
  // blocks until every rank of the communicator has joined
  Comm(const std::string& unique_id, int world, int rank, int device);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;
  void destroy();
  int world() const { return world_; }
  int rank() const { return rank_; }
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int op, void* stream);
  void broadcast(const void* send, void* recv, size_t count, int dtype, int root, void* stream);
  void all_gather(const void* send, void* recv, size_t count, int dtype, void* stream);
  void reduce_scatter(const void* send, void* recv, size_t count, int dtype, int op, void* stream);
  void send(const void* buf, size_t count, int dtype, int peer, void* stream);
  void recv(void* buf, size_t count, int dtype, int peer, void* stream);

 private:
  void* live() const;
  void* comm_ = nullptr;  // ncclComm_t
  int world_, rank_;
};

}  // namespace coll
}  // namespace dcnn
