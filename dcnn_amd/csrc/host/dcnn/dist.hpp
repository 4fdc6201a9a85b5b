// Data parallelism of the C++ host API: one process per GPU, gradients all-reduced over the
// in-tree RCCL communicator (csrc/kernels/collective.h) on the calling thread's flow, so the
// collective is part of a captured training step (TrainGraph::set_gradient_hook).
//
// Launch: the torch.distributed launcher's variables (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR,
// MASTER_PORT) — `python -m torch.distributed.run --nproc-per-node N ... <program>` or any script
// that sets them. Rank 0 creates the RCCL unique id and hands it to the other ranks over a TCP
// socket at MASTER_ADDR:MASTER_PORT + port_offset (the launcher's own store holds MASTER_PORT).
//
// Reference parity: the reference has no data parallelism (SURVEY §2.13 maps DP over RCCL to
// MI355X as an addition); the Python front end's counterpart is parallel/dp.py.
#pragma once
#include <memory>
#include <string>

#include "tensor.hpp"

namespace dcnn {
namespace coll {
class Comm;
}

namespace dist {

struct Env {
  int rank = 0, world = 1, local_rank = 0;
  std::string addr = "127.0.0.1";
  int port = 29500;
  static Env from_env();  // defaults: a single process
};

// the 128-byte RCCL unique id of rank 0 on every rank (TCP at e.addr : e.port + port_offset)
std::string exchange_unique_id(const Env& e, int port_offset = 17, double timeout_s = 120.0);

class DataParallel {
 public:
  // selects GPU local_rank, rendezvous, creates the communicator (every rank must construct it)
  explicit DataParallel(const Env& e, int port_offset = 17);
  ~DataParallel();
  int rank() const { return env_.rank; }
  int world() const { return env_.world; }
  // in place: data <- mean over ranks (fp32), on the current flow (capturable)
  void all_reduce_mean(float* data, size_t n);
  // host scalar maximum over ranks (e.g. the slowest rank's step time)
  double max(double v);

 private:
  Env env_;
  std::unique_ptr<coll::Comm> comm_;
  Tensor scratch_;
};

}  // namespace dist
}  // namespace dcnn
