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
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "tensor.hpp"

namespace dcnn {
namespace coll {
class Comm;
}
class Sequential;

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

  // Overlapped bucketed gradient mean over `model`'s GPU parameter arena (the Python plane's
  // scheme, parallel/dp.py): the flat gradient is cut at top-level layer boundaries into buckets
  // of >= bucket_mb; each bucket's mean starts on this communicator's own flow as soon as the
  // backward has produced it (the layer hook, after the weight-gradient reduces queued so far are
  // flushed), while the earlier layers' backward continues on the compute flow; finish() reduces
  // the rest and makes the current flow wait for every bucket. Fork / join are events, so the
  // whole pattern is captured into a training step graph.
  void attach(Sequential& model, double bucket_mb = 4.0);
  void on_layer_done(size_t layer);  // Sequential::set_backward_hook
  void finish();                     // between the backward and the optimizer
  int buckets_last_step() const { return nb_last_; }

 private:
  Env env_;
  std::unique_ptr<coll::Comm> comm_;
  Tensor scratch_;
  // overlap state: gradient base, per top-level layer the first arena element of its parameters
  // (SIZE_MAX: none), the reduced suffix [reduced_lo, n)
  float* g_ = nullptr;
  size_t n_ = 0, reduced_lo_ = 0, bucket_elems_ = 0;
  std::vector<size_t> lo_;
  void* flow_ = nullptr;  // gpu::Flow
  void* ev_ = nullptr;    // gpu::Event
  int nb_ = 0, nb_last_ = 0;
  void fork_bucket(size_t lo, size_t hi);
};

// One direction of a stage-to-stage device data plane (the native pipeline's transport "rccl",
// dcnn/pipeline.hpp): a two-rank RCCL communicator (rank 0 = the lower stage) that carries one
// kind of tensor one way — activations down or gradients up — on a flow of its own, so a send
// waiting for its receiver never sits in front of the opposite direction's traffic or of compute.
// Hand-offs are event-ordered on the device: a send starts after the work the calling thread's
// flow holds so far; the flow that asks for a receive waits for it. No host synchronisation per
// tensor (the IPC transport copies and waits on the host).
//
// Reference parity: the reference moves activations as host fp32 over TCP
// (include/pipeline/tcp_communicator.hpp:190,455); the Python front end's counterpart of this
// plane is parallel/rccl.py's RcclP2P (one communicator and one stream per direction).
class P2PLink {
 public:
  // blocks until the peer has joined with the same id (rank 0 / 1 of the pair)
  P2PLink(const std::string& unique_id, int rank, bool sender, int device);
  ~P2PLink();
  P2PLink(const P2PLink&) = delete;
  P2PLink& operator=(const P2PLink&) = delete;
  bool sender() const { return sender_; }
  // t's bytes to the peer after the current flow's work so far; t stays referenced (slot `key`,
  // e.g. the micro-batch) until that send has completed
  void send(const Tensor& t, uint64_t key);
  // a fresh device tensor filled by the peer's next send; the current flow waits for it
  Tensor recv(const std::vector<int64_t>& shape, DType dt, Layout layout, Device dev);
  // host: every send so far has completed (its peer posted the receive); slots released
  void drain();
  // world-1 self loop of the same code path (tests): t's bytes through a one-rank communicator's
  // send + receive pair (one group) into a fresh tensor, ordered like send() / recv()
  static Tensor loopback(const Tensor& t);

 private:
  P2PLink() = default;
  void* flow_ = nullptr;   // gpu::Flow
  void* ready_ = nullptr;  // gpu::Event: the caller's flow reached the hand-off
  void* done_ = nullptr;   // gpu::Event: the last transfer on the link flow
  std::unique_ptr<coll::Comm> comm_;
  bool sender_ = false;
  int peer_ = 0;
  struct Held {
    Tensor t;
    void* ev = nullptr;  // gpu::Event recorded after its send
  };
  std::map<uint64_t, Held> held_;
};

}  // namespace dist
}  // namespace dcnn
