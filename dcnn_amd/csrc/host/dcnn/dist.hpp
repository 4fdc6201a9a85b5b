// Data parallelism of the C++ host API: one process per GPU, gradients all-reduced over the
// in-tree RCCL communicator (csrc/kernels/collective.h) on the calling thread's flow, so the
// collective is part of a captured training step (TrainGraph::set_gradient_hook); on the CPU
// device the same schedule runs over a TCP ring of the processes (HostRing).
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
  double timeout_s = 120.0;  // rendezvous / host-plane wait limit (DCNN_DIST_TIMEOUT)
  static Env from_env();     // defaults: a single process
};

// the 128-byte RCCL unique id of rank 0 on every rank (TCP at e.addr : e.port + port_offset);
// every wait — rank 0 for the other ranks, a rank for rank 0 — ends after e.timeout_s with an error
std::string exchange_unique_id(const Env& e, int port_offset = 17);

// Host data plane of the CPU device: a TCP ring of the ranks' processes (rank r sends to r + 1 and
// receives from r - 1). Rendezvous at e.addr : e.port + port_offset: rank 0 collects every rank's
// listening address and hands out the table, then each rank connects to its successor. All
// reductions run in a fixed order (ring reduce-scatter + all-gather over W chunks), so every rank
// ends with bitwise the same result and reruns are deterministic.
class HostRing {
 public:
  HostRing(const Env& e, int port_offset);
  ~HostRing();
  HostRing(const HostRing&) = delete;
  HostRing& operator=(const HostRing&) = delete;
  int rank() const { return rank_; }
  int world() const { return world_; }
  enum Op { kSum, kMax };
  void all_reduce(float* x, size_t n, Op op = kSum);
  void broadcast(void* x, size_t nbytes, int root = 0);  // down the ring from `root`
  void barrier();

 private:
  int rank_ = 0, world_ = 1;
  int next_ = -1, prev_ = -1;  // sockets: to rank + 1, from rank - 1
  double timeout_s_ = 120.0;
  // send `sn` bytes to the successor while receiving `rn` from the predecessor (poll-driven, so a
  // ring of blocking senders cannot deadlock)
  void exchange(const char* s, size_t sn, char* r, size_t rn);
};

// Data parallelism over the processes of one job: the mean of the model's gradients over the
// ranks between the backward and the optimizer. GPU: the in-tree RCCL communicator on GPU
// local_rank, inside the captured step. CPU: the HostRing above (same bucket schedule, host
// reduction), so the schedule and the rendezvous run multi-process in CPU CI.
class DataParallel {
 public:
  // selects GPU local_rank (GPU), rendezvous, creates the plane (every rank must construct it)
  DataParallel(const Env& e, Device dev, int port_offset = 17);
  explicit DataParallel(const Env& e, int port_offset = 17) : DataParallel(e, Device::gpu(e.local_rank), port_offset) {}
  ~DataParallel();
  int rank() const { return env_.rank; }
  int world() const { return env_.world; }
  Device device() const { return dev_; }
  const char* plane() const { return dev_.is_gpu() ? "rccl" : "tcp"; }
  // in place: data <- mean over ranks (fp32); GPU: device memory, on the current flow (capturable)
  void all_reduce_mean(float* data, size_t n);
  // host scalar maximum over ranks (e.g. the slowest rank's step time)
  double max(double v);
  // every rank has reached this point (GPU: and the current flow's work so far has completed)
  void barrier();
  // rank 0's parameter values (and bf16 shadows, BatchNorm running statistics) on every rank, so
  // replicas start identical whatever each rank's seed or checkpoint was
  void broadcast_parameters(Sequential& model);

  // Overlapped bucketed gradient mean over `model`'s parameters (the Python plane's scheme,
  // parallel/dp.py): the gradients are cut at top-level layer boundaries into buckets of
  // >= bucket_mb; a bucket's mean starts as soon as the backward has produced it (the layer hook).
  // GPU: the parameters live in one arena, a bucket is a contiguous range whose mean runs on this
  // communicator's own flow (after the weight-gradient reduces queued so far are flushed) while
  // the earlier layers' backward continues; finish() reduces the rest and makes the current flow
  // wait for every bucket. Fork / join are events, so the pattern is captured into a step graph.
  // CPU: a bucket's gradients are packed, ring-reduced and unpacked at the hook (synchronously).
  void attach(Sequential& model, double bucket_mb = 4.0);
  void on_layer_done(size_t layer);  // Sequential::set_backward_hook
  void finish();                     // between the backward and the optimizer
  int buckets_last_step() const { return nb_last_; }

 private:
  Env env_;
  Device dev_;
  std::unique_ptr<coll::Comm> comm_;
  std::unique_ptr<HostRing> ring_;
  Tensor scratch_;
  // bucket state: per top-level layer its gradient segments (GPU: the first arena element of its
  // parameters, SIZE_MAX = none), layers [next_, L) already reduced this step
  float* g_ = nullptr;
  size_t n_ = 0, reduced_lo_ = 0, bucket_elems_ = 0, next_ = 0;
  std::vector<size_t> lo_;
  std::vector<std::vector<std::pair<float*, size_t>>> segs_;
  std::vector<size_t> layer_elems_;
  std::vector<float> pack_;
  void* flow_ = nullptr;  // gpu::Flow
  void* ev_ = nullptr;    // gpu::Event
  int nb_ = 0, nb_last_ = 0;
  void reduce_layers(size_t lo_layer, size_t hi_layer);
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
  // a sender / receiver pair on one one-rank communicator (tests of send() / recv() themselves,
  // each on its own link flow): a send and its receive must be posted inside one
  // coll::group_start() / group_end() (a rank's send to itself is matched within its group)
  static std::pair<std::unique_ptr<P2PLink>, std::unique_ptr<P2PLink>> self_pair(int device);

 private:
  P2PLink() = default;
  void* flow_ = nullptr;   // gpu::Flow
  void* ready_ = nullptr;  // gpu::Event: the caller's flow reached the hand-off
  void* done_ = nullptr;   // gpu::Event: the last transfer on the link flow
  std::shared_ptr<coll::Comm> comm_;  // (shared by a self_pair)
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
