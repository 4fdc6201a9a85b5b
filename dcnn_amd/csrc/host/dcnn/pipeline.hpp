// Native pipeline stage of the C++ host API: the stage event loop that a pipeline coordinator
// (Python `parallel/pipeline/coordinator.py`, in-process or over TCP) drives by messages, with the
// stage's partition as a C++ `Sequential` on the CPU or the GPU backend.
//
// Reference parity: include/pipeline/pipeline_stage.hpp:29-308 (the event loop and its command
// handlers), include/pipeline/stage_config.hpp:8-35 / endpoint.hpp:17-94 (the JSON configuration),
// include/pipeline/network_stage_worker.hpp:25-114 + examples/network_worker.cpp:14-194 (the
// worker process: `dcnn_amd/bin/network_worker`), include/pipeline/coordinator.hpp:30-599 +
// distributed_coordinator.hpp (the coordinator: `PipelineCoordinator`, driven by
// `dcnn_amd/bin/pipeline_coordinator`, examples/semi_async_pipeline_coordinator.cpp).
//
// Wire compatibility with the Python stage (parallel/pipeline/stage.py): the same commands, the
// same StageConfig JSON, tensors as typed job payloads (fp32 NCHW on the CPU; bf16 channels-last
// on the GPU, flagged 0x10 like the Python transport), flat parameter state = parameters in
// checkpoint order then every BatchNorm's running mean / variance (fp32, logical NCHW order),
// SEND_PARAMS "full" / LOAD_PARAMS micro-batch 1 = that state plus the optimizer state in fp64.
#pragma once
#include <atomic>
#include <chrono>
#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include <stdexcept>

#include "json.hpp"
#include "nn.hpp"
#include "train.hpp"

namespace dcnn_native {
struct Message;
class Communicator;
}  // namespace dcnn_native

namespace dcnn {
namespace dist {
class P2PLink;
}

struct Endpoint {
  std::string communication_type = "tcp";  // "tcp" | "in_process"
  json::Value parameters = json::Value::object();
  std::string host() const { return parameters.get_string("host", "127.0.0.1"); }
  int port() const { return (int)parameters.get_int("port", 0); }
  std::string id() const { return parameters.get_string("id", ""); }
};

struct StageConfig {
  std::string stage_id;
  int stage_index = 0, num_stages = 1;
  json::Value model_config, optimizer_config;
  std::optional<Endpoint> next_stage, prev_stage, coordinator;
  std::string device = "CPU", transport = "message", codec = "none";
  std::optional<int64_t> seed;
  bool first_layer_input_grad = false;
  double heartbeat_s = 0;
  static StageConfig parse(const std::string& text);
};

// a TCP control-plane endpoint listening on host:port (0: any free port) for a stage worker
// process; *bound_port receives the port actually bound
std::unique_ptr<dcnn_native::Communicator> make_tcp_communicator(const std::string& id, const std::string& host,
                                                                 int port, int* bound_port = nullptr);

// {"type": "sgd" | "adam" | "adamw", "parameters": {...}} (the Python OptimizerConfig)
std::unique_ptr<Optimizer> create_optimizer(const json::Value& cfg);

// flat state of a run of layers: every parameter in checkpoint order, then every BatchNorm's
// running mean / variance (depth-first through residual blocks), fp32 values in logical order
std::vector<double> pack_state(const std::vector<Layer*>& layers);
// LABELS_TRANSFER micro-batch id of the stage-loss configuration message
constexpr uint64_t kLossConfigMb = ~0ull;
void unpack_state(const std::vector<Layer*>& layers, const double* v, size_t n);

class PipelineStage {
 public:
  // `comm` must outlive the stage; a TcpCommunicator is dialled / aliased on CONFIG_TRANSFER
  explicit PipelineStage(dcnn_native::Communicator* comm, bool verbose = false);
  ~PipelineStage();
  // pop and handle messages until SHUTDOWN (or stop())
  void run(int poll_ms = 200);
  void stop() { running_ = false; }
  void process(dcnn_native::Message& m);
  const std::string& id() const { return id_; }
  Sequential* model() { return model_.get(); }

 private:
  void configure(const std::string& text);
  void connect_peers();
  void forward(dcnn_native::Message& m);
  void backward(dcnn_native::Message& m);
  void run_backward(uint64_t mb, Tensor g, const std::chrono::steady_clock::time_point& t0);
  void take_labels(dcnn_native::Message& m);
  Tensor labels_for(uint64_t mb);
  void reply(uint16_t cmd, const std::string& text = std::string());
  void send_tensor(const std::string& to, uint16_t cmd, uint64_t mb, const Tensor& t, bool as_logits);
  Tensor decode(dcnn_native::Message& m) const;
  std::vector<double> flat_state();
  void load_flat_state(const double* v, size_t n);
  std::vector<double> optimizer_state();
  void load_optimizer_state(const double* v, size_t n);
  std::string status_json();
  void start_heartbeat();
  void stop_heartbeat();

  dcnn_native::Communicator* comm_;
  bool verbose_;
  std::string id_;
  std::atomic<bool> running_{false};
  StageConfig cfg_;
  std::unique_ptr<Sequential> model_;
  std::unique_ptr<Optimizer> opt_;
  Device dev_ = Device::cpu();
  // per micro-batch: the forward output's dtype / layout / logical shape (the incoming gradient
  // is converted to it)
  struct OutKind {
    DType dt = DType::F32;
    Layout layout = Layout::NCHW;
    std::vector<int64_t> shape;
  };
  std::map<uint64_t, OutKind> out_kind_;
  // GPU stages: one hipGraph per (phase, micro-batch), captured from the second step on (the
  // first step runs eagerly, so every workspace already has its final size) and replayed after
  // that: a micro-batch's forward / backward on this stage is one graph launch instead of hundreds
  // of eager kernel launches. A micro-batch's backward graph reads the activations its forward
  // graph leaves in that graph's buffers, so both phases of a micro-batch run captured or both
  // eagerly; an eager forward (first step, DCNN_STAGE_GRAPHS=0, or a new input shape / train-eval
  // mode) drops that micro-batch's graphs, and the next step captures them again.
  struct MbGraph {
    std::unique_ptr<gpu::Graph> g;
    Tensor in, out;  // the graph's static input buffer and output
    std::vector<int64_t> shape;
    DType dt = DType::F32;
    Layout layout = Layout::NCHW;
    bool training = true;
  };
  // the loss on this (last) stage's device (LABELS_TRANSFER; native coordinator): every forward
  // output's loss + gradient (scaled by grad_scale_) right here, the backward starts at once and
  // only the loss value goes to the coordinator — no logits / gradient round trip over the host
  std::unique_ptr<Loss> stage_loss_;
  float grad_scale_ = 1.f;
  std::map<uint64_t, Tensor> labels_;  // device int64 labels per micro-batch (until its forward)
  std::map<uint64_t, MbGraph> fwd_graph_, bwd_graph_;
  std::map<uint64_t, bool> fwd_graphed_;  // the micro-batch's last forward ran its graph
  bool graphs_ = false;
  Tensor run_graph(std::map<uint64_t, MbGraph>& tab, uint64_t mb, const Tensor& in, bool training,
                   const std::function<Tensor(const Tensor&)>& body);
  void drop_graphs(uint64_t mb);
  void drop_all_graphs();
  // transport "ipc" (same node, GPU stages): stage-to-stage tensors stay on the device. The sender
  // copies into its exported buffer for (peer, micro-batch) and sends only the 64-byte handle; the
  // receiver maps the buffer once and copies out on arrival. A (peer, micro-batch) buffer is
  // rewritten only in a later step / batch, after the receiver has consumed it (the coordinator
  // joins every micro-batch before the next one starts).
  // The hand-off (DCNN_IPC_HANDOFF): "host" (default) — the sender's host waits for its copy
  // before the message goes out, the receiver's host for its copy out; "event" — an interprocess
  // event the sender records after its copy, the receiver's flow waits on it; "flag" — each buffer
  // starts with a 32-bit flag the sender's flow sets to the hand-off's sequence number after its
  // copy (stream write-value), the receiver's flow waits for it (stream wait-value). In the device-
  // ordered modes a receiver's copies are complete before it answers UPDATE_PARAMETERS; within a
  // step every later hand-off on its flow follows them. (Measured: profiles/pipeline_ipc_handoff_r6.md.)
  struct IpcSlot {
    void* ptr = nullptr;  // flag header (kIpcHeader bytes), then the tensor bytes
    size_t bytes = 0;     // tensor capacity
    std::string handle;
    uint32_t seq = 0;     // "flag": the last hand-off's sequence number
    void* ev = nullptr;   // "event": gpu::Event (interprocess), recorded after each copy
    std::string ev_handle;
  };
  std::map<std::pair<std::string, uint64_t>, IpcSlot> ipc_out_;
  std::vector<void*> ipc_retired_;                  // outgrown exports (a peer may still map them)
  mutable std::map<std::string, void*> ipc_in_;     // handle -> this process's mapping
  mutable std::map<std::string, void*> ipc_ev_in_;  // event handle -> this process's event
  mutable bool ipc_device_ordered_ = false;         // a device-ordered receive since the last update
  void release_ipc();
  // transport "rccl" (GPU stages on distinct devices, any node): stage-to-stage tensors as RCCL
  // sends on per-direction two-rank links (dist::P2PLink); the job message carries only the shape.
  // Opened on the coordinator's P2P_CONNECT (after every stage is configured): a stage sends its
  // next stage the pair's two unique ids, joins its previous stage's links, then its next stage's.
  std::unique_ptr<dist::P2PLink> act_out_, act_in_, grad_out_, grad_in_;
  std::string prev_ids_;  // the previous stage's ids, when they arrive before the coordinator's request
  void connect_links(dcnn_native::Message& m);
  void release_links();
  long n_fwd_ = 0, n_bwd_ = 0, n_upd_ = 0;
  double fwd_ms_ = 0, bwd_ms_ = 0;
  std::thread beat_;
  std::atomic<bool> beat_stop_{false};
};

// The RCCL transport's tensor hand-off (PipelineStage's sends / receives on transport "rccl",
// exposed for the GPU test that drives it through a one-rank link pair, dist::P2PLink::self_pair):
// send_rccl fills m's typed-job header (shape / dtype code with the RCCL flag; no payload bytes)
// and sends t's bytes on l; recv_rccl reads that header and receives the bytes from l into a fresh
// tensor on dev (the current flow waits for it).
namespace wire {
void send_rccl(dist::P2PLink& l, const Tensor& t, uint64_t mb, bool as_logits, dcnn_native::Message& m);
Tensor recv_rccl(dist::P2PLink& l, const dcnn_native::Message& m, Device dev);
}  // namespace wire

// ---------------------------------------------------------------- coordinator
class PipelineError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// a stage stopped answering: missed heartbeats or a lost control-plane connection
class StageFailure : public PipelineError {
 public:
  StageFailure(const std::string& stage, const std::string& why) : PipelineError(stage + ": " + why), stage(stage) {}
  std::string stage;
};

struct Partition {
  int start = 0, end = 0;  // top-level layers [start, end)
  bool operator==(const Partition& o) const { return start == o.start && end == o.end; }
};
// equal layer counts, the first L % S stages one layer more (reference naive_partitioner.hpp:13-32)
std::vector<Partition> naive_partitions(int num_layers, int num_stages);
// contiguous split minimising the largest per-stage cost (exact DP; the Python CostPartitioner)
std::vector<Partition> balanced_partitions(const std::vector<double>& costs, int num_stages);

enum class Schedule { Sync, SemiAsync, OneFOneB };
// "sync" | "gpipe", "semi_async" | "async", "1f1b" | "one_f_one_b"
Schedule parse_schedule(const std::string& s);

struct CoordinatorOptions {
  int num_microbatches = 1;
  std::vector<std::string> stage_devices;  // per stage ("CPU", "GPU:0", ...); default CPU
  std::string loss = "softmax_crossentropy";
  std::string codec = "none";               // inline payload compression of the stages' sends
  // "ipc": GPU stage-to-stage tensors via device IPC buffers (one node); "rccl": as RCCL sends over
  // per-direction stage-pair links (native GPU stages on distinct devices)
  std::string transport = "message";
  bool grad_scale_mean = true;              // micro-batch gradients * 1 / num_microbatches
  double timeout_s = 120.0;
  double heartbeat_s = 0.0;                 // > 0: stages beat every heartbeat_s ...
  int heartbeat_misses = 3;                 // ... and are declared failed after this many misses
  std::optional<int64_t> seed;              // stage i initialises with seed + i
  // the loss on the last stage's device (LABELS_TRANSFER): -1 when the last stage is a native GPU
  // stage, 0 never (logits to this coordinator, the loss on its CPU), 1 whenever it is native
  int stage_loss = -1;
  std::string host = "127.0.0.1";           // the address stages reach the coordinator at
  int port = 0;                             // 0: any free port
};

struct StepResult {
  double loss = 0;  // mean of the micro-batch mean losses
  long correct = 0;
  long samples = 0;
};

// Coordinator of separate stage processes (native `network_worker`s or Python workers: the same
// commands, StageConfig JSON and payloads) over the TCP control plane. The loss runs on the last
// stage's GPU when that stage is native (CoordinatorOptions::stage_loss), else here on the CPU;
// activations and gradients travel inline in the job messages or as device IPC references.
class PipelineCoordinator {
 public:
  PipelineCoordinator(json::Value model_config, json::Value optimizer_config, std::vector<Endpoint> stages,
                      CoordinatorOptions opts = {});
  ~PipelineCoordinator();
  // partition (default: naive over the top-level layers), dial every stage, build the configs
  void initialize(std::vector<Partition> parts = {});
  void deploy_stages();  // CONFIG_TRANSFER back to front, join CONFIG_RECEIVED
  void start();          // TRAIN_MODE
  void stop();           // SHUTDOWN + close
  void train_mode();
  void eval_mode();

  // one optimisation step over x (fp32 NCHW host) / labels (int64 host): split into micro-batches,
  // run the schedule, UPDATE_PARAMETERS
  StepResult train_step(const Tensor& x, const Tensor& labels, Schedule s = Schedule::SemiAsync);
  StepResult evaluate_batch(const Tensor& x, const Tensor& labels);  // forward only
  void update_parameters();

  // LOAD_PARAMS: each stage's slice of a full model (same architecture) / flat states as given
  void send_parameters(Sequential& model);
  void load_parameters(const std::vector<std::vector<double>>& flats, bool full);
  // SEND_PARAMS: per stage, pack_state (full: [n, state, optimizer state])
  std::vector<std::vector<double>> collect_parameters(bool full = false);
  // the trained weights / statistics into `model` (the full architecture)
  void gather_into(Sequential& model);

  float learning_rate() const { return lr_.learning_rate(); }
  void set_learning_rate(float lr) { lr_.set_learning_rate(lr); }
  // an Optimizer whose learning rate the next UPDATE_PARAMETERS broadcasts: give it to a Scheduler
  Optimizer& lr_control() { return lr_; }

  std::vector<json::Value> status();
  std::vector<std::string> print_profiling();
  void clear_profiling();
  void barrier();
  std::map<std::string, bool> health_check(double timeout_s = 10.0);
  // re-partition from the stages' measured per-layer times (when they report them) and redeploy,
  // carrying the trained weights over; returns the partitions in effect
  std::vector<Partition> balance_load();

  int num_stages() const { return (int)stages_.size(); }
  const std::vector<Partition>& partitions() const { return parts_; }
  const std::vector<std::string>& stage_names() const { return names_; }
  int port() const { return port_; }
  long steps() const { return steps_; }

 private:
  class LrControl : public Optimizer {
   public:
    using Optimizer::Optimizer;
    void step(const std::vector<Param*>&) override {}
  };
  struct Pending;
  json::Value stage_config(int i) const;
  json::Value part_config(const Partition& p) const;
  void broadcast(uint16_t cmd, const std::string& text = std::string());
  std::vector<dcnn_native::Message> join(uint16_t cmd, size_t n, double timeout_s = 0);
  bool recv_any(const std::vector<uint16_t>& cmds, dcnn_native::Message& out, int timeout_ms);
  void check_errors();
  bool take_beat(const dcnn_native::Message& m);
  void send_job(const std::string& to, uint16_t cmd, uint64_t mb, const float* data, const std::vector<int64_t>& shape);
  void forward_mb(const Pending& p);
  void loss_and_backward(dcnn_native::Message& out, Pending& p, StepResult& r);
  void take_output(dcnn_native::Message& out, Pending& p, StepResult& r);
  void enable_stage_loss();
  void send_f64(const std::string& to, uint16_t cmd, uint64_t mb, const std::vector<double>& v);
  StepResult run_sync(std::vector<Pending>& mbs);
  StepResult run_semi_async(std::vector<Pending>& mbs);
  StepResult run_1f1b(std::vector<Pending>& mbs);
  std::vector<Pending> split(const Tensor& x, const Tensor& labels) const;

  json::Value model_cfg_, opt_cfg_;
  std::vector<Endpoint> stages_;
  CoordinatorOptions o_;
  Loss loss_;
  std::unique_ptr<dcnn_native::Communicator> comm_;
  int port_ = 0;
  std::vector<std::string> names_;
  std::vector<Partition> parts_;
  LrControl lr_;
  float sent_lr_;
  bool deployed_ = false;
  bool stage_loss_on_ = false;  // the last stage computes the loss (enable_stage_loss)
  long steps_ = 0;
  std::map<std::string, std::chrono::steady_clock::time_point> last_beat_;
  struct Stash;  // messages taken off the queue while waiting for another kind
  std::unique_ptr<Stash> stash_;
};

}  // namespace dcnn
