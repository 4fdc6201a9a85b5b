// Native pipeline stage of the C++ host API: the stage event loop that a pipeline coordinator
// (Python `parallel/pipeline/coordinator.py`, in-process or over TCP) drives by messages, with the
// stage's partition as a C++ `Sequential` on the CPU or the GPU backend.
//
// Reference parity: include/pipeline/pipeline_stage.hpp:29-308 (the event loop and its command
// handlers), include/pipeline/stage_config.hpp:8-35 / endpoint.hpp:17-94 (the JSON configuration),
// include/pipeline/network_stage_worker.hpp:25-114 + examples/network_worker.cpp:14-194 (the
// worker process: `dcnn_amd/bin/network_worker`).
//
// Wire compatibility with the Python stage (parallel/pipeline/stage.py): the same commands, the
// same StageConfig JSON, tensors as typed job payloads (fp32 NCHW on the CPU; bf16 channels-last
// on the GPU, flagged 0x10 like the Python transport), flat parameter state = parameters in
// checkpoint order then every BatchNorm's running mean / variance (fp32, logical NCHW order),
// SEND_PARAMS "full" / LOAD_PARAMS micro-batch 1 = that state plus the optimizer state in fp64.
#pragma once
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <thread>
#include <vector>

#include "json.hpp"
#include "nn.hpp"

namespace dcnn_native {
struct Message;
class Communicator;
}  // namespace dcnn_native

namespace dcnn {

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
  long n_fwd_ = 0, n_bwd_ = 0, n_upd_ = 0;
  double fwd_ms_ = 0, bwd_ms_ = 0;
  std::thread beat_;
  std::atomic<bool> beat_stop_{false};
};

}  // namespace dcnn
