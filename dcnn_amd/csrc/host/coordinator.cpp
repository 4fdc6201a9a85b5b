// Native pipeline coordinator (dcnn/pipeline.hpp): partitions, deployment, the three schedules,
// parameter traffic and monitoring over the TCP control plane (csrc/native/comm.cpp).
//
// Schedules (the Python coordinator's, parallel/pipeline/coordinator.py):
//   sync       — GPipe: every forward, then every loss + backward;
//   semi_async — every forward at once, each output's loss + backward the moment it arrives
//                (reference include/pipeline/coordinator.hpp:273-326);
//   1f1b       — at most num_stages micro-batches between their forward and the end of their
//                backward; a new forward is admitted each time a backward completes.
// Reference parity: include/pipeline/coordinator.hpp:30-599, distributed_coordinator.hpp,
// include/partitioner/naive_partitioner.hpp:13-32.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>
#include <limits>
#include <thread>

#include "../native/comm.h"
#include "dcnn/pipeline.hpp"

using namespace dcnn_native;

namespace dcnn {

namespace {
using Clock = std::chrono::steady_clock;

double seconds_since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

json::Value endpoint_json(const std::string& host, int port, const std::string& id) {
  json::Value p = json::Value::object();
  p["host"] = host;
  p["port"] = port;
  p["id"] = id;
  json::Value e = json::Value::object();
  e["communication_type"] = "tcp";
  e["parameters"] = std::move(p);
  return e;
}

// a typed job payload (fp32 / bf16 / fp64, optionally compressed) as fp64 values
std::vector<double> payload_values(Message& m) {
  if (m.codec) {
    m.data = decompress(m.data, (Codec)m.codec, 0);
    m.codec = CODEC_NONE;
  }
  const int code = m.payload_type == P_TYPED_JOB ? (m.dtype & 0x0F) : 0;
  std::vector<double> v;
  if (code == 0) {
    v.resize(m.data.size() / 4);
    const float* f = reinterpret_cast<const float*>(m.data.data());
    for (size_t i = 0; i < v.size(); ++i) v[i] = f[i];
  } else if (code == 1) {
    v.resize(m.data.size() / 2);
    const uint16_t* b = reinterpret_cast<const uint16_t*>(m.data.data());
    for (size_t i = 0; i < v.size(); ++i) v[i] = bf16_to_f32(b[i]);
  } else if (code == 5) {
    v.resize(m.data.size() / 8);
    std::memcpy(v.data(), m.data.data(), v.size() * 8);
  } else {
    throw PipelineError("unsupported payload dtype " + std::to_string(code));
  }
  return v;
}
}  // namespace

std::vector<Partition> naive_partitions(int L, int S) {
  if (S <= 0 || S > L)
    throw std::invalid_argument("cannot split " + std::to_string(L) + " layers into " + std::to_string(S) + " stages");
  std::vector<Partition> out;
  const int base = L / S, rem = L % S;
  for (int i = 0, s = 0; i < S; ++i) {
    const int n = base + (i < rem ? 1 : 0);
    out.push_back({s, s + n});
    s += n;
  }
  return out;
}

std::vector<Partition> balanced_partitions(const std::vector<double>& costs, int S) {
  const int L = (int)costs.size();
  if (S <= 0 || S > L)
    throw std::invalid_argument("cannot split " + std::to_string(L) + " layers into " + std::to_string(S) + " stages");
  std::vector<double> pre(L + 1, 0.0);
  for (int i = 0; i < L; ++i) pre[i + 1] = pre[i] + costs[i];
  const double inf = std::numeric_limits<double>::infinity();
  // best[s][i]: the smallest largest-stage cost of the first i layers in s stages
  std::vector<std::vector<double>> best(S + 1, std::vector<double>(L + 1, inf));
  std::vector<std::vector<int>> cut(S + 1, std::vector<int>(L + 1, 0));
  best[0][0] = 0;
  for (int s = 1; s <= S; ++s)
    for (int i = s; i <= L - (S - s); ++i)
      for (int j = s - 1; j < i; ++j) {
        const double v = std::max(best[s - 1][j], pre[i] - pre[j]);
        if (v < best[s][i]) {
          best[s][i] = v;
          cut[s][i] = j;
        }
      }
  std::vector<Partition> out(S);
  for (int s = S, i = L; s > 0; --s) {
    out[s - 1] = {cut[s][i], i};
    i = cut[s][i];
  }
  return out;
}

Schedule parse_schedule(const std::string& s) {
  if (s == "sync" || s == "gpipe") return Schedule::Sync;
  if (s == "semi_async" || s == "async") return Schedule::SemiAsync;
  if (s == "1f1b" || s == "one_f_one_b") return Schedule::OneFOneB;
  throw std::invalid_argument("unknown pipeline schedule '" + s + "' (sync, semi_async, 1f1b)");
}

struct PipelineCoordinator::Stash {
  std::map<uint16_t, std::deque<Message>> q;
};

struct PipelineCoordinator::Pending {
  uint64_t mb = 0;
  const float* x = nullptr;  // the micro-batch's rows of the step's input (alive for the step)
  std::shared_ptr<std::vector<float>> hold;  // (a converted copy when the input is not host fp32)
  std::vector<int64_t> shape;
  std::vector<int64_t> y;
};

PipelineCoordinator::PipelineCoordinator(json::Value model_config, json::Value optimizer_config,
                                         std::vector<Endpoint> stages, CoordinatorOptions opts)
    : model_cfg_(std::move(model_config)),
      opt_cfg_(std::move(optimizer_config)),
      stages_(std::move(stages)),
      o_(std::move(opts)),
      loss_(LossFactory::create(o_.loss)),
      lr_(0.f),
      stash_(std::make_unique<Stash>()) {
  const json::Value* p = opt_cfg_.find("parameters");
  lr_.set_learning_rate(p != nullptr ? (float)p->get_number("learning_rate", 1e-3) : 1e-3f);
  sent_lr_ = lr_.learning_rate();
  if (stages_.empty()) throw std::invalid_argument("PipelineCoordinator: no stage endpoints");
  if (o_.num_microbatches <= 0) throw std::invalid_argument("PipelineCoordinator: num_microbatches must be > 0");
  if (o_.stage_devices.empty()) o_.stage_devices.assign(stages_.size(), "CPU");
  if (o_.stage_devices.size() != stages_.size()) throw std::invalid_argument("one device per stage required");
  if (o_.transport == "rccl")  // (RCCL refuses two ranks of one communicator on one device)
    for (size_t i = 0; i + 1 < stages_.size(); ++i)
      if (o_.stage_devices[i].rfind("GPU", 0) != 0 || o_.stage_devices[i] == o_.stage_devices[i + 1])
        throw std::invalid_argument("transport 'rccl': adjacent stages need distinct GPUs (" + o_.stage_devices[i] +
                                    ", " + o_.stage_devices[i + 1] + ")");
}

PipelineCoordinator::~PipelineCoordinator() {
  try {
    stop();
  } catch (...) {
  }
}

json::Value PipelineCoordinator::part_config(const Partition& p) const {
  const auto& layers = model_cfg_.at("layers").items();
  if (!(0 <= p.start && p.start < p.end && p.end <= (int)layers.size()))
    throw std::out_of_range("partition indices out of range");
  json::Value c = json::Value::object();
  c["name"] = model_cfg_.get_string("name", "sequential") + "_part_" + std::to_string(p.start) + "_" +
              std::to_string(p.end);
  c["is_training"] = true;
  json::Value ls = json::Value::array();
  for (int i = p.start; i < p.end; ++i) ls.push(layers[i]);
  c["layers"] = std::move(ls);
  if (p.start == 0)
    if (const json::Value* in = model_cfg_.find("input_shape")) c["input_shape"] = *in;
  return c;
}

json::Value PipelineCoordinator::stage_config(int i) const {
  const int S = num_stages();
  json::Value c = json::Value::object();
  c["stage_id"] = names_[i];
  c["stage_index"] = i;
  c["num_stages"] = S;
  c["model_config"] = part_config(parts_[i]);
  json::Value oc = opt_cfg_;
  oc["parameters"]["learning_rate"] = (double)lr_.learning_rate();
  c["optimizer_config"] = std::move(oc);
  c["next_stage_endpoint"] =
      i + 1 < S ? endpoint_json(stages_[i + 1].host(), stages_[i + 1].port(), names_[i + 1]) : json::Value();
  c["prev_stage_endpoint"] = i > 0 ? endpoint_json(stages_[i - 1].host(), stages_[i - 1].port(), names_[i - 1]) : json::Value();
  c["coordinator_endpoint"] = endpoint_json(o_.host, port_, "coordinator");
  c["device"] = o_.stage_devices[i];
  c["transport"] = o_.transport;
  c["codec"] = o_.codec;
  c["compute_dtype"] = "auto";
  c["seed"] = o_.seed ? json::Value(*o_.seed + i) : json::Value();
  c["first_layer_input_grad"] = false;
  c["ranks"] = json::Value();
  c["profiling"] = true;
  c["use_graph"] = o_.stage_devices[i].rfind("GPU", 0) == 0;
  c["heartbeat_s"] = o_.heartbeat_s;
  c["fault"] = json::Value();
  return c;
}

void PipelineCoordinator::initialize(std::vector<Partition> parts) {
  const int L = (int)model_cfg_.at("layers").items().size();
  parts_ = parts.empty() ? naive_partitions(L, num_stages()) : std::move(parts);
  if ((int)parts_.size() != num_stages()) throw std::invalid_argument("one partition per stage required");
  names_.clear();
  for (int i = 0; i < num_stages(); ++i) names_.push_back("stage_" + std::to_string(i));
  comm_ = make_tcp_communicator("coordinator", "0.0.0.0", o_.port, &port_);
  auto* tcp = dynamic_cast<TcpCommunicator*>(comm_.get());
  for (int i = 0; i < num_stages(); ++i) tcp->connect(names_[i], stages_[i].host(), stages_[i].port(), 60000);
}

void PipelineCoordinator::deploy_stages() {
  if (!comm_) initialize();
  // back to front, so every stage's next stage is listening with its configuration
  for (int i = num_stages() - 1; i >= 0; --i) {
    Message m;
    m.recipient = names_[i];
    m.command = CONFIG_TRANSFER;
    m.payload_type = P_STRING;
    m.text = stage_config(i).dump(-1);
    comm_->send(std::move(m));
    join(CONFIG_RECEIVED, 1);
  }
  deployed_ = true;
  const auto now = Clock::now();
  for (const auto& s : names_) last_beat_[s] = now;
  sent_lr_ = lr_.learning_rate();
  enable_stage_loss();
  if (o_.transport == "rccl" && num_stages() > 1) {
    // every stage is configured: open the stage-pair RCCL links (the stages chain their joins)
    broadcast(P2P_CONNECT);
    join(P2P_CONNECT, (size_t)num_stages());
  }
}

void PipelineCoordinator::send_f64(const std::string& to, uint16_t cmd, uint64_t mb, const std::vector<double>& v) {
  Message m;
  m.recipient = to;
  m.command = cmd;
  m.payload_type = P_TYPED_JOB;
  m.mb_id = mb;
  m.dtype = 5;  // f64
  m.shape = {(uint64_t)v.size()};
  m.data.assign(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(double));
  comm_->send(std::move(m));
}

void PipelineCoordinator::enable_stage_loss() {
  stage_loss_on_ = false;
  if (o_.stage_loss == 0 || names_.empty()) return;
  bool native = false, gpu = false;
  for (const json::Value& st : status())
    if (st.get_string("id", "") == names_.back()) {
      native = st.get_bool("native", false);
      gpu = st.get_string("device", "").rfind("GPU", 0) == 0;
    }
  if (o_.stage_loss == 1 && !native) throw PipelineError("stage loss: the last stage is not a native stage");
  if (!native || (o_.stage_loss < 0 && !gpu)) return;
  const int M = o_.num_microbatches;
  const double scale = o_.grad_scale_mean && M > 1 ? 1.0 / M : 1.0;
  send_f64(names_.back(), LABELS_TRANSFER, kLossConfigMb, {(double)loss_.kind(), (double)loss_.param(), scale});
  join(LABELS_TRANSFER, 1);
  stage_loss_on_ = true;
}

void PipelineCoordinator::broadcast(uint16_t cmd, const std::string& text) {
  for (const auto& s : names_) {
    Message m;
    m.recipient = s;
    m.command = cmd;
    if (!text.empty()) {
      m.payload_type = P_STRING;
      m.text = text;
    }
    comm_->send(std::move(m));
  }
}

void PipelineCoordinator::start() { broadcast(TRAIN_MODE); }
void PipelineCoordinator::train_mode() { broadcast(TRAIN_MODE); }
void PipelineCoordinator::eval_mode() { broadcast(EVAL_MODE); }

void PipelineCoordinator::stop() {
  if (!comm_) return;
  try {
    broadcast(SHUTDOWN);
  } catch (...) {
  }
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  comm_->close();
  comm_.reset();
  deployed_ = false;
}

bool PipelineCoordinator::take_beat(const Message& m) {
  if (m.command != HEALTH_CHECK || m.payload_type != P_STRING || m.text != "heartbeat") return false;
  const auto slash = m.sender.find('/');
  last_beat_[slash == std::string::npos ? m.sender : m.sender.substr(slash + 1)] = Clock::now();
  return true;
}

void PipelineCoordinator::check_errors() {
  MessageQueue& q = comm_->queue();
  for (uint16_t kind : {(uint16_t)ERROR_REPORT, (uint16_t)JOB_FAILURE}) {
    Message m;
    if (q.count(kind) && q.pop_command(kind, m, 0)) throw PipelineError(m.text.empty() ? "stage error" : m.text);
  }
  if (!deployed_) return;
  if (o_.heartbeat_s > 0) {
    Message m;
    while (q.count(HEALTH_CHECK) && q.pop_command(HEALTH_CHECK, m, 0))
      if (!take_beat(m)) stash_->q[HEALTH_CHECK].push_back(std::move(m));
    const double limit = o_.heartbeat_s * o_.heartbeat_misses;
    for (const auto& s : names_) {
      const double quiet = seconds_since(last_beat_[s]);
      if (quiet > limit)
        throw StageFailure(s, "no heartbeat for " + std::to_string(quiet) + " s (interval " +
                                  std::to_string(o_.heartbeat_s) + " s)");
    }
  }
  const std::vector<std::string> alive = comm_->peers();
  for (const auto& s : names_)
    if (std::find(alive.begin(), alive.end(), s) == alive.end()) throw StageFailure(s, "control-plane connection lost");
}

std::vector<Message> PipelineCoordinator::join(uint16_t cmd, size_t n, double timeout_s) {
  const auto t0 = Clock::now();
  const double limit = timeout_s > 0 ? timeout_s : o_.timeout_s;
  std::vector<Message> out;
  auto& st = stash_->q[cmd];
  while (!st.empty() && out.size() < n) {
    out.push_back(std::move(st.front()));
    st.pop_front();
  }
  while (out.size() < n) {
    check_errors();
    Message m;
    if (comm_->queue().pop_command(cmd, m, 50)) {
      if (!take_beat(m)) out.push_back(std::move(m));
    } else if (seconds_since(t0) > limit) {
      throw PipelineError("timeout waiting for " + std::to_string(n) + " x " + command_name(cmd) + " (got " +
                          std::to_string(out.size()) + ")");
    }
  }
  return out;
}

bool PipelineCoordinator::recv_any(const std::vector<uint16_t>& cmds, Message& out, int timeout_ms) {
  for (uint16_t c : cmds) {
    auto& st = stash_->q[c];
    if (!st.empty()) {
      out = std::move(st.front());
      st.pop_front();
      return true;
    }
  }
  return comm_->queue().pop_any(cmds, out, timeout_ms);
}

void PipelineCoordinator::send_job(const std::string& to, uint16_t cmd, uint64_t mb, const float* data,
                                   const std::vector<int64_t>& shape) {
  Message m;
  m.recipient = to;
  m.command = cmd;
  m.payload_type = P_TYPED_JOB;
  m.mb_id = mb;
  m.dtype = 0;
  size_t n = 1;
  for (auto d : shape) {
    m.shape.push_back((uint64_t)d);
    n *= (size_t)d;
  }
  m.data.assign(reinterpret_cast<const char*>(data), n * sizeof(float));
  comm_->send(std::move(m));
}

std::vector<PipelineCoordinator::Pending> PipelineCoordinator::split(const Tensor& x_in, const Tensor& labels) const {
  if (x_in.rank() < 2) throw std::invalid_argument("train_step: x must be (N, ...)");
  // host fp32 input: the micro-batches point into it (the caller keeps x alive for the step);
  // anything else is converted once
  std::shared_ptr<std::vector<float>> hold;
  const float* x = nullptr;
  if (!x_in.device().is_gpu() && x_in.dtype() == DType::F32 && x_in.layout() == Layout::NCHW) {
    x = x_in.ptr<float>();
  } else {
    hold = std::make_shared<std::vector<float>>(x_in.to_host_f32());
    x = hold->data();
  }
  const std::vector<int64_t> y = labels.to_host_i64();
  const int64_t N = x_in.dim(0), per = x_in.numel() / N;
  if ((int64_t)y.size() != N) throw std::invalid_argument("train_step: one label per sample required");
  const int M = o_.num_microbatches;
  if (N < M) throw std::invalid_argument("train_step: fewer samples than micro-batches");
  // the last micro-batch takes the remainder (the reference's split)
  std::vector<Pending> out(M);
  const int64_t base = N / M;
  for (int i = 0, s = 0; i < M; ++i) {
    const int64_t e = i == M - 1 ? N : s + base;
    Pending& p = out[i];
    p.mb = (uint64_t)i;
    p.x = x + s * per;
    p.hold = hold;
    p.shape = x_in.shape();
    p.shape[0] = e - s;
    p.y.assign(y.begin() + s, y.begin() + e);
    s = (int)e;
  }
  return out;
}

void PipelineCoordinator::forward_mb(const Pending& p) {
  // (the labels first: the last stage needs them when the micro-batch's activations arrive)
  if (stage_loss_on_) send_f64(names_.back(), LABELS_TRANSFER, p.mb, std::vector<double>(p.y.begin(), p.y.end()));
  send_job(names_.front(), FORWARD_JOB, p.mb, p.x, p.shape);
}

// (a P_STRING payload carries no micro-batch id field: the last stage's loss report names it)
static Message& with_mb(Message& m) {
  if (m.payload_type == P_STRING) m.mb_id = (uint64_t)json::Value::parse(m.text).get_int("mb", 0);
  return m;
}

// a micro-batch's output: the last stage's loss report (its backward already started there), or
// its logits (the loss here, the gradient back to the last stage)
void PipelineCoordinator::take_output(Message& out, Pending& p, StepResult& r) {
  if (out.payload_type == P_STRING) {
    const json::Value v = json::Value::parse(out.text);
    r.loss += v.get_number("loss", 0.0);
    r.correct += (long)v.get_int("correct", 0);
    r.samples += v.get_int("samples", 0);
    return;
  }
  loss_and_backward(out, p, r);
}

void PipelineCoordinator::loss_and_backward(Message& out, Pending& p, StepResult& r) {
  const std::vector<double> v = payload_values(out);
  const int64_t N = (int64_t)p.y.size();
  if (N == 0 || v.size() % (size_t)N) throw PipelineError("pipeline output does not match the micro-batch");
  const int64_t C = (int64_t)v.size() / N;
  const Tensor pred = Tensor::from_host(std::vector<float>(v.begin(), v.end()), {N, C}, Device::cpu());
  const Tensor lab = Tensor::from_host_i64(p.y, Device::cpu());
  LossResult lr = loss_.compute(pred, &lab);
  // the accumulated gradient is the full-batch mean with the 1 / num_microbatches scale
  const int M = o_.num_microbatches;
  if (o_.grad_scale_mean && M > 1) {
    float* g = lr.grad.ptr<float>();
    for (int64_t i = 0; i < N * C; ++i) g[i] *= 1.f / (float)M;
  }
  send_job(names_.back(), BACKWARD_JOB, p.mb, lr.grad.ptr<float>(), {N, C});
  r.loss += lr.loss;
  r.correct += lr.correct;
  r.samples += N;
}

StepResult PipelineCoordinator::run_sync(std::vector<Pending>& mbs) {
  StepResult r;
  for (auto& p : mbs) forward_mb(p);
  std::map<uint64_t, Message> outs;
  for (auto& m : join(FORWARD_JOB, mbs.size())) outs[with_mb(m).mb_id] = std::move(m);
  for (auto& p : mbs) take_output(outs.at(p.mb), p, r);
  join(BACKWARD_JOB, mbs.size());
  return r;
}

StepResult PipelineCoordinator::run_semi_async(std::vector<Pending>& mbs) {
  StepResult r;
  for (auto& p : mbs) forward_mb(p);
  const auto t0 = Clock::now();
  for (size_t done = 0; done < mbs.size();) {
    check_errors();
    Message m;
    if (!recv_any({FORWARD_JOB}, m, 50)) {
      if (seconds_since(t0) > o_.timeout_s) throw PipelineError("timeout waiting for pipeline outputs");
      continue;
    }
    take_output(m, mbs.at(with_mb(m).mb_id), r);
    ++done;
  }
  join(BACKWARD_JOB, mbs.size());
  return r;
}

StepResult PipelineCoordinator::run_1f1b(std::vector<Pending>& mbs) {
  StepResult r;
  const size_t m = mbs.size(), cap = (size_t)std::max(1, num_stages());
  size_t sent = 0, done = 0, outs = 0;
  while (sent < std::min(m, cap)) forward_mb(mbs[sent++]);
  const auto t0 = Clock::now();
  // every output AND every backward: with the loss on the last stage, that stage starts a
  // micro-batch's backward before it reports the loss, so on a transport that does not block its
  // host (device-ordered IPC, RCCL) the first stage's backward can finish first
  while (done < m || outs < m) {
    check_errors();
    Message msg;
    // either completion: an output (loss, then its backward) or a finished backward (admit the
    // next forward)
    if (!recv_any({FORWARD_JOB, BACKWARD_JOB}, msg, 20)) {
      if (seconds_since(t0) > o_.timeout_s)
        throw PipelineError("1F1B: timeout (" + std::to_string(done) + "/" + std::to_string(m) + " backwards, " +
                            std::to_string(outs) + "/" + std::to_string(m) + " outputs)");
      continue;
    }
    if (msg.command == FORWARD_JOB) {
      take_output(msg, mbs.at(with_mb(msg).mb_id), r);
      ++outs;
    } else {
      ++done;
      if (sent < m) forward_mb(mbs[sent++]);
    }
  }
  return r;
}

StepResult PipelineCoordinator::train_step(const Tensor& x, const Tensor& labels, Schedule s) {
  if (!deployed_) throw PipelineError("train_step before deploy_stages()");
  std::vector<Pending> mbs = split(x, labels);
  StepResult r = s == Schedule::Sync ? run_sync(mbs) : s == Schedule::SemiAsync ? run_semi_async(mbs) : run_1f1b(mbs);
  update_parameters();
  ++steps_;
  r.loss /= (double)mbs.size();
  return r;
}

StepResult PipelineCoordinator::evaluate_batch(const Tensor& x, const Tensor& labels) {
  std::vector<Pending> mbs = split(x, labels);
  for (auto& p : mbs) forward_mb(p);
  StepResult r;
  for (auto& m : join(FORWARD_JOB, mbs.size())) {
    Pending& p = mbs.at(with_mb(m).mb_id);
    if (m.payload_type == P_STRING) {  // (the last stage's loss; no backward in eval mode)
      take_output(m, p, r);
      continue;
    }
    const std::vector<double> v = payload_values(m);
    const int64_t N = (int64_t)p.y.size(), C = (int64_t)v.size() / N;
    const Tensor pred = Tensor::from_host(std::vector<float>(v.begin(), v.end()), {N, C}, Device::cpu());
    const Tensor lab = Tensor::from_host_i64(p.y, Device::cpu());
    const LossResult lr = loss_.compute(pred, &lab);
    r.loss += lr.loss;
    r.correct += lr.correct;
    r.samples += N;
  }
  r.loss /= (double)mbs.size();
  return r;
}

void PipelineCoordinator::update_parameters() {
  std::string text;
  if (lr_.learning_rate() != sent_lr_) {
    json::Value hp = json::Value::object();
    hp["learning_rate"] = (double)lr_.learning_rate();
    text = hp.dump(-1);
    sent_lr_ = lr_.learning_rate();
  }
  broadcast(UPDATE_PARAMETERS, text);
  join(PARAMETERS_UPDATED, names_.size());
}

void PipelineCoordinator::load_parameters(const std::vector<std::vector<double>>& flats, bool full) {
  if ((int)flats.size() != num_stages()) throw std::invalid_argument("one flat state per stage required");
  for (int i = 0; i < num_stages(); ++i) {
    Message m;
    m.recipient = names_[i];
    m.command = LOAD_PARAMS;
    m.payload_type = P_TYPED_JOB;
    m.mb_id = full ? 1 : 0;
    if (full) {
      m.dtype = 5;
      m.data.assign(reinterpret_cast<const char*>(flats[i].data()), flats[i].size() * sizeof(double));
    } else {
      const std::vector<float> f(flats[i].begin(), flats[i].end());
      m.dtype = 0;
      m.data.assign(reinterpret_cast<const char*>(f.data()), f.size() * sizeof(float));
    }
    m.shape = {(uint64_t)flats[i].size()};
    comm_->send(std::move(m));
  }
  join(PARAMS_LOADED, names_.size());
}

void PipelineCoordinator::send_parameters(Sequential& model) {
  std::vector<std::vector<double>> flats;
  for (const Partition& p : parts_) {
    std::vector<Layer*> ls;
    for (int i = p.start; i < p.end; ++i) ls.push_back(model.layers().at(i).get());
    flats.push_back(pack_state(ls));
  }
  load_parameters(flats, false);
}

std::vector<std::vector<double>> PipelineCoordinator::collect_parameters(bool full) {
  broadcast(SEND_PARAMS, full ? "full" : "");
  std::map<std::string, std::vector<double>> got;
  for (auto& m : join(PARAMS_TRANSFER, names_.size())) got[m.sender] = payload_values(m);
  std::vector<std::vector<double>> out;
  for (const auto& s : names_) {
    auto it = got.find(s);
    if (it == got.end()) throw PipelineError("no parameters from " + s);
    out.push_back(std::move(it->second));
  }
  return out;
}

void PipelineCoordinator::gather_into(Sequential& model) {
  const auto flats = collect_parameters(false);
  for (size_t k = 0; k < parts_.size(); ++k) {
    std::vector<Layer*> ls;
    for (int i = parts_[k].start; i < parts_[k].end; ++i) ls.push_back(model.layers().at(i).get());
    unpack_state(ls, flats[k].data(), flats[k].size());
  }
}

std::vector<json::Value> PipelineCoordinator::status() {
  broadcast(STATUS_REQUEST);
  std::vector<json::Value> out;
  for (auto& m : join(STATUS_RESPONSE, names_.size())) out.push_back(json::Value::parse(m.text));
  std::sort(out.begin(), out.end(),
            [](const json::Value& a, const json::Value& b) { return a.get_string("id", "") < b.get_string("id", ""); });
  return out;
}

std::vector<std::string> PipelineCoordinator::print_profiling() {
  broadcast(PRINT_PROFILING);
  std::vector<std::string> out;
  for (auto& m : join(PROFILING_PRINTED, names_.size())) out.push_back(m.text);
  return out;
}

void PipelineCoordinator::clear_profiling() {
  broadcast(CLEAR_PROFILING);
  join(PROFILING_CLEARED, names_.size());
}

void PipelineCoordinator::barrier() {
  broadcast(BARRIER_SYNC);
  join(BARRIER_SYNC, names_.size());
}

std::map<std::string, bool> PipelineCoordinator::health_check(double timeout_s) {
  broadcast(HEALTH_CHECK);
  std::map<std::string, bool> alive;
  for (const auto& s : names_) alive[s] = false;
  try {
    for (auto& m : join(HEALTH_CHECK, names_.size(), timeout_s)) alive[m.sender] = m.flag;
  } catch (const PipelineError&) {
  }
  return alive;
}

std::vector<Partition> PipelineCoordinator::balance_load() {
  const std::vector<json::Value> st = status();
  std::vector<double> costs;
  bool any = false;
  const auto& layers = model_cfg_.at("layers").items();
  for (size_t k = 0; k < st.size(); ++k) {
    const json::Value* f = st[k].find("forward_times_us");
    const json::Value* b = st[k].find("backward_times_us");
    for (int i = parts_[k].start; i < parts_[k].end; ++i) {
      const std::string key = layers[i].get_string("name", layers[i].get_string("type", ""));
      double c = 0;
      if (f != nullptr) c += f->get_number(key, 0.0);
      if (b != nullptr) c += b->get_number(key, 0.0);
      any = any || c > 0;
      costs.push_back(c);
    }
  }
  if (!any) return parts_;
  std::vector<Partition> next = balanced_partitions(costs, num_stages());
  if (next == parts_) return parts_;
  // carry the trained weights over through a host copy of the whole model (a stage's flat state
  // cannot be re-cut at other layer boundaries without the layer shapes)
  Sequential model = Sequential::load_from_config(model_cfg_);
  model.initialize(0);
  gather_into(model);
  parts_ = std::move(next);
  deploy_stages();
  send_parameters(model);
  return parts_;
}

}  // namespace dcnn
