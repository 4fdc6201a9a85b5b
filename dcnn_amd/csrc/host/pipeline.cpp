// Native pipeline stage (dcnn/pipeline.hpp): configuration, tensor payloads, the command handlers.
#include "dcnn/pipeline.hpp"
#include "dcnn/dist.hpp"
#include "dcnn/ops.hpp"

#include <unistd.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "../kernels/collective.h"
#include "../native/comm.h"

using namespace dcnn_native;

namespace dcnn {

namespace {
constexpr uint8_t kChannelsLast = 0x10;  // dtype flag: NHWC physical buffer of an NCHW tensor
// dtype flag: the payload is an IPC reference (64-byte handle + byte count), not the bytes
// (transport "ipc", native stages only)
constexpr uint8_t kIpcRef = 0x20;
constexpr size_t kIpcRefBytes = gpu::kIpcHandleBytes + sizeof(uint64_t);
// ... + the hand-off's sequence number ("flag" mode; 0: no flag to wait for) [+ the sender's
// interprocess event handle ("event" mode)]
constexpr size_t kIpcRefSeqBytes = kIpcRefBytes + sizeof(uint64_t);
constexpr size_t kIpcRefEvBytes = kIpcRefSeqBytes + gpu::kIpcHandleBytes;
constexpr size_t kIpcHeader = 256;  // flag word, padded (the tensor bytes stay 256-byte aligned)
// dtype flag: the tensor travels on the stage pair's RCCL link; the payload is empty (transport
// "rccl", native stages only)
constexpr uint8_t kRcclRef = 0x40;
constexpr size_t kIdBytes = 128;  // ncclUniqueId
constexpr uint64_t kFullState = 1;        // SEND_PARAMS "full" / LOAD_PARAMS micro-batch id

enum class Handoff { Host, Event, Flag };
Handoff ipc_handoff() {
  static const Handoff h = [] {
    const char* e = std::getenv("DCNN_IPC_HANDOFF");
    const std::string v = e ? e : "host";
    if (v == "event") return Handoff::Event;
    if (v == "flag") return gpu::stream_values_supported() ? Handoff::Flag : Handoff::Host;
    if (v != "host") throw std::runtime_error("DCNN_IPC_HANDOFF: host | event | flag");
    return Handoff::Host;
  }();
  return h;
}

// t's typed-job header: m.shape (logical NCHW dims; NHWC buffers as N, H, W, C with the channels-
// last flag; logits as (N, classes)), returns the dtype code
uint8_t encode_header(const Tensor& t, bool as_logits, Message& m) {
  const auto& s = t.shape();
  uint8_t code = t.dtype() == DType::F32 ? 0 : t.dtype() == DType::BF16 ? 1 : 0xff;
  if (code == 0xff) throw std::runtime_error("activation dtype must be fp32 or bf16");
  m.shape.clear();
  if (s.size() == 4 && s[2] == 1 && s[3] == 1 && as_logits) {
    m.shape = {(uint64_t)s[0], (uint64_t)s[1]};  // logits (N, classes)
  } else if (s.size() == 4 && t.layout() == Layout::NHWC) {
    m.shape = {(uint64_t)s[0], (uint64_t)s[2], (uint64_t)s[3], (uint64_t)s[1]};
    code |= kChannelsLast;
  } else {
    for (auto d : s) m.shape.push_back((uint64_t)d);
  }
  return code;
}

struct Header {
  std::vector<int64_t> shape;
  DType dt = DType::F32;
  Layout layout = Layout::NCHW;
  int code = 0;
};
Header decode_header(const Message& m) {
  Header h;
  h.code = m.payload_type == P_TYPED_JOB ? m.dtype : 0;
  h.shape.assign(m.shape.begin(), m.shape.end());
  if ((h.code & kChannelsLast) && h.shape.size() == 4) {
    h.shape = {h.shape[0], h.shape[3], h.shape[1], h.shape[2]};
    h.layout = Layout::NHWC;
  }
  switch (h.code & 0x0F) {
    case 0: h.dt = DType::F32; break;
    case 1: h.dt = DType::BF16; break;
    default: throw std::runtime_error("activation payloads must be fp32 or bf16");
  }
  return h;
}

// (N, F) tensors travel as rank 2: 1x1 spatial again on arrival
Tensor as_4d(Tensor t, const std::vector<int64_t>& shape) {
  if (t.rank() == 2) t = t.view({shape[0], shape[1], 1, 1}, Layout::NCHW);
  return t;
}

std::optional<Endpoint> parse_endpoint(const json::Value* v) {
  if (v == nullptr || v->is_null()) return std::nullopt;
  Endpoint e;
  e.communication_type = v->get_string("communication_type", "tcp");
  if (const json::Value* p = v->find("parameters")) e.parameters = *p;
  return e;
}

std::string str_or(const json::Value& j, const char* k, const std::string& d) {
  const json::Value* v = j.find(k);
  return (v == nullptr || v->is_null()) ? d : v->as_string();
}

int64_t numel_of(const std::vector<int64_t>& s) {
  int64_t n = 1;
  for (auto d : s) n *= d;
  return n;
}

// dst's storage <- src's bytes (same byte count, same device kind as dst)
void copy_into(const Tensor& dst, const Tensor& src) {
  if (dst.nbytes() != src.nbytes()) throw std::runtime_error("state size mismatch");
  if (dst.device().is_gpu())
    gpu::copy(dst.data(), src.data(), src.nbytes(), src.device().is_gpu() ? 2 : 0);
  else
    std::memcpy(dst.data(), src.data(), src.nbytes());
}

// t as (dt, layout) on dev
Tensor convert(const Tensor& t, DType dt, Layout layout, Device dev) {
  if (t.dtype() == dt && t.layout() == layout) return t.device() == dev ? t : t.to(dev);
  return Tensor::from_host(t.to_host_f32(), t.shape(), dev, dt, layout);
}

double rss_mb() {
  std::ifstream f("/proc/self/statm");
  long pages = 0, rss = 0;
  f >> pages >> rss;
  return (double)rss * (double)sysconf(_SC_PAGESIZE) / (1024.0 * 1024.0);
}
}  // namespace

StageConfig StageConfig::parse(const std::string& text) {
  const json::Value j = json::Value::parse(text);
  StageConfig c;
  c.stage_id = str_or(j, "stage_id", "");
  c.stage_index = (int)j.get_int("stage_index", 0);
  c.num_stages = (int)j.get_int("num_stages", 1);
  c.model_config = j.at("model_config");
  c.optimizer_config = j.at("optimizer_config");
  c.next_stage = parse_endpoint(j.find("next_stage_endpoint"));
  c.prev_stage = parse_endpoint(j.find("prev_stage_endpoint"));
  c.coordinator = parse_endpoint(j.find("coordinator_endpoint"));
  c.device = str_or(j, "device", "CPU");
  c.transport = str_or(j, "transport", "message");
  c.codec = str_or(j, "codec", "none");
  if (const json::Value* s = j.find("seed"); s != nullptr && !s->is_null()) c.seed = s->as_int();
  if (const json::Value* f = j.find("first_layer_input_grad"); f != nullptr && !f->is_null())
    c.first_layer_input_grad = f->as_bool();
  if (const json::Value* h = j.find("heartbeat_s"); h != nullptr && !h->is_null()) c.heartbeat_s = h->as_number();
  return c;
}

std::unique_ptr<Communicator> make_tcp_communicator(const std::string& id, const std::string& host, int port,
                                                   int* bound_port) {
  auto c = std::make_unique<TcpCommunicator>(id, host, port);
  if (bound_port != nullptr) *bound_port = c->port();
  return c;
}

std::unique_ptr<Optimizer> create_optimizer(const json::Value& cfg) {
  std::string type = str_or(cfg, "type", "sgd");
  for (auto& ch : type) ch = (char)std::tolower((unsigned char)ch);
  const json::Value* pp = cfg.find("parameters");
  const json::Value p = pp != nullptr ? *pp : json::Value::object();
  const float lr = (float)p.get_number("learning_rate", type == "sgd" ? 0.01 : 0.001);
  if (type == "sgd") return std::make_unique<SGD>(lr, (float)p.get_number("momentum", 0.0));
  if (type == "adam" || type == "adamw") {
    const bool dec = type == "adamw" || p.get_bool("decouple_weight_decay", false);
    return std::make_unique<Adam>(lr, (float)p.get_number("beta1", 0.9), (float)p.get_number("beta2", 0.999),
                                  (float)p.get_number("epsilon", 1e-8), (float)p.get_number("weight_decay", 0.0), dec);
  }
  throw std::runtime_error("unknown optimizer type '" + type + "'");
}

PipelineStage::PipelineStage(Communicator* comm, bool verbose) : comm_(comm), verbose_(verbose), id_(comm->id()) {}

PipelineStage::~PipelineStage() {
  stop_heartbeat();
  try {
    release_links();
    release_ipc();
  } catch (...) {
  }
}

void PipelineStage::release_links() {
  act_out_.reset();
  act_in_.reset();
  grad_out_.reset();
  grad_in_.reset();
}

void PipelineStage::connect_links(Message& m) {
  if (m.payload_type == P_TYPED_JOB) {  // the previous stage's ids, ahead of the coordinator's request
    if (m.data.size() != 2 * kIdBytes) throw std::runtime_error("P2P_CONNECT: malformed unique ids");
    prev_ids_ = m.data;
    return;
  }
  if (cfg_.transport != "rccl") throw std::runtime_error("P2P_CONNECT: the stage transport is '" + cfg_.transport + "'");
  release_links();
  const int dev = dev_.index;
  const bool has_prev = cfg_.stage_index > 0, has_next = cfg_.stage_index < cfg_.num_stages - 1;
  std::string next_ids;
  if (has_next) {
    next_ids = coll::unique_id() + coll::unique_id();  // activations down, gradients up
    Message u;
    u.recipient = "next_stage";
    u.command = P2P_CONNECT;
    u.payload_type = P_TYPED_JOB;
    u.dtype = 4;  // u8
    u.shape = {(uint64_t)next_ids.size()};
    u.data = next_ids;
    comm_->send(std::move(u));
  }
  // the previous pair first, then the next: stage i's next pair is stage i + 1's previous pair,
  // so the blocking joins chain from the first stage down without a cycle
  if (has_prev) {
    const auto t0 = std::chrono::steady_clock::now();
    while (prev_ids_.empty()) {
      Message q;
      if (comm_->queue().pop_command(P2P_CONNECT, q, 50)) {
        if (q.payload_type != P_TYPED_JOB) throw std::runtime_error("P2P_CONNECT: second request before the links opened");
        connect_links(q);
      } else if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
        throw std::runtime_error("P2P_CONNECT: no unique ids from the previous stage");
      }
    }
    act_in_ = std::make_unique<dist::P2PLink>(prev_ids_.substr(0, kIdBytes), 1, false, dev);
    grad_out_ = std::make_unique<dist::P2PLink>(prev_ids_.substr(kIdBytes), 1, true, dev);
    prev_ids_.clear();
  }
  if (has_next) {
    act_out_ = std::make_unique<dist::P2PLink>(next_ids.substr(0, kIdBytes), 0, true, dev);
    grad_in_ = std::make_unique<dist::P2PLink>(next_ids.substr(kIdBytes), 0, false, dev);
  }
  reply(P2P_CONNECT, "ok");
}

void PipelineStage::release_ipc() {
  if ((!ipc_out_.empty() || !ipc_in_.empty()) && dev_.is_gpu()) gpu::synchronize();  // (no hand-off in flight)
  for (auto& kv : ipc_in_) gpu::ipc_close(kv.second);
  ipc_in_.clear();
  for (auto& kv : ipc_ev_in_) gpu::event_destroy(kv.second);
  ipc_ev_in_.clear();
  for (auto& kv : ipc_out_) {
    gpu::ipc_free(kv.second.ptr);
    if (kv.second.ev) gpu::event_destroy(kv.second.ev);
  }
  ipc_out_.clear();
  for (void* p : ipc_retired_) gpu::ipc_free(p);
  ipc_retired_.clear();
}

void PipelineStage::run(int poll_ms) {
  running_ = true;
  while (running_) {
    Message m;
    if (!comm_->queue().pop(m, poll_ms)) {
      if (comm_->queue().closed()) break;
      continue;
    }
    process(m);
  }
  stop_heartbeat();
}

void PipelineStage::reply(uint16_t cmd, const std::string& text) {
  Message m;
  m.recipient = "coordinator";
  m.command = cmd;
  if (!text.empty()) {
    m.payload_type = P_STRING;
    m.text = text;
  }
  if (auto* tcp = dynamic_cast<TcpCommunicator*>(comm_)) tcp->wait_for_peer("coordinator", 30000);
  comm_->send(std::move(m));
}

void PipelineStage::process(Message& m) {
  const uint16_t cmd = m.command;
  try {
    switch (cmd) {
      case FORWARD_JOB: forward(m); break;
      case BACKWARD_JOB: backward(m); break;
      case LABELS_TRANSFER: take_labels(m); break;
      case P2P_CONNECT: connect_links(m); break;
      case UPDATE_PARAMETERS: {
        if (m.payload_type == P_STRING && !m.text.empty()) {
          const json::Value hp = json::Value::parse(m.text);
          if (hp.has("learning_rate")) opt_->set_learning_rate((float)hp.at("learning_rate").as_number());
        }
        // every micro-batch's sends have their receives posted by now: release their slots
        if (act_out_) act_out_->drain();
        if (grad_out_) grad_out_->drain();
        opt_->step(model_->parameters());
        model_->zero_grad();
        // the step's IPC copies out of the peers' buffers are complete before this answer (the
        // peers rewrite them in the next step)
        if (ipc_device_ordered_) gpu::flow_synchronize();
        ipc_device_ordered_ = false;
        ++n_upd_;
        reply(PARAMETERS_UPDATED);
        break;
      }
      case TRAIN_MODE: model_->set_training(true); break;
      case EVAL_MODE: model_->set_training(false); break;
      case SHUTDOWN: stop(); break;
      case CONFIG_TRANSFER: configure(m.text); break;
      case SEND_PARAMS: {
        const bool full = m.payload_type == P_STRING && m.text == "full";
        Message r;
        r.recipient = "coordinator";
        r.command = PARAMS_TRANSFER;
        r.payload_type = P_TYPED_JOB;
        r.mb_id = full ? kFullState : 0;
        std::vector<double> st = flat_state();
        if (full) {
          std::vector<double> v{(double)st.size()};
          v.insert(v.end(), st.begin(), st.end());
          std::vector<double> o = optimizer_state();
          v.insert(v.end(), o.begin(), o.end());
          r.dtype = 5;  // f64
          r.shape = {(uint64_t)v.size()};
          r.data.assign(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(double));
        } else {
          std::vector<float> f(st.begin(), st.end());
          r.dtype = 0;
          r.shape = {(uint64_t)f.size()};
          r.data.assign(reinterpret_cast<const char*>(f.data()), f.size() * sizeof(float));
        }
        if (auto* tcp = dynamic_cast<TcpCommunicator*>(comm_)) tcp->wait_for_peer("coordinator", 30000);
        comm_->send(std::move(r));
        break;
      }
      case LOAD_PARAMS:
      case PARAMS_TRANSFER: {
        if (m.codec) m.data = decompress(m.data, (Codec)m.codec, 0);
        const int code = m.payload_type == P_TYPED_JOB ? (m.dtype & 0x0F) : 0;
        std::vector<double> v;
        if (code == 5) {
          v.resize(m.data.size() / sizeof(double));
          std::memcpy(v.data(), m.data.data(), v.size() * sizeof(double));
        } else if (code == 0) {
          std::vector<float> f(m.data.size() / sizeof(float));
          std::memcpy(f.data(), m.data.data(), f.size() * sizeof(float));
          v.assign(f.begin(), f.end());
        } else {
          throw std::runtime_error("parameter state must be fp32 or fp64");
        }
        if (m.mb_id == kFullState && code == 5) {
          const size_t n = (size_t)v.at(0);
          load_flat_state(v.data() + 1, n);
          load_optimizer_state(v.data() + 1 + n, v.size() - 1 - n);
        } else {
          load_flat_state(v.data(), v.size());
        }
        reply(PARAMS_LOADED);
        break;
      }
      case STATUS_REQUEST: reply(STATUS_RESPONSE, status_json()); break;
      case HEALTH_CHECK: {
        Message r;
        r.recipient = "coordinator";
        r.command = HEALTH_CHECK;
        r.payload_type = P_BOOL;
        r.flag = true;
        comm_->send(std::move(r));
        break;
      }
      case BARRIER_SYNC:
        if (dev_.is_gpu()) gpu::synchronize();
        reply(BARRIER_SYNC);
        break;
      case CHECKPOINT_REQUEST:
        model_->save_to_file(m.text);
        reply(CHECKPOINT_COMPLETE, m.text);
        break;
      case REPORT_LOAD: {
        Message r;
        r.recipient = "coordinator";
        r.command = LOAD_REPORT;
        r.payload_type = P_LOAD;
        r.load.avg_forward_ms = n_fwd_ ? (float)(fwd_ms_ / (double)n_fwd_) : 0.f;
        r.load.avg_backward_ms = n_bwd_ ? (float)(bwd_ms_ / (double)n_bwd_) : 0.f;
        r.load.avg_cpu_utilization = -1.f;
        r.load.max_memory_mb = (float)rss_mb();
        comm_->send(std::move(r));
        break;
      }
      case UPDATE_LOAD: reply(LOAD_REPORT, status_json()); break;
      case PRINT_PROFILING: {
        char buf[256];
        std::snprintf(buf, sizeof buf, "%s (native): %ld forward, %ld backward, %ld updates; avg forward %.3f ms, "
                      "avg backward %.3f ms\n", id_.c_str(), n_fwd_, n_bwd_, n_upd_,
                      n_fwd_ ? fwd_ms_ / (double)n_fwd_ : 0.0, n_bwd_ ? bwd_ms_ / (double)n_bwd_ : 0.0);
        reply(PROFILING_PRINTED, buf);
        break;
      }
      case CLEAR_PROFILING:
        fwd_ms_ = bwd_ms_ = 0;
        n_fwd_ = n_bwd_ = 0;
        reply(PROFILING_CLEARED);
        break;
      default: throw std::runtime_error(std::string("unhandled command ") + command_name(cmd));
    }
  } catch (const std::exception& e) {
    const uint16_t kind = (cmd == FORWARD_JOB || cmd == BACKWARD_JOB) ? JOB_FAILURE : ERROR_REPORT;
    const std::string what = id_ + ": " + command_name(cmd) + " failed\n" + e.what();
    if (verbose_) std::fprintf(stderr, "%s\n", what.c_str());
    try {
      reply(kind, what);
    } catch (...) {
    }
  }
}

void PipelineStage::configure(const std::string& text) {
  cfg_ = StageConfig::parse(text);
  if (cfg_.transport != "message" && cfg_.transport != "ipc" && cfg_.transport != "rccl")
    throw std::runtime_error("native stage: transport '" + cfg_.transport + "' not supported ('message' | 'ipc' | 'rccl')");
  stop_heartbeat();
  dev_ = Device::parse(cfg_.device);
  if (cfg_.transport != "message" && !dev_.is_gpu())
    throw std::runtime_error("native stage: transport '" + cfg_.transport + "' needs a GPU stage");
  release_links();
  prev_ids_.clear();
  release_ipc();  // (a redeploy may change the neighbours)
  drop_all_graphs();  // (they hold the previous model's buffers)
  if (dev_.is_gpu()) gpu::set_device(dev_.index);
  const char* ge = std::getenv("DCNN_STAGE_GRAPHS");
  graphs_ = dev_.is_gpu() && !(ge != nullptr && std::string(ge) == "0");
  model_ = std::make_unique<Sequential>(Sequential::load_from_config(cfg_.model_config));
  model_->set_device(dev_);
  model_->initialize((uint64_t)cfg_.seed.value_or(0));
  // the first stage's input gradient goes nowhere unless asked for: skip its data-gradient GEMM
  if (cfg_.stage_index == 0 && !cfg_.first_layer_input_grad && !model_->layers().empty())
    model_->layers()[0]->set_input_grad(false);
  opt_ = create_optimizer(cfg_.optimizer_config);
  out_kind_.clear();
  n_fwd_ = n_bwd_ = n_upd_ = 0;
  fwd_ms_ = bwd_ms_ = 0;
  id_ = cfg_.stage_id;
  comm_->set_id(id_);
  connect_peers();
  if (cfg_.heartbeat_s > 0) start_heartbeat();
  reply(CONFIG_RECEIVED, id_);
}

void PipelineStage::connect_peers() {
  auto* tcp = dynamic_cast<TcpCommunicator*>(comm_);
  auto* inproc = dynamic_cast<InProcessCommunicator*>(comm_);
  const std::pair<const char*, const std::optional<Endpoint>*> eps[] = {
      {"next_stage", &cfg_.next_stage}, {"prev_stage", &cfg_.prev_stage}, {"coordinator", &cfg_.coordinator}};
  for (const auto& [name, ep] : eps) {
    if (!ep->has_value()) continue;
    const Endpoint& e = **ep;
    const std::string peer = e.id();
    if (e.communication_type == "in_process") {
      if (inproc == nullptr) throw std::runtime_error("in_process endpoint needs an in-process communicator");
      if (peer != name) inproc->alias(name, peer);
    } else if (tcp != nullptr) {
      if (std::string(name) == "next_stage") {
        tcp->connect(name, e.host(), e.port(), 60000);
        if (!peer.empty()) tcp->alias(peer, name);
      } else if (!peer.empty()) {
        tcp->alias(name, peer);  // prev stage / coordinator dial us
      }
    } else {
      throw std::runtime_error("endpoint type " + e.communication_type + " needs a TCP communicator");
    }
  }
}

Tensor PipelineStage::decode(Message& m) const {
  if (m.payload_type != P_JOB && m.payload_type != P_TYPED_JOB) throw std::runtime_error("job message without a tensor");
  if (m.shape.empty()) return Tensor();
  if (m.codec) {
    m.data = decompress(m.data, (Codec)m.codec, 0);
    m.codec = CODEC_NONE;
  }
  const Header hd = decode_header(m);
  const std::vector<int64_t>& shape = hd.shape;
  const DType dt = hd.dt;
  const Layout layout = hd.layout;
  if (hd.code & kRcclRef) {
    // the peer's send on this pair's link (sent before the message; RCCL matches in order)
    dist::P2PLink* l = m.command == FORWARD_JOB ? act_in_.get() : m.command == BACKWARD_JOB ? grad_in_.get() : nullptr;
    if (l == nullptr || !dev_.is_gpu()) throw std::runtime_error("RCCL tensor reference without an open link");
    return wire::recv_rccl(*l, m, dev_);
  }
  if (hd.code & kIpcRef) {
    // a peer stage's device buffer: map it once, copy out on this stage's flow once the sender's
    // copy into it has completed (its flag; the sender rewrites the buffer only in a later step)
    if (!dev_.is_gpu() || (m.data.size() != kIpcRefSeqBytes && m.data.size() != kIpcRefEvBytes))
      throw std::runtime_error("malformed IPC tensor reference");
    Tensor t = Tensor::empty(shape, dt, dev_, layout);
    uint64_t nbytes = 0, seq = 0;
    std::memcpy(&nbytes, m.data.data() + gpu::kIpcHandleBytes, sizeof nbytes);
    std::memcpy(&seq, m.data.data() + kIpcRefBytes, sizeof seq);
    if (nbytes != t.nbytes()) throw std::runtime_error("IPC tensor size does not match its shape");
    const std::string key(m.data.data(), gpu::kIpcHandleBytes);
    auto it = ipc_in_.find(key);
    if (it == ipc_in_.end()) it = ipc_in_.emplace(key, gpu::ipc_open(key.data())).first;
    char* base = static_cast<char*>(it->second);
    bool device_ordered = false;
    if (m.data.size() == kIpcRefEvBytes) {
      const std::string ek(m.data.data() + kIpcRefSeqBytes, gpu::kIpcHandleBytes);
      auto e = ipc_ev_in_.find(ek);
      if (e == ipc_ev_in_.end()) e = ipc_ev_in_.emplace(ek, gpu::ipc_event_open(ek.data())).first;
      gpu::flow_wait(nullptr, e->second);
      device_ordered = true;
    } else if (seq != 0) {
      gpu::flow_wait_u32_geq(base, (uint32_t)seq);
      device_ordered = true;
    }
    gpu::copy(t.data(), base + kIpcHeader, t.nbytes(), 2);
    if (device_ordered)
      ipc_device_ordered_ = true;
    else
      gpu::flow_synchronize();  // (host-waited hand-off: the copy is done before any reply goes out)
    return as_4d(t, shape);
  }
  // a GPU stage's own activation form (bf16 NHWC) goes straight from the payload to the device
  const bool direct = dev_.is_gpu() && dt == DType::BF16 && layout == Layout::NHWC;
  Tensor t = Tensor::empty(shape, dt, direct ? dev_ : Device::cpu(), layout);
  if (m.data.size() != t.nbytes()) throw std::runtime_error("tensor payload size does not match its shape");
  if (direct)
    gpu::copy(t.data(), m.data.data(), t.nbytes(), 0);
  else
    std::memcpy(t.data(), m.data.data(), t.nbytes());
  if (t.rank() == 2) t = t.view({shape[0], shape[1], 1, 1}, Layout::NCHW);  // (N, F): 1x1 spatial
  return t;
}

void PipelineStage::send_tensor(const std::string& to, uint16_t cmd, uint64_t mb, const Tensor& t, bool as_logits) {
  Message m;
  m.recipient = to;
  m.command = cmd;
  m.payload_type = P_TYPED_JOB;
  m.mb_id = mb;
  if (t.defined()) {
    if (cfg_.transport == "rccl" && t.device().is_gpu() && (to == "next_stage" || to == "prev_stage")) {
      dist::P2PLink* l = to == "next_stage" ? act_out_.get() : grad_out_.get();
      if (l == nullptr) throw std::runtime_error("transport 'rccl': the stage links are not open (P2P_CONNECT)");
      wire::send_rccl(*l, t, mb, as_logits, m);
      comm_->send(std::move(m));
      return;
    }
    const uint8_t code = encode_header(t, as_logits, m);
    m.dtype = code;
    if (cfg_.transport == "ipc" && t.device().is_gpu() && (to == "next_stage" || to == "prev_stage")) {
      IpcSlot& slot = ipc_out_[{to, mb}];
      if (slot.bytes < t.nbytes()) {
        if (slot.ptr != nullptr) ipc_retired_.push_back(slot.ptr);
        slot.handle.assign(gpu::kIpcHandleBytes, '\0');
        slot.ptr = gpu::ipc_alloc(kIpcHeader + t.nbytes(), slot.handle.data());
        slot.bytes = t.nbytes();
        gpu::zero(slot.ptr, kIpcHeader);
        slot.seq = 0;
      }
      gpu::copy(static_cast<char*>(slot.ptr) + kIpcHeader, t.data(), t.nbytes(), 2);
      uint64_t seq = 0;
      Handoff mode = ipc_handoff();
      if (mode == Handoff::Event && slot.ev == nullptr) {
        std::string h(gpu::kIpcHandleBytes, '\0');
        slot.ev = gpu::ipc_event_create(h.data());
        if (slot.ev) slot.ev_handle = h;
      }
      if (mode == Handoff::Event && slot.ev == nullptr) mode = Handoff::Host;  // (no exportable events)
      if (mode == Handoff::Flag) {
        seq = ++slot.seq;
        if (seq == 0xffffffffull) throw std::runtime_error("IPC hand-off sequence exhausted");
        gpu::flow_write_u32(slot.ptr, (uint32_t)seq);  // (after the copy: the receiver's flow waits for it)
      } else if (mode == Handoff::Event) {
        gpu::event_record(slot.ev);  // (after the copy: the receiver's flow waits for it)
      } else {
        gpu::flow_synchronize();  // the slot is complete (this stage's flow) before the peer process reads it
      }
      const uint64_t nbytes = t.nbytes();
      m.dtype = code | kIpcRef;
      m.data.assign(slot.handle);
      m.data.append(reinterpret_cast<const char*>(&nbytes), sizeof nbytes);
      m.data.append(reinterpret_cast<const char*>(&seq), sizeof seq);
      if (mode == Handoff::Event) m.data.append(slot.ev_handle);
      comm_->send(std::move(m));
      return;
    }
    m.data.resize(t.nbytes());  // (device tensors copy straight into the payload)
    if (t.device().is_gpu())
      gpu::copy(m.data.data(), t.data(), t.nbytes(), 1);
    else
      std::memcpy(m.data.data(), t.data(), t.nbytes());
    if (cfg_.codec == "zlib" || cfg_.codec == "zstd") {
      const Codec c = cfg_.codec == "zlib" ? CODEC_ZLIB : CODEC_ZSTD;
      m.data = compress(m.data, c, 3);
      m.codec = c;
    }
  }
  comm_->send(std::move(m));
}

void PipelineStage::forward(Message& m) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t mb = m.mb_id;
  Tensor x = decode(m);
  Tensor a;
  if (cfg_.stage_index == 0 && x.dtype() == DType::F32 && x.layout() == Layout::NCHW) {
    a = model_->input_activation(x);  // the network input (fp32 NCHW)
  } else if (dev_.is_gpu()) {
    a = convert(x, DType::BF16, Layout::NHWC, dev_);
  } else {
    a = convert(x, DType::F32, Layout::NCHW, dev_);
  }
  Tensor out;
  if (graphs_ && n_upd_ >= 1) {
    out = run_graph(fwd_graph_, mb, a, model_->is_training(),
                    [&](const Tensor& in) { return model_->forward_activation(in, (int)mb); });
    fwd_graphed_[mb] = true;
  } else {
    drop_graphs(mb);
    out = model_->forward_activation(a, (int)mb);
    fwd_graphed_[mb] = false;
  }
  out_kind_[mb] = OutKind{out.dtype(), out.layout(), out.shape()};
  const bool last = cfg_.stage_index == cfg_.num_stages - 1;
  if (last && stage_loss_) {
    // loss + d loss / d logits on this device; the coordinator gets the value, the backward starts
    const Tensor labels = labels_for(mb);
    const int64_t N = out.dim(0), C = out.numel() / N;
    LossResult lr;
    const bool train = model_->is_training();
    if (dev_.is_gpu()) {
      // the loss kernel and the backward go out first; one read of the value after them
      lr.grad = Tensor::empty({N, C}, DType::BF16, dev_, Layout::NHWC);
      gpu_ops::loss_launch(stage_loss_->kind(), out.data(), nullptr, labels.ptr<int64_t>(), lr.grad.data(), (int)N,
                           (int)C, stage_loss_->param(), grad_scale_);
      ++n_fwd_;
      fwd_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (train) run_backward(mb, lr.grad, std::chrono::steady_clock::now());
      lr.loss = gpu_ops::read_last_loss(&lr.correct);
    } else {
      lr = stage_loss_->compute(out.view({N, C}, out.layout()), &labels, nullptr, grad_scale_);
      ++n_fwd_;
      fwd_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    Message r;
    r.recipient = "coordinator";
    r.command = FORWARD_JOB;
    r.payload_type = P_STRING;
    json::Value v = json::Value::object();
    v["mb"] = (int64_t)mb;
    v["loss"] = lr.loss;
    v["correct"] = (int64_t)lr.correct;
    v["samples"] = N;
    r.text = v.dump(-1);
    comm_->send(std::move(r));
    if (train && !dev_.is_gpu()) run_backward(mb, lr.grad, std::chrono::steady_clock::now());
    return;
  }
  send_tensor(last ? "coordinator" : "next_stage", FORWARD_JOB, mb, out, last);
  ++n_fwd_;
  fwd_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void PipelineStage::take_labels(Message& m) {
  if (m.payload_type != P_TYPED_JOB || (m.dtype & 0x0F) != 5) throw std::runtime_error("LABELS_TRANSFER: f64 payload expected");
  std::vector<double> v(m.data.size() / sizeof(double));
  std::memcpy(v.data(), m.data.data(), v.size() * sizeof(double));
  if (m.mb_id == kLossConfigMb) {
    if (v.size() != 3) throw std::runtime_error("LABELS_TRANSFER: loss configuration is [kind, param, scale]");
    if (cfg_.stage_index != cfg_.num_stages - 1) throw std::runtime_error("the stage loss runs on the last stage");
    stage_loss_ = std::make_unique<Loss>((int)v[0], (float)v[1], "stage_loss");
    grad_scale_ = (float)v[2];
    labels_.clear();
    reply(LABELS_TRANSFER, "ok");
    return;
  }
  std::vector<int64_t> y(v.size());
  for (size_t i = 0; i < v.size(); ++i) y[i] = (int64_t)v[i];
  labels_[m.mb_id] = Tensor::from_host_i64(y, dev_);
}

// the micro-batch's labels: sent by the coordinator before its input, but the queue serves
// LABELS_TRANSFER after FORWARD_JOB, so they may still be queued when the forward gets here
Tensor PipelineStage::labels_for(uint64_t mb) {
  const auto t0 = std::chrono::steady_clock::now();
  while (labels_.find(mb) == labels_.end()) {
    Message m;
    if (comm_->queue().pop_command(LABELS_TRANSFER, m, 50)) {
      take_labels(m);
    } else if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
      throw std::runtime_error("no labels for micro-batch " + std::to_string(mb));
    }
  }
  Tensor y = labels_.at(mb);
  labels_.erase(mb);
  return y;
}

void PipelineStage::backward(Message& m) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t mb = m.mb_id;
  auto it = out_kind_.find(mb);
  if (it == out_kind_.end()) throw std::runtime_error("backward for micro-batch " + std::to_string(mb) + " without a forward");
  const OutKind k = it->second;
  Tensor g = decode(m);
  if (g.shape() != k.shape) {
    if (g.numel() != numel_of(k.shape)) throw std::runtime_error("gradient shape does not match the forward output");
    // (N, C) logits gradient for an (N, C, 1, 1) output: the same bytes in either layout
    g = g.view(k.shape, k.layout);
  }
  g = convert(g, k.dt, k.layout, dev_);
  run_backward(mb, g, t0);
}

void PipelineStage::run_backward(uint64_t mb, Tensor g, const std::chrono::steady_clock::time_point& t0) {
  const OutKind& k = out_kind_.at(mb);
  if (g.shape() != k.shape) g = g.view(k.shape, k.layout);  // ((N, C) logits gradient of an (N, C, 1, 1) output)
  Tensor gin;
  auto fg = fwd_graphed_.find(mb);
  if (graphs_ && fg != fwd_graphed_.end() && fg->second)
    gin = run_graph(bwd_graph_, mb, g, true, [&](const Tensor& in) { return model_->backward_activation(in, (int)mb); });
  else
    gin = model_->backward_activation(g, (int)mb);
  const bool first = cfg_.stage_index == 0;
  if (first && !cfg_.first_layer_input_grad) gin = Tensor();
  send_tensor(first ? "coordinator" : "prev_stage", BACKWARD_JOB, mb, gin, false);
  ++n_bwd_;
  bwd_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

Tensor PipelineStage::run_graph(std::map<uint64_t, MbGraph>& tab, uint64_t mb, const Tensor& in, bool training,
                                const std::function<Tensor(const Tensor&)>& body) {
  MbGraph& G = tab[mb];
  if (G.g && (G.shape != in.shape() || G.dt != in.dtype() || G.layout != in.layout() || G.training != training)) {
    drop_graphs(mb);  // (both phases: the backward graph reads the forward graph's buffers)
    return run_graph(tab, mb, in, training, body);
  }
  if (!G.g) {
    G.in = Tensor::empty(in.shape(), in.dtype(), dev_, in.layout());
    copy_into(G.in, in);
    G.g = std::make_unique<gpu::Graph>();
    G.g->begin();
    try {
      G.out = body(G.in);
    } catch (...) {
      G.g.reset();  // (ends the capture)
      tab.erase(mb);
      throw;
    }
    G.g->end();
    G.shape = in.shape();
    G.dt = in.dtype();
    G.layout = in.layout();
    G.training = training;
  } else {
    copy_into(G.in, in);
  }
  G.g->replay();
  return G.out;
}

void PipelineStage::drop_graphs(uint64_t mb) {
  fwd_graph_.erase(mb);
  bwd_graph_.erase(mb);
  fwd_graphed_.erase(mb);
}

void PipelineStage::drop_all_graphs() {
  fwd_graph_.clear();
  bwd_graph_.clear();
  fwd_graphed_.clear();
}

namespace {
void params_and_bns(const std::vector<Layer*>& layers, std::vector<Param*>& ps, std::vector<BatchNorm*>& bns) {
  std::vector<Layer*> all;
  for (Layer* l : layers) {
    l->collect_params(ps);
    l->collect_layers(all);
  }
  for (Layer* l : all)
    if (auto* bn = dynamic_cast<BatchNorm*>(l)) bns.push_back(bn);
}

std::vector<Layer*> layers_of(const Sequential& m) {
  std::vector<Layer*> out;
  for (auto& l : m.layers()) out.push_back(l.get());
  return out;
}
}  // namespace

std::vector<double> pack_state(const std::vector<Layer*>& layers) {
  std::vector<Param*> ps;
  std::vector<BatchNorm*> bns;
  params_and_bns(layers, ps, bns);
  std::vector<double> out;
  for (Param* p : ps) {
    const std::vector<float> v = p->value.view(p->shape, p->layout).to_host_f32();
    out.insert(out.end(), v.begin(), v.end());
  }
  for (BatchNorm* bn : bns) {
    for (const Tensor* t : {&bn->running_mean, &bn->running_var}) {
      const std::vector<float> v = t->to_host_f32();
      out.insert(out.end(), v.begin(), v.end());
    }
  }
  return out;
}

void unpack_state(const std::vector<Layer*>& layers, const double* v, size_t n) {
  std::vector<Param*> ps;
  std::vector<BatchNorm*> bns;
  params_and_bns(layers, ps, bns);
  size_t off = 0;
  auto take = [&](int64_t k) {
    if (off + (size_t)k > n) throw std::runtime_error("flat state too short");
    std::vector<float> f(v + off, v + off + k);
    off += (size_t)k;
    return f;
  };
  for (Param* p : ps) {
    const Tensor t = Tensor::from_host(take(numel_of(p->shape)), p->shape, p->value.device(), DType::F32, p->layout);
    copy_into(p->value, t);
  }
  for (BatchNorm* bn : bns) {
    for (Tensor* t : {&bn->running_mean, &bn->running_var}) {
      const Tensor h = Tensor::from_host(take(t->numel()), t->shape(), t->device(), DType::F32, t->layout());
      copy_into(*t, h);
    }
  }
  if (off != n) throw std::runtime_error("flat state size mismatch: consumed " + std::to_string(off) + " of " +
                                         std::to_string(n));
  for (Layer* l : layers) l->sync_shadow();
}

std::vector<double> PipelineStage::flat_state() { return pack_state(layers_of(*model_)); }

void PipelineStage::load_flat_state(const double* v, size_t n) { unpack_state(layers_of(*model_), v, n); }

// [learning rate, step count, then the state tensors by name (Adam: m, v; SGD with momentum:
// velocity), each over every parameter in checkpoint order]
std::vector<double> PipelineStage::optimizer_state() {
  std::vector<double> out{(double)opt_->learning_rate(), 0.0};
  auto* adam = dynamic_cast<Adam*>(opt_.get());
  auto* sgd = dynamic_cast<SGD*>(opt_.get());
  auto params = model_->parameters();
  auto append = [&](Tensor Param::*field) {
    for (Param* p : params) {
      const Tensor& t = p->*field;
      if (t.defined()) {
        const std::vector<float> v = t.view(p->shape, p->layout).to_host_f32();
        out.insert(out.end(), v.begin(), v.end());
      } else {
        out.insert(out.end(), (size_t)numel_of(p->shape), 0.0);
      }
    }
  };
  if (adam != nullptr) {
    out[1] = (double)adam->step_count();
    append(&Param::m);
    append(&Param::v);
  } else if (sgd != nullptr && sgd->momentum() != 0.f) {
    append(&Param::m);  // (SGD keeps its velocity in Param::m)
  }
  return out;
}

void PipelineStage::load_optimizer_state(const double* v, size_t n) {
  if (n < 2) throw std::runtime_error("optimizer state too short");
  opt_->set_learning_rate((float)v[0]);
  size_t off = 2;
  auto params = model_->parameters();
  auto fill = [&](Tensor Param::*field) {
    for (Param* p : params) {
      const int64_t k = numel_of(p->shape);
      if (off + (size_t)k > n) throw std::runtime_error("optimizer state too short");
      std::vector<float> f(v + off, v + off + k);
      off += (size_t)k;
      Tensor& dst = p->*field;
      if (!dst.defined()) dst = Tensor::zeros(p->value.shape(), DType::F32, p->value.device(), p->value.layout());
      copy_into(dst, Tensor::from_host(f, p->shape, p->value.device(), DType::F32, p->layout));
    }
  };
  if (auto* adam = dynamic_cast<Adam*>(opt_.get())) {
    adam->set_step_count((long)v[1]);
    fill(&Param::m);
    fill(&Param::v);
  } else if (auto* sgd = dynamic_cast<SGD*>(opt_.get()); sgd != nullptr && sgd->momentum() != 0.f) {
    fill(&Param::m);
  }
  if (off != n) throw std::runtime_error("optimizer state size mismatch");
}

std::string PipelineStage::status_json() {
  json::Value d = json::Value::object();
  d["id"] = id_;
  json::Value c = json::Value::object();
  c["forward"] = (int64_t)n_fwd_;
  c["backward"] = (int64_t)n_bwd_;
  c["update"] = (int64_t)n_upd_;
  d["counts"] = std::move(c);
  d["pid"] = (int64_t)getpid();
  d["native"] = true;
  if (model_) {
    d["device"] = dev_.str();
    json::Value ls = json::Value::array();
    for (auto& l : model_->layers()) ls.push(l->name());
    d["layers"] = std::move(ls);
    d["num_parameters"] = (int64_t)model_->num_parameters();
  }
  return d.dump(-1);
}

void PipelineStage::start_heartbeat() {
  beat_stop_ = false;
  const double every = cfg_.heartbeat_s;
  beat_ = std::thread([this, every] {
    while (!beat_stop_) {
      Message m;
      m.recipient = "coordinator";
      m.command = HEALTH_CHECK;
      m.payload_type = P_STRING;
      m.text = "heartbeat";
      try {
        comm_->send(std::move(m));
      } catch (...) {
      }
      const auto until = std::chrono::steady_clock::now() + std::chrono::duration<double>(every);
      while (!beat_stop_ && std::chrono::steady_clock::now() < until)
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
  });
}

void PipelineStage::stop_heartbeat() {
  beat_stop_ = true;
  if (beat_.joinable()) beat_.join();
}

namespace wire {
void send_rccl(dist::P2PLink& l, const Tensor& t, uint64_t mb, bool as_logits, Message& m) {
  const uint8_t code = encode_header(t, as_logits, m);
  m.payload_type = P_TYPED_JOB;
  m.mb_id = mb;
  m.data.clear();
  l.send(t, mb);  // (before the message: the receiver posts its receive when the message arrives)
  m.dtype = code | kRcclRef;
}

Tensor recv_rccl(dist::P2PLink& l, const Message& m, Device dev) {
  const Header hd = decode_header(m);
  if (!(hd.code & kRcclRef)) throw std::runtime_error("not an RCCL tensor reference");
  if (!dev.is_gpu()) throw std::runtime_error("RCCL tensor reference on a CPU stage");
  return as_4d(l.recv(hd.shape, hd.dt, hd.layout, dev), hd.shape);
}
}  // namespace wire

}  // namespace dcnn
