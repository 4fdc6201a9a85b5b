// Data parallelism of the C++ host API (dcnn/dist.hpp).
#include "dcnn/dist.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

#include <algorithm>
#include <cstdint>

#include "../kernels/collective.h"
#include "dcnn/nn.hpp"
#include "dcnn/ops.hpp"

namespace dcnn {
namespace dist {

namespace {
int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}
void send_all(int fd, const char* p, size_t n) {
  while (n) {
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) throw std::runtime_error("dist: send failed");
    p += k;
    n -= (size_t)k;
  }
}
void recv_all(int fd, char* p, size_t n) {
  while (n) {
    const ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) throw std::runtime_error("dist: recv failed");
    p += k;
    n -= (size_t)k;
  }
}
}  // namespace

Env Env::from_env() {
  Env e;
  e.rank = env_int("RANK", 0);
  e.world = env_int("WORLD_SIZE", 1);
  e.local_rank = env_int("LOCAL_RANK", e.rank);
  if (const char* a = std::getenv("MASTER_ADDR")) e.addr = a;
  e.port = env_int("MASTER_PORT", 29500);
  if (e.world < 1 || e.rank < 0 || e.rank >= e.world) throw std::invalid_argument("dist: bad RANK / WORLD_SIZE");
  return e;
}

std::string exchange_unique_id(const Env& e, int port_offset, double timeout_s) {
  if (e.world == 1) return coll::unique_id();
  const int port = e.port + port_offset;
  const auto t0 = std::chrono::steady_clock::now();
  auto expired = [&] {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s;
  };
  if (e.rank == 0) {
    const std::string id = coll::unique_id();
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) throw std::runtime_error("dist: socket failed");
    const int one = 1;
    ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    a.sin_port = htons((uint16_t)port);
    if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || ::listen(fd, e.world) != 0) {
      ::close(fd);
      throw std::runtime_error("dist: rank 0 cannot listen on port " + std::to_string(port));
    }
    for (int served = 1; served < e.world; ++served) {
      const int c = ::accept(fd, nullptr, nullptr);
      if (c < 0) {
        ::close(fd);
        throw std::runtime_error("dist: accept failed");
      }
      send_all(c, id.data(), id.size());
      ::close(c);
    }
    ::close(fd);
    return id;
  }
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(e.addr.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("dist: cannot resolve " + e.addr);
  std::string id(128, '\0');
  while (true) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      recv_all(fd, &id[0], id.size());
      ::close(fd);
      break;
    }
    if (fd >= 0) ::close(fd);
    if (expired()) {
      ::freeaddrinfo(res);
      throw std::runtime_error("dist: no rank 0 at " + e.addr + ":" + std::to_string(port));
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  ::freeaddrinfo(res);
  return id;
}

DataParallel::DataParallel(const Env& e, int port_offset) : env_(e) {
  if (!coll::available()) throw std::runtime_error("dist: RCCL unavailable: " + coll::load_error());
  gpu::set_device(e.local_rank);
  const std::string id = exchange_unique_id(e, port_offset);
  comm_ = std::make_unique<coll::Comm>(id, e.world, e.rank, e.local_rank);
  scratch_ = Tensor::zeros({1}, DType::F32, Device::gpu(e.local_rank));
}

DataParallel::~DataParallel() {
  try {
    if (flow_) gpu::flow_synchronize(flow_);
    if (ev_) gpu::event_destroy(ev_);
    if (flow_) gpu::flow_destroy(flow_);
  } catch (...) {
  }
}

void DataParallel::all_reduce_mean(float* data, size_t n) {
  if (n == 0) return;
  comm_->all_reduce(data, data, n, 0, 4, gpu::flow());  // fp32, average (world 1 too: one code path)
}

void DataParallel::attach(Sequential& model, double bucket_mb) {
  const auto params = model.parameters();
  if (params.empty() || !params[0]->arena) throw std::runtime_error("DataParallel::attach: no GPU parameter arena");
  ParamArena* a = params[0]->arena.get();
  g_ = a->grad.ptr<float>();
  n_ = (size_t)a->grad.numel();
  bucket_elems_ = (size_t)(bucket_mb * (1 << 20) / sizeof(float));
  if (bucket_elems_ < 1) bucket_elems_ = 1;
  lo_.clear();
  for (const auto& l : model.layers()) {
    size_t lo = SIZE_MAX;
    std::vector<Param*> ps;
    l->collect_params(ps);
    for (Param* p : ps) {
      if (p->arena.get() != a) throw std::runtime_error("DataParallel::attach: parameters outside the arena");
      lo = std::min(lo, (size_t)(p->grad.ptr<float>() - g_));
    }
    lo_.push_back(lo);
  }
  // the backward completes layers last to first: the suffix from a layer's first element is final
  // only if the arena holds the layers in order
  size_t prev = 0;
  for (size_t lo : lo_) {
    if (lo == SIZE_MAX) continue;
    if (lo < prev) throw std::runtime_error("DataParallel::attach: arena not in layer order");
    prev = lo;
  }
  if (!flow_) flow_ = gpu::flow_create();
  if (!ev_) ev_ = gpu::event_create();
  reduced_lo_ = n_;
  nb_ = 0;
  model.set_backward_hook([this](size_t i) { on_layer_done(i); });
}

void DataParallel::fork_bucket(size_t lo, size_t hi) {
  gpu_ops::flush_deferred_reduce();  // the bucket's weight gradients are summed first
  gpu::event_record(ev_);            // (the compute flow up to here)
  gpu::flow_wait(flow_, ev_);
  comm_->all_reduce(g_ + lo, g_ + lo, hi - lo, 0, 4, flow_);
  ++nb_;
}

void DataParallel::on_layer_done(size_t layer) {
  if (!g_ || layer >= lo_.size()) return;
  // the final suffix: from the first element of the lowest layer done so far that has parameters
  size_t lo = SIZE_MAX;
  for (size_t j = layer; j < lo_.size(); ++j) lo = std::min(lo, lo_[j]);
  if (lo == SIZE_MAX || lo >= reduced_lo_) return;
  if (reduced_lo_ - lo < bucket_elems_) return;
  fork_bucket(lo, reduced_lo_);
  reduced_lo_ = lo;
}

void DataParallel::finish() {
  if (!g_) {
    throw std::runtime_error("DataParallel::finish: attach() first");
  }
  if (reduced_lo_ > 0) fork_bucket(0, reduced_lo_);
  gpu::event_record(ev_, flow_);  // join: the optimizer reads every bucket's mean
  gpu::flow_wait(gpu::flow(), ev_);
  nb_last_ = nb_;
  nb_ = 0;
  reduced_lo_ = n_;
}

double DataParallel::max(double v) {
  float f = (float)v;
  gpu::copy(scratch_.data(), &f, sizeof f, 0);
  comm_->all_reduce(scratch_.data(), scratch_.data(), 1, 0, 2, gpu::flow());
  gpu::copy(&f, scratch_.data(), sizeof f, 1);
  return f;
}

P2PLink::P2PLink(const std::string& unique_id, int rank, bool sender, int device) : sender_(sender) {
  if (!coll::available()) throw std::runtime_error("dist: RCCL unavailable: " + coll::load_error());
  if (rank != 0 && rank != 1) throw std::invalid_argument("P2PLink: rank 0 or 1");
  gpu::set_device(device);
  peer_ = 1 - rank;
  comm_ = std::make_unique<coll::Comm>(unique_id, 2, rank, device);
  flow_ = gpu::flow_create();
  ready_ = gpu::event_create();
  done_ = gpu::event_create();
}

P2PLink::~P2PLink() {
  try {
    drain();
  } catch (...) {
  }
  for (auto& kv : held_)
    if (kv.second.ev) gpu::event_destroy(kv.second.ev);
  if (ready_) gpu::event_destroy(ready_);
  if (done_) gpu::event_destroy(done_);
  comm_.reset();
  if (flow_) gpu::flow_destroy(flow_);
}

void P2PLink::send(const Tensor& t, uint64_t key) {
  if (!sender_) throw std::logic_error("P2PLink: receive-only link");
  if (!t.device().is_gpu()) throw std::invalid_argument("P2PLink: device tensors only");
  Held& h = held_[key];
  if (h.ev) gpu::event_synchronize(h.ev);  // the slot's previous send has completed
  else h.ev = gpu::event_create();
  gpu::event_record(ready_);  // (current flow)
  gpu::flow_wait(flow_, ready_);
  comm_->send(t.data(), t.nbytes(), 4, peer_, flow_);  // bytes (uint8)
  gpu::event_record(h.ev, flow_);
  h.t = t;
}

Tensor P2PLink::recv(const std::vector<int64_t>& shape, DType dt, Layout layout, Device dev) {
  if (sender_) throw std::logic_error("P2PLink: send-only link");
  // the buffer comes from the current flow's cache: the link flow starts after that flow's work
  // so far (a recycled block's last reader), and the current flow continues after the receive
  Tensor t = Tensor::empty(shape, dt, dev, layout);
  gpu::event_record(ready_);
  gpu::flow_wait(flow_, ready_);
  comm_->recv(t.data(), t.nbytes(), 4, peer_, flow_);
  gpu::event_record(done_, flow_);
  gpu::flow_wait(gpu::flow(), done_);
  return t;
}

void P2PLink::drain() {
  for (auto& kv : held_) {
    if (kv.second.ev) gpu::event_synchronize(kv.second.ev);
    kv.second.t = Tensor();
  }
}

Tensor P2PLink::loopback(const Tensor& t) {
  if (!coll::available()) throw std::runtime_error("dist: RCCL unavailable: " + coll::load_error());
  if (!t.device().is_gpu()) throw std::invalid_argument("P2PLink: device tensors only");
  P2PLink l;
  l.comm_ = std::make_unique<coll::Comm>(coll::unique_id(), 1, 0, t.device().index);
  l.flow_ = gpu::flow_create();
  l.ready_ = gpu::event_create();
  l.done_ = gpu::event_create();
  Tensor out = Tensor::empty(t.shape(), t.dtype(), t.device(), t.layout());
  gpu::event_record(l.ready_);
  gpu::flow_wait(l.flow_, l.ready_);
  coll::group_start();  // (a rank's send to itself and its receive must be one group)
  l.comm_->send(t.data(), t.nbytes(), 4, 0, l.flow_);
  l.comm_->recv(out.data(), out.nbytes(), 4, 0, l.flow_);
  coll::group_end();
  gpu::event_record(l.done_, l.flow_);
  gpu::flow_wait(gpu::flow(), l.done_);
  gpu::flow_synchronize(l.flow_);  // (the link and its flow go away here)
  return out;
}

}  // namespace dist
}  // namespace dcnn
