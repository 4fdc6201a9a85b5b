// Data parallelism of the C++ host API (dcnn/dist.hpp): RCCL rendezvous, the host TCP ring of
// the CPU device, the bucketed gradient mean and the pipeline's device links.
#include "dcnn/dist.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
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
using Clock = std::chrono::steady_clock;

int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}
double seconds_since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }
// milliseconds left of a timeout_s wait that started at t0 (>= 0)
int ms_left(Clock::time_point t0, double timeout_s) {
  const double left = timeout_s - seconds_since(t0);
  return left <= 0 ? 0 : (int)std::min(left * 1e3 + 1, 2e9);
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
void no_delay(int fd) {
  const int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

// listening socket on `port` (0: an ephemeral one; *bound = the port it got)
int listen_on(int port, int backlog, int* bound = nullptr) {
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) throw std::runtime_error("dist: socket failed");
  const int one = 1;
  ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons((uint16_t)port);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || ::listen(fd, backlog) != 0) {
    ::close(fd);
    throw std::runtime_error("dist: cannot listen on port " + std::to_string(port));
  }
  if (bound) {
    socklen_t len = sizeof a;
    ::getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
    *bound = ntohs(a.sin_port);
  }
  return fd;
}

// one connection from `lfd`, or an error once the wait that started at t0 exceeds timeout_s
int accept_until(int lfd, Clock::time_point t0, double timeout_s, const std::string& what) {
  while (true) {
    pollfd p{lfd, POLLIN, 0};
    const int r = ::poll(&p, 1, ms_left(t0, timeout_s));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0)
      throw std::runtime_error("dist: timed out after " + std::to_string((int)timeout_s) + " s waiting for " + what);
    const int c = ::accept(lfd, nullptr, nullptr);
    if (c >= 0) return c;
    if (errno != EINTR && errno != ECONNABORTED) throw std::runtime_error("dist: accept failed");
  }
}

// a connection to host:port, retried until the wait that started at t0 exceeds timeout_s
int connect_until(const std::string& host, int port, Clock::time_point t0, double timeout_s, const std::string& what) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("dist: cannot resolve " + host);
  while (true) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      ::freeaddrinfo(res);
      return fd;
    }
    if (fd >= 0) ::close(fd);
    if (seconds_since(t0) > timeout_s) {
      ::freeaddrinfo(res);
      throw std::runtime_error("dist: timed out after " + std::to_string((int)timeout_s) + " s connecting to " + what +
                               " at " + host + ":" + std::to_string(port));
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
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
  if (const char* t = std::getenv("DCNN_DIST_TIMEOUT"))
    if (*t) e.timeout_s = std::atof(t);
  if (e.world < 1 || e.rank < 0 || e.rank >= e.world) throw std::invalid_argument("dist: bad RANK / WORLD_SIZE");
  if (!(e.timeout_s > 0)) throw std::invalid_argument("dist: DCNN_DIST_TIMEOUT must be > 0");
  return e;
}

std::string exchange_unique_id(const Env& e, int port_offset) {
  if (e.world == 1) return coll::unique_id();
  const int port = e.port + port_offset;
  const auto t0 = Clock::now();
  if (e.rank == 0) {
    const std::string id = coll::unique_id();
    const int fd = listen_on(port, e.world);
    try {
      for (int served = 1; served < e.world; ++served) {
        const int c = accept_until(fd, t0, e.timeout_s,
                                   "rank " + std::to_string(served) + " of " + std::to_string(e.world - 1) +
                                       " other ranks (port " + std::to_string(port) + ")");
        try {
          send_all(c, id.data(), id.size());
        } catch (...) {
          ::close(c);
          throw;
        }
        ::close(c);
      }
    } catch (...) {
      ::close(fd);
      throw;
    }
    ::close(fd);
    return id;
  }
  const int fd = connect_until(e.addr, port, t0, e.timeout_s, "rank 0");
  std::string id(128, '\0');
  try {
    recv_all(fd, &id[0], id.size());
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
  return id;
}

// ------------------------------------------------------------------ HostRing
HostRing::HostRing(const Env& e, int port_offset) : rank_(e.rank), world_(e.world), timeout_s_(e.timeout_s) {
  if (world_ == 1) return;
  const auto t0 = Clock::now();
  int my_port = 0;
  const int lfd = listen_on(0, 4, &my_port);
  // rendezvous: every rank's (IPv4, port) at rank 0, the table back to everyone
  std::vector<uint32_t> table((size_t)world_ * 2, 0);
  try {
    if (rank_ == 0) {
      const int cfd = listen_on(e.port + port_offset, world_);
      std::vector<int> conns;
      try {
        for (int k = 1; k < world_; ++k) {
          const int c = accept_until(cfd, t0, timeout_s_,
                                     "the host ring's rank " + std::to_string(k) + " of " + std::to_string(world_ - 1) +
                                         " other ranks (port " + std::to_string(e.port + port_offset) + ")");
          conns.push_back(c);
          int32_t hello[2];
          recv_all(c, reinterpret_cast<char*>(hello), sizeof hello);
          if (hello[0] <= 0 || hello[0] >= world_ || table[2 * hello[0] + 1]) throw std::runtime_error("dist: bad host-ring hello");
          sockaddr_in peer{};
          socklen_t len = sizeof peer;
          ::getpeername(c, reinterpret_cast<sockaddr*>(&peer), &len);
          table[2 * hello[0]] = peer.sin_addr.s_addr;
          table[2 * hello[0] + 1] = (uint32_t)hello[1];
          if (k == 1) {  // rank 0's own address as its peers reach it
            sockaddr_in self{};
            len = sizeof self;
            ::getsockname(c, reinterpret_cast<sockaddr*>(&self), &len);
            table[0] = self.sin_addr.s_addr;
            table[1] = (uint32_t)my_port;
          }
        }
        for (int c : conns) send_all(c, reinterpret_cast<const char*>(table.data()), table.size() * 4);
      } catch (...) {
        for (int c : conns) ::close(c);
        ::close(cfd);
        throw;
      }
      for (int c : conns) ::close(c);
      ::close(cfd);
    } else {
      const int c = connect_until(e.addr, e.port + port_offset, t0, timeout_s_, "the host ring's rank 0");
      try {
        const int32_t hello[2] = {rank_, my_port};
        send_all(c, reinterpret_cast<const char*>(hello), sizeof hello);
        recv_all(c, reinterpret_cast<char*>(table.data()), table.size() * 4);
      } catch (...) {
        ::close(c);
        throw;
      }
      ::close(c);
    }
    // the ring: connect to the successor (its listener exists already), accept the predecessor
    const int nx = (rank_ + 1) % world_;
    char ip[INET_ADDRSTRLEN] = {0};
    in_addr ia{};
    ia.s_addr = table[2 * nx];
    ::inet_ntop(AF_INET, &ia, ip, sizeof ip);
    next_ = connect_until(ip, (int)table[2 * nx + 1], t0, timeout_s_, "host-ring rank " + std::to_string(nx));
    const int32_t me = rank_;
    send_all(next_, reinterpret_cast<const char*>(&me), sizeof me);
    prev_ = accept_until(lfd, t0, timeout_s_, "host-ring rank " + std::to_string((rank_ + world_ - 1) % world_));
    int32_t who = -1;
    recv_all(prev_, reinterpret_cast<char*>(&who), sizeof who);
    if (who != (rank_ + world_ - 1) % world_) throw std::runtime_error("dist: host ring wired to the wrong rank");
    no_delay(next_);
    no_delay(prev_);
  } catch (...) {
    ::close(lfd);
    if (next_ >= 0) ::close(next_);
    if (prev_ >= 0) ::close(prev_);
    next_ = prev_ = -1;
    throw;
  }
  ::close(lfd);
}

HostRing::~HostRing() {
  if (next_ >= 0) ::close(next_);
  if (prev_ >= 0) ::close(prev_);
}

void HostRing::exchange(const char* s, size_t sn, char* r, size_t rn) {
  size_t sent = 0, got = 0;
  while (sent < sn || got < rn) {
    pollfd p[2];
    int k = 0, is = -1, ir = -1;
    if (sent < sn) {
      p[k] = {next_, POLLOUT, 0};
      is = k++;
    }
    if (got < rn) {
      p[k] = {prev_, POLLIN, 0};
      ir = k++;
    }
    const int n = ::poll(p, (nfds_t)k, (int)std::min(timeout_s_ * 1e3, 2e9));
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) throw std::runtime_error("dist: host ring timed out (a peer rank stopped)");
    if (is >= 0 && (p[is].revents & (POLLOUT | POLLERR | POLLHUP))) {
      const ssize_t m = ::send(next_, s + sent, sn - sent, MSG_NOSIGNAL | MSG_DONTWAIT);
      if (m > 0) sent += (size_t)m;
      else if (m < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
        throw std::runtime_error("dist: host ring send failed");
    }
    if (ir >= 0 && (p[ir].revents & (POLLIN | POLLERR | POLLHUP))) {
      const ssize_t m = ::recv(prev_, r + got, rn - got, MSG_DONTWAIT);
      if (m > 0) got += (size_t)m;
      else if (m == 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR))
        throw std::runtime_error("dist: host ring peer closed the connection");
    }
  }
}

void HostRing::all_reduce(float* x, size_t n, Op op) {
  if (world_ == 1 || n == 0) return;
  const size_t W = (size_t)world_, r = (size_t)rank_;
  auto lo = [&](size_t c) { return c * n / W; };
  auto len = [&](size_t c) { return lo(c + 1) - lo(c); };
  std::vector<float> tmp(n / W + 1);
  // reduce-scatter: after W - 1 steps rank r holds the complete chunk (r + 1) mod W, summed in the
  // fixed ring order starting at the chunk's own rank
  for (size_t s = 0; s + 1 < W; ++s) {
    const size_t cs = (r + W - s) % W, cr = (r + 2 * W - s - 1) % W;
    exchange(reinterpret_cast<const char*>(x + lo(cs)), len(cs) * 4, reinterpret_cast<char*>(tmp.data()), len(cr) * 4);
    float* d = x + lo(cr);
    const size_t m = len(cr);
    if (op == kSum)
      for (size_t i = 0; i < m; ++i) d[i] += tmp[i];
    else
      for (size_t i = 0; i < m; ++i) d[i] = std::max(d[i], tmp[i]);
  }
  // all-gather of the complete chunks
  for (size_t s = 0; s + 1 < W; ++s) {
    const size_t cs = (r + 1 + W - s) % W, cr = (r + W - s) % W;
    exchange(reinterpret_cast<const char*>(x + lo(cs)), len(cs) * 4, reinterpret_cast<char*>(x + lo(cr)), len(cr) * 4);
  }
}

void HostRing::broadcast(void* x, size_t nbytes, int root) {
  if (world_ == 1 || nbytes == 0) return;
  if (rank_ != root) exchange(nullptr, 0, static_cast<char*>(x), nbytes);
  if ((rank_ + 1) % world_ != root) exchange(static_cast<const char*>(x), nbytes, nullptr, 0);
}

void HostRing::barrier() {
  float z = 0.f;
  all_reduce(&z, 1);
}

// ------------------------------------------------------------------ DataParallel
DataParallel::DataParallel(const Env& e, Device dev, int port_offset) : env_(e), dev_(dev) {
  if (dev.is_gpu()) {
    if (!coll::available()) throw std::runtime_error("dist: RCCL unavailable: " + coll::load_error());
    dev_ = Device::gpu(e.local_rank);
    gpu::set_device(e.local_rank);
    const std::string id = exchange_unique_id(e, port_offset);
    comm_ = std::make_unique<coll::Comm>(id, e.world, e.rank, e.local_rank);
    scratch_ = Tensor::zeros({1}, DType::F32, dev_);
  } else {
    ring_ = std::make_unique<HostRing>(e, port_offset);
  }
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
  if (comm_) {
    comm_->all_reduce(data, data, n, 0, 4, gpu::flow());  // fp32, average (world 1 too: one code path)
    return;
  }
  ring_->all_reduce(data, n);
  if (env_.world > 1) {
    const float s = 1.f / (float)env_.world;
    for (size_t i = 0; i < n; ++i) data[i] *= s;
  }
}

double DataParallel::max(double v) {
  float f = (float)v;
  if (ring_) {
    ring_->all_reduce(&f, 1, HostRing::kMax);
    return f;
  }
  gpu::copy(scratch_.data(), &f, sizeof f, 0);
  comm_->all_reduce(scratch_.data(), scratch_.data(), 1, 0, 2, gpu::flow());
  gpu::copy(&f, scratch_.data(), sizeof f, 1);
  return f;
}

void DataParallel::barrier() {
  if (ring_) {
    ring_->barrier();
    return;
  }
  comm_->all_reduce(scratch_.data(), scratch_.data(), 1, 0, 2, gpu::flow());
  gpu::flow_synchronize();
}

void DataParallel::broadcast_parameters(Sequential& model) {
  std::vector<Tensor*> ts;  // fp32 tensors to broadcast
  const auto params = model.parameters();
  ParamArena* a = params.empty() ? nullptr : params[0]->arena.get();
  if (!a)
    for (Param* p : params) ts.push_back(&p->value);
  for (BatchNorm* bn : model.batchnorms()) {
    if (bn->running_mean.defined()) ts.push_back(&bn->running_mean);
    if (bn->running_var.defined()) ts.push_back(&bn->running_var);
  }
  for (Tensor* t : ts)
    if (t->dtype() != DType::F32) throw std::runtime_error("DataParallel::broadcast_parameters: fp32 tensors only");
  if (ring_) {
    for (Tensor* t : ts) ring_->broadcast(t->data(), t->nbytes());
    return;
  }
  if (a) {
    comm_->broadcast(a->value.data(), a->value.data(), (size_t)a->value.numel(), 0, 0, gpu::flow());
    comm_->broadcast(a->shadow.data(), a->shadow.data(), (size_t)a->shadow.numel(), 1, 0, gpu::flow());
  }
  for (Tensor* t : ts) comm_->broadcast(t->data(), t->data(), (size_t)t->numel(), 0, 0, gpu::flow());
  if (a) a->refresh_transposes();
  else
    for (auto& l : model.layers()) l->sync_shadow();
  gpu::flow_synchronize();
}

void DataParallel::attach(Sequential& model, double bucket_mb) {
  const auto params = model.parameters();
  if (params.empty()) throw std::runtime_error("DataParallel::attach: the model has no parameters");
  bucket_elems_ = (size_t)(bucket_mb * (1 << 20) / sizeof(float));
  if (bucket_elems_ < 1) bucket_elems_ = 1;
  lo_.clear();
  segs_.clear();
  layer_elems_.clear();
  ParamArena* a = nullptr;
  if (comm_) {
    if (!params[0]->arena) throw std::runtime_error("DataParallel::attach: no GPU parameter arena");
    a = params[0]->arena.get();
    g_ = a->grad.ptr<float>();
    n_ = (size_t)a->grad.numel();
  }
  for (const auto& l : model.layers()) {
    size_t lo = SIZE_MAX, elems = 0;
    std::vector<Param*> ps;
    l->collect_params(ps);
    std::vector<std::pair<float*, size_t>> seg;
    for (Param* p : ps) {
      elems += (size_t)p->grad.numel();
      if (a) {
        if (p->arena.get() != a) throw std::runtime_error("DataParallel::attach: parameters outside the arena");
        lo = std::min(lo, (size_t)(p->grad.ptr<float>() - g_));
      } else {
        if (p->grad.device().is_gpu()) throw std::runtime_error("DataParallel::attach: device mismatch");
        seg.emplace_back(p->grad.ptr<float>(), (size_t)p->grad.numel());
      }
    }
    lo_.push_back(lo);
    segs_.push_back(std::move(seg));
    layer_elems_.push_back(elems);
  }
  if (a) {
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
  }
  reduced_lo_ = n_;
  next_ = lo_.size();
  nb_ = 0;
  model.set_backward_hook([this](size_t i) { on_layer_done(i); });
}

void DataParallel::reduce_layers(size_t lo_layer, size_t hi_layer) {
  if (comm_) {
    size_t lo = SIZE_MAX;
    for (size_t j = lo_layer; j < hi_layer; ++j) lo = std::min(lo, lo_[j]);
    if (lo == SIZE_MAX || lo >= reduced_lo_) return;
    gpu_ops::flush_deferred_reduce();  // the bucket's weight gradients are summed first
    gpu::event_record(ev_);            // (the compute flow up to here)
    gpu::flow_wait(flow_, ev_);
    comm_->all_reduce(g_ + lo, g_ + lo, reduced_lo_ - lo, 0, 4, flow_);
    reduced_lo_ = lo;
    ++nb_;
    return;
  }
  size_t total = 0;
  for (size_t j = lo_layer; j < hi_layer; ++j) total += layer_elems_[j];
  if (total == 0) return;
  pack_.resize(total);
  size_t o = 0;
  for (size_t j = lo_layer; j < hi_layer; ++j)
    for (const auto& s : segs_[j]) {
      std::memcpy(pack_.data() + o, s.first, s.second * 4);
      o += s.second;
    }
  all_reduce_mean(pack_.data(), total);
  o = 0;
  for (size_t j = lo_layer; j < hi_layer; ++j)
    for (const auto& s : segs_[j]) {
      std::memcpy(s.first, pack_.data() + o, s.second * 4);
      o += s.second;
    }
  ++nb_;
}

void DataParallel::on_layer_done(size_t layer) {
  if (lo_.empty() || layer >= next_) return;
  size_t pending = 0;
  for (size_t j = layer; j < next_; ++j) pending += layer_elems_[j];
  if (pending == 0 || pending < bucket_elems_) return;
  reduce_layers(layer, next_);
  next_ = layer;
}

void DataParallel::finish() {
  if (lo_.empty()) throw std::runtime_error("DataParallel::finish: attach() first");
  if (next_ > 0) reduce_layers(0, next_);
  if (comm_) {
    gpu::event_record(ev_, flow_);  // join: the optimizer reads every bucket's mean
    gpu::flow_wait(gpu::flow(), ev_);
  }
  nb_last_ = nb_;
  nb_ = 0;
  reduced_lo_ = n_;
  next_ = lo_.size();
}

P2PLink::P2PLink(const std::string& unique_id, int rank, bool sender, int device) : sender_(sender) {
  if (!coll::available()) throw std::runtime_error("dist: RCCL unavailable: " + coll::load_error());
  if (rank != 0 && rank != 1) throw std::invalid_argument("P2PLink: rank 0 or 1");
  gpu::set_device(device);
  peer_ = 1 - rank;
  comm_ = std::make_shared<coll::Comm>(unique_id, 2, rank, device);
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
  // (inside a group the send is enqueued at the group's end: the record follows it there)
  coll::after_group([ev = h.ev, fl = flow_] { gpu::event_record(ev, fl); });
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
  coll::after_group([this] {
    gpu::event_record(done_, flow_);
    gpu::flow_wait(gpu::flow(), done_);
  });
  return t;
}

void P2PLink::drain() {
  for (auto& kv : held_) {
    if (kv.second.ev) gpu::event_synchronize(kv.second.ev);
    kv.second.t = Tensor();
  }
}

std::pair<std::unique_ptr<P2PLink>, std::unique_ptr<P2PLink>> P2PLink::self_pair(int device) {
  if (!coll::available()) throw std::runtime_error("dist: RCCL unavailable: " + coll::load_error());
  gpu::set_device(device);
  auto comm = std::make_shared<coll::Comm>(coll::unique_id(), 1, 0, device);
  std::unique_ptr<P2PLink> tx(new P2PLink()), rx(new P2PLink());
  for (P2PLink* l : {tx.get(), rx.get()}) {
    l->comm_ = comm;
    l->peer_ = 0;
    l->flow_ = gpu::flow_create();
    l->ready_ = gpu::event_create();
    l->done_ = gpu::event_create();
  }
  tx->sender_ = true;
  return {std::move(tx), std::move(rx)};
}

Tensor P2PLink::loopback(const Tensor& t) {
  if (!coll::available()) throw std::runtime_error("dist: RCCL unavailable: " + coll::load_error());
  if (!t.device().is_gpu()) throw std::invalid_argument("P2PLink: device tensors only");
  P2PLink l;
  l.comm_ = std::make_shared<coll::Comm>(coll::unique_id(), 1, 0, t.device().index);
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
