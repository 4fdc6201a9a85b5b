// Control plane implementation (see comm.h).  Reference behaviour studied:
// include/pipeline/tcp_communicator.hpp:29-546 (asio; per-peer write queue, io threads),
// include/pipeline/communicator.hpp:27-169 (priority input queues), in_process_communicator.hpp.
// This implementation uses plain POSIX sockets + std::thread: one blocking reader per
// connection (a stage has at most 3 peers), synchronous writev for sends.
#include "comm.h"

#include <arpa/inet.h>
#include <dlfcn.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>
#include <zlib.h>

#include <chrono>
#include <cstring>
#include <stdexcept>

namespace dcnn_native {

static const char* kNames[] = {
    "_START", "FORWARD_JOB", "BACKWARD_JOB", "UPDATE_PARAMETERS", "TRAIN_MODE", "EVAL_MODE", "SHUTDOWN",
    "CONFIG_TRANSFER", "CONFIG_RECEIVED", "LOAD_PARAMS", "PARAMS_LOADED", "SEND_PARAMS", "PARAMS_TRANSFER",
    "STATUS_REQUEST", "STATUS_RESPONSE", "PARAMETERS_UPDATED", "HEALTH_CHECK", "ERROR_REPORT", "JOB_FAILURE",
    "BARRIER_SYNC", "CHECKPOINT_REQUEST", "CHECKPOINT_COMPLETE", "UPDATE_LOAD", "REPORT_LOAD", "LOAD_REPORT",
    "PRINT_PROFILING", "PROFILING_PRINTED", "CLEAR_PROFILING", "PROFILING_CLEARED", "LABELS_TRANSFER",
    "P2P_CONNECT"};
static_assert(sizeof(kNames) / sizeof(kNames[0]) == CMD_COUNT, "command table");

const char* command_name(uint16_t c) { return c < CMD_COUNT ? kNames[c] : "UNKNOWN"; }

// ------------------------------------------------------------------ serialisation
namespace {
inline bool host_little() {
  const uint16_t x = 1;
  return *reinterpret_cast<const uint8_t*>(&x) == 1;
}
template <typename T>
inline void put(std::string& o, T v) {
  o.append(reinterpret_cast<const char*>(&v), sizeof(T));
}
inline void put_str(std::string& o, const std::string& s) {
  put<uint64_t>(o, s.size());
  o.append(s);
}
template <typename T>
inline T bswap_t(T v) {
  T r;
  auto* a = reinterpret_cast<uint8_t*>(&v);
  auto* b = reinterpret_cast<uint8_t*>(&r);
  for (size_t i = 0; i < sizeof(T); ++i) b[i] = a[sizeof(T) - 1 - i];
  return r;
}
struct Reader {
  const char* p;
  size_t n, off = 0;
  bool swap;
  void need(size_t k) {
    if (off + k > n) throw std::runtime_error("truncated message");
  }
  template <typename T>
  T get() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, p + off, sizeof(T));
    off += sizeof(T);
    return swap ? bswap_t(v) : v;
  }
  std::string bytes(size_t k) {
    need(k);
    std::string s(p + off, k);
    off += k;
    return s;
  }
  std::string str() { return bytes(get<uint64_t>()); }
};
size_t elem_size(uint8_t dt) {
  switch (dt) {
    case 0: return 4;
    case 1: case 2: return 2;
    case 3: return 8;
    default: return 1;
  }
}
}  // namespace

size_t Message::body_size() const {
  size_t s = 8 + recipient.size() + 8 + sender.size() + 2 + 8;
  switch (payload_type) {
    case P_JOB: s += 16 + 8 * shape.size() + data.size(); break;
    case P_STRING: s += 8 + text.size(); break;
    case P_BOOL: s += 1; break;
    case P_LOAD: s += 16; break;
    case P_TYPED_JOB: s += 8 + 2 + 8 + 8 * shape.size() + 8 + data.size(); break;
    default: break;
  }
  return s;
}

static void serialize_meta(const Message& m, std::string& o) {
  // everything of the body except the trailing raw tensor bytes
  put_str(o, m.recipient);
  put_str(o, m.sender);
  put<uint16_t>(o, m.command);
  put<uint64_t>(o, m.payload_type);
  switch (m.payload_type) {
    case P_NONE: break;
    case P_JOB:
      put<uint64_t>(o, m.mb_id);
      put<uint64_t>(o, m.shape.size());
      for (auto d : m.shape) put<uint64_t>(o, d);
      break;
    case P_STRING: put_str(o, m.text); break;
    case P_BOOL: put<uint8_t>(o, m.flag ? 1 : 0); break;
    case P_LOAD:
      put<float>(o, m.load.avg_forward_ms);
      put<float>(o, m.load.avg_backward_ms);
      put<float>(o, m.load.avg_cpu_utilization);
      put<float>(o, m.load.max_memory_mb);
      break;
    case P_TYPED_JOB:
      put<uint64_t>(o, m.mb_id);
      put<uint8_t>(o, m.dtype);
      put<uint8_t>(o, m.codec);
      put<uint64_t>(o, m.shape.size());
      for (auto d : m.shape) put<uint64_t>(o, d);
      put<uint64_t>(o, m.data.size());
      break;
    default: throw std::runtime_error("unsupported payload type");
  }
}

static bool has_raw(const Message& m) { return m.payload_type == P_JOB || m.payload_type == P_TYPED_JOB; }

void serialize_body(const Message& m, std::string& o) {
  serialize_meta(m, o);
  if (has_raw(m)) o.append(m.data);
}

std::string serialize(const Message& m) {
  std::string body;
  body.reserve(m.body_size());
  serialize_body(m, body);
  std::string o;
  o.reserve(kFixedHeader + body.size());
  put<uint8_t>(o, 1);
  put<uint8_t>(o, host_little() ? 1 : 0);
  put<uint64_t>(o, body.size());
  o.append(body);
  return o;
}

Message deserialize_body(const char* p, size_t n, bool swap) {
  Reader r{p, n, 0, swap};
  Message m;
  m.recipient = r.str();
  m.sender = r.str();
  m.command = r.get<uint16_t>();
  m.payload_type = r.get<uint64_t>();
  switch (m.payload_type) {
    case P_NONE: break;
    case P_JOB: {
      m.mb_id = r.get<uint64_t>();
      const uint64_t nd = r.get<uint64_t>();
      if (nd > 16) throw std::runtime_error("bad tensor rank");
      uint64_t cnt = 1;
      for (uint64_t i = 0; i < nd; ++i) {
        m.shape.push_back(r.get<uint64_t>());
        cnt *= m.shape.back();
      }
      m.dtype = 0;
      m.data = r.bytes(cnt * 4);
      if (swap) {
        auto* f = reinterpret_cast<uint32_t*>(&m.data[0]);
        for (uint64_t i = 0; i < cnt; ++i) f[i] = bswap_t(f[i]);
      }
      break;
    }
    case P_STRING: m.text = r.str(); break;
    case P_BOOL: m.flag = r.get<uint8_t>() != 0; break;
    case P_LOAD:
      m.load.avg_forward_ms = r.get<float>();
      m.load.avg_backward_ms = r.get<float>();
      m.load.avg_cpu_utilization = r.get<float>();
      m.load.max_memory_mb = r.get<float>();
      break;
    case P_TYPED_JOB: {
      m.mb_id = r.get<uint64_t>();
      m.dtype = r.get<uint8_t>();
      m.codec = r.get<uint8_t>();
      const uint64_t nd = r.get<uint64_t>();
      if (nd > 16) throw std::runtime_error("bad tensor rank");
      for (uint64_t i = 0; i < nd; ++i) m.shape.push_back(r.get<uint64_t>());
      m.data = r.bytes(r.get<uint64_t>());
      if (swap && m.codec == CODEC_NONE) throw std::runtime_error("typed job across endianness unsupported");
      break;
    }
    default: throw std::runtime_error("unsupported payload type " + std::to_string(m.payload_type));
  }
  (void)elem_size;
  return m;
}

Message deserialize(const std::string& f) {
  if (f.size() < kFixedHeader) throw std::runtime_error("frame too short");
  const uint8_t ver = static_cast<uint8_t>(f[0]);
  if (ver != 1) throw std::runtime_error("unsupported protocol version");
  const bool swap = (static_cast<uint8_t>(f[1]) != 0) != host_little();
  uint64_t len;
  std::memcpy(&len, f.data() + 2, 8);
  if (swap) len = bswap_t(len);
  if (len != f.size() - kFixedHeader) throw std::runtime_error("frame length mismatch");
  return deserialize_body(f.data() + kFixedHeader, len, swap);
}

// ------------------------------------------------------------------ compression
namespace {
struct Zstd {
  size_t (*compress)(void*, size_t, const void*, size_t, int) = nullptr;
  size_t (*decompress)(void*, size_t, const void*, size_t) = nullptr;
  size_t (*bound)(size_t) = nullptr;
  unsigned (*is_error)(size_t) = nullptr;
  unsigned long long (*content_size)(const void*, size_t) = nullptr;
  bool ok = false;
  Zstd() {
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    compress = reinterpret_cast<decltype(compress)>(dlsym(h, "ZSTD_compress"));
    decompress = reinterpret_cast<decltype(decompress)>(dlsym(h, "ZSTD_decompress"));
    bound = reinterpret_cast<decltype(bound)>(dlsym(h, "ZSTD_compressBound"));
    is_error = reinterpret_cast<decltype(is_error)>(dlsym(h, "ZSTD_isError"));
    content_size = reinterpret_cast<decltype(content_size)>(dlsym(h, "ZSTD_getFrameContentSize"));
    ok = compress && decompress && bound && is_error && content_size;
  }
};
Zstd& zstd() {
  static Zstd z;
  return z;
}
}  // namespace

bool zstd_available() { return zstd().ok; }

std::string compress(const std::string& in, Codec codec, int level) {
  if (codec == CODEC_NONE) return in;
  if (codec == CODEC_ZSTD) {
    auto& z = zstd();
    if (!z.ok) throw std::runtime_error("libzstd.so.1 not available");
    std::string out(z.bound(in.size()), '\0');
    size_t r = z.compress(&out[0], out.size(), in.data(), in.size(), level);
    if (z.is_error(r)) throw std::runtime_error("zstd compression failed");
    out.resize(r);
    return out;
  }
  uLongf cap = compressBound(in.size());
  std::string out(cap + 8, '\0');
  const uint64_t raw = in.size();
  std::memcpy(&out[0], &raw, 8);
  if (::compress2(reinterpret_cast<Bytef*>(&out[8]), &cap, reinterpret_cast<const Bytef*>(in.data()), in.size(),
                  level < 0 ? Z_DEFAULT_COMPRESSION : std::min(level, 9)) != Z_OK)
    throw std::runtime_error("zlib compression failed");
  out.resize(cap + 8);
  return out;
}

std::string decompress(const std::string& in, Codec codec, size_t hint) {
  if (codec == CODEC_NONE) return in;
  if (codec == CODEC_ZSTD) {
    auto& z = zstd();
    if (!z.ok) throw std::runtime_error("libzstd.so.1 not available");
    unsigned long long n = z.content_size(in.data(), in.size());
    if (n == (unsigned long long)-1 || n == (unsigned long long)-2) n = hint;
    std::string out(n, '\0');
    size_t r = z.decompress(&out[0], out.size(), in.data(), in.size());
    if (z.is_error(r)) throw std::runtime_error("zstd decompression failed");
    out.resize(r);
    return out;
  }
  if (in.size() < 8) throw std::runtime_error("zlib frame too short");
  uint64_t raw;
  std::memcpy(&raw, in.data(), 8);
  std::string out(raw, '\0');
  uLongf n = raw;
  if (::uncompress(reinterpret_cast<Bytef*>(&out[0]), &n, reinterpret_cast<const Bytef*>(in.data() + 8),
                   in.size() - 8) != Z_OK || n != raw)
    throw std::runtime_error("zlib decompression failed");
  return out;
}

// ------------------------------------------------------------------ queue
// Deadlines on system_clock: libstdc++ then waits with pthread_cond_timedwait, which
// ThreadSanitizer intercepts (its steady_clock path, pthread_cond_clockwait, is invisible to
// the GCC 11 TSan runtime and produces false double-lock reports).
static std::chrono::system_clock::time_point deadline_ms(int ms) {
  return std::chrono::system_clock::now() + std::chrono::milliseconds(ms);
}

void MessageQueue::push(Message&& m) {
  const uint16_t c = m.command < CMD_COUNT ? m.command : CMD_START;
  {
    std::lock_guard<std::mutex> g(mu_);
    q_[c].push_back(std::move(m));
    ++total_;
  }
  cv_.notify_all();
}

bool MessageQueue::pop(Message& out, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return total_ > 0 || closed_; };
  if (timeout_ms < 0)
    cv_.wait(lk, ready);
  else if (!cv_.wait_until(lk, deadline_ms(timeout_ms), ready))
    return false;
  if (total_ == 0) return false;
  for (int c = 0; c < CMD_COUNT; ++c) {
    if (!q_[c].empty()) {
      out = std::move(q_[c].front());
      q_[c].pop_front();
      --total_;
      return true;
    }
  }
  return false;
}

bool MessageQueue::pop_command(uint16_t cmd, Message& out, int timeout_ms) {
  if (cmd >= CMD_COUNT) return false;
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return !q_[cmd].empty() || closed_; };
  if (timeout_ms < 0)
    cv_.wait(lk, ready);
  else if (!cv_.wait_until(lk, deadline_ms(timeout_ms), ready))
    return false;
  if (q_[cmd].empty()) return false;
  out = std::move(q_[cmd].front());
  q_[cmd].pop_front();
  --total_;
  return true;
}

bool MessageQueue::pop_any(const std::vector<uint16_t>& cmds, Message& out, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] {
    if (closed_) return true;
    for (uint16_t c : cmds)
      if (c < CMD_COUNT && !q_[c].empty()) return true;
    return false;
  };
  if (timeout_ms < 0)
    cv_.wait(lk, ready);
  else if (!cv_.wait_until(lk, deadline_ms(timeout_ms), ready))
    return false;
  uint16_t best = CMD_COUNT;
  for (uint16_t c : cmds)
    if (c < CMD_COUNT && !q_[c].empty() && c < best) best = c;
  if (best == CMD_COUNT) return false;
  out = std::move(q_[best].front());
  q_[best].pop_front();
  --total_;
  return true;
}

size_t MessageQueue::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return total_;
}

size_t MessageQueue::count(uint16_t cmd) const {
  std::lock_guard<std::mutex> g(mu_);
  return cmd < CMD_COUNT ? q_[cmd].size() : 0;
}

void MessageQueue::close() {
  closed_ = true;
  cv_.notify_all();
}

// ------------------------------------------------------------------ in-process
namespace {
std::mutex g_reg_mu;
std::map<std::string, InProcessCommunicator*>& registry() {
  static std::map<std::string, InProcessCommunicator*> r;
  return r;
}
}  // namespace

InProcessCommunicator::InProcessCommunicator(std::string id) : Communicator(std::move(id)) {
  std::lock_guard<std::mutex> g(g_reg_mu);
  if (registry().count(id_)) throw std::runtime_error("in-process communicator id already registered: " + id_);
  registry()[id_] = this;
}

InProcessCommunicator::~InProcessCommunicator() { close(); }

void InProcessCommunicator::close() {
  {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = registry().find(id_);
    if (it != registry().end() && it->second == this) registry().erase(it);
  }
  Communicator::close();
}

void InProcessCommunicator::alias(const std::string& name, const std::string& target) {
  std::lock_guard<std::mutex> g(mu_);
  alias_[name] = target;
}

std::vector<std::string> InProcessCommunicator::peers() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (auto& kv : alias_) out.push_back(kv.first);
  return out;
}

void InProcessCommunicator::send(Message&& m) {
  std::string target = m.recipient;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = alias_.find(target);
    if (it != alias_.end()) target = it->second;
  }
  m.sender = id_;
  const size_t sz = m.body_size();
  std::lock_guard<std::mutex> g(g_reg_mu);
  auto it = registry().find(target);
  if (it == registry().end()) throw std::runtime_error("in-process recipient not found: " + target);
  bytes_sent_ += sz;
  ++msgs_sent_;
  it->second->bytes_recv_ += sz;
  ++it->second->msgs_recv_;
  it->second->queue().push(std::move(m));
}

// ------------------------------------------------------------------ TCP
namespace {
bool write_all(int fd, struct iovec* iov, int cnt) {
  while (cnt > 0) {
    ssize_t w = ::writev(fd, iov, cnt);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    size_t left = static_cast<size_t>(w);
    while (cnt > 0 && left >= iov->iov_len) {
      left -= iov->iov_len;
      ++iov;
      --cnt;
    }
    if (cnt > 0) {
      iov->iov_base = static_cast<char*>(iov->iov_base) + left;
      iov->iov_len -= left;
    }
  }
  return true;
}
bool read_all(int fd, char* p, size_t n) {
  while (n > 0) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}
void tune_socket(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}
constexpr uint64_t kMaxFrame = 1ull << 36;  // 64 GiB sanity bound
}  // namespace

TcpCommunicator::TcpCommunicator(std::string id, const std::string& host, int port) : Communicator(std::move(id)) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("socket() failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (host.empty() || host == "0.0.0.0")
    a.sin_addr.s_addr = htonl(INADDR_ANY);
  else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1)
    throw std::runtime_error("bad listen address " + host);
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("bind() failed on port " + std::to_string(port) + ": " + strerror(errno));
  }
  socklen_t len = sizeof(a);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&a), &len);
  port_ = ntohs(a.sin_port);
  if (::listen(listen_fd_, 64) != 0) throw std::runtime_error("listen() failed");
  acceptor_ = std::thread([this] { accept_loop(); });
}

TcpCommunicator::~TcpCommunicator() { close(); }

void TcpCommunicator::accept_loop() {
  while (!stopping_) {
    pollfd p{listen_fd_, POLLIN, 0};
    int r = ::poll(&p, 1, 100);
    if (r <= 0) continue;
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    tune_socket(fd);
    auto c = std::make_shared<Conn>();
    c->fd = fd;
    {
      std::lock_guard<std::mutex> g(mu_);
      all_.push_back(c);
    }
    c->reader = std::thread([this, c] { reader_loop(c, true); });
  }
}

void TcpCommunicator::register_conn(const std::string& name, std::shared_ptr<Conn> c) {
  {
    std::lock_guard<std::mutex> g(mu_);
    conns_[name] = c;
    if (c->name.empty()) c->name = name;
  }
  cv_.notify_all();
}

void TcpCommunicator::reader_loop(std::shared_ptr<Conn> c, bool expect_hello) {
  std::string body;
  char hdr[kFixedHeader];
  while (!stopping_ && c->alive) {
    if (!read_all(c->fd, hdr, kFixedHeader)) break;
    if (static_cast<uint8_t>(hdr[0]) != 1) break;
    const bool swap = (static_cast<uint8_t>(hdr[1]) != 0) != host_little();
    uint64_t len;
    std::memcpy(&len, hdr + 2, 8);
    if (swap) len = bswap_t(len);
    if (len > kMaxFrame) break;
    body.resize(len);
    if (len && !read_all(c->fd, &body[0], len)) break;
    Message m;
    try {
      m = deserialize_body(body.data(), len, swap);
    } catch (const std::exception&) {
      break;
    }
    bytes_recv_ += kFixedHeader + len;
    if (m.command == CMD_START && m.payload_type == P_STRING) {  // HELLO: peer announces its id
      if (expect_hello) register_conn(m.text, c);
      continue;
    }
    ++msgs_recv_;
    m.sender = c->name.empty() ? m.sender : c->name;
    queue_.push(std::move(m));
  }
  c->alive = false;
}

void TcpCommunicator::connect(const std::string& name, const std::string& host, int port, int timeout_ms) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("cannot resolve " + host);
  int fd = -1;
  while (true) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
    ::close(fd);
    fd = -1;
    if (std::chrono::steady_clock::now() > deadline || stopping_) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  freeaddrinfo(res);
  if (fd < 0) throw std::runtime_error("connect to " + host + ":" + std::to_string(port) + " timed out");
  tune_socket(fd);
  auto c = std::make_shared<Conn>();
  c->fd = fd;
  c->name = name;
  {
    std::lock_guard<std::mutex> g(mu_);
    all_.push_back(c);
  }
  Message hello;
  hello.command = CMD_START;
  hello.payload_type = P_STRING;
  hello.text = id();
  write_frame(*c, hello);
  register_conn(name, c);
  c->reader = std::thread([this, c] { reader_loop(c, false); });
}

void TcpCommunicator::alias(const std::string& name, const std::string& target) {
  std::lock_guard<std::mutex> g(mu_);
  alias_[name] = target;
}

std::shared_ptr<TcpCommunicator::Conn> TcpCommunicator::lookup(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  std::string n = name;
  auto a = alias_.find(n);
  if (a != alias_.end()) n = a->second;
  auto it = conns_.find(n);
  return it == conns_.end() ? nullptr : it->second;
}

bool TcpCommunicator::wait_for_peer(const std::string& name, int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  auto have = [&] {
    std::string n = name;
    auto a = alias_.find(n);
    if (a != alias_.end()) n = a->second;
    return conns_.count(n) > 0;
  };
  return cv_.wait_until(lk, deadline_ms(timeout_ms), have);
}

void TcpCommunicator::write_frame(Conn& c, const Message& m) {
  std::string meta;
  serialize_meta(m, meta);
  const uint64_t raw = has_raw(m) ? m.data.size() : 0;
  const uint64_t body = meta.size() + raw;
  char hdr[kFixedHeader];
  hdr[0] = 1;
  hdr[1] = host_little() ? 1 : 0;
  std::memcpy(hdr + 2, &body, 8);
  struct iovec iov[3];
  iov[0] = {hdr, kFixedHeader};
  iov[1] = {const_cast<char*>(meta.data()), meta.size()};
  iov[2] = {const_cast<char*>(m.data.data()), static_cast<size_t>(raw)};
  std::lock_guard<std::mutex> g(c.wmu);
  if (!write_all(c.fd, iov, raw ? 3 : 2)) {
    c.alive = false;
    throw std::runtime_error("send to peer '" + c.name + "' failed: " + strerror(errno));
  }
  bytes_sent_ += kFixedHeader + body;
}

void TcpCommunicator::send(Message&& m) {
  auto c = lookup(m.recipient);
  if (!c || !c->alive) throw std::runtime_error("no live connection to '" + m.recipient + "'");
  m.sender = id();
  write_frame(*c, m);
  ++msgs_sent_;
}

std::vector<std::string> TcpCommunicator::peers() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (auto& kv : conns_)
    if (kv.second->alive) out.push_back(kv.first);
  return out;
}

void TcpCommunicator::close() {
  if (stopping_.exchange(true)) return;
  Communicator::close();
  if (acceptor_.joinable()) acceptor_.join();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  std::vector<std::shared_ptr<Conn>> all;
  {
    std::lock_guard<std::mutex> g(mu_);
    all = all_;
  }
  for (auto& c : all) {
    c->alive = false;
    ::shutdown(c->fd, SHUT_RDWR);
  }
  for (auto& c : all) {
    if (c->reader.joinable()) c->reader.join();
    ::close(c->fd);
  }
}

}  // namespace dcnn_native
