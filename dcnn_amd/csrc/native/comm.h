// Control plane of the pipeline runtime: message model, wire serialisation, priority message
// queue, TCP and in-process communicators, payload compression.
//
// Wire format (compatible with the reference, include/pipeline/message.hpp:23-58 and
// include/pipeline/binary_serializer.hpp:27-78):
//   u8 version=1 | u8 endianness (1 = little) | u64 body_len
//   body: u64 len, recipient | u64 len, sender | u16 command | u64 payload_type | payload
//   payload 0 none | 1 Job<f32>: u64 mb_id, u64 ndim, u64 dims[ndim], f32 data[]
//           2 string: u64 len, bytes | 3 bool: u8 | 4 LoadTracker: 4 x f32 (the reference
//           declares but never serialises it)
//   extension (not in the reference): 5 typed job: u64 mb_id, u8 dtype, u8 codec,
//           u64 ndim, u64 dims[], u64 nbytes, bytes[] (bf16 activations, compressed payloads)
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dcnn_native {

// Order == dequeue priority (reference include/pipeline/command_type.hpp:20-68).
enum Command : uint16_t {
  CMD_START = 0,
  FORWARD_JOB, BACKWARD_JOB, UPDATE_PARAMETERS,
  TRAIN_MODE, EVAL_MODE, SHUTDOWN,
  CONFIG_TRANSFER, CONFIG_RECEIVED, LOAD_PARAMS, PARAMS_LOADED, SEND_PARAMS, PARAMS_TRANSFER,
  STATUS_REQUEST, STATUS_RESPONSE, PARAMETERS_UPDATED, HEALTH_CHECK,
  ERROR_REPORT, JOB_FAILURE,
  BARRIER_SYNC, CHECKPOINT_REQUEST, CHECKPOINT_COMPLETE,
  UPDATE_LOAD, REPORT_LOAD, LOAD_REPORT,
  PRINT_PROFILING, PROFILING_PRINTED, CLEAR_PROFILING, PROFILING_CLEARED,
  // native extension (the loss on the last stage's GPU, dcnn/pipeline.hpp): coordinator -> last
  // stage, f64 payload [kind, param, gradient scale] with micro-batch id kLossConfig = enable (the
  // stage answers with this command), else [label...] of that micro-batch
  LABELS_TRANSFER,
  // native extension (transport "rccl"): coordinator -> every stage = open the stage-to-stage RCCL
  // links (each stage answers with this command when its links are up); stage -> next stage = the
  // two 128-byte unique ids of that pair's links (u8 payload: activations down, gradients up)
  P2P_CONNECT,
  CMD_COUNT
};
const char* command_name(uint16_t c);

enum PayloadType : uint64_t { P_NONE = 0, P_JOB = 1, P_STRING = 2, P_BOOL = 3, P_LOAD = 4, P_TYPED_JOB = 5 };
enum Codec : uint8_t { CODEC_NONE = 0, CODEC_ZLIB = 1, CODEC_ZSTD = 2 };

struct LoadTracker {
  float avg_forward_ms = 0, avg_backward_ms = 0, avg_cpu_utilization = -1, max_memory_mb = -1;
};

struct Message {
  std::string recipient, sender;
  uint16_t command = CMD_START;
  uint64_t payload_type = P_NONE;
  // job payloads
  uint64_t mb_id = 0;
  uint8_t dtype = 0;   // 0 f32, 1 bf16, 2 f16, 3 i64, 4 u8, 5 f64
  uint8_t codec = CODEC_NONE;
  std::vector<uint64_t> shape;
  std::string data;    // raw (possibly compressed) tensor bytes
  // scalar payloads
  std::string text;
  bool flag = false;
  LoadTracker load;

  size_t body_size() const;
};

// ---- serialisation
void serialize_body(const Message& m, std::string& out);          // body only
std::string serialize(const Message& m);                          // fixed header + body
Message deserialize_body(const char* p, size_t n, bool swap);
Message deserialize(const std::string& frame);
constexpr size_t kFixedHeader = 10;

// ---- compression (zstd via dlopen(libzstd.so.1) when present, zlib otherwise)
bool zstd_available();
std::string compress(const std::string& in, Codec codec, int level);
std::string decompress(const std::string& in, Codec codec, size_t raw_size_hint);

// ---- priority queue of incoming messages
class MessageQueue {
 public:
  void push(Message&& m);
  // Pops the highest-priority (lowest command value) message; false on timeout (ms < 0: wait).
  bool pop(Message& out, int timeout_ms);
  bool pop_command(uint16_t cmd, Message& out, int timeout_ms);
  // Pops the first queued message of the lowest-valued command in `cmds` that has one, waiting up
  // to timeout_ms for any of them (a scheduler serving several kinds of completion at once)
  bool pop_any(const std::vector<uint16_t>& cmds, Message& out, int timeout_ms);
  size_t size() const;
  size_t count(uint16_t cmd) const;
  void close();
  bool closed() const { return closed_; }

 private:
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Message> q_[CMD_COUNT];
  size_t total_ = 0;
  std::atomic<bool> closed_{false};
};

// ---- communicators
class Communicator {
 public:
  explicit Communicator(std::string id) : id_(std::move(id)) {}
  virtual ~Communicator() = default;
  std::string id() const {
    std::lock_guard<std::mutex> g(id_mu_);
    return id_;
  }
  // Renames this endpoint (a network worker learns its stage name from CONFIG_TRANSFER);
  // affects the HELLO of later connections and the sender field of later messages.
  void set_id(const std::string& id) {
    std::lock_guard<std::mutex> g(id_mu_);
    id_ = id;
  }
  MessageQueue& queue() { return queue_; }
  virtual void send(Message&& m) = 0;
  virtual void close() { queue_.close(); }
  virtual std::vector<std::string> peers() const = 0;
  uint64_t bytes_sent() const { return bytes_sent_; }
  uint64_t bytes_received() const { return bytes_recv_; }
  uint64_t messages_sent() const { return msgs_sent_; }
  uint64_t messages_received() const { return msgs_recv_; }

 protected:
  std::string id_;
  mutable std::mutex id_mu_;
  MessageQueue queue_;
  std::atomic<uint64_t> bytes_sent_{0}, bytes_recv_{0}, msgs_sent_{0}, msgs_recv_{0};
};

// Routes directly into the recipient's queue through a process-wide registry; no delivery
// thread (the reference's delivery loop double-locks).
class InProcessCommunicator : public Communicator {
 public:
  explicit InProcessCommunicator(std::string id);
  ~InProcessCommunicator() override;
  void send(Message&& m) override;
  void alias(const std::string& name, const std::string& target);
  std::vector<std::string> peers() const override;
  void close() override;

 private:
  mutable std::mutex mu_;
  std::map<std::string, std::string> alias_;
};

// POSIX TCP control plane: listener + one reader thread per connection; sends are
// synchronous writev()s under a per-connection mutex (called with the GIL released).
class TcpCommunicator : public Communicator {
 public:
  TcpCommunicator(std::string id, const std::string& host, int port);
  ~TcpCommunicator() override;
  int port() const { return port_; }
  // Connects and registers the connection under `name` (logical name such as
  // "next_stage"); retries until timeout_ms.  The peer learns our id from a HELLO frame.
  void connect(const std::string& name, const std::string& host, int port, int timeout_ms);
  void alias(const std::string& name, const std::string& target);
  bool wait_for_peer(const std::string& name, int timeout_ms);
  void send(Message&& m) override;
  std::vector<std::string> peers() const override;
  void close() override;

 private:
  struct Conn {
    int fd = -1;
    std::string name;
    std::mutex wmu;
    std::thread reader;
    std::atomic<bool> alive{true};
  };
  void accept_loop();
  void reader_loop(std::shared_ptr<Conn> c, bool expect_hello);
  void register_conn(const std::string& name, std::shared_ptr<Conn> c);
  std::shared_ptr<Conn> lookup(const std::string& name);
  void write_frame(Conn& c, const Message& m);

  int listen_fd_ = -1;
  int port_ = 0;
  std::thread acceptor_;
  std::atomic<bool> stopping_{false};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::shared_ptr<Conn>> conns_;
  std::vector<std::shared_ptr<Conn>> all_;
  std::map<std::string, std::string> alias_;
};

}  // namespace dcnn_native
