// Standalone C++ self-test of the host runtime (no Python): message serialisation, priority
// queue, in-process + TCP communicators under concurrent senders, compression, JPEG decode of a
// malformed stream.  Built three ways by tests/test_native_sanitizers.py:
//   plain, -fsanitize=address,undefined, and -fsanitize=thread (race detection on the comm
//   runtime — the reference advertises sanitizers but never enables any).
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../comm.h"
#include "../native.h"

using namespace dcnn_native;

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                  \
    }                                                                \
  } while (0)

static Message job(const std::string& to, uint16_t cmd, uint64_t mb, size_t n) {
  Message m;
  m.recipient = to;
  m.command = cmd;
  m.payload_type = P_JOB;
  m.mb_id = mb;
  m.shape = {n};
  m.data.resize(n * 4);
  for (size_t i = 0; i < n; ++i) {
    float v = static_cast<float>(mb * 1000 + i);
    std::memcpy(&m.data[i * 4], &v, 4);
  }
  return m;
}

static void test_serialization() {
  Message m = job("stage_1", FORWARD_JOB, 7, 33);
  m.sender = "coordinator";
  Message r = deserialize(serialize(m));
  CHECK(r.recipient == "stage_1" && r.sender == "coordinator" && r.command == FORWARD_JOB);
  CHECK(r.mb_id == 7 && r.shape.size() == 1 && r.shape[0] == 33 && r.data == m.data);
  Message t;
  t.recipient = "x";
  t.payload_type = P_TYPED_JOB;
  t.dtype = 1;
  t.codec = CODEC_ZLIB;
  t.shape = {2, 3};
  std::string raw(12, 'a');
  t.data = compress(raw, CODEC_ZLIB, 3);
  Message t2 = deserialize(serialize(t));
  CHECK(decompress(t2.data, CODEC_ZLIB, 0) == raw);
  std::string frame = serialize(m);
  bool threw = false;
  try {
    deserialize(frame.substr(0, frame.size() - 3));
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_queue_priority() {
  MessageQueue q;
  for (uint16_t c : {SHUTDOWN, BACKWARD_JOB, FORWARD_JOB, UPDATE_PARAMETERS}) {
    Message m;
    m.command = c;
    q.push(std::move(m));
  }
  Message out;
  std::vector<uint16_t> got;
  while (q.pop(out, 0)) got.push_back(out.command);
  CHECK((got == std::vector<uint16_t>{FORWARD_JOB, BACKWARD_JOB, UPDATE_PARAMETERS, SHUTDOWN}));
}

static void test_inprocess_concurrent() {
  InProcessCommunicator dst("st_dst");
  const int T = 4, N = 500;
  std::vector<std::thread> th;
  std::vector<std::unique_ptr<InProcessCommunicator>> srcs;
  for (int t = 0; t < T; ++t) srcs.emplace_back(new InProcessCommunicator("st_src" + std::to_string(t)));
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      for (int i = 0; i < N; ++i) srcs[t]->send(job("st_dst", i % 2 ? BACKWARD_JOB : FORWARD_JOB, i, 8));
    });
  std::atomic<int> got{0};
  std::thread consumer([&] {
    Message m;
    while (got < T * N)
      if (dst.queue().pop(m, 1000)) ++got;
  });
  for (auto& x : th) x.join();
  consumer.join();
  CHECK(got == T * N && dst.messages_received() == static_cast<uint64_t>(T * N));
}

static void test_tcp_concurrent() {
  TcpCommunicator server("server", "127.0.0.1", 0);
  const int C = 3, N = 200;
  std::vector<std::unique_ptr<TcpCommunicator>> clients;
  for (int c = 0; c < C; ++c) {
    clients.emplace_back(new TcpCommunicator("client" + std::to_string(c), "127.0.0.1", 0));
    clients.back()->connect("server", "127.0.0.1", server.port(), 5000);
  }
  for (int c = 0; c < C; ++c) CHECK(server.wait_for_peer("client" + std::to_string(c), 5000));
  std::vector<std::thread> th;
  for (int c = 0; c < C; ++c)
    th.emplace_back([&, c] {
      for (int i = 0; i < N; ++i) clients[c]->send(job("server", FORWARD_JOB, i, 64 + (i % 7) * 1000));
    });
  // replies from the server to every client on their accepted connections, concurrently
  std::thread replier([&] {
    for (int i = 0; i < N; ++i)
      for (int c = 0; c < C; ++c) {
        Message m;
        m.recipient = "client" + std::to_string(c);
        m.command = HEALTH_CHECK;
        m.payload_type = P_BOOL;
        m.flag = true;
        server.send(std::move(m));
      }
  });
  std::vector<int> next(C, 0);
  int got = 0;
  Message m;
  while (got < C * N) {
    CHECK(server.queue().pop(m, 5000));
    const int c = m.sender.back() - '0';
    CHECK(static_cast<int>(m.mb_id) == next[c]);  // per-connection FIFO
    ++next[c];
    float v;
    std::memcpy(&v, m.data.data() + 4, 4);
    CHECK(v == static_cast<float>(m.mb_id * 1000 + 1));
    ++got;
  }
  for (auto& x : th) x.join();
  replier.join();
  for (int c = 0; c < C; ++c) {
    int h = 0;
    while (h < N && clients[c]->queue().pop(m, 5000)) ++h;
    CHECK(h == N);
  }
  for (auto& c : clients) c->close();
  server.close();
}

static void test_jpeg_garbage() {
  std::vector<unsigned char> rgb;
  int w = 0, h = 0;
  std::string err;
  const unsigned char bad[] = {0xFF, 0xD8, 0xFF, 0xC0, 0x00, 0x11, 0x08, 0x00};
  CHECK(!decode_jpeg(bad, sizeof(bad), rgb, w, h, &err));
  std::vector<unsigned char> noise(4096);
  for (size_t i = 0; i < noise.size(); ++i) noise[i] = static_cast<unsigned char>(i * 131 + 7);
  noise[0] = 0xFF;
  noise[1] = 0xD8;
  decode_jpeg(noise.data(), noise.size(), rgb, w, h, &err);  // must not crash
}

int main() {
  test_serialization();
  test_queue_priority();
  test_inprocess_concurrent();
  test_tcp_concurrent();
  test_jpeg_garbage();
  std::printf("native selftest OK\n");
  return 0;
}
