// Self-test of the C++ host API (run by tests/test_cpp_host_api.py; exit code 0 = pass):
// layout traits, relayout, bf16 rounding, JSON round trip, tensor records, grow-only ensure,
// config round trip through the layer factory, and a finite-difference gradient check of every
// layer type on the CPU backend. With "--device GPU" it also checks the GPU backend's forward /
// backward against the CPU backend on the same weights.
#include <cmath>
#include <cstdio>
#include <sstream>
#include <string>

#include "../../dcnn_amd/csrc/kernels/collective.h"
#include "../../dcnn_amd/csrc/native/comm.h"  // (Message: the stage's job messages)
#include "dcnn/dist.hpp"
#include "dcnn/nn.hpp"
#include "dcnn/pipeline.hpp"

using namespace dcnn;

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static void test_layout() {
  using NHWC = LayoutTrait<Layout::NHWC>;
  static_assert(NHWC::rank == 4 && NHWC::channels_last, "NHWC trait");
  static_assert(LayoutTrait<Layout::NDHWC>::perm[4] == 1, "NDHWC keeps C innermost");
  constexpr std::array<int64_t, 4> d{2, 3, 4, 5};
  constexpr auto s = strides_of<Layout::NHWC>(d);
  static_assert(s[1] == 1 && s[3] == 3 && s[2] == 15 && s[0] == 60, "NHWC strides");
  static_assert(offset_of<Layout::NCHW>(d, {1, 2, 3, 4}) == 60 + 40 + 15 + 4, "NCHW offset");
  static_assert(physical_dims<Layout::NHWC>(d)[3] == 3, "NHWC physical dims");
  const auto s5 = layout_strides(Layout::NDHWC, {2, 3, 4, 5, 6});
  CHECK(s5[1] == 1 && s5[4] == 3 && s5[3] == 18 && s5[2] == 90 && s5[0] == 360);
  CHECK(layout_info(Layout::NCDHW).rank == 5 && !layout_info(Layout::NCDHW).channels_last);
  std::vector<float> a(120), b(120), c(120);
  for (int i = 0; i < 120; ++i) a[i] = (float)i;
  relayout(a.data(), Layout::NCHW, b.data(), Layout::NHWC, {2, 3, 4, 5});
  CHECK(b[1] == a[20]);  // NHWC element (n0, h0, w0, c1) = NCHW (0, 1, 0, 0)
  relayout(b.data(), Layout::NHWC, c.data(), Layout::NCHW, {2, 3, 4, 5});
  CHECK(a == c);
}

static void test_bf16_json_tensor() {
  CHECK(bf16_to_f32(f32_to_bf16(1.0f)) == 1.0f);
  CHECK(f32_to_bf16(1.00390625f) == 0x3f80);   // tie -> even
  CHECK(f32_to_bf16(1.01171875f) == 0x3f82);   // tie -> even (odd below)
  json::Value v = json::Value::object();
  v["name"] = "m";
  v["x"] = 1.5;
  v["n"] = 3;
  v["b"] = true;
  json::Value arr = json::Value::array();
  arr.push("a\"b");
  arr.push(json::Value());
  v["arr"] = arr;
  const json::Value w = json::Value::parse(v.dump(2));
  CHECK(w.at("x").as_number() == 1.5 && w.at("n").as_int() == 3 && w.at("b").as_bool());
  CHECK(w.at("arr").items()[0].as_string() == "a\"b" && w.at("arr").items()[1].is_null());
  CHECK(w.dump(0) == v.dump(0));

  std::vector<float> vals(2 * 3 * 2 * 2);
  for (size_t i = 0; i < vals.size(); ++i) vals[i] = 0.25f * (float)i - 1.f;
  Tensor t = Tensor::from_host(vals, {2, 3, 2, 2}, Device::cpu(), DType::F32, Layout::NHWC);
  CHECK(t.to_host_f32() == vals);  // logical order survives the NHWC storage
  std::stringstream ss;
  t.save(ss);
  Tensor u = Tensor::load(ss);
  CHECK(u.to_host_f32() == vals && u.shape() == t.shape());
  Tensor g;
  g.ensure({4, 4}, DType::F32, Device::cpu());
  void* p0 = g.data();
  g.ensure({2, 2}, DType::F32, Device::cpu());
  CHECK(g.data() == p0 && g.numel() == 4);  // grow-only: no reallocation when smaller
  g.ensure({8, 8}, DType::F32, Device::cpu());
  CHECK(g.numel() == 64);
  // slices share the storage at a byte offset (parameter arenas)
  Tensor flat = Tensor::from_host(std::vector<float>{0, 1, 2, 3, 4, 5, 6, 7}, {8}, Device::cpu());
  Tensor s1 = flat.slice(4 * 4, {2, 2}, DType::F32);
  CHECK(s1.data() == static_cast<char*>(flat.data()) + 16);
  CHECK((s1.to_host_f32() == std::vector<float>{4, 5, 6, 7}));
  s1.ptr<float>()[0] = 40.f;
  CHECK(flat.to_host_f32()[4] == 40.f);
  bool threw = false;
  try {
    flat.slice(6 * 4, {4}, DType::F32);  // runs past the storage
  } catch (const std::out_of_range&) {
    threw = true;
  }
  CHECK(threw);
}

static Sequential small_model(bool with_bn) {
  SequentialBuilder b("selftest");
  b.input({2, 6, 6}).conv2d(4, 3, 3, 1, 1, 1, 1);
  if (with_bn) b.batchnorm();
  b.activation("tanh").maxpool2d(2, 2).conv2d(3, 2, 2, 1, 1, 0, 0).activation("elu").avgpool2d(2, 2, 1, 1)
      .flatten().dense(5);
  return b.build();
}

static double loss_of(Sequential& m, const Tensor& x, const Tensor& y) {
  return softmax_cross_entropy(m.forward(x), y).loss;
}

// central differences of the mean loss against the analytic gradients (fp32 CPU backend)
static void test_gradcheck(bool with_bn) {
  Sequential m = small_model(with_bn);
  m.initialize(3);
  SyntheticClassification src(4, 2, 6, 6, 5, 11, 1.0f);
  src.reset(0);
  Tensor x, y;
  src.next(4, x, y);
  m.set_training(true);
  m.zero_grad();
  auto r = softmax_cross_entropy(m.forward(x), y);
  m.backward(r.grad);
  double worst = 0;
  int checked = 0;
  for (auto* p : m.parameters()) {
    float* v = p->value.ptr<float>();
    const float* g = p->grad.ptr<float>();
    const int64_t n = p->value.numel();
    for (int64_t i = 0; i < n; i += std::max<int64_t>(1, n / 6)) {
      const float keep = v[i], h = 1e-3f;
      v[i] = keep + h;
      const double lp = loss_of(m, x, y);
      v[i] = keep - h;
      const double lm = loss_of(m, x, y);
      v[i] = keep;
      const double num = (lp - lm) / (2.0 * h);
      const double err = std::abs(num - g[i]) / std::max(1e-3, std::abs(num) + std::abs((double)g[i]));
      worst = std::max(worst, err);
      if (err > 5e-2) std::printf("  %s[%ld] num %.6g ana %.6g\n", p->name.c_str(), (long)i, num, (double)g[i]);
      ++checked;
    }
  }
  std::printf("gradcheck (bn=%d): %d entries, worst rel err %.3g\n", (int)with_bn, checked, worst);
  CHECK(checked > 20 && worst < 5e-2);
}

static void test_config_roundtrip() {
  Sequential m = small_model(true);
  const json::Value c = m.get_config();
  Sequential n = Sequential::load_from_config(json::Value::parse(c.dump(4)));
  CHECK(n.get_config().dump(0) == c.dump(0));
  CHECK(n.layers().size() == m.layers().size());
}

// GPU-comparison model: smooth layers only (a max-pool's argmax flips under bf16 rounding)
static Sequential smooth_model() {
  SequentialBuilder b("gpu_vs_cpu");
  b.input({8, 8, 8}).conv2d(16, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu").avgpool2d(2, 2, 2, 2)
      .conv2d(16, 3, 3, 1, 1, 1, 1, false).batchnorm().activation("tanh").flatten().dense(10);
  return b.build();
}

// GPU backend vs CPU backend on identical weights (bf16 activations: loose tolerance)
static void test_gpu_vs_cpu() {
  Sequential c = smooth_model(), g = smooth_model();
  c.initialize(5);
  g.set_device(Device::gpu(0));
  g.initialize(5);
  SyntheticClassification src(64, 8, 8, 8, 10, 13, 1.0f);
  src.reset(0);
  Tensor x, y;
  src.next(64, x, y);
  auto rc = softmax_cross_entropy(c.forward(x), y);
  auto rg = softmax_cross_entropy(g.forward(x), y);
  std::printf("gpu vs cpu loss %.5f %.5f\n", rg.loss, rc.loss);
  CHECK(std::abs(rg.loss - rc.loss) < 2e-2 * std::max(1.0, std::abs(rc.loss)));
  c.zero_grad();
  g.zero_grad();
  c.backward(rc.grad);
  g.backward(rg.grad);
  auto pc = c.parameters(), pg = g.parameters();
  std::vector<std::vector<float>> ga, gb;
  double top = 0;
  for (size_t k = 0; k < pc.size(); ++k) {
    ga.push_back(pc[k]->grad.view(pc[k]->shape, pc[k]->layout).to_host_f32());
    gb.push_back(pg[k]->grad.view(pg[k]->shape, pg[k]->layout).to_host_f32());
    double n2 = 0;
    for (float v : ga.back()) n2 += (double)v * v;
    top = std::max(top, std::sqrt(n2));
  }
  for (size_t k = 0; k < pc.size(); ++k) {
    const auto& a = ga[k];
    const auto& b = gb[k];
    double num = 0, den = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      num += (double)(a[i] - b[i]) * (a[i] - b[i]);
      den += (double)a[i] * a[i];
    }
    // bf16 activations: a few percent on gradients that pass a BatchNorm backward (a difference
    // of nearly equal terms); a conv bias feeding a BatchNorm has an exactly-zero gradient, so
    // it is held to an absolute bound relative to the model's largest gradient instead
    const bool degenerate = std::sqrt(den) < 1e-3 * top;
    const double rel = degenerate ? std::sqrt(num) / top : std::sqrt(num / den);
    std::printf("  grad %zu/%s %s %.3g\n", k, pc[k]->name.c_str(), degenerate ? "abs/top" : "rel l2", rel);
    CHECK(rel < 6e-2);
  }
}

// the native pipeline's RCCL stage link (transport "rccl") at world size 1: a GPU-produced bf16
// NHWC activation through a one-rank communicator's send / receive on the link's own flow, read
// back on the caller's flow (event ordering both ways), then a second round trip of another size
static void test_p2p_loopback() {
  Sequential g = smooth_model();
  g.set_device(Device::gpu(0));
  g.initialize(3);
  SyntheticClassification src(16, 8, 8, 8, 10, 3, 1.0f);
  src.reset(0);
  Tensor x, y;
  src.next(16, x, y);
  const Tensor a = g.forward(x);  // produced on the caller's flow just before the hand-off
  const Tensor b = dist::P2PLink::loopback(a);
  CHECK(b.shape() == a.shape() && b.dtype() == a.dtype() && b.layout() == a.layout());
  const auto ha = a.to_host_f32(), hb = b.to_host_f32();
  size_t diff = 0;
  for (size_t i = 0; i < ha.size(); ++i) diff += ha[i] != hb[i];
  CHECK(diff == 0);
  std::vector<float> v(3 * 5 * 7 * 11);
  for (size_t i = 0; i < v.size(); ++i) v[i] = (float)i * 0.25f - 100.f;
  const Tensor c = Tensor::from_host(v, {3, 5, 7, 11}, Device::gpu(0), DType::F32);
  const auto hc = dist::P2PLink::loopback(c).to_host_f32();
  CHECK(hc == v);
  std::printf("p2p loopback ok (%zu + %zu values, %zu differ)\n", ha.size(), v.size(), diff);
}

// the RCCL stage transport's own send / receive (dist::P2PLink::send / recv, each link on its own
// flow, and the stage's job-message header: wire::send_rccl / recv_rccl, the functions
// PipelineStage's transport "rccl" calls) through a one-rank sender / receiver pair — a send to
// itself is matched within one RCCL group, so each hand-off is one group here, where two stage
// processes post theirs independently. Activations (bf16 NHWC, produced on the caller's flow just
// before the send), logits (fp32 (N, classes): rank 2 on the wire) and gradients, interleaved over
// two micro-batch slots and read back on the caller's flow.
static void test_p2p_pair() {
  auto pair = dist::P2PLink::self_pair(0);
  dist::P2PLink& tx = *pair.first;
  dist::P2PLink& rx = *pair.second;
  SequentialBuilder b("p2p_pair");
  b.input({8, 8, 8}).conv2d(16, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu");
  Sequential g = b.build();
  g.set_device(Device::gpu(0));
  g.initialize(7);
  size_t checked = 0, differ = 0;
  for (int k = 0; k < 6; ++k) {
    SyntheticClassification src(8, 8, 8, 8, 10, 11 + k, 1.0f);
    src.reset(0);
    Tensor x, y;
    src.next(8, x, y);
    std::vector<float> lv(8 * 10), gv(8 * 16 * 8 * 8);
    for (size_t i = 0; i < lv.size(); ++i) lv[i] = std::sin(0.37f * (float)(i + 13 * k));
    for (size_t i = 0; i < gv.size(); ++i) gv[i] = std::cos(0.11f * (float)(i + 7 * k)) * 1e-3f;
    struct Case {
      Tensor t;
      bool logits;
    } cases[] = {{g.forward(x), false},
                 {Tensor::from_host(lv, {8, 10, 1, 1}, Device::gpu(0), DType::F32), true},
                 {Tensor::from_host(gv, {8, 16, 8, 8}, Device::gpu(0), DType::BF16, Layout::NHWC), false}};
    for (const Case& c : cases) {
      dcnn_native::Message m;
      m.command = dcnn_native::FORWARD_JOB;
      coll::group_start();
      wire::send_rccl(tx, c.t, (uint64_t)(k % 2), c.logits, m);
      Tensor r = wire::recv_rccl(rx, m, Device::gpu(0));
      coll::group_end();
      CHECK((m.dtype & 0x40) != 0 && m.data.empty() && m.mb_id == (uint64_t)(k % 2));
      // ((N, F) tensors — the GPU forward's flattened output — arrive as (N, F, 1, 1) NCHW: the same
      // bytes, features in logical order)
      const bool flat = c.t.rank() == 2;
      const std::vector<int64_t> want = flat ? std::vector<int64_t>{c.t.dim(0), c.t.dim(1), 1, 1} : c.t.shape();
      const Layout want_layout = flat ? Layout::NCHW : c.t.layout();
      if (!(r.shape() == want && r.dtype() == c.t.dtype() && r.layout() == want_layout)) {
        auto str = [](const Tensor& t) {
          std::string o = "[";
          for (auto d : t.shape()) o += std::to_string(d) + ",";
          return o + "] dt " + std::to_string((int)t.dtype()) + " layout " + std::to_string((int)t.layout());
        };
        std::printf("p2p pair: sent %s, received %s\n", str(c.t).c_str(), str(r).c_str());
      }
      CHECK(r.shape() == want && r.dtype() == c.t.dtype() && r.layout() == want_layout);
      const auto ht = c.t.to_host_f32(), hr = r.to_host_f32();
      CHECK(ht.size() == hr.size());
      for (size_t i = 0; i < std::min(ht.size(), hr.size()); ++i) differ += ht[i] != hr[i];
      checked += ht.size();
    }
  }
  tx.drain();
  CHECK(differ == 0);
  std::printf("p2p pair ok (%zu values over 18 hand-offs, %zu differ)\n", checked, differ);
}

int main(int argc, char** argv) {
  const bool gpu = argc > 2 && std::string(argv[1]) == "--device" && std::string(argv[2]) == "GPU";
  try {
    test_layout();
    test_bf16_json_tensor();
    test_config_roundtrip();
    test_gradcheck(false);
    test_gradcheck(true);
    if (gpu) test_gpu_vs_cpu();
    if (gpu) test_p2p_loopback();
    if (gpu) test_p2p_pair();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 1;
  }
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures ? 1 : 0;
}
