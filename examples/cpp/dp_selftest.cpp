// Multi-process check of the C++ host API's data parallelism (dcnn/dist.hpp): run one process per
// rank under the launcher variables (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT; tests/
// test_cpp_dp.py starts them), each trains one step on its shard of a fixed global batch, and the
// averaged gradient / updated parameters are written for comparison against a world-1 run on the
// whole batch.
//
//   dcnn_amd/bin/dp_selftest --device CPU|GPU|UID --out DIR [--batch 16] [--bucket-mb 0.004]
//   (UID: only the RCCL unique-id rendezvous of the GPU plane, exchange_unique_id)
//                            [--graph]   (GPU: Adam + the captured TrainGraph step)
//                            [--no-dp]   (the same step without the gradient mean: world-1 baseline)
//
// Writes DIR/w<W>r<R>.bin: u64 n_grad, f32 grad[n_grad], u64 n_param, f32 params[n_param],
// u64 n_bn, f32 bn_params_and_running_stats[n_bn] (a BatchNorm model whose ranks start from
// different seeds, after broadcast_parameters), and prints one JSON line (buckets, loss).
// Reference parity: none (the reference has no data parallelism).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "dcnn/dist.hpp"
#include "dcnn/nn.hpp"
#include "dcnn/train.hpp"

using namespace dcnn;

namespace {
// the fixed global batch (every rank generates all of it and takes its shard)
void global_batch(int n, std::vector<float>& x, std::vector<int64_t>& y) {
  uint64_t s = 0x9E3779B97F4A7C15ull;
  auto next = [&] {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return (double)(s >> 11) / (double)(1ull << 53);
  };
  x.resize((size_t)n * 3 * 16 * 16);
  for (auto& v : x) v = (float)(2.0 * next() - 1.0);
  y.resize((size_t)n);
  for (auto& v : y) v = (int64_t)(next() * 10.0);
}

void append(std::vector<float>& out, const std::vector<Param*>& ps, bool grads) {
  for (Param* p : ps) {
    const auto h = (grads ? p->grad : p->value).to_host_f32();
    out.insert(out.end(), h.begin(), h.end());
  }
}
void write_block(std::ofstream& f, const std::vector<float>& v) {
  const uint64_t n = v.size();
  f.write(reinterpret_cast<const char*>(&n), 8);
  f.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)(v.size() * 4));
}
}  // namespace

int main(int argc, char** argv) {
  std::string device = "CPU", out = ".";
  int batch = 16;
  double bucket_mb = 0.004;  // ~1 KB buckets: several fire points inside the backward
  bool graph = false, no_dp = false;
  for (int i = 1; i < argc; ++i) {
    const std::string k = argv[i];
    if (k == "--graph") { graph = true; continue; }
    if (k == "--no-dp") { no_dp = true; continue; }
    if (i + 1 >= argc) break;
    const std::string v = argv[++i];
    if (k == "--device") device = v;
    else if (k == "--out") out = v;
    else if (k == "--batch") batch = std::atoi(v.c_str());
    else if (k == "--bucket-mb") bucket_mb = std::atof(v.c_str());
  }
  try {
    const dist::Env env = dist::Env::from_env();
    if (device == "UID") {  // the RCCL unique-id rendezvous alone (no device work): every rank
                            // prints a hash of the id it holds
      const std::string id = dist::exchange_unique_id(env);
      uint64_t h = 1469598103934665603ull;
      for (unsigned char ch : id) h = (h ^ ch) * 1099511628211ull;
      std::printf("{\"rank\": %d, \"uid_hash\": \"%016llx\", \"uid_bytes\": %zu}\n", env.rank,
                  (unsigned long long)h, id.size());
      return 0;
    }
    Device dev = Device::parse(device);
    dist::DataParallel dp(env, dev);
    dev = dp.device();
    if (batch % env.world) throw std::invalid_argument("--batch must divide by WORLD_SIZE");
    const int per = batch / env.world;

    // 1) BN-free model, SGD (or Adam + TrainGraph): averaged shard gradients == whole-batch gradient
    Sequential m = SequentialBuilder("dp_exact").input({3, 16, 16})
                       .conv2d(16, 3, 3, 1, 1, 1, 1).activation("relu").maxpool2d(2, 2, 2, 2)
                       .conv2d(32, 3, 3, 1, 1, 1, 1).activation("relu").flatten().dense(10).build();
    m.set_device(dev);
    m.initialize(3 + 11 * (uint64_t)env.rank);  // replicas differ until the broadcast
    dp.broadcast_parameters(m);
    if (!no_dp) dp.attach(m, bucket_mb);
    std::vector<float> xg;
    std::vector<int64_t> yg;
    global_batch(batch, xg, yg);
    const std::vector<float> xs(xg.begin() + (size_t)env.rank * per * 3 * 256, xg.begin() + (size_t)(env.rank + 1) * per * 3 * 256);
    const std::vector<int64_t> ys(yg.begin() + (size_t)env.rank * per, yg.begin() + (size_t)(env.rank + 1) * per);
    const Tensor x = Tensor::from_host(xs, {per, 3, 16, 16}, dev);
    const Tensor y = Tensor::from_host_i64(ys, dev);
    Loss loss = LossFactory::create("softmax_ce");
    double l = 0;
    if (graph) {
      if (!dev.is_gpu()) throw std::invalid_argument("--graph: GPU only");
      Adam opt(1e-3f);
      TrainGraph tg(m, opt, loss);
      if (!no_dp) tg.set_gradient_hook([&dp] { dp.finish(); });
      tg.step(x, y);  // capture (after two restored warm-up steps) + one replay
      l = tg.last_loss();
    } else {
      SGD opt(0.1f);
      m.zero_grad();
      LossResult r = loss(m.forward(x), y);
      m.backward(r.grad);
      if (!no_dp) dp.finish();
      opt.step(m.parameters());
      l = r.loss;
    }
    if (dev.is_gpu()) gpu::synchronize();
    std::vector<float> g, p;
    append(g, m.parameters(), true);
    append(p, m.parameters(), false);

    // 2) BatchNorm model from rank-dependent seeds: broadcast_parameters makes every replica rank 0's
    Sequential b = SequentialBuilder("dp_bcast").input({3, 16, 16})
                       .conv2d(8, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu").flatten().dense(10).build();
    b.set_device(dev);
    b.initialize(100 + 7 * (uint64_t)env.rank);
    for (BatchNorm* bn : b.batchnorms()) {  // rank-dependent running statistics too
      std::vector<float> mu(bn->running_mean.numel(), 0.01f * (float)env.rank);
      const Tensor h = Tensor::from_host(mu, bn->running_mean.shape(), dev);
      if (dev.is_gpu()) gpu::copy(bn->running_mean.data(), h.data(), h.nbytes(), 2);
      else std::memcpy(bn->running_mean.data(), h.data(), h.nbytes());
    }
    dp.broadcast_parameters(b);
    if (dev.is_gpu()) gpu::synchronize();
    std::vector<float> bv;
    append(bv, b.parameters(), false);
    for (BatchNorm* bn : b.batchnorms()) {
      const auto rm = bn->running_mean.to_host_f32(), rv = bn->running_var.to_host_f32();
      bv.insert(bv.end(), rm.begin(), rm.end());
      bv.insert(bv.end(), rv.begin(), rv.end());
    }
    const double slow = dp.max((double)env.rank);
    dp.barrier();

    std::ofstream f(out + "/w" + std::to_string(env.world) + "r" + std::to_string(env.rank) + ".bin", std::ios::binary);
    write_block(f, g);
    write_block(f, p);
    write_block(f, bv);
    std::printf("{\"rank\": %d, \"world\": %d, \"plane\": \"%s\", \"buckets\": %d, \"loss\": %.6f, \"max_rank\": %.1f}\n",
                env.rank, env.world, dp.plane(), dp.buckets_last_step(), l, slow);
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
