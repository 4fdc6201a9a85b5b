// Cross-language parity probe of the C++ host API (tests/test_cpp_host_blocks.py drives it):
//
//   host_api_parity schedulers                 LR sequence of every scheduler type, one line each
//   host_api_parity losses <in.bin> <C>        loss + gradient of the six losses on a [N, C] record
//                                              (labels = row index % C), CPU backend
//   host_api_parity forward <model> <x.bin> [--device GPU]
//                                              logits of a saved model (path.json/.bin/.bnstats) in
//                                              eval mode for an (N, C, H, W) .bin record
//   host_api_parity grads <model_name> <batch> <out.bin> [<prefix>] [--device GPU]
//                                              one forward + backward; every parameter gradient
//                                              (logical NCHW fp32 records) into out.bin; with a
//                                              prefix also the initial model (prefix.json/.bin)
//                                              and the batch (prefix.x.bin, prefix.y.bin)
//   host_api_parity blocks <model_name> <batch> [--device GPU]
//                                              teacher-forced per-layer errors against the CPU backend
//   host_api_parity train <model_name> <steps> <batch> <save> [--device GPU] [--graph]
//                                              Adam steps on a synthetic set, then save
// Output is plain text: one "key v0 v1 ..." line per item.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>

#include "dcnn/nn.hpp"
#include "dcnn/train.hpp"

using namespace dcnn;

static Device device_arg(int argc, char** argv) {
  for (int i = 1; i + 1 < argc; ++i)
    if (std::string(argv[i]) == "--device") return Device::parse(argv[i + 1]);
  return Device::cpu();
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: host_api_parity schedulers|losses|forward|train ...\n");
    return 2;
  }
  const std::string cmd = argv[1];
  try {
    if (cmd == "schedulers") {
      const char* cfgs[] = {
          R"({"type": "step_lr", "parameters": {"step_size": 3, "gamma": 0.5}})",
          R"({"type": "multi_step_lr", "parameters": {"milestones": [2, 5, 9], "gamma": 0.3}})",
          R"({"type": "exponential_lr", "parameters": {"gamma": 0.9}})",
          R"({"type": "cosine_annealing_lr", "parameters": {"T_max": 7, "eta_min": 0.001}})",
          R"({"type": "cosine_annealing_warm_restarts", "parameters": {"T_0": 3, "T_mult": 2, "eta_min": 0.0}})",
          R"({"type": "linear_warmup", "parameters": {"warmup_steps": 4, "start_lr": 0.01}})",
          R"({"type": "warmup_cosine_annealing", "parameters": {"warmup_steps": 3, "total_steps": 10, "start_lr": 0.0, "eta_min": 0.01}})",
          R"({"type": "reduce_lr_on_plateau", "parameters": {"mode": "min", "factor": 0.5, "patience": 2, "threshold": 0.0001, "min_lr": 0.001}})",
          R"({"type": "polynomial_lr", "parameters": {"total_steps": 8, "power": 2.0, "end_lr": 0.001}})",
          R"({"type": "one_cycle_lr", "parameters": {"max_lr": 0.5, "total_steps": 10, "pct_start": 0.3, "div_factor": 25.0, "final_div_factor": 10000.0}})",
      };
      for (const char* c : cfgs) {
        SGD opt(0.1f);
        auto s = SchedulerFactory::create_from_config(json::Value::parse(c), &opt);
        std::printf("%s %.9g", s->type().c_str(), (double)opt.learning_rate());
        const double metrics[] = {1.0, 0.9, 0.95, 0.95, 0.96, 0.97, 0.5, 0.6, 0.6, 0.6, 0.7, 0.8};
        for (int k = 0; k < 12; ++k) {
          if (s->type() == "reduce_lr_on_plateau")
            s->step(metrics[k]);
          else
            s->step();
          std::printf(" %.9g", (double)opt.learning_rate());
        }
        std::printf("\n");
      }
      return 0;
    }
    if (cmd == "losses" && argc >= 4) {
      std::ifstream f(argv[2], std::ios::binary);
      Tensor x = Tensor::load(f);
      const int C = std::atoi(argv[3]);
      const int N = (int)(x.numel() / C);
      Tensor pred = x.view({N, C});
      std::vector<int64_t> lab(N);
      for (int i = 0; i < N; ++i) lab[i] = i % C;
      Tensor labels = Tensor::from_host_i64(lab, Device::cpu());
      const char* names[] = {"crossentropy", "softmax_crossentropy", "logsoftmax_crossentropy", "mse", "mae", "huber"};
      for (const char* n : names) {
        Loss l = LossFactory::create(n);
        LossResult r = l.compute(pred, &labels);
        std::printf("%s %.9g %ld", n, r.loss, r.correct);
        for (float g : r.grad.to_host_f32()) std::printf(" %.9g", (double)g);
        std::printf("\n");
      }
      return 0;
    }
    if (cmd == "forward" && argc >= 4) {
      const Device dev = device_arg(argc, argv);
      Sequential m = Sequential::from_file(argv[2], dev);
      m.set_training(false);
      std::ifstream f(argv[3], std::ios::binary);
      Tensor x = Tensor::load(f);
      Tensor logits = m.forward(x);
      std::printf("params %zu\nlogits", m.num_parameters());
      for (float v : logits.to_host_f32()) std::printf(" %.9g", (double)v);
      std::printf("\n");
      return 0;
    }
    if (cmd == "grads" && argc >= 5) {
      // one forward + backward on the first synthetic batch; every parameter's gradient is
      // written (logical NCHW fp32 records, parameter order) to argv[4]
      const Device dev = device_arg(argc, argv);
      Sequential m = create_model(argv[2]);
      m.set_device(dev);
      m.initialize(11);
      const int batch = std::atoi(argv[3]);
      const bool cifar = std::string(argv[2]).find("cifar") != std::string::npos;
      const int hw = cifar ? 32 : 64, classes = cifar ? 10 : 200;
      SyntheticClassification data((size_t)batch, 3, hw, hw, classes, 5, 0.3f);
      Loss loss = LossFactory::create("softmax_crossentropy");
      data.reset(0);
      Tensor x, y;
      if (!data.next(batch, x, y)) throw std::runtime_error("no batch");
      if (argc >= 6 && argv[5][0] != '-') {
        // the initial weights and the batch, for another front end to run the same step
        const std::string pre = argv[5];
        m.save_to_file(pre);
        std::ofstream fx(pre + ".x.bin", std::ios::binary);
        x.to(Device::cpu()).save(fx);
        std::vector<float> yl;
        for (int64_t v : y.to(Device::cpu()).to_host_i64()) yl.push_back((float)v);
        std::ofstream fy(pre + ".y.bin", std::ios::binary);
        Tensor::from_host(yl, {(int64_t)yl.size(), 1, 1, 1}, Device::cpu()).save(fy);
      }
      m.zero_grad();
      LossResult r = loss(m.forward(x), y);
      m.backward(r.grad);
      std::ofstream f(argv[4], std::ios::binary);
      std::printf("loss %.9g\nparams", r.loss);
      for (Param* p : m.parameters()) {
        p->grad.view(p->shape, p->layout).save(f);
        std::printf(" %s", p->name.c_str());
      }
      std::printf("\n");
      return 0;
    }
    if (cmd == "blocks" && argc >= 4) {
      // teacher-forced per segment (a top-level layer, or a BatchNorm with the activation / pool
      // the GPU backend fuses into it): the CPU backend's fp32 activations and gradients of one
      // step are the reference; every GPU segment gets the CPU input and output gradient, and its
      // output, input gradient and parameter gradients are compared. Errors do not compound
      // through the network, so each layer's bound is absolute (tests/test_cpp_host_blocks.py).
      const std::string name = argv[2];
      const int batch = std::atoi(argv[3]);
      const Device gdev = device_arg(argc, argv);
      Sequential mc = create_model(name), mg = create_model(name);
      mc.set_device(Device::cpu());
      mc.initialize(11);
      mg.set_device(gdev);
      mg.initialize(11);
      mc.set_training(true);
      mg.set_training(true);
      const bool cifar = name.find("cifar") != std::string::npos;
      const int hw = cifar ? 32 : 64, classes = cifar ? 10 : 200;
      SyntheticClassification data((size_t)batch, 3, hw, hw, classes, 5, 0.3f);
      data.reset(0);
      Tensor x, y;
      if (!data.next(batch, x, y)) throw std::runtime_error("no batch");
      const auto& lc = mc.layers();
      const auto& lg = mg.layers();
      const size_t L = lc.size();
      // CPU reference: every top-level activation and gradient
      mc.zero_grad();
      std::vector<Tensor> act(L + 1), grad(L + 1);
      act[0] = mc.input_activation(x);
      for (size_t i = 0; i < L; ++i) act[i + 1] = lc[i]->forward(act[i], true);
      const Tensor logits = act[L].view({act[L].dim(0), act[L].numel() / act[L].dim(0)});
      Loss loss = LossFactory::create("softmax_crossentropy");
      LossResult r = loss(logits, y);
      grad[L] = r.grad.view(act[L].shape(), Layout::NCHW);
      lc[0]->set_input_grad(false);
      for (size_t i = L; i-- > 0;) grad[i] = lc[i]->backward(grad[i + 1]);
      auto cosine = [](const std::vector<float>& a, const std::vector<float>& b) {
        double ab = 0, aa = 0, bb = 0;
        for (size_t k = 0; k < a.size() && k < b.size(); ++k) {
          ab += (double)a[k] * b[k];
          aa += (double)a[k] * a[k];
          bb += (double)b[k] * b[k];
        }
        return aa > 0 && bb > 0 ? ab / std::sqrt(aa * bb) : (aa == bb ? 1.0 : 0.0);
      };
      auto rel = [](const std::vector<float>& a, const std::vector<float>& b) {
        double num = 0, den = 0;
        for (size_t k = 0; k < a.size() && k < b.size(); ++k) {
          num += ((double)a[k] - b[k]) * ((double)a[k] - b[k]);
          den += (double)b[k] * b[k];
        }
        return a.size() != b.size() ? 1e9 : std::sqrt(num / (den > 1e-300 ? den : 1e-300));
      };
      // GPU activation of a CPU tensor (bf16 NHWC for 4-D activations)
      auto to_gpu = [&](const Tensor& t) {
        return Tensor::from_host(t.to_host_f32(), t.shape(), gdev, gdev.is_gpu() ? DType::BF16 : DType::F32,
                                 gdev.is_gpu() ? Layout::NHWC : Layout::NCHW);
      };
      mg.zero_grad();
      lg[0]->set_input_grad(false);
      for (size_t i = 0; i < L;) {
        size_t j = i + 1;
        if (auto* bn = dynamic_cast<BatchNorm*>(lg[i].get())) {
          if (gdev.is_gpu() && bn->fused_relu() && j < L) ++j;  // (its ReLU runs in the BatchNorm)
          if (gdev.is_gpu() && bn->fused_pool() && j < L) ++j;  // (and the max-pool)
        }
        Tensor h = i == 0 ? mg.input_activation(x) : to_gpu(act[i]);
        for (size_t k = i; k < j; ++k) h = lg[k]->forward(h, true);
        const double ef = rel(h.to_host_f32(), act[j].to_host_f32());
        Tensor g = to_gpu(grad[j]);
        for (size_t k = j; k-- > i;) g = lg[k]->backward(g);
        double eb = 0, cb = 1;
        if (i > 0 && g.defined()) {
          // (a conv whose input a BatchNorm + ReLU produced returns its data gradient already
          // masked by that ReLU — the mask runs in the dgrad epilogue with the BatchNorm's backward
          // statistics — so the reference is the CPU gradient masked by input > 0 there; the
          // closer of the two references is reported)
          const auto gg = g.to_host_f32(), gc = grad[i].to_host_f32(), xin = act[i].to_host_f32();
          std::vector<float> gm(gc.size());
          for (size_t k = 0; k < gc.size(); ++k) gm[k] = xin[k] > 0.f ? gc[k] : 0.f;
          const double e0 = rel(gg, gc), e1 = rel(gg, gm);
          eb = std::min(e0, e1);
          cb = e1 < e0 ? cosine(gg, gm) : cosine(gg, gc);
        }
        // parameter gradients: error relative to max(|ref|, 5% of the segment's largest gradient)
        // (a conv bias in front of a BatchNorm has a mathematically zero gradient: noise on both)
        double ep = 0, cp = 1;
        std::string pn;
        std::vector<std::pair<std::vector<float>, std::vector<float>>> pairs;
        std::vector<std::string> names;
        double scale = 0;
        for (size_t k = i; k < j; ++k) {
          std::vector<Param*> pc, pg;
          lc[k]->collect_params(pc);
          lg[k]->collect_params(pg);
          for (size_t q = 0; q < pc.size() && q < pg.size(); ++q) {
            pairs.emplace_back(pg[q]->grad.view(pg[q]->shape, pg[q]->layout).to_host_f32(),
                               pc[q]->grad.view(pc[q]->shape, pc[q]->layout).to_host_f32());
            names.push_back(pg[q]->name);
            double nb = 0;
            for (float v : pairs.back().second) nb += (double)v * v;
            scale = std::max(scale, std::sqrt(nb));
          }
        }
        for (size_t q = 0; q < pairs.size(); ++q) {
          const auto& [a, b] = pairs[q];
          double num = 0, nb = 0;
          for (size_t k = 0; k < a.size(); ++k) {
            num += ((double)a[k] - b[k]) * ((double)a[k] - b[k]);
            nb += (double)b[k] * b[k];
          }
          const double e = std::sqrt(num) / std::max(std::sqrt(nb), 0.05 * scale + 1e-30);
          if (e > ep) {
            ep = e;
            pn = names[q];
          }
          if (std::sqrt(nb) >= 0.05 * scale) cp = std::min(cp, cosine(a, b));
        }
        std::printf("segment %zu %zu %s fwd %.6g bwd %.6g param %.6g %s bcos %.6g pcos %.6g\n", i, j,
                    lg[i]->name().c_str(), ef, eb, ep, pn.empty() ? "-" : pn.c_str(), cb, cp);
        i = j;
      }
      return 0;
    }
    if (cmd == "train" && argc >= 6) {
      const Device dev = device_arg(argc, argv);
      Sequential m = create_model(argv[2]);
      m.set_device(dev);
      m.initialize(11);
      const int steps = std::atoi(argv[3]), batch = std::atoi(argv[4]);
      const bool cifar = std::string(argv[2]).find("cifar") != std::string::npos;
      const int hw = cifar ? 32 : 64, classes = cifar ? 10 : 200;
      SyntheticClassification data((size_t)batch * steps, 3, hw, hw, classes, 5, 0.3f);
      Adam opt(1e-3f);
      Loss loss = LossFactory::create("softmax_crossentropy");
      data.reset(0);
      Tensor x, y;
      bool graph = false;  // --graph: the GPU step captured once (TrainGraph) and replayed
      for (int i = 1; i < argc; ++i) graph = graph || std::string(argv[i]) == "--graph";
      TrainGraph tg(m, opt, loss);
      std::printf("losses");
      for (int i = 0; i < steps && data.next(batch, x, y); ++i) {
        if (graph && dev.is_gpu()) {
          tg.step(x, y);
          std::printf(" %.6g", tg.last_loss());
          continue;
        }
        m.zero_grad();
        LossResult r = loss(m.forward(x), y);
        m.backward(r.grad);
        opt.step(m.parameters());
        std::printf(" %.6g", r.loss);
      }
      std::printf("\n");
      m.save_to_file(argv[5]);
      return 0;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  std::fprintf(stderr, "bad arguments\n");
  return 2;
}
