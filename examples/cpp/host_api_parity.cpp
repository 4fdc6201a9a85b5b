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
//   host_api_parity train <model_name> <steps> <batch> <save> [--device GPU] [--graph]
//                                              Adam steps on a synthetic set, then save
// Output is plain text: one "key v0 v1 ..." line per item.
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
