// ResNet-18 (or -34 / -50 / ResNet-9) on Tiny-ImageNet trained from C++ on the dcnn host API —
// residual blocks, the routed MFMA conv kernels, a scheduler and a loss of the factories; no Python.
//
//   dcnn_amd/bin/tiny_imagenet_resnet18 [--device CPU|GPU] [--model resnet18_tiny_imagenet]
//        [--data data/tiny-imagenet-200] [--epochs E] [--steps S] [--batch B] [--lr 1e-3]
//        [--loss logsoftmax_ce] [--scheduler cosine_annealing_lr] [--max-per-class K]
//        [--save model_snapshots/resnet18] [--bench [--eager] [--warmup W]] [--dp] [--device-data]
//
// Without --data it trains on a learnable synthetic 3x64x64 200-class set. --device-data (GPU, with
// --data): the GPU data path (DeviceImageDataset): the decoded set lives in HBM as uint8 and every
// batch is one augment_batch launch (random crop +-4, horizontal flip, ImageNet normalisation) on
// the training flow — with --bench that launch is inside every timed step. --bench times
// --steps training steps after --warmup (3) warm-up steps on two device-resident synthetic batches and
// prints one JSON line (images/sec); on the GPU the step is captured into a hipGraph
// (dcnn::TrainGraph) and replayed, --eager launches every kernel from the host instead. The saved
// model (path.json + path.bin + path.bnstats) loads in Python with Sequential.from_file.
// --dp (--bench): data parallel, one process per GPU under the torch.distributed launcher's
// variables (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT; dcnn/dist.hpp): rank 0's
// weights are broadcast, each rank trains --batch samples per step, the bucketed gradient mean runs
// inside the captured step over RCCL (--device CPU: over the host TCP ring), the timed steps are
// fenced by barriers and rank 0 prints the whole job's images/sec with the slowest rank's time.
// Honours the reference's .env keys DEVICE_TYPE / EPOCHS / BATCH_SIZE / LR_INITIAL.
// Reference parity: examples/tiny_imagenet_resnet18.cpp:23-107 (Adam, logsoftmax-CE, profiling),
// include/nn/example_models.hpp:306-331 (the model).
#include <algorithm>
#include <chrono>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <string>

#include "dcnn/dist.hpp"
#include "dcnn/nn.hpp"
#include "dcnn/train.hpp"

using namespace dcnn;

namespace {
std::string env_or(const char* k, const std::string& d) {
  const char* v = std::getenv(k);
  return v && *v ? v : d;
}
}  // namespace

int main(int argc, char** argv) {
  std::string device = env_or("DEVICE_TYPE", "CPU"), data, save, model_name = "resnet18_tiny_imagenet";
  std::string loss_name = "logsoftmax_ce", sched_name;
  int epochs = std::atoi(env_or("EPOCHS", "1").c_str()), steps = -1, max_per_class = 0, warmup = 3;
  int batch = std::atoi(env_or("BATCH_SIZE", "64").c_str());
  float lr = std::atof(env_or("LR_INITIAL", "0.001").c_str());
  bool bench = false, eager = false, dp_on = false, device_data = false;
  for (int i = 1; i < argc; ++i) {
    const std::string k = argv[i];
    if (k == "--bench") { bench = true; continue; }
    if (k == "--eager") { eager = true; continue; }
    if (k == "--dp") { dp_on = true; continue; }
    if (k == "--device-data") { device_data = true; continue; }
    if (i + 1 >= argc) break;
    const std::string v = argv[++i];
    if (k == "--device") device = v;
    else if (k == "--model") model_name = v;
    else if (k == "--data") data = v;
    else if (k == "--epochs") epochs = std::atoi(v.c_str());
    else if (k == "--steps") steps = std::atoi(v.c_str());
    else if (k == "--batch") batch = std::atoi(v.c_str());
    else if (k == "--lr") lr = std::atof(v.c_str());
    else if (k == "--loss") loss_name = v;
    else if (k == "--scheduler") sched_name = v;
    else if (k == "--max-per-class") max_per_class = std::atoi(v.c_str());
    else if (k == "--save") save = v;
    else if (k == "--warmup") warmup = std::atoi(v.c_str());
  }
  try {
    Sequential model = create_model(model_name);
    std::unique_ptr<dist::DataParallel> dp;
    Device dev = Device::parse(device);
    if (dp_on) {
      if (!bench) throw std::invalid_argument("--dp: --bench runs only");
      const dist::Env env = dist::Env::from_env();
      dp = std::make_unique<dist::DataParallel>(env, dev);  // (GPU: selects GPU LOCAL_RANK)
      dev = dp->device();
    }
    model.set_device(dev);
    model.initialize(42);
    if (dp) dp->broadcast_parameters(model);  // identical replicas whatever each rank's seed
    std::printf("%s on %s: %zu parameters\n", model.name().c_str(), dev.str().c_str(), model.num_parameters());
    Adam opt(lr);
    Loss loss = LossFactory::create(loss_name);
    const bool cifar = model_name.find("cifar") != std::string::npos;
    const int C = 3, HW = cifar ? 32 : 64, classes = cifar ? 10 : 200;
    std::unique_ptr<DataSource> train, val;
    if (!data.empty() && device_data) {
      // the GPU data path: decoded once into HBM (uint8), every batch one augment_batch launch
      if (!dev.is_gpu()) throw std::invalid_argument("--device-data: GPU runs only");
      const uint64_t rs = dp ? (uint64_t)dp->rank() : 0;
      auto tr = std::make_unique<DeviceImageDataset>(load_tiny_imagenet(data, "train", max_per_class, 1), dev,
                                                     1 + rs);
      tr->random_crop(1.f, 4).horizontal_flip(0.5f).normalize();
      std::printf("device dataset: %zu images, %.1f MB of HBM (%s)\n", tr->size(), tr->device_bytes() / 1e6,
                  tr->stored_u8() ? "uint8" : "fp32");
      train = std::move(tr);
      auto va = std::make_unique<DeviceImageDataset>(load_tiny_imagenet(data, "val", 0, 2), dev, 2, false, false);
      va->normalize();
      val = std::move(va);
    } else if (!data.empty()) {
      auto tr = std::make_unique<ImageDataset>(load_tiny_imagenet(data, "train", max_per_class, 1));
      tr->set_random_flip(0.5f);
      train = std::move(tr);
      val = std::make_unique<ImageDataset>(load_tiny_imagenet(data, "val", 0, 2));
    } else {
      // (data parallel: each rank draws its own samples)
      train = std::make_unique<SyntheticClassification>(bench ? (size_t)batch * (steps + 4) : (size_t)4 * batch, C, HW,
                                                        HW, classes, 7 + (dp ? (uint64_t)dp->rank() : 0), 0.5f);
      val = std::make_unique<SyntheticClassification>((size_t)batch, C, HW, HW, classes, 7, 0.5f);
    }
    if (bench) {
      // steady-state throughput: warm-up steps (kernel instances, workspaces), then timed steps on
      // device-resident synthetic batches (as bench.py: the timed region is the training step,
      // not host-side data synthesis)
      train->reset(0);
      std::vector<std::pair<Tensor, Tensor>> staged;
      // the device dataset assembles a fresh augmented batch inside every timed step instead
      uint64_t epoch = 0;
      auto fresh = [&](Tensor& xb, Tensor& yb) {
        if (!train->next(batch, xb, yb)) {
          train->reset(++epoch);
          if (!train->next(batch, xb, yb)) throw std::runtime_error("--bench: fewer samples than one batch");
        }
      };
      for (int i = 0; i < (device_data ? 0 : 2); ++i) {
        Tensor xh, yh;
        if (!train->next(batch, xh, yh)) {
          train->reset(1);
          train->next(batch, xh, yh);
        }
        staged.emplace_back(xh.to(dev), yh.to(dev));
      }
      const int timed = steps > 0 ? steps : 20;
      int k = 0;
      // GPU: the step captured into a hipGraph (TrainGraph: gpu::Graph on the thread's flow) and
      // replayed with one launch per step; --eager launches every kernel from the host
      const bool graph = dev.is_gpu() && !eager;
      TrainGraph tg(model, opt, loss);
      // data parallel: the mean of the flat arena gradient over the ranks, inside the captured
      // step: bucketed and started from the backward's layer hook on the communicator's own flow
      // (overlapping the earlier layers' backward), joined before the optimizer; DCNN_DP_OVERLAP=0:
      // one all-reduce of the whole arena after the backward
      std::function<void()> allreduce;
      if (dp) {
        ParamArena* arena = model.parameters().at(0)->arena.get();
        const char* ov = std::getenv("DCNN_DP_OVERLAP");
        if (!(ov && std::string(ov) == "0") || !arena) {
          const char* mb = std::getenv("DCNN_DP_BUCKET_MB");
          dp->attach(model, mb && *mb ? std::atof(mb) : 4.0);
          allreduce = [&dp] { dp->finish(); };
        } else {
          allreduce = [&dp, arena] { dp->all_reduce_mean(arena->grad.ptr<float>(), (size_t)arena->grad.numel()); };
        }
        tg.set_gradient_hook(allreduce);
      }
      auto one = [&] {
        Tensor dx, dy;
        if (device_data) fresh(dx, dy);
        const auto& [x, y] = device_data ? std::pair<Tensor, Tensor>{dx, dy} : staged[(size_t)(k++) % staged.size()];
        if (graph) return tg.step(x, y);
        model.zero_grad();
        Tensor logits = model.forward(x);
        LossResult r = loss(logits, y);
        model.backward(r.grad);
        if (allreduce) allreduce();
        opt.step(model.parameters());
        return r.loss;
      };
      for (int i = 0; i < std::max(1, warmup); ++i) one();
      // the timed region is bracketed by a device synchronisation + a barrier over the ranks on
      // both sides; the slowest rank's time is reported
      auto fence = [&] {
        if (dev.is_gpu()) gpu::synchronize();
        if (dp) dp->barrier();
      };
      fence();
      const auto t0 = std::chrono::steady_clock::now();
      double last = 0;
      for (int i = 0; i < timed; ++i) last = one();
      fence();
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (graph) last = tg.last_loss();
      const int world = dp ? dp->world() : 1;
      if (dp) s = dp->max(s);  // the slowest rank
      if (!dp || dp->rank() == 0)
        std::printf("{\"metric\": \"images/sec %s training (C++ host API)\", \"value\": %.1f, \"ms_per_step\": %.3f, "
                    "\"batch\": %d, \"steps\": %d, \"device\": \"%s\", \"hipgraph\": %s, \"loss\": %.6f, "
                    "\"world\": %d, \"data_parallel\": %s%s%s, \"dp_buckets\": %d, \"data\": \"%s, random init\"}\n",
                    model_name.c_str(), (double)batch * world * timed / s, 1e3 * s / timed, batch, timed,
                    dev.str().c_str(), graph ? "true" : "false", last, world, dp ? "\"" : "", dp ? dp->plane() : "null",
                    dp ? "\"" : "", dp ? dp->buckets_last_step() : 0,
                    data.empty() ? "synthetic: 2 device-resident batches per rank of a learnable class-template set "
                                   "(SyntheticClassification)"
                    : device_data ? "--data decoded into HBM, one augment_batch launch per step (crop, flip, normalise)"
                                  : "2 device-resident batches per rank staged from --data");
      return 0;
    }
    std::unique_ptr<Scheduler> sched;
    if (!sched_name.empty()) {
      json::Value p = json::Value::object();
      const long total = (long)epochs * (long)(steps > 0 ? steps : (long)(train->size() / batch));
      p["T_max"] = (int64_t)std::max(1l, total);
      p["total_steps"] = (int64_t)std::max(1l, total);
      sched = SchedulerFactory::create(sched_name, &opt, p);
    }
    TrainingConfig cfg;
    cfg.epochs = epochs;
    cfg.batch_size = batch;
    cfg.max_steps = steps;
    cfg.progress_interval = 20;
    train_model(model, *train, val.get(), opt, loss, cfg, sched.get());
    if (!save.empty()) {
      model.save_to_file(save);
      std::printf("saved %s.json / .bin / .bnstats\n", save.c_str());
    }
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
