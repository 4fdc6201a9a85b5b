// Pipeline-parallel training driven from C++: the native coordinator (dcnn::PipelineCoordinator)
// partitions a model over stage worker processes (dcnn_amd/bin/network_worker, or Python
// workers) and trains it with the sync (GPipe), semi-async or 1F1B schedule. No Python.
//
//   dcnn_amd/bin/pipeline_coordinator (--workers H:P,H:P,... | --spawn N)
//        [--model mnist_cnn|resnet9_cifar10|... | --config arch.json | --init snapshot] [--schedule semi_async]
//        [--microbatches 4] [--batch 64] [--steps 20] [--optimizer adam|sgd] [--lr 1e-3]
//        [--momentum 0.9] [--devices CPU,CPU | --device GPU:0] [--loss softmax_crossentropy]
//        [--data-x x.f32 --data-y y.i64] [--input C,H,W] [--classes K] [--save out]
//        [--heartbeat S] [--transport message|ipc|rccl] [--stage-loss auto|0|1] [--partitioner naive|flops]
//        [--json] [--bench W]
//
// --spawn N starts N local native workers (this program never touches the GPU itself, so starting
// them is safe). --init loads a saved model (path.json + path.bin [+ .bnstats]) whose weights are
// pushed to the stages. --data-x / --data-y are raw fp32 NCHW images and int64 labels, batch after
// batch; without them a learnable synthetic set of --input / --classes is used. --json prints one
// JSON line per step; --bench W times the steps after W untimed warm-up steps (images/sec).
// --transport ipc (GPU stages on one node): stage-to-stage activations and gradients stay on the
// device (HIP IPC buffers); only their handles travel in the messages. --transport rccl (GPU stages
// on distinct devices, one node or several): they travel as RCCL sends on per-direction stage-pair
// links, the messages carry only their shapes. --stage-loss: the loss on
// the last stage's GPU (auto: when that stage is a native GPU stage) — the labels go there, only
// the loss value comes back, and the backward starts without a round trip through this process.
// Reference parity: examples/semi_async_pipeline_coordinator.cpp, sync_pipeline_coordinator.cpp,
// coordinator_tiny_imagenet.cpp; include/pipeline/distributed_coordinator.hpp.
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "dcnn/pipeline.hpp"

extern char** environ;

using namespace dcnn;

namespace {
std::vector<std::string> split_list(const std::string& s, char sep = ',') {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, sep))
    if (!t.empty()) out.push_back(t);
  return out;
}

std::string self_dir() {
  char buf[4096];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return ".";
  std::string p(buf, (size_t)n);
  return p.substr(0, p.rfind('/'));
}

// local native workers on free ports: (pid, port)
struct Spawned {
  pid_t pid;
  int port;
  int out_fd;  // the worker's stdout (kept open: a later write must not raise SIGPIPE)
};
void spawn_workers(int n, std::vector<Spawned>& out) {
  const std::string exe = self_dir() + "/network_worker";
  for (int i = 0; i < n; ++i) {
    int fds[2];
    if (pipe(fds) != 0) throw std::runtime_error("pipe failed");
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_adddup2(&fa, fds[1], 1);
    posix_spawn_file_actions_addclose(&fa, fds[0]);
    std::vector<std::string> args{exe, "0", "--host", "127.0.0.1"};
    std::vector<char*> argv;
    for (auto& a : args) argv.push_back(a.data());
    argv.push_back(nullptr);
    pid_t pid = 0;
    const int rc = posix_spawn(&pid, exe.c_str(), &fa, nullptr, argv.data(), environ);
    posix_spawn_file_actions_destroy(&fa);
    close(fds[1]);
    if (rc != 0) throw std::runtime_error("cannot start " + exe);
    // "native stage worker listening on port P (pid X)"
    std::string line;
    char ch;
    while (read(fds[0], &ch, 1) == 1 && ch != '\n') line.push_back(ch);
    const auto at = line.find("port ");
    out.push_back({pid, at == std::string::npos ? 0 : std::atoi(line.c_str() + at + 5), fds[0]});
    if (at == std::string::npos) throw std::runtime_error("worker did not report its port: " + line);
  }
}

std::vector<char> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  return std::vector<char>(std::istreambuf_iterator<char>(f), {});
}
}  // namespace

int main(int argc, char** argv) {
  std::string workers, model_name = "mnist_cnn", config_path, init, schedule = "semi_async", opt_name = "adam";
  std::string devices, loss_name = "softmax_crossentropy", data_x, data_y, save, input = "1,28,28";
  std::string transport = "message", partitioner = "naive";
  int spawn = 0, microbatches = 4, batch = 64, steps = 20, classes = 10, bench = -1, stage_loss = -1;
  float lr = 1e-3f, momentum = 0.f;
  double heartbeat = 0;
  bool json_out = false;
  for (int i = 1; i < argc; ++i) {
    const std::string k = argv[i];
    if (k == "--json") { json_out = true; continue; }
    if (i + 1 >= argc) {
      std::fprintf(stderr, "missing value for %s\n", k.c_str());
      return 2;
    }
    const std::string v = argv[++i];
    if (k == "--workers") workers = v;
    else if (k == "--spawn") spawn = std::atoi(v.c_str());
    else if (k == "--model") model_name = v;
    else if (k == "--config") config_path = v;
    else if (k == "--init") init = v;
    else if (k == "--schedule") schedule = v;
    else if (k == "--microbatches") microbatches = std::atoi(v.c_str());
    else if (k == "--batch") batch = std::atoi(v.c_str());
    else if (k == "--steps") steps = std::atoi(v.c_str());
    else if (k == "--optimizer") opt_name = v;
    else if (k == "--lr") lr = std::atof(v.c_str());
    else if (k == "--momentum") momentum = std::atof(v.c_str());
    else if (k == "--devices" || k == "--device") devices = v;
    else if (k == "--loss") loss_name = v;
    else if (k == "--data-x") data_x = v;
    else if (k == "--data-y") data_y = v;
    else if (k == "--input") input = v;
    else if (k == "--classes") classes = std::atoi(v.c_str());
    else if (k == "--save") save = v;
    else if (k == "--heartbeat") heartbeat = std::atof(v.c_str());
    else if (k == "--bench") bench = std::atoi(v.c_str());
    else if (k == "--transport") transport = v;
    else if (k == "--stage-loss") stage_loss = v == "auto" ? -1 : std::atoi(v.c_str());
    else if (k == "--partitioner") partitioner = v;
    else {
      std::fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  std::vector<Spawned> local;
  int rc = 0;
  try {
    std::vector<Endpoint> eps;
    if (spawn > 0) {
      spawn_workers(spawn, local);
      for (auto& s : local) {
        Endpoint e;
        e.parameters["host"] = "127.0.0.1";
        e.parameters["port"] = s.port;
        eps.push_back(e);
      }
    } else {
      for (const auto& w : split_list(workers)) {
        const auto c = w.rfind(':');
        if (c == std::string::npos) throw std::invalid_argument("worker endpoint must be host:port, got " + w);
        Endpoint e;
        e.parameters["host"] = w.substr(0, c);
        e.parameters["port"] = std::atoi(w.c_str() + c + 1);
        eps.push_back(e);
      }
    }
    if (eps.empty()) throw std::invalid_argument("no workers: give --workers H:P,... or --spawn N");

    // the full model on the host: its architecture is partitioned, its weights pushed
    Sequential model;
    if (!init.empty()) {
      model = Sequential::from_file(init);
    } else {
      if (!config_path.empty()) {
        const std::vector<char> b = read_file(config_path);
        model = Sequential::load_from_config(json::Value::parse(std::string(b.begin(), b.end())));
      } else {
        model = create_model(model_name);
      }
      model.initialize(42);
    }

    json::Value oc = json::Value::object();
    oc["type"] = opt_name;
    json::Value op = json::Value::object();
    op["learning_rate"] = (double)lr;
    if (opt_name == "sgd") op["momentum"] = (double)momentum;
    oc["parameters"] = std::move(op);

    CoordinatorOptions o;
    o.num_microbatches = microbatches;
    o.loss = loss_name;
    o.heartbeat_s = heartbeat;
    o.transport = transport;
    o.stage_loss = stage_loss;
    if (!devices.empty()) {
      o.stage_devices = split_list(devices);
      if (o.stage_devices.size() == 1) o.stage_devices.assign(eps.size(), o.stage_devices[0]);
    }
    PipelineCoordinator coord(model.get_config(), oc, eps, o);
    std::vector<Partition> parts;
    if (partitioner == "flops") {
      // FLOP-balanced stages (forward + backward of each top-level layer at the micro-batch shape)
      std::vector<int64_t> shape{std::max(1, batch / std::max(1, microbatches))};
      for (const auto& d : split_list(input)) shape.push_back(std::atoll(d.c_str()));
      parts = balanced_partitions(model.layer_flops(shape), (int)eps.size());
    } else if (partitioner != "naive") {
      throw std::invalid_argument("unknown partitioner " + partitioner + " (naive, flops)");
    }
    coord.initialize(parts);
    coord.deploy_stages();
    coord.start();
    coord.send_parameters(model);
    for (size_t i = 0; i < coord.partitions().size(); ++i)
      std::fprintf(stderr, "stage_%zu: layers [%d, %d) on %s\n", i, coord.partitions()[i].start,
                   coord.partitions()[i].end, (o.stage_devices.empty() ? "CPU" : o.stage_devices[i].c_str()));

    // data: raw files batch after batch, or the synthetic set
    const std::vector<std::string> chw_s = split_list(input);
    if (chw_s.size() != 3) throw std::invalid_argument("--input must be C,H,W");
    const int C = std::atoi(chw_s[0].c_str()), H = std::atoi(chw_s[1].c_str()), W = std::atoi(chw_s[2].c_str());
    std::vector<char> xb, yb;
    std::unique_ptr<SyntheticClassification> synth;
    if (!data_x.empty()) {
      xb = read_file(data_x);
      yb = read_file(data_y);
    } else {
      synth = std::make_unique<SyntheticClassification>((size_t)batch * 8, C, H, W, classes, 7, 0.5f);
      synth->reset(0);
    }
    const size_t per = (size_t)C * H * W;
    const Schedule sched = parse_schedule(schedule);
    std::vector<std::pair<Tensor, Tensor>> staged;
    auto next_batch = [&](int step, Tensor& x, Tensor& y) {
      if (!xb.empty()) {
        const size_t off = (size_t)step * batch;
        if ((off + batch) * per * 4 > xb.size() || (off + batch) * 8 > yb.size())
          throw std::runtime_error("--data-x / --data-y hold fewer than " + std::to_string(step + 1) + " batches");
        std::vector<float> xv(batch * per);
        std::memcpy(xv.data(), xb.data() + off * per * 4, xv.size() * 4);
        std::vector<int64_t> yv(batch);
        std::memcpy(yv.data(), yb.data() + off * 8, yv.size() * 8);
        x = Tensor::from_host(xv, {batch, C, H, W}, Device::cpu());
        y = Tensor::from_host_i64(yv, Device::cpu());
      } else if (bench >= 0 && !staged.empty()) {
        x = staged[(size_t)step % staged.size()].first;  // (bench: batches synthesised once)
        y = staged[(size_t)step % staged.size()].second;
      } else if (!synth->next(batch, x, y)) {
        synth->reset((uint64_t)step);
        synth->next(batch, x, y);
      }
    };
    if (bench >= 0 && xb.empty())
      for (int i = 0; i < 2; ++i) {
        Tensor sx, sy;
        if (!synth->next(batch, sx, sy)) {
          synth->reset(1);
          synth->next(batch, sx, sy);
        }
        staged.emplace_back(sx, sy);
      }
    const int warm = bench > 0 ? bench : 0;
    Tensor x, y;
    std::chrono::steady_clock::time_point t0;
    double last = 0;
    for (int s = 0; s < warm + steps; ++s) {
      if (s == warm) {
        coord.barrier();
        t0 = std::chrono::steady_clock::now();
      }
      next_batch(s, x, y);
      const auto ts = std::chrono::steady_clock::now();
      const StepResult r = coord.train_step(x, y, sched);
      last = r.loss;
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
      if (json_out)
        std::printf("{\"step\": %d, \"loss\": %.9g, \"correct\": %ld, \"samples\": %ld, \"ms\": %.3f}\n", s, r.loss,
                    r.correct, r.samples, ms);
      else if (bench < 0)
        std::printf("step %d: loss %.5f acc %.3f (%.1f ms)\n", s, r.loss, (double)r.correct / (double)r.samples, ms);
      std::fflush(stdout);
    }
    if (bench >= 0) {
      coord.barrier();
      const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      std::printf("{\"metric\": \"images/sec pipeline training (native coordinator + %d stages, %s, %d micro-batches)\", "
                  "\"value\": %.1f, \"ms_per_step\": %.3f, \"batch\": %d, \"steps\": %d, \"loss\": %.4f, "
                  "\"transport\": \"%s\"}\n",
                  coord.num_stages(), schedule.c_str(), microbatches, (double)batch * steps / sec, 1e3 * sec / steps,
                  batch, steps, last, transport.c_str());
    }
    for (const auto& line : coord.print_profiling()) std::fprintf(stderr, "%s", line.c_str());
    if (!save.empty()) {
      coord.gather_into(model);
      model.save_to_file(save);
      std::fprintf(stderr, "saved %s.json / .bin / .bnstats\n", save.c_str());
    }
    coord.stop();
  } catch (const std::exception& e) {
    std::cerr << "pipeline_coordinator: " << e.what() << std::endl;
    rc = 1;
  }
  for (auto& s : local) {
    int st = 0;
    // (SHUTDOWN ends them; a worker that never got a configuration is stopped)
    for (int k = 0; k < 40 && waitpid(s.pid, &st, WNOHANG) == 0; ++k) usleep(50000);
    if (waitpid(s.pid, &st, WNOHANG) == 0) {
      kill(s.pid, SIGKILL);
      waitpid(s.pid, &st, 0);
    }
    close(s.out_fd);
  }
  return rc;
}
