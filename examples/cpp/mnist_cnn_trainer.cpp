// MNIST-shaped CNN trained from C++ on the dcnn host API (no Python).
//
//   dcnn_amd/bin/mnist_cnn_trainer [--device CPU|GPU] [--epochs E] [--steps S] [--batch B]
//                                  [--csv data/mnist/train.csv] [--save model_snapshots/mnist_cnn]
//
// Without --csv it trains on a learnable synthetic 1x28x28 ten-class set. The saved model
// (path.json + path.bin) loads in Python with dcnn_amd.nn.Sequential.from_file. Also honours the
// reference's .env keys DEVICE_TYPE / EPOCHS / BATCH_SIZE / LR_INITIAL.
// Reference parity: examples/mnist_cnn_trainer.cpp, include/nn/example_models.hpp (create_mnist_trainer).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>

#include "dcnn/nn.hpp"

using namespace dcnn;

namespace {
std::string env_or(const char* k, const std::string& d) {
  const char* v = std::getenv(k);
  return v && *v ? v : d;
}

// label,pixel0,...,pixel783 rows (the reference's MNIST CSV)
class MnistCsv : public DataSource {
 public:
  explicit MnistCsv(const std::string& path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot read " + path);
    std::string line;
    while (std::getline(f, line)) {
      if (line.empty() || !std::isdigit((unsigned char)line[0])) continue;  // header
      std::stringstream ss(line);
      std::string tok;
      std::getline(ss, tok, ',');
      labels_.push_back(std::stoll(tok));
      while (std::getline(ss, tok, ',')) pix_.push_back(std::stof(tok) / 255.f);
    }
  }
  void reset(uint64_t) override { pos_ = 0; }
  bool next(int batch, Tensor& x, Tensor& y) override {
    if (pos_ >= labels_.size()) return false;
    const size_t b = std::min<size_t>((size_t)batch, labels_.size() - pos_);
    std::vector<float> xs(pix_.begin() + pos_ * 784, pix_.begin() + (pos_ + b) * 784);
    std::vector<int64_t> ys(labels_.begin() + pos_, labels_.begin() + pos_ + b);
    x = Tensor::from_host(xs, {(int64_t)b, 1, 28, 28}, Device::cpu());
    y = Tensor::from_host_i64(ys, Device::cpu());
    pos_ += b;
    return true;
  }
  size_t size() const override { return labels_.size(); }

 private:
  std::vector<int64_t> labels_;
  std::vector<float> pix_;
  size_t pos_ = 0;
};
}  // namespace

int main(int argc, char** argv) {
  std::string device = env_or("DEVICE_TYPE", "CPU"), csv, save = "model_snapshots/mnist_cnn";
  int epochs = std::atoi(env_or("EPOCHS", "1").c_str()), steps = -1;
  int batch = std::atoi(env_or("BATCH_SIZE", "64").c_str());
  float lr = std::atof(env_or("LR_INITIAL", "0.001").c_str());
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i], v = argv[i + 1];
    if (k == "--device") device = v;
    else if (k == "--epochs") epochs = std::atoi(v.c_str());
    else if (k == "--steps") steps = std::atoi(v.c_str());
    else if (k == "--batch") batch = std::atoi(v.c_str());
    else if (k == "--csv") csv = v;
    else if (k == "--save") save = v;
    else if (k == "--lr") lr = std::atof(v.c_str());
  }
  try {
    const Device dev = Device::parse(device);
    auto model = SequentialBuilder("mnist_cnn")
                     .input({1, 28, 28})
                     .conv2d(16, 3, 3, 1, 1, 1, 1)
                     .batchnorm()
                     .activation("relu")
                     .maxpool2d(2, 2)
                     .conv2d(32, 3, 3, 1, 1, 1, 1)
                     .batchnorm()
                     .activation("relu")
                     .maxpool2d(2, 2)
                     .flatten()
                     .dense(64)
                     .activation("relu")
                     .dense(10)
                     .build();
    model.set_device(dev);
    model.initialize(42);
    model.print_config();
    std::printf("device %s, %zu parameters\n", dev.str().c_str(), model.num_parameters());

    std::unique_ptr<DataSource> train, val;
    if (!csv.empty()) {
      train = std::make_unique<MnistCsv>(csv);
    } else {
      train = std::make_unique<SyntheticClassification>(4096, 1, 28, 28, 10, 7, 3.0f);
      val = std::make_unique<SyntheticClassification>(512, 1, 28, 28, 10, 7, 3.0f);
    }
    Adam opt(lr);
    TrainingConfig cfg;
    cfg.epochs = epochs;
    cfg.batch_size = batch;
    cfg.max_steps = steps;
    cfg.progress_interval = 20;
    auto hist = train_classification_model(model, *train, val.get(), opt, cfg);

    model.save_to_file(save);
    // reload and check the saved model reproduces the trained one's logits
    Sequential back = Sequential::from_file(save, dev);
    back.set_training(false);
    model.set_training(false);
    Tensor x, y;
    SyntheticClassification probe(8, 1, 28, 28, 10, 99);
    probe.reset(0);
    probe.next(8, x, y);
    const auto a = model.forward(x).to_host_f32(), b = back.forward(x).to_host_f32();
    double md = 0;
    for (size_t i = 0; i < a.size(); ++i) md = std::max(md, (double)std::abs(a[i] - b[i]));
    std::printf("saved %s.{json,bin}; reload max |dlogit| = %.3g\n", save.c_str(), md);
    {
      std::ofstream f(save + ".probe.txt");
      for (float v : a) f << v << "\n";
      std::ofstream fx(save + ".probe_x.bin", std::ios::binary);
      x.save(fx);  // the probe batch as a .bin record (first dim 8, then 1 x 28 x 28)
    }
    if (dev.is_gpu()) {
      // the same saved model on the CPU backend (fp32): the bf16 GPU path must agree closely
      Sequential cpu = Sequential::from_file(save, Device::cpu());
      cpu.set_training(false);
      const auto c = cpu.forward(x).to_host_f32();
      double num = 0, den = 0;
      for (size_t i = 0; i < a.size(); ++i) {
        num += (double)(a[i] - c[i]) * (a[i] - c[i]);
        den += (double)c[i] * c[i];
      }
      std::printf("GPU vs CPU logits: rel l2 %.3g\n", std::sqrt(num / std::max(den, 1e-30)));
    }
    std::printf("RESULT first_loss=%.5f last_loss=%.5f val_acc=%.4f reload_diff=%.3g\n",
                hist.empty() ? 0.0 : hist.front().train_loss, hist.empty() ? 0.0 : hist.back().train_loss,
                hist.empty() ? 0.0 : hist.back().val_acc, md);
    return md == 0.0 ? 0 : 2;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
