// Losses, schedulers, dataset loaders and the model zoo of the C++ host API (dcnn/train.hpp).
#include "dcnn/train.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <thread>

namespace dcnn_native {
bool decode_jpeg(const unsigned char* data, size_t n, std::vector<unsigned char>& rgb, int& w, int& h,
                 std::string* err);  // csrc/native/jpeg.cpp
}

namespace dcnn {

// ================================================================= losses
LossResult Loss::compute(const Tensor& pred, const Tensor* labels_in, const Tensor* target_in, float grad_scale) const {
  if (pred.rank() != 2) throw std::runtime_error("loss: expected [N, C] predictions");
  const int N = (int)pred.dim(0), C = (int)pred.dim(1);
  const Device dev = pred.device();
  Tensor labels, target;
  if (labels_in) labels = labels_in->device() == dev ? *labels_in : labels_in->to(dev);
  if (target_in) {
    if (target_in->numel() != (int64_t)N * C) throw std::runtime_error("loss: target must be [N, C]");
    target = target_in->device() == dev ? *target_in : target_in->to(dev);
  }
  if (!labels.defined() && !target.defined()) throw std::runtime_error("loss: labels or a target are required");
  const int64_t* lp = labels.defined() ? labels.ptr<int64_t>() : nullptr;
  const float* tp = target.defined() ? target.ptr<float>() : nullptr;
  LossResult r;
  if (dev.is_gpu()) {
    r.grad = Tensor::empty({N, C}, DType::BF16, dev, Layout::NHWC);
    r.loss = gpu_ops::loss(kind_, pred.data(), tp, lp, r.grad.data(), N, C, param_, &r.correct, grad_scale);
  } else {
    r.grad = Tensor::empty({N, C}, DType::F32, dev);
    r.loss = cpu_ops::loss(kind_, pred.ptr<float>(), tp, lp, r.grad.ptr<float>(), N, C, param_, &r.correct);
    if (grad_scale != 1.f) {
      float* g = r.grad.ptr<float>();
      for (int64_t i = 0; i < (int64_t)N * C; ++i) g[i] *= grad_scale;
    }
  }
  return r;
}

// ================================================================= captured training step
void TrainGraph::capture(const Tensor& x, const Tensor& labels) {
  const Device dev = model_.device();
  sx_ = x.to(dev).clone();
  sy_ = labels.to(dev).clone();
  std::vector<Param*> params = model_.parameters();
  ParamArena* a = params.empty() ? nullptr : params[0]->arena.get();
  if (!a) throw std::runtime_error("TrainGraph: the model's parameters are not in a GPU arena");
  // the warm-up steps must not train: snapshot what they change (parameters, moments, shadow,
  // BatchNorm running statistics)
  const Tensor v0 = a->value.clone(), m0 = a->m.clone(), w0 = a->v.clone(), s0 = a->shadow.clone();
  std::vector<std::pair<Tensor, Tensor>> bn0;  // (live buffer, its snapshot)
  for (BatchNorm* bn : model_.batchnorms())
    for (Tensor* t : {&bn->running_mean, &bn->running_var})
      if (t->defined()) bn0.emplace_back(*t, t->clone());
  const long t0 = opt_.step_count();
  auto eager = [&] {
    model_.zero_grad();
    LossResult r = loss_(model_.forward(sx_), sy_);
    model_.backward(r.grad);
    if (grad_hook_) grad_hook_();
    opt_.step(params);
  };
  for (int i = 0; i < 2; ++i) eager();
  gpu::copy(a->value.data(), v0.data(), v0.nbytes(), 2);
  gpu::copy(a->m.data(), m0.data(), m0.nbytes(), 2);
  gpu::copy(a->v.data(), w0.data(), w0.nbytes(), 2);
  gpu::copy(a->shadow.data(), s0.data(), s0.nbytes(), 2);
  for (auto& [live, snap] : bn0) gpu::copy(live.data(), snap.data(), snap.nbytes(), 2);
  a->refresh_transposes();
  opt_.set_step_count(t0);
  opt_.upload_hyper();
  gpu::flow_synchronize();
  graph_.begin();
  try {
    eager();
  } catch (...) {
    graph_.end();
    throw;
  }
  graph_.end();
  opt_.set_step_count(t0);  // the captured step has not run yet: each replay advances it
  opt_.upload_hyper();
  captured_ = true;
}

double TrainGraph::step(const Tensor& x, const Tensor& labels) {
  const Device dev = model_.device();
  if (!dev.is_gpu()) {  // the CPU backend runs the same step eagerly
    model_.zero_grad();
    LossResult r = loss_(model_.forward(x), labels);
    model_.backward(r.grad);
    if (grad_hook_) grad_hook_();
    opt_.step(model_.parameters());
    return r.loss;
  }
  if (!captured_) capture(x, labels);
  if (x.numel() != sx_.numel() || labels.numel() != sy_.numel())
    throw std::runtime_error("TrainGraph: the batch shape changed after capture");
  // the batch into the static slots (device-resident batches: stream-ordered D2D copies, both in
  // one kernel launch)
  if (x.device() == dev && labels.device() == dev) {
    gpu::copy2_d2d(sx_.data(), x.data(), sx_.nbytes(), sy_.data(), labels.data(), sy_.nbytes());
  } else {
    if (x.device() == dev) gpu::copy(sx_.data(), x.data(), sx_.nbytes(), 2);
    else gpu::copy(sx_.data(), x.to(dev).data(), sx_.nbytes(), 2);
    if (labels.device() == dev) gpu::copy(sy_.data(), labels.data(), sy_.nbytes(), 2);
    else gpu::copy(sy_.data(), labels.to(dev).data(), sy_.nbytes(), 2);
  }
  opt_.before_replay();
  graph_.replay();
  return std::nan("");
}

double TrainGraph::last_loss() {
  if (!model_.device().is_gpu() || !captured_) return std::nan("");
  float l = 0.f;
  gpu::copy(&l, gpu_ops::loss_device(), sizeof l, 1);
  return l;
}

Loss LossFactory::create(const std::string& name, float param) {
  std::string n = name;
  std::transform(n.begin(), n.end(), n.begin(), ::tolower);
  if (n == "ce" || n == "crossentropy" || n == "cross_entropy")
    return Loss(0, param >= 0 ? param : 1e-15f, "crossentropy");
  if (n == "softmax_ce" || n == "softmax_crossentropy" || n == "softmax_cross_entropy")
    return Loss(1, param >= 0 ? param : 1e-15f, "softmax_crossentropy");
  if (n == "logsoftmax_ce" || n == "logsoftmax_crossentropy" || n == "log_softmax_crossentropy")
    return Loss(2, param >= 0 ? param : 1e-15f, "logsoftmax_crossentropy");
  if (n == "mse") return Loss(3, 0.f, "mse");
  if (n == "mae") return Loss(4, 0.f, "mae");
  if (n == "huber") return Loss(5, param >= 0 ? param : 1.0f, "huber");
  throw std::invalid_argument("unknown loss '" + name + "'");
}

// ================================================================= schedulers
namespace {
constexpr double kPi = 3.14159265358979323846;
}

json::Value Scheduler::get_config() const {
  json::Value c = json::Value::object();
  c["type"] = type();
  c["name"] = type();
  c["parameters"] = parameters_config();
  return c;
}

void StepLR::step() {
  ++step_;
  if (step_ % size_ == 0) set_lr(get_lr() * gamma_);
}
json::Value StepLR::parameters_config() const {
  json::Value p = json::Value::object();
  p["step_size"] = size_;
  p["gamma"] = gamma_;
  return p;
}

MultiStepLR::MultiStepLR(Optimizer* o, std::vector<int> milestones, double gamma)
    : Scheduler(o), ms_(std::move(milestones)), gamma_(gamma) {
  std::sort(ms_.begin(), ms_.end());
}
void MultiStepLR::step() {
  ++step_;
  if (idx_ < ms_.size() && step_ >= ms_[idx_]) {
    set_lr(get_lr() * gamma_);
    ++idx_;
  }
}
void MultiStepLR::reset() {
  Scheduler::reset();
  idx_ = 0;
}
json::Value MultiStepLR::parameters_config() const {
  json::Value p = json::Value::object();
  json::Value m = json::Value::array();
  for (int v : ms_) m.push(v);
  p["milestones"] = std::move(m);
  p["gamma"] = gamma_;
  return p;
}

void ExponentialLR::step() {
  ++step_;
  set_lr(get_lr() * gamma_);
}
json::Value ExponentialLR::parameters_config() const {
  json::Value p = json::Value::object();
  p["gamma"] = gamma_;
  return p;
}

void CosineAnnealingLR::step() {
  ++step_;
  const long s = step_ % tmax_;
  set_lr(eta_min_ + (base_lr_ - eta_min_) * (1 + std::cos(kPi * s / tmax_)) / 2);
}
json::Value CosineAnnealingLR::parameters_config() const {
  json::Value p = json::Value::object();
  p["T_max"] = tmax_;
  p["eta_min"] = eta_min_;
  return p;
}

void CosineAnnealingWarmRestarts::step() {
  ++step_;
  ++tcur_;
  if (tcur_ >= ti_) {
    tcur_ = 0;
    ti_ *= tmult_;
  }
  set_lr(eta_min_ + (base_lr_ - eta_min_) * (1 + std::cos(kPi * (double)tcur_ / (double)ti_)) / 2);
}
void CosineAnnealingWarmRestarts::reset() {
  Scheduler::reset();
  tcur_ = 0;
  ti_ = t0_;
}
json::Value CosineAnnealingWarmRestarts::parameters_config() const {
  json::Value p = json::Value::object();
  p["T_0"] = t0_;
  p["T_mult"] = tmult_;
  p["eta_min"] = eta_min_;
  return p;
}

LinearWarmup::LinearWarmup(Optimizer* o, int warmup_steps, double start_lr)
    : Scheduler(o), warm_(warmup_steps), start_(start_lr) {
  set_lr(start_);
}
void LinearWarmup::step() {
  ++step_;
  if (step_ <= warm_) set_lr(start_ + (double)step_ / warm_ * (base_lr_ - start_));
}
json::Value LinearWarmup::parameters_config() const {
  json::Value p = json::Value::object();
  p["warmup_steps"] = warm_;
  p["start_lr"] = start_;
  return p;
}

WarmupCosineAnnealing::WarmupCosineAnnealing(Optimizer* o, int warmup_steps, int total_steps, double start_lr,
                                             double eta_min)
    : Scheduler(o), warm_(warmup_steps), total_(total_steps), start_(start_lr), eta_min_(eta_min) {
  set_lr(start_);
}
void WarmupCosineAnnealing::step() {
  ++step_;
  if (step_ <= warm_) {
    set_lr(start_ + (double)step_ / warm_ * (base_lr_ - start_));
  } else {
    const double p = std::min((double)(step_ - warm_) / (double)(total_ - warm_), 1.0);
    set_lr(eta_min_ + (base_lr_ - eta_min_) * (1 + std::cos(kPi * p)) / 2);
  }
}
json::Value WarmupCosineAnnealing::parameters_config() const {
  json::Value p = json::Value::object();
  p["warmup_steps"] = warm_;
  p["total_steps"] = total_;
  p["start_lr"] = start_;
  p["eta_min"] = eta_min_;
  return p;
}

ReduceLROnPlateau::ReduceLROnPlateau(Optimizer* o, std::string mode, double factor, int patience, double threshold,
                                     double min_lr)
    : Scheduler(o), mode_(std::move(mode)), factor_(factor), patience_(patience), threshold_(threshold),
      min_lr_(min_lr), best_(mode_ == "min" ? 1e10 : -1e10) {}
void ReduceLROnPlateau::step(double metric) {
  ++step_;
  const bool better = mode_ == "min" ? metric < best_ - threshold_ : metric > best_ + threshold_;
  if (better) {
    best_ = metric;
    bad_ = 0;
  } else if (++bad_ >= patience_) {
    set_lr(std::max((double)get_lr() * factor_, min_lr_));
    bad_ = 0;
  }
}
void ReduceLROnPlateau::reset() {
  Scheduler::reset();
  best_ = mode_ == "min" ? 1e10 : -1e10;
  bad_ = 0;
}
json::Value ReduceLROnPlateau::parameters_config() const {
  json::Value p = json::Value::object();
  p["mode"] = mode_;
  p["factor"] = factor_;
  p["patience"] = patience_;
  p["threshold"] = threshold_;
  p["min_lr"] = min_lr_;
  return p;
}

void PolynomialLR::step() {
  ++step_;
  const double p = std::min((double)step_ / total_, 1.0);
  set_lr((base_lr_ - end_) * std::pow(1 - p, power_) + end_);
}
json::Value PolynomialLR::parameters_config() const {
  json::Value p = json::Value::object();
  p["total_steps"] = total_;
  p["power"] = power_;
  p["end_lr"] = end_;
  return p;
}

OneCycleLR::OneCycleLR(Optimizer* o, double max_lr, int total_steps, double pct_start, double div_factor,
                       double final_div_factor)
    : Scheduler(o), max_lr_(max_lr), total_(total_steps), pct_(pct_start), div_(div_factor),
      final_div_(final_div_factor) {
  initial_ = max_lr_ / div_;
  min_lr_ = initial_ / final_div_;
  up_ = (int)(total_ * pct_);
  down_ = total_ - up_;
  set_lr(initial_);
}
void OneCycleLR::step() {
  ++step_;
  double lr;
  if (step_ <= up_) {
    lr = initial_ + (double)step_ / up_ * (max_lr_ - initial_);
  } else {
    const double p = (double)(step_ - up_) / down_;
    lr = min_lr_ + (max_lr_ - min_lr_) * (1 + std::cos(kPi * p)) / 2;
  }
  set_lr(lr);
}
json::Value OneCycleLR::parameters_config() const {
  json::Value p = json::Value::object();
  p["max_lr"] = max_lr_;
  p["total_steps"] = total_;
  p["pct_start"] = pct_;
  p["div_factor"] = div_;
  p["final_div_factor"] = final_div_;
  return p;
}

std::unique_ptr<Scheduler> SchedulerFactory::create(const std::string& type, Optimizer* opt, const json::Value& params) {
  json::Value c = json::Value::object();
  c["type"] = type;
  c["parameters"] = params;
  return create_from_config(c, opt);
}

std::unique_ptr<Scheduler> SchedulerFactory::create_from_config(const json::Value& cfg, Optimizer* opt) {
  const std::string t = cfg.get_string("type", "");
  static const json::Value empty = json::Value::object();
  const json::Value& p = cfg.has("parameters") ? cfg.at("parameters") : empty;
  auto I = [&](const char* k, int64_t d) { return (int)p.get_int(k, d); };
  auto D = [&](const char* k, double d) { return p.get_number(k, d); };
  if (t == "step_lr") return std::make_unique<StepLR>(opt, I("step_size", 10), D("gamma", 0.1));
  if (t == "multi_step_lr") {
    std::vector<int> ms;
    if (const json::Value* m = p.find("milestones"))
      for (auto& v : m->items()) ms.push_back((int)v.as_int());
    return std::make_unique<MultiStepLR>(opt, ms, D("gamma", 0.1));
  }
  if (t == "exponential_lr") return std::make_unique<ExponentialLR>(opt, D("gamma", 0.95));
  if (t == "cosine_annealing_lr") return std::make_unique<CosineAnnealingLR>(opt, I("T_max", 100), D("eta_min", 0.0));
  if (t == "cosine_annealing_warm_restarts")
    return std::make_unique<CosineAnnealingWarmRestarts>(opt, I("T_0", 10), I("T_mult", 1), D("eta_min", 0.0));
  if (t == "linear_warmup") return std::make_unique<LinearWarmup>(opt, I("warmup_steps", 100), D("start_lr", 0.0));
  if (t == "warmup_cosine_annealing")
    return std::make_unique<WarmupCosineAnnealing>(opt, I("warmup_steps", 100), I("total_steps", 1000),
                                                   D("start_lr", 0.0), D("eta_min", 0.0));
  if (t == "reduce_lr_on_plateau")
    return std::make_unique<ReduceLROnPlateau>(opt, p.get_string("mode", "min"), D("factor", 0.1), I("patience", 10),
                                               D("threshold", 1e-4), D("min_lr", 0.0));
  if (t == "polynomial_lr")
    return std::make_unique<PolynomialLR>(opt, I("total_steps", 100), D("power", 1.0), D("end_lr", 0.0));
  if (t == "one_cycle_lr")
    return std::make_unique<OneCycleLR>(opt, D("max_lr", 0.1), I("total_steps", 100), D("pct_start", 0.3),
                                        D("div_factor", 25.0), D("final_div_factor", 1e4));
  throw std::invalid_argument("unknown scheduler type '" + t + "'");
}

// ================================================================= data
namespace {
uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

template <class F>
void parallel_for(size_t n, F&& fn) {
  const int T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::atomic<size_t> next{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < T; ++t)
    ts.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
    });
  for (auto& t : ts) t.join();
}
}  // namespace

ImageDataset::ImageDataset(std::vector<float> images, std::vector<int64_t> labels, int c, int h, int w, int classes,
                           uint64_t seed, bool shuffle)
    : img_(std::move(images)), labels_(std::move(labels)), c_(c), h_(h), w_(w), classes_(classes), seed_(seed),
      shuffle_(shuffle) {
  if (img_.size() != labels_.size() * (size_t)c * h * w) throw std::invalid_argument("ImageDataset: size mismatch");
  order_.resize(labels_.size());
  for (size_t i = 0; i < order_.size(); ++i) order_[i] = i;
}

void ImageDataset::normalize(const std::vector<float>& mean, const std::vector<float>& stdev) {
  if ((int)mean.size() != c_ || (int)stdev.size() != c_) throw std::invalid_argument("normalize: one value per channel");
  const size_t hw = (size_t)h_ * w_;
  for (size_t n = 0; n < labels_.size(); ++n)
    for (int c = 0; c < c_; ++c) {
      float* p = img_.data() + (n * c_ + c) * hw;
      for (size_t k = 0; k < hw; ++k) p[k] = (p[k] - mean[c]) / stdev[c];
    }
}

void ImageDataset::reset(uint64_t epoch) {
  epoch_ = epoch;
  for (size_t i = 0; i < order_.size(); ++i) order_[i] = i;
  if (shuffle_) {
    uint64_t s = seed_ * 1000003ull + epoch;
    for (size_t i = order_.size(); i > 1; --i) {
      s = mix64(s);
      std::swap(order_[i - 1], order_[(size_t)(s % i)]);
    }
  }
  pos_ = 0;
}

bool ImageDataset::next(int batch, Tensor& x, Tensor& labels) {
  if (pos_ >= order_.size()) return false;
  const int b = (int)std::min<size_t>((size_t)batch, order_.size() - pos_);
  const size_t per = (size_t)c_ * h_ * w_;
  std::vector<float> xs((size_t)b * per);
  std::vector<int64_t> ys((size_t)b);
  for (int i = 0; i < b; ++i) {
    const size_t idx = order_[pos_ + i];
    ys[i] = labels_[idx];
    const float* src = img_.data() + idx * per;
    float* dst = xs.data() + (size_t)i * per;
    const bool flip = flip_ > 0.f && (float)(mix64(seed_ ^ (epoch_ * 0x100000001b3ull) ^ idx) >> 40) * (1.f / 16777216.f) < flip_;
    if (!flip) {
      std::memcpy(dst, src, per * sizeof(float));
    } else {
      for (int c = 0; c < c_; ++c)
        for (int y = 0; y < h_; ++y)
          for (int xx = 0; xx < w_; ++xx)
            dst[((size_t)c * h_ + y) * w_ + xx] = src[((size_t)c * h_ + y) * w_ + (w_ - 1 - xx)];
    }
  }
  pos_ += (size_t)b;
  x = Tensor::from_host(xs, {b, c_, h_, w_}, Device::cpu());
  labels = Tensor::from_host_i64(ys, Device::cpu());
  return true;
}

ImageDataset load_mnist_csv(const std::string& path, uint64_t seed) {
  std::istringstream in(read_file(path));
  std::string line;
  std::vector<float> img;
  std::vector<int64_t> lab;
  bool first = true;
  while (std::getline(in, line)) {
    if (line.empty() || line == "\r") continue;
    if (first) {
      first = false;
      if (!std::isdigit((unsigned char)line[0])) continue;  // header row
    }
    std::istringstream ls(line);
    std::string cell;
    if (!std::getline(ls, cell, ',')) continue;
    lab.push_back(std::stoll(cell));
    int k = 0;
    while (std::getline(ls, cell, ',') && k < 784) {
      img.push_back(std::stof(cell) / 255.f);
      ++k;
    }
    if (k != 784) throw std::runtime_error(path + ": row with " + std::to_string(k) + " pixels");
  }
  return ImageDataset(std::move(img), std::move(lab), 1, 28, 28, 10, seed);
}

ImageDataset load_cifar_bin(const std::vector<std::string>& files, int label_bytes, int label_index, int classes,
                            uint64_t seed) {
  std::vector<float> img;
  std::vector<int64_t> lab;
  const size_t rec = (size_t)label_bytes + 3072;
  for (auto& f : files) {
    const std::string b = read_file(f);
    if (b.size() % rec) throw std::runtime_error(f + ": not a CIFAR binary batch");
    for (size_t o = 0; o < b.size(); o += rec) {
      lab.push_back((unsigned char)b[o + label_index]);
      for (size_t k = 0; k < 3072; ++k) img.push_back((unsigned char)b[o + label_bytes + k] / 255.f);
    }
  }
  return ImageDataset(std::move(img), std::move(lab), 3, 32, 32, classes, seed);
}

ImageDataset load_tiny_imagenet(const std::string& root, const std::string& split, int max_per_class, uint64_t seed) {
  std::vector<std::string> wnids;
  {
    std::istringstream ss(read_file(root + "/wnids.txt"));
    std::string l;
    while (std::getline(ss, l)) {
      while (!l.empty() && (l.back() == '\r' || l.back() == ' ')) l.pop_back();
      if (!l.empty()) wnids.push_back(l);
    }
  }
  std::vector<std::pair<std::string, int>> files;
  if (split == "train") {
    for (size_t c = 0; c < wnids.size(); ++c) {
      const std::string dir = root + "/train/" + wnids[c] + "/images";
      std::vector<std::string> names;
      for (auto& e : std::filesystem::directory_iterator(dir)) names.push_back(e.path().filename().string());
      std::sort(names.begin(), names.end());
      int k = 0;
      for (auto& n : names) {
        if (max_per_class > 0 && k++ >= max_per_class) break;
        files.emplace_back(dir + "/" + n, (int)c);
      }
    }
  } else {
    std::istringstream ss(read_file(root + "/val/val_annotations.txt"));
    std::string l;
    while (std::getline(ss, l)) {
      std::istringstream ls(l);
      std::string f, w;
      if (!std::getline(ls, f, '\t') || !std::getline(ls, w, '\t')) continue;
      auto it = std::find(wnids.begin(), wnids.end(), w);
      if (it != wnids.end()) files.emplace_back(root + "/val/images/" + f, (int)(it - wnids.begin()));
    }
  }
  const size_t N = files.size();
  std::vector<float> img(N * 3 * 64 * 64, 0.f);
  std::vector<int64_t> lab(N);
  std::atomic<int> failures{0};
  parallel_for(N, [&](size_t i) {
    lab[i] = files[i].second;
    std::vector<unsigned char> rgb;
    int w = 0, h = 0;
    bool ok = false;
    try {
      const std::string blob = read_file(files[i].first);
      ok = dcnn_native::decode_jpeg(reinterpret_cast<const unsigned char*>(blob.data()), blob.size(), rgb, w, h,
                                    nullptr);
    } catch (...) {
    }
    if (!ok || w != 64 || h != 64) {
      ++failures;
      return;
    }
    float* o = img.data() + i * 3 * 4096;
    for (int c = 0; c < 3; ++c)
      for (int p = 0; p < 4096; ++p) o[c * 4096 + p] = rgb[(size_t)p * 3 + c] / 255.f;
  });
  if (failures) std::fprintf(stderr, "load_tiny_imagenet: %d undecodable images zero-filled\n", failures.load());
  return ImageDataset(std::move(img), std::move(lab), 3, 64, 64, (int)wnids.size(), seed);
}

// ================================================================= model zoo
Sequential create_model(const std::string& name) {
  if (name == "mnist_cnn")
    return SequentialBuilder("mnist_cnn_model").input({1, 28, 28})
        .conv2d(8, 5, 5, 1, 1, 0, 0, true, "conv1").batchnorm(1e-5f, 0.1f, true, "bn1")
        .activation("relu", "relu1").maxpool2d(3, 3, 3, 3, 0, 0, "pool1")
        .conv2d(16, 1, 1, 1, 1, 0, 0, true, "conv2_1x1").batchnorm(1e-5f, 0.1f, true, "bn2")
        .activation("relu", "relu2")
        .conv2d(48, 5, 5, 1, 1, 0, 0, true, "conv3").batchnorm(1e-5f, 0.1f, true, "bn3")
        .activation("relu", "relu3").maxpool2d(2, 2, 2, 2, 0, 0, "pool2")
        .flatten("flatten").dense(10, true, "output").build();
  if (name == "resnet9_cifar10")
    return SequentialBuilder("ResNet-9-CIFAR10").input({3, 32, 32})
        .conv2d(64, 3, 3, 1, 1, 1, 1, true, "conv1").batchnorm(1e-5f, 0.1f, true, "bn1").activation("relu", "relu1")
        .conv2d(128, 3, 3, 1, 1, 1, 1, true, "conv2").batchnorm(1e-5f, 0.1f, true, "bn2").activation("relu", "relu2")
        .maxpool2d(2, 2, 2, 2, 0, 0, "pool1")
        .basic_residual_block(128, 128, 1, "res_block1").basic_residual_block(128, 128, 1, "res_block2")
        .conv2d(256, 3, 3, 1, 1, 1, 1, true, "conv3").batchnorm(1e-5f, 0.1f, true, "bn3").activation("relu", "relu3")
        .maxpool2d(2, 2, 2, 2, 0, 0, "pool2")
        .basic_residual_block(256, 256, 1, "res_block3").basic_residual_block(256, 256, 1, "res_block4")
        .conv2d(512, 3, 3, 1, 1, 1, 1, true, "conv4").batchnorm(1e-5f, 0.1f, true, "bn4").activation("relu", "relu4")
        .maxpool2d(2, 2, 2, 2, 0, 0, "pool3")
        .basic_residual_block(512, 512, 1, "res_block5")
        .avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(10, true, "output").build();
  if (name == "resnet18_tiny_imagenet" || name == "resnet34_tiny_imagenet") {
    const bool r34 = name == "resnet34_tiny_imagenet";
    SequentialBuilder b(r34 ? "ResNet-34-Tiny-ImageNet" : "ResNet-18-Tiny-ImageNet");
    b.input({3, 64, 64}).conv2d(32, 3, 3, 1, 1, 1, 1, false, "conv1").batchnorm(1e-3f, 0.1f, true, "bn1")
        .activation("relu", "relu1").maxpool2d(2, 2, 2, 2, 0, 0, "maxpool");
    const int per[4] = {r34 ? 3 : 2, r34 ? 4 : 2, r34 ? 6 : 2, r34 ? 3 : 2};
    const int width[4] = {64, 128, 256, 512};
    int in = 32;
    for (int L = 0; L < 4; ++L)
      for (int i = 1; i <= per[L]; ++i) {
        b.basic_residual_block(in, width[L], (i == 1 && L > 0) ? 2 : 1,
                               "layer" + std::to_string(L + 1) + "_block" + std::to_string(i));
        in = width[L];
      }
    return b.avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(200, true, "fc").build();
  }
  if (name == "resnet50_tiny_imagenet") {
    SequentialBuilder b("ResNet-50-Tiny-ImageNet");
    b.input({3, 64, 64}).conv2d(64, 3, 3, 1, 1, 1, 1, true, "conv1").batchnorm(1e-5f, 0.1f, true, "bn1")
        .activation("relu", "relu1").maxpool2d(3, 3, 2, 2, 1, 1, "maxpool");
    const int per[4] = {3, 4, 6, 3}, mid[4] = {64, 128, 256, 512};
    int in = 64;
    for (int L = 0; L < 4; ++L)
      for (int i = 1; i <= per[L]; ++i) {
        b.bottleneck_residual_block(in, mid[L], 4 * mid[L], (i == 1 && L > 0) ? 2 : 1,
                                    "layer" + std::to_string(L + 1) + "_block" + std::to_string(i));
        in = 4 * mid[L];
      }
    return b.avgpool2d(4, 4, 1, 1, 0, 0, "avgpool").flatten("flatten").dense(200, true, "fc").build();
  }
  throw std::invalid_argument("unknown model '" + name + "'");
}

// ================================================================= training loop
std::vector<EpochStats> train_model(Sequential& model, DataSource& train, DataSource* val, Optimizer& opt,
                                    const Loss& loss, const TrainingConfig& cfg, Scheduler* sched) {
  const bool plateau = sched && sched->type() == "reduce_lr_on_plateau";
  std::vector<EpochStats> hist;
  for (int e = 0; e < cfg.epochs; ++e) {
    const auto t0 = std::chrono::steady_clock::now();
    train.reset(cfg.seed + (uint64_t)e);
    model.set_training(true);
    Tensor x, y;
    double lsum = 0;
    long correct = 0, seen = 0;
    int step = 0;
    while ((cfg.max_steps < 0 || step < cfg.max_steps) && train.next(cfg.batch_size, x, y)) {
      model.zero_grad();
      Tensor logits = model.forward(x);
      LossResult r = loss(logits, y);
      model.backward(r.grad);
      opt.step(model.parameters());
      if (sched && !plateau) sched->step();
      lsum += r.loss * x.dim(0);
      correct += r.correct;
      seen += x.dim(0);
      ++step;
      if (cfg.progress_interval > 0 && step % cfg.progress_interval == 0)
        std::printf("epoch %d step %d  loss %.4f  acc %.2f%%  lr %.3g\n", e + 1, step, lsum / seen,
                    100.0 * correct / seen, (double)opt.learning_rate());
    }
    EpochStats s;
    s.train_loss = seen ? lsum / seen : 0;
    s.train_acc = seen ? (double)correct / seen : 0;
    if (val) {
      model.set_training(false);
      val->reset(0);
      double vl = 0;
      long vc = 0, vn = 0;
      while (val->next(cfg.batch_size, x, y)) {
        LossResult r = loss.compute(model.forward(x), &y);
        vl += r.loss * x.dim(0);
        vc += r.correct;
        vn += x.dim(0);
      }
      model.set_training(true);
      s.val_loss = vn ? vl / vn : 0;
      s.val_acc = vn ? (double)vc / vn : 0;
    }
    if (plateau) sched->step(val ? s.val_loss : s.train_loss);
    if (model.device().is_gpu()) gpu::synchronize();
    s.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("epoch %d/%d  train loss %.4f acc %.2f%%  val loss %.4f acc %.2f%%  (%.2f s)\n", e + 1, cfg.epochs,
                s.train_loss, 100 * s.train_acc, s.val_loss, 100 * s.val_acc, s.seconds);
    hist.push_back(s);
    if (!sched) opt.set_learning_rate(opt.learning_rate() * cfg.lr_decay);
  }
  return hist;
}

}  // namespace dcnn
