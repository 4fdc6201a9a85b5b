// Training components of the C++ host API beyond nn.hpp: the six losses (LossFactory), the ten
// learning-rate schedulers (SchedulerFactory) and the dataset loaders (MNIST CSV, CIFAR-10/100
// binary batches, Tiny-ImageNet JPEG folders) as DataSources, plus the model zoo builders.
//
// Semantics follow the Python front end (dcnn_amd/nn/loss.py, nn/schedulers.py, data/datasets.py)
// so a schedule or a loss value is the same number from either language.
// Reference parity: include/nn/loss.hpp:59-343 (losses + factory :403),
// include/nn/schedulers.hpp:42-698 (schedulers + factory :598),
// include/data_loading/{mnist,cifar10,cifar100,tiny_imagenet}_data_loader.hpp,
// include/nn/example_models.hpp:13-437 (model zoo).
#pragma once
#include <functional>
#include <initializer_list>
#include <memory>
#include <string>
#include <vector>

#include "json.hpp"
#include "nn.hpp"

namespace dcnn {

// ---------------------------------------------------------------- losses
// Mean over the batch; targets are class labels (one-hot) or, for the regression losses, an
// optional dense [N, C] fp32 target. kind codes match the fused kernels: 0 crossentropy (on
// probabilities, eps-clamped), 1 softmax crossentropy, 2 log-softmax crossentropy, 3 mse, 4 mae,
// 5 huber(delta).
class Loss {
 public:
  Loss(int kind, float param, std::string type) : kind_(kind), param_(param), type_(std::move(type)) {}
  // logits / predictions [N, C] (device), labels int64 [N] or target fp32 [N, C] (any device)
  // grad_scale multiplies the gradient (e.g. 1 / micro-batches), not the loss value
  LossResult compute(const Tensor& pred, const Tensor* labels, const Tensor* target = nullptr,
                     float grad_scale = 1.f) const;
  LossResult operator()(const Tensor& pred, const Tensor& labels) const { return compute(pred, &labels); }
  const std::string& type() const { return type_; }
  int kind() const { return kind_; }
  float param() const { return param_; }

 private:
  int kind_;
  float param_;
  std::string type_;
};

// One training step (zero_grad, forward, loss, backward, optimizer) captured into a gpu::Graph
// and replayed with one launch (the C++ counterpart of the Python front end's runtime/step.py).
// The batch is copied into static device tensors before each replay; the loss stays on the
// device until loss() reads it. capture() runs two eager warm-up steps first (workspaces, kernel
// instances, allocator size classes) and restores the parameters and optimizer moments they
// changed, so the first replay is the first update.
class TrainGraph {
 public:
  TrainGraph(Sequential& model, Adam& opt, const Loss& loss) : model_(model), opt_(opt), loss_(loss) {}
  double step(const Tensor& x, const Tensor& labels);  // eager on the first call: captures, then replays
  double last_loss();                                  // host read of the last replay's loss
  // runs between the backward and the optimizer of every step, inside the capture (e.g. the
  // data-parallel gradient all-reduce, dist::DataParallel::all_reduce_mean on the arena gradient)
  void set_gradient_hook(std::function<void()> f) { grad_hook_ = std::move(f); }

 private:
  void capture(const Tensor& x, const Tensor& labels);
  Sequential& model_;
  Adam& opt_;
  const Loss& loss_;
  gpu::Graph graph_;
  Tensor sx_, sy_;
  bool captured_ = false;
  std::function<void()> grad_hook_;
};

struct LossFactory {
  // "crossentropy"|"ce", "softmax_crossentropy"|"softmax_ce", "logsoftmax_crossentropy"|
  // "logsoftmax_ce", "mse", "mae", "huber" (param: delta)
  static Loss create(const std::string& name, float param = -1.f);
};

// ---------------------------------------------------------------- schedulers
class Scheduler {
 public:
  explicit Scheduler(Optimizer* opt) : opt_(opt), base_lr_(opt ? opt->learning_rate() : 0.f) {}
  virtual ~Scheduler() = default;
  virtual void step() = 0;
  virtual void step(double metric) { (void)metric; step(); }
  virtual void reset() {
    step_ = 0;
    set_lr(base_lr_);
  }
  virtual std::string type() const = 0;
  virtual json::Value parameters_config() const = 0;
  json::Value get_config() const;
  float get_lr() const { return opt_ ? opt_->learning_rate() : base_lr_; }
  float base_lr() const { return base_lr_; }
  long current_step() const { return step_; }

 protected:
  void set_lr(double lr) {
    if (opt_) opt_->set_learning_rate((float)lr);
  }
  Optimizer* opt_;
  float base_lr_;
  long step_ = 0;
};

class StepLR : public Scheduler {
 public:
  StepLR(Optimizer* o, int step_size, double gamma = 0.1) : Scheduler(o), size_(step_size), gamma_(gamma) {}
  void step() override;
  std::string type() const override { return "step_lr"; }
  json::Value parameters_config() const override;

 private:
  int size_;
  double gamma_;
};

class MultiStepLR : public Scheduler {
 public:
  MultiStepLR(Optimizer* o, std::vector<int> milestones, double gamma = 0.1);
  void step() override;
  void reset() override;
  std::string type() const override { return "multi_step_lr"; }
  json::Value parameters_config() const override;

 private:
  std::vector<int> ms_;
  double gamma_;
  size_t idx_ = 0;
};

class ExponentialLR : public Scheduler {
 public:
  ExponentialLR(Optimizer* o, double gamma = 0.95) : Scheduler(o), gamma_(gamma) {}
  void step() override;
  std::string type() const override { return "exponential_lr"; }
  json::Value parameters_config() const override;

 private:
  double gamma_;
};

class CosineAnnealingLR : public Scheduler {
 public:
  CosineAnnealingLR(Optimizer* o, int T_max, double eta_min = 0.0) : Scheduler(o), tmax_(T_max), eta_min_(eta_min) {}
  void step() override;
  std::string type() const override { return "cosine_annealing_lr"; }
  json::Value parameters_config() const override;

 private:
  int tmax_;
  double eta_min_;
};

class CosineAnnealingWarmRestarts : public Scheduler {
 public:
  CosineAnnealingWarmRestarts(Optimizer* o, int T_0, int T_mult = 1, double eta_min = 0.0)
      : Scheduler(o), t0_(T_0), tmult_(T_mult), eta_min_(eta_min), ti_(T_0) {}
  void step() override;
  void reset() override;
  std::string type() const override { return "cosine_annealing_warm_restarts"; }
  json::Value parameters_config() const override;

 private:
  int t0_, tmult_;
  double eta_min_;
  long tcur_ = 0, ti_;
};

class LinearWarmup : public Scheduler {
 public:
  LinearWarmup(Optimizer* o, int warmup_steps, double start_lr = 0.0);
  void step() override;
  bool is_warmup_complete() const { return step_ >= warm_; }
  std::string type() const override { return "linear_warmup"; }
  json::Value parameters_config() const override;

 private:
  int warm_;
  double start_;
};

class WarmupCosineAnnealing : public Scheduler {
 public:
  WarmupCosineAnnealing(Optimizer* o, int warmup_steps, int total_steps, double start_lr = 0.0, double eta_min = 0.0);
  void step() override;
  std::string type() const override { return "warmup_cosine_annealing"; }
  json::Value parameters_config() const override;

 private:
  int warm_, total_;
  double start_, eta_min_;
};

class ReduceLROnPlateau : public Scheduler {
 public:
  ReduceLROnPlateau(Optimizer* o, std::string mode = "min", double factor = 0.1, int patience = 10,
                    double threshold = 1e-4, double min_lr = 0.0);
  void step() override { ++step_; }
  void step(double metric) override;
  void reset() override;
  std::string type() const override { return "reduce_lr_on_plateau"; }
  json::Value parameters_config() const override;

 private:
  std::string mode_;
  double factor_;
  int patience_;
  double threshold_, min_lr_, best_;
  int bad_ = 0;
};

class PolynomialLR : public Scheduler {
 public:
  PolynomialLR(Optimizer* o, int total_steps, double power = 1.0, double end_lr = 0.0)
      : Scheduler(o), total_(total_steps), power_(power), end_(end_lr) {}
  void step() override;
  std::string type() const override { return "polynomial_lr"; }
  json::Value parameters_config() const override;

 private:
  int total_;
  double power_, end_;
};

class OneCycleLR : public Scheduler {
 public:
  OneCycleLR(Optimizer* o, double max_lr, int total_steps, double pct_start = 0.3, double div_factor = 25.0,
             double final_div_factor = 1e4);
  void step() override;
  std::string type() const override { return "one_cycle_lr"; }
  json::Value parameters_config() const override;

 private:
  double max_lr_;
  int total_;
  double pct_, div_, final_div_, initial_, min_lr_;
  int up_, down_;
};

struct SchedulerFactory {
  // {"type": ..., "parameters": {...}} (the Python SchedulerConfig / reference JSON)
  static std::unique_ptr<Scheduler> create_from_config(const json::Value& cfg, Optimizer* opt);
  static std::unique_ptr<Scheduler> create(const std::string& type, Optimizer* opt,
                                           const json::Value& params = json::Value::object());
};

// ---------------------------------------------------------------- data
// In-memory image classification set: fp32 NCHW images in [0, 1] (+ optional per-channel
// normalisation) and int64 labels, reshuffled every epoch (deterministic in the seed).
class ImageDataset : public DataSource {
 public:
  ImageDataset(std::vector<float> images, std::vector<int64_t> labels, int c, int h, int w, int classes,
               uint64_t seed = 0, bool shuffle = true);
  void reset(uint64_t epoch) override;
  bool next(int batch, Tensor& x, Tensor& labels) override;
  size_t size() const override { return labels_.size(); }
  int channels() const { return c_; }
  int height() const { return h_; }
  int width() const { return w_; }
  int num_classes() const { return classes_; }
  // x = (x - mean[c]) / std[c]
  void normalize(const std::vector<float>& mean, const std::vector<float>& stdev);
  // horizontal flip with probability p per sample (applied at batch time)
  void set_random_flip(float p) { flip_ = p; }
  const std::vector<float>& images() const { return img_; }
  const std::vector<int64_t>& labels() const { return labels_; }

 private:
  std::vector<float> img_;
  std::vector<int64_t> labels_;
  int c_, h_, w_, classes_;
  uint64_t seed_, epoch_ = 0;
  bool shuffle_;
  float flip_ = 0.f;
  std::vector<size_t> order_;
  size_t pos_ = 0;
};

// HBM-resident image classification set (the GPU data path): the whole set lives in device memory
// (uint8 when every value is an exact k / 255, as decoded images are: 1.2 GB for Tiny-ImageNet's
// 100k training images, else fp32) and every batch is assembled by ONE kernel launch on the current
// flow (augment.hip: gather by the epoch order + the augmentation chain + labels), so training never
// waits on host decoding, augmentation or host-to-device copies. The chain's draws are a counter
// hash of (epoch seed, sample, op, draw) — the Python DeviceDataLoader's kernel and semantics
// (data/device_loader.py): a rerun reproduces every batch.
// Reference parity: include/data_loading/tiny_imagenet_data_loader.hpp:481 (batches of the epoch
// order), include/data_augmentation/augmentation.hpp:114 (the op chain: crop, flips, rotation,
// brightness, contrast, noise, cutout, normalisation).
class DeviceImageDataset : public DataSource {
 public:
  DeviceImageDataset(const ImageDataset& host, Device dev, uint64_t seed = 0, bool shuffle = true,
                     bool drop_last = true);
  // the augmentation chain, applied in the order added (at most 12 ops; p = probability per sample)
  DeviceImageDataset& horizontal_flip(float p = 0.5f);
  DeviceImageDataset& vertical_flip(float p = 0.5f);
  DeviceImageDataset& rotation(float p, float max_degrees);
  DeviceImageDataset& brightness(float p, float delta);
  DeviceImageDataset& contrast(float p, float delta);
  DeviceImageDataset& gaussian_noise(float p, float sigma);
  DeviceImageDataset& random_crop(float p, int pad);  // shift by up to +-pad pixels, zero fill
  DeviceImageDataset& cutout(float p, int size);
  DeviceImageDataset& normalize(const std::vector<float>& mean = {0.485f, 0.456f, 0.406f},
                                const std::vector<float>& stdev = {0.229f, 0.224f, 0.225f});
  void reset(uint64_t epoch) override;
  // x: fp32 [B, C, H, W] and labels int64 [B], both on the device
  bool next(int batch, Tensor& x, Tensor& labels) override;
  size_t size() const override { return n_; }
  bool stored_u8() const { return u8_; }
  size_t device_bytes() const { return data_.nbytes(); }
  uint64_t epoch_seed() const;

 private:
  struct Op {
    int kind;
    float p;
    float a[6];
  };
  DeviceImageDataset& add(int kind, float p, std::initializer_list<float> a);
  Device dev_;
  Tensor data_, labels_, order_dev_;
  std::vector<int64_t> order_;
  std::vector<Op> ops_;
  size_t n_ = 0, pos_ = 0;
  int c_, h_, w_;
  uint64_t seed_, epoch_ = 0;
  bool shuffle_, drop_last_, u8_ = false;
};

// MNIST CSV (label, 784 pixels per row; header row auto-detected) -> [N, 1, 28, 28] / 255
ImageDataset load_mnist_csv(const std::string& path, uint64_t seed = 0);
// CIFAR binary batches (label bytes + 3072 pixel bytes per record): CIFAR-10 (label_bytes 1) or
// CIFAR-100 (label_bytes 2, fine label = byte 1, coarse = byte 0)
ImageDataset load_cifar_bin(const std::vector<std::string>& files, int label_bytes, int label_index, int classes,
                            uint64_t seed = 0);
// Tiny-ImageNet-200 folder (wnids.txt, train/<wnid>/images/*.JPEG, val/val_annotations.txt);
// split "train" or "val"; max_per_class <= 0: all images
ImageDataset load_tiny_imagenet(const std::string& root, const std::string& split, int max_per_class = 0,
                                uint64_t seed = 0);

// ---------------------------------------------------------------- model zoo
// the reference's builders (include/nn/example_models.hpp): mnist_cnn, cifar10_resnet9,
// resnet18_tiny_imagenet, resnet34_tiny_imagenet, resnet50_tiny_imagenet
Sequential create_model(const std::string& name);

// training loop with an optional scheduler stepped once per optimizer step (ReduceLROnPlateau:
// once per epoch with the validation loss) and a loss of the factory
std::vector<EpochStats> train_model(Sequential& model, DataSource& train, DataSource* val, Optimizer& opt,
                                    const Loss& loss, const TrainingConfig& cfg, Scheduler* sched = nullptr);

}  // namespace dcnn
