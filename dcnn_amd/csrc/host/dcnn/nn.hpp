// C++ host API: layers, Sequential / SequentialBuilder, loss, optimizers, training loop.
//
// A C++ program builds, trains, saves and reloads a model without Python:
//
//   auto model = dcnn::SequentialBuilder("mnist_cnn").input({1, 28, 28})
//                    .conv2d(16, 3, 3, 1, 1, 1, 1).batchnorm().activation("relu").maxpool2d(2, 2)
//                    .flatten().dense(10).build();
//   model.set_device(dcnn::Device::gpu(0));
//   model.initialize(42);
//   dcnn::Adam opt(1e-3f);
//   dcnn::train_classification_model(model, train_source, &test_source, opt, cfg);
//   model.save_to_file("snapshots/mnist_cnn");   // path.json + path.bin, readable by Python
//
// CPU: fp32 NCHW on the native CPU kernels. GPU: bf16 NHWC activations on the HIP/CDNA4 kernel
// library with fp32 master parameters (Adam / SGD write the bf16 operand shadows in the same
// kernel). The architecture JSON and the .bin weight records are the formats of the Python front
// end (dcnn_amd/nn/sequential.py) and of the reference, so a model moves between the two.
// Reference parity: include/nn/sequential.hpp:39-1340 (Sequential, SequentialBuilder),
// include/nn/train.hpp:202 (train_classification_model), include/nn/optimizers.hpp,
// include/nn/loss.hpp, examples/mnist_cnn_trainer.cpp.
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "json.hpp"
#include "ops.hpp"
#include "tensor.hpp"

namespace dcnn {

// One trainable tensor. `value` / `grad` are fp32 on the layer's device in `layout` (GPU conv
// weights: physical [Co][KH][KW][Ci] = NHWC of the logical (Co, Ci, KH, KW)); `shadow` is the bf16
// GEMM operand copy on the GPU. `shape` is the logical 4-D shape of the .bin record.
struct ParamArena;
struct Param {
  std::string name;
  std::vector<int64_t> shape;
  Layout layout = Layout::NCHW;
  Tensor value, grad, shadow;
  Tensor m, v;  // optimizer state (lazily created)
  std::shared_ptr<ParamArena> arena;  // GPU: the flat buffers value / grad / m / v / shadow live in
};

// GPU parameter arena of a Sequential: every parameter's value, gradient, optimizer moments and
// bf16 shadow as slices of five flat buffers (64-element aligned), so zero_grad is one memset and
// an optimizer step one fused kernel over all `count` parameters (`n` elements, gaps stay zero)
struct ParamArena {
  Tensor value, grad, m, v, shadow;
  size_t n = 0, count = 0;
  // every eligible conv's dgrad operand ([C][KH][KW][Co] bf16), regenerated from the shadows in
  // one batched launch after each fused optimizer step (rows: src, dst, Co, T, C)
  Tensor wt_table;
  int n_wt = 0;
  long wt_tiles = 0;
  bool wt_valid = false;
  void refresh_transposes();
};

class Layer {
 public:
  explicit Layer(std::string name) : name_(std::move(name)) {}
  virtual ~Layer() = default;
  virtual std::string type() const = 0;
  virtual json::Value parameters_config() const = 0;
  // logical (N, C, H, W) output shape for a logical input shape
  virtual std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const = 0;
  // create parameters for the given input shape on `dev` (deterministic in `seed`)
  virtual void build(const std::vector<int64_t>& in, Device dev, uint64_t seed) { (void)in; (void)seed; dev_ = dev; }
  virtual Tensor forward(const Tensor& x, bool training) = 0;
  virtual Tensor backward(const Tensor& dy) = 0;
  // refresh the bf16 operand shadows from the fp32 masters (after loading weights)
  virtual void sync_shadow();
  // this layer's parameters, then those of its sub-layers (ResidualBlock), in checkpoint order
  virtual void collect_params(std::vector<Param*>& out) {
    for (auto& p : params_) out.push_back(&p);
  }
  // this layer and, depth-first, every sub-layer (BatchNorm statistics sidecar order)
  virtual void collect_layers(std::vector<Layer*>& out) { out.push_back(this); }
  std::vector<Param>& params() { return params_; }
  const std::string& name() const { return name_; }
  Device device() const { return dev_; }
  // micro-batch whose forward state the next forward / backward call uses: every layer keeps its
  // forward caches per micro-batch (the reference's unordered_map<size_t, ...> caches), so a
  // pipeline stage can hold several micro-batches in flight (semi-async, 1F1B)
  virtual void set_micro_batch(int mb) { mb_ = mb; }
  void clear_caches() { caches_.clear(); }
  // false: backward need not produce the input gradient (the network's first layer); the layers
  // that can skip their data-gradient GEMM (Conv2D, Dense) then return an undefined tensor
  void set_input_grad(bool b) { input_grad_ = b; }
  bool input_grad() const { return input_grad_; }
  // the network input (fp32 NCHW, logical input shape `in`) is consumed as is (GPU RGB stem conv)
  virtual bool takes_raw_input(const std::vector<int64_t>& in) const { (void)in; return false; }
  // forward + backward FLOPs for a logical input shape (the pipeline's FLOP-balanced partition;
  // the Python layers' forward_flops + backward_flops)
  virtual double flops(const std::vector<int64_t>& in) const { (void)in; return 0; }

 protected:
  struct MbCache {
    Tensor a, b, c, d;
    std::vector<int64_t> shape;
    uint64_t u = 0;
    bool flag = false;
  };
  MbCache& mbc() { return caches_[mb_]; }
  std::map<int, MbCache> caches_;
  int mb_ = 0;
  bool input_grad_ = true;
  Param& add_param(const std::string& n, const std::vector<int64_t>& shape, Layout phys, const std::vector<float>& init);
  std::string name_;
  Device dev_ = Device::cpu();
  std::vector<Param> params_;
};

class Conv2D : public Layer {
 public:
  Conv2D(int in_ch, int out_ch, int kh, int kw, int sh = 1, int sw = 1, int ph = 0, int pw = 0, bool bias = true,
         std::string name = "conv2d");
  std::string type() const override { return "conv2d"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override;
  void build(const std::vector<int64_t>& in, Device dev, uint64_t seed) override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;
  bool takes_raw_input(const std::vector<int64_t>& in) const override;
  double flops(const std::vector<int64_t>& in) const override;
  // GPU: hand the output's BatchNorm statistics, computed in the conv epilogue, to `bn` (the
  // BatchNorm that consumes this conv's output; fuse_bn_relu wires it)
  void set_stats_consumer(class BatchNorm* bn) { stats_to_ = bn; }
  // GPU: the BatchNorm (+ ReLU) producing this conv's input; the data gradient's epilogue applies
  // its ReLU mask and computes its backward statistics (fuse_bn_relu wires it)
  void set_bnb_producer(class BatchNorm* bn) { bnb_from_ = bn; }
  // the same across a residual-block boundary: the previous block's tail BatchNorm (its mask is
  // the block output), applied only by backward_residual (after the shortcut gradient is added)
  void set_block_bnb_producer(class BatchNorm* bn) { bnb_block_from_ = bn; }
  // GPU: backward whose input gradient also adds `residual` in the data-gradient epilogue
  Tensor backward_residual(const Tensor& dy, const Tensor& residual);
  // GPU RGB stem (the network input, fp32, on the stem kernel): true when this micro-batch's
  // forward ran it, so backward_stem_bn applies
  bool ran_stem() const;
  // the stem's weight gradient with its BatchNorm's backward applied to `dy` on the fly
  // (Sequential::backward_activation; gpu_ops::stem_wgrad_bn)
  void backward_stem_bn(const Tensor& dy, const gpu_ops::StemBn& bn);
  void sync_shadow() override;
  // GPU parameter arena: allocate this conv's pre-transposed dgrad operand; the arena's batched
  // transpose row and tile count (false: not eligible)
  bool make_transposed_operand(std::vector<int64_t>& row, long& tiles);

 private:
  ConvShape shape_for(const std::vector<int64_t>& in) const;
  int ci_, co_, kh_, kw_, sh_, sw_, ph_, pw_;
  bool bias_;
  class BatchNorm* stats_to_ = nullptr;
  class BatchNorm* bnb_from_ = nullptr;
  class BatchNorm* bnb_block_from_ = nullptr;
  Tensor wt_;  // pre-transposed dgrad operand (arena-managed)
  const void* dgrad_operand(bool& transposed) const;
};

class Dense : public Layer {
 public:
  Dense(int in_features, int out_features, bool bias = true, std::string name = "dense");
  std::string type() const override { return "dense"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override;
  void build(const std::vector<int64_t>& in, Device dev, uint64_t seed) override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;
  double flops(const std::vector<int64_t>& in) const override { return 6.0 * in[0] * in_ * out_; }

 private:
  int in_, out_;
  bool bias_;
};

class BatchNorm : public Layer {
 public:
  explicit BatchNorm(int num_features, float eps = 1e-5f, float momentum = 0.1f, bool affine = true,
                     std::string name = "batchnorm");
  std::string type() const override { return "batchnorm"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override { return in; }
  double flops(const std::vector<int64_t>& in) const override {
    return 15.0 * (double)in[0] * (double)in[1] * (double)in[2] * (double)in[3];  // 6 forward + 9 backward
  }
  void build(const std::vector<int64_t>& in, Device dev, uint64_t seed) override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;
  // GPU: the following ReLU runs inside this layer's apply / backward kernels (fuse_bn_relu)
  void set_fused_relu(bool b) { fused_relu_ = b; }
  bool fused_relu() const { return fused_relu_; }
  // GPU: y = act(bn(x) + residual) in one pass (a residual block's tail BatchNorm, act = ReLU when
  // `relu`), and its backward: the BatchNorm input gradient, *branch = the (masked) dy the
  // shortcut branch receives
  Tensor forward_residual(const Tensor& x, const Tensor& residual, bool relu, bool training);
  Tensor backward_residual(const Tensor& dy, Tensor* branch);
  // GPU pairing with a projection shortcut's BatchNorm (`deferred`): forward_deferred takes that
  // layer's statistics rows now; the tail's forward_dual applies both BatchNorms, the residual add
  // and the activation in one pass. backward_dual: both data gradients from one pass over the
  // tail's masked gradient (false: not applicable, the caller runs the two backwards)
  void forward_deferred(const Tensor& x, bool training);
  Tensor forward_dual(const Tensor& x, BatchNorm& deferred, bool relu, bool training);
  bool backward_dual(const Tensor& dy, BatchNorm& deferred, Tensor& dx, Tensor& dx_deferred);
  // GPU: the following ReLU + max-pool run inside this layer's training apply (fuse_bn_relu; the
  // stem's BatchNorm -> ReLU -> max-pool)
  void set_fused_pool(class Pool2D* p) { fused_pool_ = p; }
  bool fused_pool() const { return fused_pool_ != nullptr; }
  // backward-fusion operands of micro-batch `mb` (its forward's input, output mask, statistics)
  gpu_ops::BnbOperands bnb_operands(int mb);
  // the next backward over the gradient at `dy` takes its statistics from this consumer slab (the
  // gradient is already masked)
  void offer_bwd_stats(const void* dy, const float* slab, int rows) {
    bwd_dy_ = dy;
    bwd_slab_ = slab;
    bwd_rows_ = rows;
  }
  // the next forward over the tensor at `x` takes its statistics from this producer slab
  void offer_stats(const void* x, const float* slab, int rows) {
    pending_x_ = x;
    pending_slab_ = slab;
    pending_rows_ = rows;
  }
  // GPU: this layer's backward over `dy` folded into the stem conv's weight gradient (its input
  // gradient has no other consumer): false when not applicable (no consumer statistics slab for
  // dy, or eval mode), the caller then runs the two backwards
  bool backward_into_stem(const Tensor& dy, Conv2D& stem);
  Tensor running_mean, running_var;

 private:
  int c_;
  float eps_, momentum_;
  bool affine_;
  bool train_ = true;
  bool fused_relu_ = false;
  Tensor forward_impl(const Tensor& x, bool training, const Tensor* residual, bool relu);
  Tensor apply_deferred(bool training);
  class Pool2D* fused_pool_ = nullptr;
  gpu_ops::BnRaw deferred_raw_{nullptr, 0};
  const void* bwd_dy_ = nullptr;
  const float* bwd_slab_ = nullptr;
  int bwd_rows_ = 0;
  const void* pending_x_ = nullptr;
  const float* pending_slab_ = nullptr;
  int pending_rows_ = 0;
};

// activation kinds: relu, leaky_relu (0.01), elu (alpha 1), sigmoid, tanh, linear, softmax (over the
// channels of every pixel)
class Activation : public Layer {
 public:
  explicit Activation(std::string kind = "relu", std::string name = "activation");
  std::string type() const override { return "activation"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override { return in; }
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;
  bool is_relu() const;
  // GPU: the preceding BatchNorm applies this ReLU (fuse_bn_relu); forward / backward pass through
  void set_passthrough(bool b) { passthrough_ = b; }

 private:
  std::string kind_;
  int code_;
  bool passthrough_ = false;
};

// GroupNorm over G channel groups per image; gamma / beta per channel
// (reference include/nn/layers_impl/groupnorm_layer.tpp:21-321)
class GroupNorm : public Layer {
 public:
  GroupNorm(int num_groups, int num_channels, float eps = 1e-5f, bool affine = true, std::string name = "groupnorm");
  std::string type() const override { return "groupnorm"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override { return in; }
  void build(const std::vector<int64_t>& in, Device dev, uint64_t seed) override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;

 private:
  int g_, c_;
  float eps_;
  bool affine_;
  bool gb_identity_ = false;
  Tensor ident_, scratch_;
};

// inverted dropout (scale 1 / (1 - p)), identity in eval; the mask is a counter-based function
// of (seed, element), regenerated in backward (reference include/nn/layers_impl/dropout_layer.tpp)
class Dropout : public Layer {
 public:
  explicit Dropout(float rate = 0.5f, std::string name = "dropout");
  std::string type() const override { return "dropout"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override { return in; }
  void build(const std::vector<int64_t>& in, Device dev, uint64_t seed) override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;

 private:
  float p_;
  uint64_t seed_ = 0, draw_ = 0;
};

class Pool2D : public Layer {
 public:
  Pool2D(bool max, int kh, int kw, int sh, int sw, int ph, int pw, std::string name);
  std::string type() const override { return max_ ? "maxpool2d" : "avgpool2d"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;
  bool is_max() const { return max_; }
  PoolShape shape_for(const std::vector<int64_t>& in) const;
  // GPU: the preceding BatchNorm + ReLU computes this pool's output in its training apply
  // (BatchNorm::set_fused_pool); forward then passes it through and backward is the max-pool
  // backward fused with that BatchNorm's backward statistics
  void set_fused_producer(class BatchNorm* bn) { bn_ = bn; }
  // the index buffer for a pre-pooled output `ypool` of an input of shape `in`
  uint8_t* accept_prepooled(const Tensor& ypool, const std::vector<int64_t>& in);
  void clear_prepooled() { mbc().flag = false; }

 private:
  class BatchNorm* bn_ = nullptr;
  bool max_;
  int kh_, kw_, sh_, sw_, ph_, pw_;
};

class Flatten : public Layer {
 public:
  explicit Flatten(std::string name = "flatten") : Layer(std::move(name)) {}
  std::string type() const override { return "flatten"; }
  json::Value parameters_config() const override { return json::Value::object(); }
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;
};

// out = act(F(x) + S(x)): F the main path, S the projection shortcut (identity when empty).
// Backward sums the main and shortcut input gradients. Config: sub-layer records as JSON strings
// ("main_path", "shortcut_path"), as the Python front end and the reference write them
// (include/nn/blocks_impl/residual_block.hpp:30-476).
class ResidualBlock : public Layer {
 public:
  ResidualBlock(std::vector<std::unique_ptr<Layer>> main, std::vector<std::unique_ptr<Layer>> shortcut,
                std::string activation = "relu", std::string name = "residual_block");
  std::string type() const override { return "residual_block"; }
  json::Value parameters_config() const override;
  std::vector<int64_t> output_shape(const std::vector<int64_t>& in) const override;
  double flops(const std::vector<int64_t>& in) const override;
  void build(const std::vector<int64_t>& in, Device dev, uint64_t seed) override;
  Tensor forward(const Tensor& x, bool training) override;
  Tensor backward(const Tensor& dy) override;
  void sync_shadow() override;
  void collect_params(std::vector<Param*>& out) override;
  void collect_layers(std::vector<Layer*>& out) override;
  void set_micro_batch(int mb) override;
  const std::vector<std::unique_ptr<Layer>>& main_path() const { return main_; }
  const std::vector<std::unique_ptr<Layer>>& shortcut_path() const { return short_; }
  // GPU: the main path's tail BatchNorm adds the shortcut and applies the block activation
  class BatchNorm* fused_tail() const;
  // the main path's first layer when it is a conv (its dgrad adds the shortcut gradient)
  class Conv2D* head_conv() const;
  // GPU: the projection shortcut's closing BatchNorm, paired with the fused tail
  // (BatchNorm::forward_dual / backward_dual); null without one
  class BatchNorm* dual_shortcut() const;

 private:
  std::vector<std::unique_ptr<Layer>> main_, short_;
  std::string act_;
};

// layer from its JSON record {"type", "name", "parameters"} (the LayerFactory of the formats)
std::unique_ptr<Layer> create_layer(const json::Value& rec);

// GPU fusion pass over a layer sequence: every BatchNorm directly followed by a ReLU applies the
// ReLU itself (one pass instead of two forward and backward; the ReLU layer passes through), and
// every conv directly followed by a BatchNorm hands it the statistics its epilogue computed (no
// statistics pass over the conv output). `on` false undoes it (CPU placement).
// Sequential::initialize / ResidualBlock::build run it.
void fuse_bn_relu(std::vector<std::unique_ptr<Layer>>& seq, bool on);
// after the layers are built: consecutive residual blocks with fused tails — the next block's
// head-conv data gradient (shortcut gradient added) also masks with the previous block's output
// and computes its tail BatchNorm's backward statistics
void fuse_blocks(std::vector<std::unique_ptr<Layer>>& seq, bool on);

class Sequential {
 public:
  explicit Sequential(std::string name = "sequential") : name_(std::move(name)) {}
  Sequential(Sequential&&) = default;
  Sequential& operator=(Sequential&&) = default;
  void add(std::unique_ptr<Layer> l) { layers_.push_back(std::move(l)); }
  void set_input_shape(const std::vector<int64_t>& chw) { input_chw_ = chw; }
  void set_device(Device d);
  Device device() const { return dev_; }
  void initialize(uint64_t seed = 0);
  void set_training(bool t) { training_ = t; }
  bool is_training() const { return training_; }
  // x: fp32 logical NCHW (host or device); returns the logits [N, classes] as a device tensor
  Tensor forward(const Tensor& x, int mb = 0);
  void backward(const Tensor& dlogits, int mb = 0);
  // one partition of a pipeline: activations in the device layout in and out (GPU: bf16 NHWC,
  // CPU: fp32 NCHW); backward returns the input gradient in the same layout
  Tensor forward_activation(const Tensor& x, int mb);
  Tensor backward_activation(const Tensor& g, int mb);
  // the network input (fp32 NCHW, any device) as the first layer's activation
  Tensor input_activation(const Tensor& x) const;
  std::vector<Param*> parameters();
  // forward + backward FLOPs of every top-level layer for an (N, C, H, W) input
  std::vector<double> layer_flops(const std::vector<int64_t>& in) const;
  // every BatchNorm, depth-first through residual blocks (the .bnstats record order)
  std::vector<BatchNorm*> batchnorms();
  void zero_grad();
  size_t num_parameters();
  const std::vector<std::unique_ptr<Layer>>& layers() const { return layers_; }
  const std::string& name() const { return name_; }
  // called with the top-level layer index after each layer's backward (in backward order), inside
  // a capture too (the data-parallel bucket all-reduces start from here: dist::DataParallel)
  void set_backward_hook(std::function<void(size_t)> f) { bwd_hook_ = std::move(f); }

  json::Value get_config() const;
  void print_config() const;
  static Sequential load_from_config(const json::Value& cfg);
  // path.json (architecture) + path.bin (parameters in layer order, logical NCHW fp32) +
  // path.bnstats (BatchNorm running statistics)
  void save_to_file(const std::string& path) const;
  void load_weights_file(const std::string& path);
  // BatchNorm running statistics sidecar (path.bnstats, written by save_to_file)
  void load_bn_stats(const std::string& path);
  static Sequential from_file(const std::string& path, Device dev = Device::cpu());

 private:
  std::string name_;
  std::vector<std::unique_ptr<Layer>> layers_;
  std::vector<int64_t> input_chw_;
  Device dev_ = Device::cpu();
  bool training_ = true;
  bool initialized_ = false;
  std::shared_ptr<ParamArena> arena_;
  std::function<void(size_t)> bwd_hook_;
  void pack_params();
};

class SequentialBuilder {
 public:
  explicit SequentialBuilder(std::string name = "sequential") : model_(std::move(name)) {}
  SequentialBuilder& input(const std::vector<int64_t>& chw);
  SequentialBuilder& conv2d(int out_ch, int kh, int kw, int sh = 1, int sw = 1, int ph = 0, int pw = 0,
                            bool bias = true, const std::string& name = "");
  SequentialBuilder& batchnorm(float eps = 1e-5f, float momentum = 0.1f, bool affine = true,
                               const std::string& name = "");
  SequentialBuilder& activation(const std::string& kind = "relu", const std::string& name = "");
  SequentialBuilder& maxpool2d(int kh, int kw, int sh = 0, int sw = 0, int ph = 0, int pw = 0,
                               const std::string& name = "");
  SequentialBuilder& avgpool2d(int kh, int kw, int sh = 1, int sw = 1, int ph = 0, int pw = 0,
                               const std::string& name = "");
  SequentialBuilder& flatten(const std::string& name = "");
  SequentialBuilder& dense(int out_features, bool bias = true, const std::string& name = "");
  SequentialBuilder& groupnorm(int num_groups, float eps = 1e-5f, bool affine = true, const std::string& name = "");
  SequentialBuilder& dropout(float rate, const std::string& name = "");
  // generic residual block from prebuilt paths (shapes must agree)
  SequentialBuilder& residual(std::vector<std::unique_ptr<Layer>> main, std::vector<std::unique_ptr<Layer>> shortcut,
                              const std::string& activation = "relu", const std::string& name = "");
  // 3x3-BN-ReLU-3x3-BN (+ 1x1-BN projection when the stride or width changes), ReLU after the add
  // (reference include/nn/sequential.hpp:1253)
  SequentialBuilder& basic_residual_block(int in_ch, int out_ch, int stride = 1, const std::string& name = "");
  // 1x1-BN-ReLU-3x3(stride)-BN-ReLU-1x1-BN, BN eps 1e-3 (reference include/nn/sequential.hpp:1288)
  SequentialBuilder& bottleneck_residual_block(int in_ch, int mid_ch, int out_ch, int stride = 1,
                                               const std::string& name = "");
  Sequential build();

 private:
  std::string auto_name(const std::string& given, const std::string& kind);
  Sequential model_;
  std::vector<int64_t> cur_;  // current (C, H, W)
  int count_ = 0;
};

// ---- loss: softmax cross-entropy over logits [N, C] (mean over the batch)
struct LossResult {
  double loss = 0;
  long correct = 0;
  Tensor grad;  // d loss / d logits, same device / dtype as the logits
};
LossResult softmax_cross_entropy(const Tensor& logits, const Tensor& labels);

class Optimizer {
 public:
  explicit Optimizer(float lr) : lr_(lr) {}
  virtual ~Optimizer() = default;
  virtual void step(const std::vector<Param*>& params) = 0;
  void set_learning_rate(float lr) { lr_ = lr; }
  float learning_rate() const { return lr_; }

 protected:
  float lr_;
};

class SGD : public Optimizer {
 public:
  explicit SGD(float lr, float momentum = 0.f) : Optimizer(lr), momentum_(momentum) {}
  void step(const std::vector<Param*>& params) override;
  float momentum() const { return momentum_; }

 private:
  float momentum_;
};

class Adam : public Optimizer {
 public:
  explicit Adam(float lr, float b1 = 0.9f, float b2 = 0.999f, float eps = 1e-8f, float wd = 0.f,
                bool decoupled = false)
      : Optimizer(lr), b1_(b1), b2_(b2), eps_(eps), wd_(wd), decoupled_(decoupled) {}
  void step(const std::vector<Param*>& params) override;
  long step_count() const { return t_; }
  void set_step_count(long t) { t_ = t; }
  // a replayed graph ran one step on the device: mirror it on the host (t) and upload a changed
  // learning rate before the replay
  void before_replay();
  // host step state (lr, t) -> the device step scalars (outside a capture)
  void upload_hyper();

 private:
  float b1_, b2_, eps_, wd_;
  bool decoupled_;
  long t_ = 0;
  // GPU arena path: step scalars in device memory {lr, bc1, bc2, t}, updated on the device
  Tensor hyper_;
  float hyper_lr_ = -1.f;
  long hyper_t_ = -1;
};


// ---- data
class DataSource {
 public:
  virtual ~DataSource() = default;
  virtual void reset(uint64_t epoch) = 0;
  // next batch: x fp32 host NCHW, labels int64; false at the end of the epoch
  virtual bool next(int batch, Tensor& x, Tensor& labels) = 0;
  virtual size_t size() const = 0;
};

// learnable synthetic classification set: class k images carry a class-specific spatial
// pattern plus noise (deterministic in the seed)
class SyntheticClassification : public DataSource {
 public:
  SyntheticClassification(size_t n, int c, int h, int w, int classes, uint64_t seed, float noise = 0.5f);
  void reset(uint64_t epoch) override;
  bool next(int batch, Tensor& x, Tensor& labels) override;
  size_t size() const override { return n_; }

 private:
  size_t n_;
  int c_, h_, w_, classes_;
  uint64_t seed_;
  float noise_;
  std::vector<float> proto_;
  std::vector<size_t> order_;
  size_t pos_ = 0;
};

struct TrainingConfig {
  int epochs = 1;
  int batch_size = 64;
  int max_steps = -1;          // per epoch, -1 = whole epoch
  int progress_interval = 50;  // steps between progress lines, 0 = quiet
  float lr_decay = 1.0f;       // multiplicative per epoch
  uint64_t seed = 0;
};

struct EpochStats {
  double train_loss = 0, train_acc = 0, val_loss = 0, val_acc = 0, seconds = 0;
};

// one optimisation step; returns (loss, correct)
LossResult train_step(Sequential& model, Optimizer& opt, const Tensor& x, const Tensor& labels);
// mean loss / accuracy over a source
EpochStats evaluate(Sequential& model, DataSource& src, int batch_size);
std::vector<EpochStats> train_classification_model(Sequential& model, DataSource& train, DataSource* val,
                                                   Optimizer& opt, const TrainingConfig& cfg);

}  // namespace dcnn
