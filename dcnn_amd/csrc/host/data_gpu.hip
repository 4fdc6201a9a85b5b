// GPU data path of the C++ host API (dcnn/train.hpp DeviceImageDataset): the HBM-resident image
// set and its one-launch batch assembly (augment.hip, the kernel the Python DeviceDataLoader runs).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../kernels/api.h"
#include "dcnn/train.hpp"

namespace dcnn {
namespace {
uint64_t mix(uint64_t z) {  // splitmix64 finaliser (data/device_loader.py _mix)
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// every value an exact k / 255 (decoded 8-bit images): stored as uint8 (4x less HBM and traffic)
bool exact_u8(const std::vector<float>& v) {
  for (float f : v) {
    const float q = std::nearbyint(f * 255.f);
    if (q < 0.f || q > 255.f || q / 255.f != f) return false;
  }
  return true;
}
}  // namespace

DeviceImageDataset::DeviceImageDataset(const ImageDataset& host, Device dev, uint64_t seed, bool shuffle,
                                       bool drop_last)
    : dev_(dev), n_(host.size()), c_(host.channels()), h_(host.height()), w_(host.width()), seed_(seed),
      shuffle_(shuffle), drop_last_(drop_last) {
  if (!dev.is_gpu()) throw std::invalid_argument("DeviceImageDataset: a GPU device");
  if (!augment_batch_supported(c_, h_, w_))
    throw std::invalid_argument("DeviceImageDataset: " + std::to_string(c_) + "x" + std::to_string(h_) + "x" +
                                std::to_string(w_) + " images exceed the batch kernel's LDS staging");
  const std::vector<float>& img = host.images();
  u8_ = exact_u8(img);
  const int64_t per = (int64_t)c_ * h_ * w_;
  if (u8_) {
    std::vector<uint8_t> q(img.size());
    for (size_t i = 0; i < img.size(); ++i) q[i] = (uint8_t)std::nearbyint(img[i] * 255.f);
    data_ = Tensor::empty({(int64_t)n_ * per}, DType::U8, dev);
    gpu::copy(data_.data(), q.data(), q.size(), 0);
  } else {
    data_ = Tensor::empty({(int64_t)n_ * per}, DType::F32, dev);
    gpu::copy(data_.data(), img.data(), img.size() * 4, 0);
  }
  labels_ = Tensor::from_host_i64(host.labels(), dev);
  order_.resize(n_);
  order_dev_ = Tensor::empty({(int64_t)std::max<size_t>(n_, 1)}, DType::I64, dev);
  reset(0);
}

DeviceImageDataset& DeviceImageDataset::add(int kind, float p, std::initializer_list<float> a) {
  if (ops_.size() >= (size_t)kAugMaxOps) throw std::invalid_argument("DeviceImageDataset: at most 12 ops");
  Op o{kind, p, {0, 0, 0, 0, 0, 0}};
  int k = 0;
  for (float v : a) o.a[k++] = v;
  ops_.push_back(o);
  return *this;
}
DeviceImageDataset& DeviceImageDataset::horizontal_flip(float p) { return add(AUG_HFLIP, p, {}); }
DeviceImageDataset& DeviceImageDataset::vertical_flip(float p) { return add(AUG_VFLIP, p, {}); }
DeviceImageDataset& DeviceImageDataset::rotation(float p, float deg) { return add(AUG_ROTATION, p, {deg}); }
DeviceImageDataset& DeviceImageDataset::brightness(float p, float d) { return add(AUG_BRIGHTNESS, p, {d}); }
DeviceImageDataset& DeviceImageDataset::contrast(float p, float d) { return add(AUG_CONTRAST, p, {d}); }
DeviceImageDataset& DeviceImageDataset::gaussian_noise(float p, float s) { return add(AUG_NOISE, p, {s}); }
DeviceImageDataset& DeviceImageDataset::random_crop(float p, int pad) { return add(AUG_CROP, p, {(float)pad}); }
DeviceImageDataset& DeviceImageDataset::cutout(float p, int size) { return add(AUG_CUTOUT, p, {(float)size}); }
DeviceImageDataset& DeviceImageDataset::normalize(const std::vector<float>& mean, const std::vector<float>& stdev) {
  if (mean.empty() || mean.size() != stdev.size()) throw std::invalid_argument("normalize: mean / std per channel");
  // (channels >= 3 use mean[c] / std[c] of the first three; one value broadcasts: data.cpp's rule)
  auto at = [](const std::vector<float>& v, int c) { return v.size() >= 3 ? v[c] : v[0]; };
  return add(AUG_NORMALIZE, 1.f, {at(mean, 0), at(mean, 1), at(mean, 2), at(stdev, 0), at(stdev, 1), at(stdev, 2)});
}

uint64_t DeviceImageDataset::epoch_seed() const { return mix(seed_ * 0x2545F4914F6CDD1Dull + epoch_); }

void DeviceImageDataset::reset(uint64_t epoch) {
  epoch_ = epoch;
  for (size_t i = 0; i < n_; ++i) order_[i] = (int64_t)i;
  if (shuffle_) {
    uint64_t s = seed_ * 1000003ull + epoch;
    for (size_t i = n_; i > 1; --i) {
      s = mix(s);
      std::swap(order_[i - 1], order_[(size_t)(s % i)]);
    }
  }
  // stream-ordered upload on the current flow: batches already assembled from the previous
  // order were enqueued before it
  if (n_) gpu::copy(order_dev_.data(), order_.data(), n_ * 8, 0);
  pos_ = 0;
}

bool DeviceImageDataset::next(int batch, Tensor& x, Tensor& labels) {
  if (batch <= 0 || pos_ >= n_) return false;
  const size_t left = n_ - pos_;
  if (drop_last_ && left < (size_t)batch) return false;
  const int b = (int)std::min<size_t>((size_t)batch, left);
  x = Tensor::empty({b, c_, h_, w_}, DType::F32, dev_);
  labels = Tensor::empty({b}, DType::I64, dev_);
  AugBatchArgs a{};
  a.src = data_.data();
  a.src_u8 = u8_ ? 1 : 0;
  a.idx = order_dev_.ptr<int64_t>() + pos_;
  a.labels = labels_.ptr<int64_t>();
  a.labels_out = labels.ptr<int64_t>();
  a.out = x.ptr<float>();
  a.B = b;
  a.C = c_;
  a.H = h_;
  a.W = w_;
  a.seed = epoch_seed();
  a.nops = (int)ops_.size();
  for (size_t k = 0; k < ops_.size(); ++k) {
    a.ops[k].kind = ops_[k].kind;
    a.ops[k].p = ops_[k].p;
    std::memcpy(a.ops[k].a, ops_[k].a, sizeof a.ops[k].a);
  }
  augment_batch(a, static_cast<hipStream_t>(gpu::flow()));
  pos_ += (size_t)b;
  return true;
}

}  // namespace dcnn
