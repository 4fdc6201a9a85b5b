// Tensor / Storage of the C++ host API (see dcnn/tensor.hpp).
#include "dcnn/tensor.hpp"

#include <cstdlib>
#include <istream>
#include <ostream>
#include <sstream>
#include <stdexcept>

namespace dcnn {

Device Device::parse(const std::string& s) {
  std::string u;
  for (char c : s) u += (char)toupper((unsigned char)c);
  if (u == "CPU" || u == "CPU:0") return cpu();
  if (u == "GPU" || u == "CUDA") return gpu(0);
  if (u.rfind("GPU:", 0) == 0) return gpu(std::stoi(u.substr(4)));
  throw std::invalid_argument("unknown device '" + s + "'");
}

std::string Device::str() const { return is_gpu() ? "GPU:" + std::to_string(index) : "CPU:0"; }

size_t dtype_size(DType t) {
  switch (t) {
    case DType::F32: return 4;
    case DType::BF16: return 2;
    case DType::I32: return 4;
    case DType::I64: return 8;
    case DType::U8: return 1;
  }
  return 0;
}

const char* dtype_name(DType t) {
  switch (t) {
    case DType::F32: return "f32";
    case DType::BF16: return "bf16";
    case DType::I32: return "i32";
    case DType::I64: return "i64";
    case DType::U8: return "u8";
  }
  return "?";
}

uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

float bf16_to_f32(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

Storage::Storage(Device d, size_t nbytes) : dev_(d), n_(nbytes) {
  const size_t n = nbytes ? nbytes : 1;
  if (d.is_gpu()) {
    gpu::set_device(d.index);
    p_ = gpu::alloc(n);
  } else {
    p_ = std::aligned_alloc(64, (n + 63) / 64 * 64);
    if (!p_) throw std::bad_alloc();
  }
}

Storage::~Storage() {
  if (!p_) return;
  if (dev_.is_gpu()) {
    gpu::set_device(dev_.index);
    gpu::free(p_);
  } else {
    std::free(p_);
  }
}

int64_t Tensor::numel() const {
  int64_t n = 1;
  for (auto s : shape_) n *= s;
  return n;
}

Tensor Tensor::empty(const std::vector<int64_t>& shape, DType dt, Device dev, Layout layout) {
  Tensor t;
  t.shape_ = shape;
  t.dt_ = dt;
  t.layout_ = layout;
  t.st_ = std::make_shared<Storage>(dev, t.nbytes());
  return t;
}

Tensor Tensor::zeros(const std::vector<int64_t>& shape, DType dt, Device dev, Layout layout) {
  Tensor t = empty(shape, dt, dev, layout);
  t.zero_();
  return t;
}

void Tensor::zero_() {
  if (!st_) return;
  if (device().is_gpu()) {
    gpu::set_device(device().index);
    gpu::zero(data(), nbytes());
  } else {
    std::memset(data(), 0, nbytes());
  }
}

Tensor Tensor::from_host(const std::vector<float>& v, const std::vector<int64_t>& shape, Device dev, DType dt,
                         Layout layout) {
  Tensor t;
  t.shape_ = shape;
  t.dt_ = dt;
  t.layout_ = layout;
  if ((int64_t)v.size() != t.numel()) throw std::invalid_argument("from_host: size does not match shape");
  std::vector<float> phys(v.size());
  relayout(v.data(), Layout::NCHW, phys.data(), layout, shape);
  std::vector<uint8_t> bytes(t.nbytes());
  if (dt == DType::F32) {
    std::memcpy(bytes.data(), phys.data(), bytes.size());
  } else if (dt == DType::BF16) {
    auto* o = reinterpret_cast<uint16_t*>(bytes.data());
    for (size_t i = 0; i < phys.size(); ++i) o[i] = f32_to_bf16(phys[i]);
  } else {
    throw std::invalid_argument("from_host: float data into a non-float dtype");
  }
  t.st_ = std::make_shared<Storage>(dev, t.nbytes());
  if (dev.is_gpu()) {
    gpu::set_device(dev.index);
    gpu::copy(t.data(), bytes.data(), bytes.size(), 0);
  } else {
    std::memcpy(t.data(), bytes.data(), bytes.size());
  }
  return t;
}

Tensor Tensor::from_host_i64(const std::vector<int64_t>& v, Device dev) {
  Tensor t = empty({(int64_t)v.size()}, DType::I64, dev);
  if (dev.is_gpu()) {
    gpu::set_device(dev.index);
    gpu::copy(t.data(), v.data(), v.size() * 8, 0);
  } else {
    std::memcpy(t.data(), v.data(), v.size() * 8);
  }
  return t;
}

Tensor Tensor::view(const std::vector<int64_t>& shape, Layout layout) const {
  Tensor t = *this;
  t.shape_ = shape;
  t.layout_ = layout;
  if (t.numel() != numel()) throw std::invalid_argument("view: element count mismatch " + shape_str(shape));
  return t;
}

Tensor Tensor::slice(size_t byte_off, const std::vector<int64_t>& shape, DType dt, Layout layout) const {
  Tensor t;
  t.st_ = st_;
  t.off_ = off_ + byte_off;
  t.shape_ = shape;
  t.dt_ = dt;
  t.layout_ = layout;
  if (!st_ || t.off_ + t.nbytes() > st_->nbytes()) throw std::out_of_range("slice: outside the storage");
  return t;
}

void Tensor::ensure(const std::vector<int64_t>& shape, DType dt, Device dev, Layout layout) {
  int64_t n = 1;
  for (auto s : shape) n *= s;
  const size_t need = (size_t)n * dtype_size(dt);
  if (!st_ || st_->device() != dev || st_->nbytes() - off_ < need) {
    st_ = std::make_shared<Storage>(dev, need);
    off_ = 0;
  }
  shape_ = shape;
  dt_ = dt;
  layout_ = layout;
}

Tensor Tensor::clone() const { return to(device()); }

Tensor Tensor::to(Device dev) const {
  Tensor t = empty(shape_, dt_, dev, layout_);
  const Device src = device();
  if (!src.is_gpu() && !dev.is_gpu()) {
    std::memcpy(t.data(), data(), nbytes());
  } else if (src.is_gpu() && dev.is_gpu()) {
    gpu::set_device(dev.index);
    gpu::copy(t.data(), data(), nbytes(), 2);
  } else if (dev.is_gpu()) {
    gpu::set_device(dev.index);
    gpu::copy(t.data(), data(), nbytes(), 0);
  } else {
    gpu::set_device(src.index);
    gpu::copy(t.data(), data(), nbytes(), 1);
  }
  return t;
}

std::vector<float> Tensor::to_host_f32() const {
  std::vector<uint8_t> bytes(nbytes());
  if (device().is_gpu()) {
    gpu::set_device(device().index);
    gpu::copy(bytes.data(), data(), bytes.size(), 1);
  } else {
    std::memcpy(bytes.data(), data(), bytes.size());
  }
  std::vector<float> phys((size_t)numel());
  if (dt_ == DType::F32) {
    std::memcpy(phys.data(), bytes.data(), bytes.size());
  } else if (dt_ == DType::BF16) {
    const auto* b = reinterpret_cast<const uint16_t*>(bytes.data());
    for (size_t i = 0; i < phys.size(); ++i) phys[i] = bf16_to_f32(b[i]);
  } else {
    throw std::invalid_argument("to_host_f32: not a float tensor");
  }
  std::vector<float> out(phys.size());
  relayout(phys.data(), layout_, out.data(), Layout::NCHW, shape_);
  return out;
}

std::vector<int64_t> Tensor::to_host_i64() const {
  if (dt_ != DType::I64) throw std::invalid_argument("to_host_i64: not an int64 tensor");
  std::vector<int64_t> v((size_t)numel());
  if (device().is_gpu()) {
    gpu::set_device(device().index);
    gpu::copy(v.data(), data(), nbytes(), 1);
  } else {
    std::memcpy(v.data(), data(), nbytes());
  }
  return v;
}

void Tensor::save(std::ostream& os) const {
  uint64_t s[4] = {1, 1, 1, 1};
  for (int k = 0; k < rank() && k < 4; ++k) s[k] = (uint64_t)shape_[k];
  for (int k = 4; k < rank(); ++k) s[3] *= (uint64_t)shape_[k];
  os.write(reinterpret_cast<const char*>(s), sizeof(s));
  const std::vector<float> v = to_host_f32();
  os.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)(v.size() * 4));
  if (!os) throw std::runtime_error("Tensor::save: write failed");
}

Tensor Tensor::load(std::istream& is, Device dev) {
  uint64_t s[4];
  is.read(reinterpret_cast<char*>(s), sizeof(s));
  if (!is) throw std::runtime_error("Failed to read tensor shape from file");
  std::vector<int64_t> shape{(int64_t)s[0], (int64_t)s[1], (int64_t)s[2], (int64_t)s[3]};
  std::vector<float> v((size_t)(s[0] * s[1] * s[2] * s[3]));
  is.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(v.size() * 4));
  if (!is) throw std::runtime_error("Failed to read tensor data from file");
  return from_host(v, shape, dev);
}

std::string shape_str(const std::vector<int64_t>& s) {
  std::ostringstream o;
  o << "(";
  for (size_t i = 0; i < s.size(); ++i) o << (i ? ", " : "") << s[i];
  o << ")";
  return o.str();
}

}  // namespace dcnn
