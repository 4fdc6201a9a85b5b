// Dataset parsers, batch gather and host-side augmentation (reference include/data_loading/*
// and include/data_augmentation/*).  All heavy loops run with the GIL released on a small
// std::thread pool; per-sample random streams are derived from (seed, sample index) so the
// result does not depend on the number of threads.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "native.h"

namespace py = pybind11;
using namespace dcnn_native;

namespace {

int default_threads() {
  unsigned n = std::thread::hardware_concurrency();
  return static_cast<int>(std::max(1u, std::min(n, 16u)));
}

template <typename F>
void parallel_for(size_t n, int threads, F&& fn) {
  if (threads <= 1 || n < 2) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> pool;
  const int T = static_cast<int>(std::min<size_t>(threads, n));
  std::exception_ptr err;
  std::mutex emu;
  for (int t = 0; t < T; ++t)
    pool.emplace_back([&] {
      try {
        for (size_t i = next++; i < n; i = next++) fn(i);
      } catch (...) {
        std::lock_guard<std::mutex> g(emu);
        if (!err) err = std::current_exception();
      }
    });
  for (auto& th : pool) th.join();
  if (err) std::rethrow_exception(err);
}

std::string read_all(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

bool is_dir(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::vector<std::string> list_dir(const std::string& p) {
  std::vector<std::string> out;
  DIR* d = opendir(p.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n != "." && n != "..") out.push_back(n);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<std::string> split_ws(const std::string& line, char sep) {
  std::vector<std::string> out;
  std::string cur;
  std::stringstream ss(line);
  while (std::getline(ss, cur, sep)) out.push_back(cur);
  return out;
}

// ---------------------------------------------------------------- MNIST CSV
py::tuple load_mnist_csv(const std::string& path, bool has_header) {
  std::string text = read_all(path);
  std::vector<size_t> starts;
  size_t pos = 0;
  if (has_header) {
    pos = text.find('\n');
    pos = pos == std::string::npos ? text.size() : pos + 1;
  }
  while (pos < text.size()) {
    size_t e = text.find('\n', pos);
    if (e == std::string::npos) e = text.size();
    if (e > pos + 1) starts.push_back(pos);
    pos = e + 1;
  }
  const size_t N = starts.size();
  py::array_t<float> img({static_cast<py::ssize_t>(N), py::ssize_t(1), py::ssize_t(28), py::ssize_t(28)});
  py::array_t<int64_t> lab({static_cast<py::ssize_t>(N)});
  float* ip = img.mutable_data();
  int64_t* lp = lab.mutable_data();
  {
    py::gil_scoped_release nogil;
    parallel_for(N, default_threads(), [&](size_t i) {
      const char* p = text.data() + starts[i];
      char* end;
      lp[i] = std::strtol(p, &end, 10);
      p = end;
      float* o = ip + i * 784;
      for (int k = 0; k < 784; ++k) {
        while (*p == ',' || *p == ' ') ++p;
        o[k] = static_cast<float>(std::strtol(p, &end, 10)) / 255.0f;
        p = end;
      }
    });
  }
  return py::make_tuple(img, lab);
}

// ---------------------------------------------------------------- CIFAR-10 / 100
py::tuple load_cifar_bin(const std::vector<std::string>& paths, int label_bytes, int label_index) {
  std::vector<std::string> blobs;
  size_t total = 0;
  const size_t rec = label_bytes + 3072;
  for (auto& p : paths) {
    blobs.push_back(read_all(p));
    if (blobs.back().size() % rec) throw std::runtime_error(p + ": size is not a multiple of the record size");
    total += blobs.back().size() / rec;
  }
  py::array_t<float> img({static_cast<py::ssize_t>(total), py::ssize_t(3), py::ssize_t(32), py::ssize_t(32)});
  py::array_t<int64_t> lab({static_cast<py::ssize_t>(total)});
  float* ip = img.mutable_data();
  int64_t* lp = lab.mutable_data();
  {
    py::gil_scoped_release nogil;
    size_t base = 0;
    for (auto& b : blobs) {
      const size_t n = b.size() / rec;
      parallel_for(n, default_threads(), [&](size_t i) {
        const unsigned char* r = reinterpret_cast<const unsigned char*>(b.data()) + i * rec;
        lp[base + i] = r[label_index];
        float* o = ip + (base + i) * 3072;
        for (int k = 0; k < 3072; ++k) o[k] = r[label_bytes + k] / 255.0f;
      });
      base += n;
    }
  }
  return py::make_tuple(img, lab);
}

// ---------------------------------------------------------------- Tiny-ImageNet
py::tuple load_tiny_imagenet(const std::string& root, const std::string& split, int threads, int max_per_class) {
  // class ids in wnids.txt order
  std::vector<std::string> wnids;
  {
    std::stringstream ss(read_all(root + "/wnids.txt"));
    std::string l;
    while (std::getline(ss, l)) {
      while (!l.empty() && (l.back() == '\r' || l.back() == ' ')) l.pop_back();
      if (!l.empty()) wnids.push_back(l);
    }
  }
  std::vector<std::pair<std::string, int>> files;
  auto class_of = [&](const std::string& w) -> int {
    auto it = std::find(wnids.begin(), wnids.end(), w);
    return it == wnids.end() ? -1 : static_cast<int>(it - wnids.begin());
  };
  if (split == "train") {
    for (size_t c = 0; c < wnids.size(); ++c) {
      std::string dir = root + "/train/" + wnids[c] + "/images";
      auto names = list_dir(dir);
      int k = 0;
      for (auto& n : names) {
        if (max_per_class > 0 && k >= max_per_class) break;
        files.emplace_back(dir + "/" + n, static_cast<int>(c));
        ++k;
      }
    }
  } else {
    std::stringstream ss(read_all(root + "/val/val_annotations.txt"));
    std::string l;
    while (std::getline(ss, l)) {
      auto cols = split_ws(l, '\t');
      if (cols.size() < 2) continue;
      const int c = class_of(cols[1]);
      if (c >= 0) files.emplace_back(root + "/val/images/" + cols[0], c);
    }
  }
  const size_t N = files.size();
  py::array_t<float> img({static_cast<py::ssize_t>(N), py::ssize_t(3), py::ssize_t(64), py::ssize_t(64)});
  py::array_t<int64_t> lab({static_cast<py::ssize_t>(N)});
  float* ip = img.mutable_data();
  int64_t* lp = lab.mutable_data();
  std::atomic<int> failures{0};
  {
    py::gil_scoped_release nogil;
    parallel_for(N, threads > 0 ? threads : default_threads(), [&](size_t i) {
      lp[i] = files[i].second;
      float* o = ip + i * 3 * 64 * 64;
      std::string blob;
      std::vector<unsigned char> rgb;
      int w = 0, h = 0;
      std::string err;
      bool ok = false;
      try {
        blob = read_all(files[i].first);
        ok = decode_jpeg(reinterpret_cast<const unsigned char*>(blob.data()), blob.size(), rgb, w, h, &err);
      } catch (...) {
      }
      if (!ok || w != 64 || h != 64) {
        ++failures;
        std::memset(o, 0, sizeof(float) * 3 * 64 * 64);
        return;
      }
      for (int c = 0; c < 3; ++c)
        for (int p = 0; p < 64 * 64; ++p) o[c * 4096 + p] = rgb[p * 3 + c] / 255.0f;
    });
  }
  return py::make_tuple(img, lab, wnids, failures.load());
}

py::dict read_tiny_imagenet_words(const std::string& path) {
  py::dict d;
  std::stringstream ss(read_all(path));
  std::string l;
  while (std::getline(ss, l)) {
    const size_t t = l.find('\t');
    if (t == std::string::npos) continue;
    d[py::str(l.substr(0, t))] = l.substr(t + 1);
  }
  return d;
}

// ---------------------------------------------------------------- WiFi / UJI CSV
py::tuple load_wifi_csv(const std::string& path, size_t f0, size_t f1, size_t t0, size_t t1, bool has_header) {
  std::stringstream ss(read_all(path));
  std::string line;
  std::vector<float> feats, tgts;
  size_t nf = 0, nt = 0, rows = 0;
  bool first = true;
  while (std::getline(ss, line)) {
    if (first && has_header) {
      first = false;
      continue;
    }
    first = false;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    auto cols = split_ws(line, ',');
    if (cols.empty()) continue;
    const size_t fe = std::min(f1, cols.size()), te = std::min(t1, cols.size());
    if (fe <= f0 || te <= t0) continue;
    std::vector<float> fr, tr;
    for (size_t i = f0; i < fe; ++i) {
      float v;
      try {
        v = std::stof(cols[i]);
        if (v == 100.0f || v == 0.0f) v = -100.0f;  // "not detected" -> weakest RSSI (reference semantics)
      } catch (...) {
        v = -100.0f;
      }
      fr.push_back(v);
    }
    bool ok = true;
    for (size_t i = t0; i < te; ++i) {
      try {
        tr.push_back(std::stof(cols[i]));
      } catch (...) {
        ok = false;
      }
    }
    if (!ok || fr.empty() || tr.empty()) continue;
    if (rows == 0) {
      nf = fr.size();
      nt = tr.size();
    }
    if (fr.size() != nf || tr.size() != nt) continue;
    feats.insert(feats.end(), fr.begin(), fr.end());
    tgts.insert(tgts.end(), tr.begin(), tr.end());
    ++rows;
  }
  py::array_t<float> F({static_cast<py::ssize_t>(rows), static_cast<py::ssize_t>(nf)});
  py::array_t<float> T({static_cast<py::ssize_t>(rows), static_cast<py::ssize_t>(nt)});
  if (rows) {
    std::memcpy(F.mutable_data(), feats.data(), feats.size() * sizeof(float));
    std::memcpy(T.mutable_data(), tgts.data(), tgts.size() * sizeof(float));
  }
  return py::make_tuple(F, T);
}

// ---------------------------------------------------------------- gather
void gather_rows(py::array src, py::array_t<int64_t> idx, py::array dst) {
  if (!(src.flags() & py::array::c_style) || !(dst.flags() & py::array::c_style))
    throw std::runtime_error("gather_rows: arrays must be C-contiguous");
  if (src.itemsize() != dst.itemsize()) throw std::runtime_error("gather_rows: dtype mismatch");
  const size_t rowb = src.shape(0) ? src.nbytes() / src.shape(0) : 0;
  const size_t n = idx.size();
  if (static_cast<size_t>(dst.shape(0)) < n || (dst.shape(0) && dst.nbytes() / dst.shape(0) != rowb))
    throw std::runtime_error("gather_rows: destination shape mismatch");
  const char* s = static_cast<const char*>(src.data());
  char* d = static_cast<char*>(dst.mutable_data());
  const int64_t* ix = idx.data();
  const int64_t N = src.shape(0);
  for (size_t i = 0; i < n; ++i)
    if (ix[i] < 0 || ix[i] >= N) throw std::runtime_error("gather_rows: index out of range");
  py::gil_scoped_release nogil;
  parallel_for(n, n * rowb > (1 << 20) ? default_threads() : 1,
               [&](size_t i) { std::memcpy(d + i * rowb, s + static_cast<size_t>(ix[i]) * rowb, rowb); });
}

// ---------------------------------------------------------------- augmentation
struct AugOp {
  std::string kind;
  float p = 0.5f;
  std::vector<float> a;
};

inline float clamp01(float v) { return v < 0 ? 0 : (v > 1 ? 1 : v); }

void apply_one(const AugOp& op, float* img, int C, int H, int W, std::mt19937& rng, std::vector<float>& tmp) {
  std::uniform_real_distribution<float> U(0.f, 1.f);
  const size_t HW = static_cast<size_t>(H) * W, n = HW * C;
  if (op.kind == "normalize") {  // always applied
    for (int c = 0; c < C; ++c) {
      const float m = op.a.size() >= 6 && C == 3 ? op.a[c] : op.a[0];
      const float s = op.a.size() >= 6 && C == 3 ? op.a[3 + c] : op.a[op.a.size() / 2];
      float* q = img + c * HW;
      for (size_t i = 0; i < HW; ++i) q[i] = (q[i] - m) / s;
    }
    return;
  }
  if (U(rng) >= op.p) return;
  if (op.kind == "horizontal_flip") {
    for (int c = 0; c < C; ++c)
      for (int y = 0; y < H; ++y) std::reverse(img + c * HW + y * W, img + c * HW + (y + 1) * W);
  } else if (op.kind == "vertical_flip") {
    for (int c = 0; c < C; ++c)
      for (int y = 0; y < H / 2; ++y)
        std::swap_ranges(img + c * HW + y * W, img + c * HW + (y + 1) * W, img + c * HW + (H - 1 - y) * W);
  } else if (op.kind == "brightness") {
    std::uniform_real_distribution<float> D(-op.a[0], op.a[0]);
    const float f = D(rng);
    for (size_t i = 0; i < n; ++i) img[i] = clamp01(img[i] + f);
  } else if (op.kind == "contrast") {
    std::uniform_real_distribution<float> D(1.f - op.a[0], 1.f + op.a[0]);
    const float f = D(rng);
    for (size_t i = 0; i < n; ++i) img[i] = clamp01(img[i] * f);
  } else if (op.kind == "gaussian_noise") {
    std::normal_distribution<float> D(0.f, op.a[0]);
    for (size_t i = 0; i < n; ++i) img[i] = clamp01(img[i] + D(rng));
  } else if (op.kind == "random_crop") {
    const int pad = static_cast<int>(op.a[0]);
    std::uniform_int_distribution<int> D(0, 2 * pad);
    const int sx = D(rng) - pad, sy = D(rng) - pad;  // offset of the crop window vs. the original
    tmp.assign(img, img + n);
    for (int c = 0; c < C; ++c)
      for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
          const int yy = y + sy, xx = x + sx;
          img[c * HW + y * W + x] = (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0.f : tmp[c * HW + yy * W + xx];
        }
  } else if (op.kind == "cutout") {
    const int s = static_cast<int>(op.a[0]);
    std::uniform_int_distribution<int> DX(0, std::max(0, W - s)), DY(0, std::max(0, H - s));
    const int x0 = DX(rng), y0 = DY(rng);
    for (int c = 0; c < C; ++c)
      for (int y = y0; y < std::min(H, y0 + s); ++y)
        for (int x = x0; x < std::min(W, x0 + s); ++x) img[c * HW + y * W + x] = 0.f;
  } else if (op.kind == "rotation") {
    std::uniform_real_distribution<float> D(-op.a[0], op.a[0]);
    const float ang = D(rng) * 3.14159265358979f / 180.f, ca = std::cos(ang), sa = std::sin(ang);
    const float cx = W / 2.f, cy = H / 2.f;
    tmp.assign(img, img + n);
    for (int c = 0; c < C; ++c)
      for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
          const float sx = (x - cx) * ca - (y - cy) * sa + cx, sy = (x - cx) * sa + (y - cy) * ca + cy;
          const int x1 = static_cast<int>(std::floor(sx)), y1 = static_cast<int>(std::floor(sy));
          const float fx = sx - x1, fy = sy - y1;
          auto at = [&](int yy, int xx) {
            return (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0.f : tmp[c * HW + yy * W + xx];
          };
          img[c * HW + y * W + x] = (1 - fx) * (1 - fy) * at(y1, x1) + fx * (1 - fy) * at(y1, x1 + 1) +
                                    (1 - fx) * fy * at(y1 + 1, x1) + fx * fy * at(y1 + 1, x1 + 1);
        }
  } else {
    throw std::runtime_error("unknown augmentation " + op.kind);
  }
}

void augment(py::array_t<float, py::array::c_style> batch, const std::vector<std::tuple<std::string, float, std::vector<float>>>& ops,
             uint64_t seed, int threads) {
  if (batch.ndim() != 4) throw std::runtime_error("augment: expected [N, C, H, W]");
  std::vector<AugOp> list;
  for (auto& t : ops) list.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
  for (auto& o : list) {
    const bool needs_arg = o.kind != "horizontal_flip" && o.kind != "vertical_flip";
    if (needs_arg && o.a.empty()) throw std::runtime_error("augmentation '" + o.kind + "' needs a parameter");
  }
  const int N = static_cast<int>(batch.shape(0)), C = static_cast<int>(batch.shape(1)),
            H = static_cast<int>(batch.shape(2)), W = static_cast<int>(batch.shape(3));
  float* base = batch.mutable_data();
  py::gil_scoped_release nogil;
  parallel_for(N, threads > 0 ? threads : default_threads(), [&](size_t i) {
    std::seed_seq ss{static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32), static_cast<uint32_t>(i)};
    std::mt19937 rng(ss);
    std::vector<float> tmp;
    float* img = base + i * static_cast<size_t>(C) * H * W;
    for (auto& op : list) apply_one(op, img, C, H, W, rng, tmp);
  });
}

py::array_t<uint8_t> decode_jpeg_py(py::bytes b) {
  std::string s(b);
  std::vector<unsigned char> rgb;
  int w = 0, h = 0;
  std::string err;
  if (!decode_jpeg(reinterpret_cast<const unsigned char*>(s.data()), s.size(), rgb, w, h, &err))
    throw std::runtime_error("decode_jpeg: " + err);
  py::array_t<uint8_t> out({static_cast<py::ssize_t>(h), static_cast<py::ssize_t>(w), py::ssize_t(3)});
  std::memcpy(out.mutable_data(), rgb.data(), rgb.size());
  return out;
}

}  // namespace

void bind_data(py::module_& m) {
  auto d = m.def_submodule("data", "dataset parsers, batch gather, augmentation");
  d.def("load_mnist_csv", &load_mnist_csv, py::arg("path"), py::arg("has_header") = true);
  d.def("load_cifar_bin", &load_cifar_bin, py::arg("paths"), py::arg("label_bytes") = 1, py::arg("label_index") = 0);
  d.def("load_tiny_imagenet", &load_tiny_imagenet, py::arg("root"), py::arg("split") = "train",
        py::arg("threads") = 0, py::arg("max_per_class") = 0);
  d.def("read_tiny_imagenet_words", &read_tiny_imagenet_words);
  d.def("load_wifi_csv", &load_wifi_csv, py::arg("path"), py::arg("feature_start"), py::arg("feature_end"),
        py::arg("target_start"), py::arg("target_end"), py::arg("has_header") = true);
  d.def("gather_rows", &gather_rows);
  d.def("augment", &augment, py::arg("batch"), py::arg("ops"), py::arg("seed"), py::arg("threads") = 0);
  d.def("decode_jpeg", &decode_jpeg_py);
}
