// Layout traits of the C++ host API: logical NCHW / NCDHW dimensions, physical order per layout.
//
// Every tensor keeps its LOGICAL shape in the reference's order (N, C, H, W) or (N, C, D, H, W);
// the layout names the PHYSICAL order in memory. NHWC / NDHWC (channels innermost) is the MFMA
// GEMM-K-contiguous form the GPU kernels read; NCHW / NCDHW is the reference's CPU form.
// LayoutTrait<L> is the compile-time description (rank, physical permutation, strides, offsets);
// layout_info(L) the same at run time for code that switches on a tensor's layout.
// Reference parity: include/tensor/layout_trait.hpp:13-135 (NCHW / NHWC / NCDHW / NDHWC).
#pragma once
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace dcnn {

enum class Layout { NCHW, NHWC, NCDHW, NDHWC };

template <Layout L>
struct LayoutTrait;

// perm[k] = logical dimension stored at physical position k (outermost first)
template <>
struct LayoutTrait<Layout::NCHW> {
  static constexpr int rank = 4;
  static constexpr std::array<int, 4> perm{0, 1, 2, 3};
  static constexpr bool channels_last = false;
  static constexpr const char* name = "NCHW";
};
template <>
struct LayoutTrait<Layout::NHWC> {
  static constexpr int rank = 4;
  static constexpr std::array<int, 4> perm{0, 2, 3, 1};
  static constexpr bool channels_last = true;
  static constexpr const char* name = "NHWC";
};
template <>
struct LayoutTrait<Layout::NCDHW> {
  static constexpr int rank = 5;
  static constexpr std::array<int, 5> perm{0, 1, 2, 3, 4};
  static constexpr bool channels_last = false;
  static constexpr const char* name = "NCDHW";
};
template <>
struct LayoutTrait<Layout::NDHWC> {
  static constexpr int rank = 5;
  static constexpr std::array<int, 5> perm{0, 2, 3, 4, 1};
  static constexpr bool channels_last = true;
  static constexpr const char* name = "NDHWC";
};

// logical-order strides (elements) of a dense tensor of logical dims `d` stored in layout L
template <Layout L>
constexpr std::array<int64_t, LayoutTrait<L>::rank> strides_of(const std::array<int64_t, LayoutTrait<L>::rank>& d) {
  constexpr int R = LayoutTrait<L>::rank;
  std::array<int64_t, R> s{};
  int64_t acc = 1;
  for (int k = R - 1; k >= 0; --k) {
    s[LayoutTrait<L>::perm[k]] = acc;
    acc *= d[LayoutTrait<L>::perm[k]];
  }
  return s;
}

// element offset of logical index `i`
template <Layout L>
constexpr int64_t offset_of(const std::array<int64_t, LayoutTrait<L>::rank>& d,
                            const std::array<int64_t, LayoutTrait<L>::rank>& i) {
  const auto s = strides_of<L>(d);
  int64_t o = 0;
  for (int k = 0; k < LayoutTrait<L>::rank; ++k) o += i[k] * s[k];
  return o;
}

// physical (memory-order) dims
template <Layout L>
constexpr std::array<int64_t, LayoutTrait<L>::rank> physical_dims(const std::array<int64_t, LayoutTrait<L>::rank>& d) {
  std::array<int64_t, LayoutTrait<L>::rank> p{};
  for (int k = 0; k < LayoutTrait<L>::rank; ++k) p[k] = d[LayoutTrait<L>::perm[k]];
  return p;
}

// ---- run-time view
struct LayoutInfo {
  Layout layout;
  int rank;
  std::vector<int> perm;
  bool channels_last;
  const char* name;
};

inline LayoutInfo layout_info(Layout l) {
  auto mk = [&](auto t) {
    using T = decltype(t);
    return LayoutInfo{l, T::rank, std::vector<int>(T::perm.begin(), T::perm.end()), T::channels_last, T::name};
  };
  switch (l) {
    case Layout::NCHW: return mk(LayoutTrait<Layout::NCHW>{});
    case Layout::NHWC: return mk(LayoutTrait<Layout::NHWC>{});
    case Layout::NCDHW: return mk(LayoutTrait<Layout::NCDHW>{});
    case Layout::NDHWC: return mk(LayoutTrait<Layout::NDHWC>{});
  }
  throw std::invalid_argument("unknown layout");
}

// logical strides of logical dims `d` in layout `l` (d.size() must equal the layout's rank; any
// other rank is dense row-major)
inline std::vector<int64_t> layout_strides(Layout l, const std::vector<int64_t>& d) {
  std::vector<int64_t> s(d.size(), 1);
  const LayoutInfo li = layout_info(l);
  if ((int)d.size() != li.rank) {
    int64_t acc = 1;
    for (int k = (int)d.size() - 1; k >= 0; --k) {
      s[k] = acc;
      acc *= d[k];
    }
    return s;
  }
  int64_t acc = 1;
  for (int k = li.rank - 1; k >= 0; --k) {
    s[li.perm[k]] = acc;
    acc *= d[li.perm[k]];
  }
  return s;
}

// copy between two layouts of the same logical dims (host memory, any element type)
template <typename T>
void relayout(const T* src, Layout ls, T* dst, Layout ld, const std::vector<int64_t>& d) {
  const auto ss = layout_strides(ls, d), sd = layout_strides(ld, d);
  int64_t n = 1;
  for (auto v : d) n *= v;
  std::vector<int64_t> idx(d.size(), 0);
  for (int64_t e = 0; e < n; ++e) {
    int64_t os = 0, od = 0;
    for (size_t k = 0; k < d.size(); ++k) {
      os += idx[k] * ss[k];
      od += idx[k] * sd[k];
    }
    dst[od] = src[os];
    for (int k = (int)d.size() - 1; k >= 0; --k) {
      if (++idx[k] < d[k]) break;
      idx[k] = 0;
    }
  }
}

}  // namespace dcnn
