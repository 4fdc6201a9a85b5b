// GPU backend of the C++ host API: the HIP/CDNA4 kernel library (csrc/kernels/*.hip) driven
// from C++ — bf16 NHWC activations, fp32 master parameters, bf16 operand shadows. Convolutions
// and dense layers run on the generic implicit-GEMM MFMA kernels (gemm_nt forward / dgrad,
// gemm_tn + split-K reduce weight gradients), BatchNorm on the deterministic slab statistics,
// the loss and the optimizers on the fused kernels. Work goes to the null stream in order;
// workspaces are grow-only device buffers reused across calls.
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../kernels/api.h"
#include "dcnn/ops.hpp"
#include "dcnn/tensor.hpp"

#define HOST_HIP_CHECK(x)                                                                    \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace dcnn {

namespace gpu {
int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
void set_device(int dev) { HOST_HIP_CHECK(hipSetDevice(dev)); }
void* alloc(size_t nbytes) {
  void* p = nullptr;
  HOST_HIP_CHECK(hipMalloc(&p, nbytes));
  return p;
}
void free(void* p) { (void)hipFree(p); }
void copy(void* dst, const void* src, size_t nbytes, int kind) {
  static const hipMemcpyKind k[] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice};
  HOST_HIP_CHECK(hipMemcpy(dst, src, nbytes, k[kind]));
}
void synchronize() { HOST_HIP_CHECK(hipDeviceSynchronize()); }
}  // namespace gpu

namespace gpu_ops {
namespace {
constexpr int kPlain = 0, kConvFwd = 1, kConvDgrad = 2;
constexpr int kBF16 = 1;
const hipStream_t S = nullptr;

// grow-only workspace per purpose
enum Slot { W_T = 0, SLAB, BSLAB, STAT_SLAB, STAT_SUMS, STAT_PART, LOSS_WS, LOSS_OUT, TICKETS, NSLOTS };
void* scratch(Slot s, size_t bytes) {
  static void* p[NSLOTS] = {};
  static size_t n[NSLOTS] = {};
  if (n[s] < bytes) {
    if (p[s]) HOST_HIP_CHECK(hipFree(p[s]));
    HOST_HIP_CHECK(hipMalloc(&p[s], bytes));
    n[s] = bytes;
  }
  return p[s];
}

// batched [rows][cols] -> [cols][rows] transpose of 16-bit elements (32 x 32 LDS tiles)
__global__ void transpose16_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int rows, int cols) {
  __shared__ uint16_t t[32][33];
  const long b = blockIdx.z;
  const uint16_t* src = in + b * rows * cols;
  uint16_t* dst = out + b * rows * cols;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  for (int k = threadIdx.y; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + threadIdx.x;
    if (r < rows && c < cols) t[k][threadIdx.x] = src[(long)r * cols + c];
  }
  __syncthreads();
  for (int k = threadIdx.y; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + threadIdx.x;
    if (r < rows && c < cols) dst[(long)c * rows + r] = t[threadIdx.x][k];
  }
}

void transpose16(const void* in, void* out, int batch, int rows, int cols) {
  dim3 grid((cols + 31) / 32, (rows + 31) / 32, batch);
  hipLaunchKernelGGL(transpose16_kernel, grid, dim3(32, 8), 0, S, static_cast<const uint16_t*>(in),
                     static_cast<uint16_t*>(out), rows, cols);
  HOST_HIP_CHECK(hipGetLastError());
}

PoolGeom geom(const PoolShape& p) { return PoolGeom{p.N, p.H, p.W, p.C, p.OH, p.OW, p.KH, p.KW, p.SH, p.SW, p.PH, p.PW}; }

void wgrad_reduce(const float* slab, float* gw, long n, const float* bslab, float* gb, long nb, int splits) {
  if (gb)
    splitk_reduce2(slab, gw, n, bslab, gb, nb, splits, 1, S);
  else
    splitk_reduce(slab, gw, n, splits, 1, S);
}
}  // namespace

void input_to_nhwc(const float* x, void* y, int N, int C, int HW) { nchw_to_nhwc(kBF16, x, y, N, C, HW, S); }
void nhwc_to_nchw(const void* x, void* y, int N, int HW, int C) { transpose16(x, y, N, HW, C); }
void nchw_to_nhwc_bf16(const void* x, void* y, int N, int HW, int C) { transpose16(x, y, N, C, HW); }
void cast_bf16(const float* x, void* y, long n) { cast_f32_bf16(x, static_cast<bf16*>(y), n, S); }
void zero(void* p, long nbytes) { zero_bytes(p, nbytes, S); }

void conv_fwd(const void* x, const void* w, const float* bias, void* y, const ConvShape& s) {
  const int K = s.KH * s.KW * s.C;
  NtArgs a{static_cast<const bf16*>(x), static_cast<const bf16*>(w), y, s.N * s.OH * s.OW, s.Co, K, 0, K, s.Co,
           kConvFwd, s.N, s.H, s.W, s.C, s.OH, s.OW, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, bias, nullptr, nullptr, 0, 0};
  gemm_nt(a, S);
}

void conv_dgrad(const void* dy, const void* w, void* dx, const ConvShape& s) {
  const int T = s.KH * s.KW, K = T * s.Co;
  bf16* wt = static_cast<bf16*>(scratch(W_T, (size_t)s.Co * T * s.C * 2));
  conv_weight_transpose(kBF16, w, wt, s.Co, T, s.C, S);  // [Co][T][C] -> [C][T][Co]
  NtArgs a{static_cast<const bf16*>(dy), wt, dx, s.N * s.H * s.W, s.C, K, 0, K, s.C, kConvDgrad, s.N, s.OH, s.OW,
           s.Co, s.H, s.W, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, nullptr, nullptr, nullptr, 0, 0};
  gemm_nt(a, S);
}

void conv_wgrad(const void* dy, const void* x, float* gw, float* gb, const ConvShape& s) {
  const int Ng = s.KH * s.KW * s.C, P = s.N * s.OH * s.OW;
  const int splits = gemm_tn_splits(s.Co, Ng, P);
  float* slab = static_cast<float*>(scratch(SLAB, (size_t)splits * s.Co * Ng * 4));
  float* bslab = gb ? static_cast<float*>(scratch(BSLAB, (size_t)splits * s.Co * 4)) : nullptr;
  TnArgs a{static_cast<const bf16*>(dy), static_cast<const bf16*>(x), slab, bslab, s.Co, Ng, P, kConvFwd, s.N, s.H,
           s.W, s.C, s.OH, s.OW, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, 0, 0};
  gemm_tn(a, splits, S);
  wgrad_reduce(slab, gw, (long)s.Co * Ng, bslab, gb, s.Co, splits);
}

void dense_fwd(const void* x, const void* w, const float* bias, void* y, int N, int In, int Out) {
  NtArgs a{static_cast<const bf16*>(x), static_cast<const bf16*>(w), y, N, Out, In, In, In, Out, kPlain, 0, 0, 0, 0,
           1, 1, 1, 1, 1, 1, 0, 0, bias, nullptr, nullptr, 0, 0};
  gemm_nt(a, S);
}

void dense_dgrad(const void* dy, const void* w, void* dx, int N, int In, int Out) {
  bf16* wt = static_cast<bf16*>(scratch(W_T, (size_t)In * Out * 2));
  conv_weight_transpose(kBF16, w, wt, Out, 1, In, S);  // [Out][In] -> [In][Out]
  NtArgs a{static_cast<const bf16*>(dy), wt, dx, N, In, Out, Out, Out, In, kPlain, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 0, 0,
           nullptr, nullptr, nullptr, 0, 0};
  gemm_nt(a, S);
}

void dense_wgrad(const void* dy, const void* x, float* gw, float* gb, int N, int In, int Out) {
  const int splits = gemm_tn_splits(Out, In, N);
  float* slab = static_cast<float*>(scratch(SLAB, (size_t)splits * Out * In * 4));
  float* bslab = gb ? static_cast<float*>(scratch(BSLAB, (size_t)splits * Out * 4)) : nullptr;
  TnArgs a{static_cast<const bf16*>(dy), static_cast<const bf16*>(x), slab, bslab, Out, In, N, kPlain, 0, 0, 0, 0, 1,
           1, 1, 1, 1, 1, 0, 0, In, 0};
  gemm_tn(a, splits, S);
  wgrad_reduce(slab, gw, (long)Out * In, bslab, gb, Out, splits);
}

// deterministic slab statistics: (pointer, parts) for bn_apply / bn_bwd_apply
static std::pair<const float*, int> reduce_stats(int mode, const float* slab, int rows, int C) {
  const int parts = bn_stat_parts(rows);
  float* sums = static_cast<float*>(scratch(STAT_SUMS, (size_t)2 * C * 4));
  float* part = parts > 1 ? static_cast<float*>(scratch(STAT_PART, (size_t)parts * 3 * C * 4)) : nullptr;
  bn_stat_reduce(mode, slab, rows, C, sums, part, nullptr, S);
  return {parts > 1 ? part : sums, parts};
}

void bn_fwd(const void* x, void* y, long R, int C, const float* g, const float* b, float eps, bool train,
            float* rmean, float* rvar, float momentum, float* smean, float* sistd) {
  if (!train) {
    bn_apply(kBF16, x, y, R, C, nullptr, 1, (float)R, g, b, eps, nullptr, 0, smean, sistd, rmean, rvar, momentum, 1, S);
    return;
  }
  const int rows = bn_partial_rows(R, C);
  float* slab = static_cast<float*>(scratch(STAT_SLAB, (size_t)rows * 3 * C * 4));
  bn_partial(kBF16, x, nullptr, nullptr, nullptr, nullptr, nullptr, R, C, slab, 0, nullptr, S);
  const auto st = reduce_stats(0, slab, rows, C);
  bn_apply(kBF16, x, y, R, C, st.first, st.second, (float)R, g, b, eps, nullptr, 0, smean, sistd, rmean, rvar,
           momentum, 0, S);
}

void bn_bwd(const void* dy, const void* x, void* dx, long R, int C, const float* mean, const float* istd,
            const float* g, float* dg, float* db, bool train) {
  const int rows = bn_partial_rows(R, C);
  float* slab = static_cast<float*>(scratch(STAT_SLAB, (size_t)rows * 2 * C * 4));
  bn_partial(kBF16, x, dy, nullptr, nullptr, mean, istd, R, C, slab, 1, nullptr, S);
  const auto st = reduce_stats(1, slab, rows, C);
  bn_bwd_apply(kBF16, dy, nullptr, x, dx, R, C, mean, istd, g, st.first, st.second, (float)R, dg, db, train ? 0 : 1,
               S);
}

void maxpool_fwd(const void* x, void* y, uint8_t* idx, const PoolShape& p) {
  if (p.KH * p.KW > 256) throw std::invalid_argument("maxpool: window larger than 256 taps");
  dcnn::maxpool_fwd(kBF16, x, y, idx, geom(p), S);
}
void maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, const PoolShape& p) {
  dcnn::maxpool_bwd(kBF16, dy, idx, dx, geom(p), S);
}
void avgpool_fwd(const void* x, void* y, const PoolShape& p) { dcnn::avgpool_fwd(kBF16, x, y, geom(p), S); }
void avgpool_bwd(const void* dy, void* dx, const PoolShape& p) { dcnn::avgpool_bwd(kBF16, dy, dx, geom(p), S); }

void act_fwd(int kind, const void* x, void* y, long n, float alpha) { dcnn::act_fwd(kBF16, x, y, n, kind, alpha, S); }
void act_bwd(int kind, const void* x, const void* dy, void* dx, long n, float alpha) {
  dcnn::act_bwd(kBF16, x, dy, dx, n, kind, alpha, S);
}

double softmax_ce(const void* pred, const int64_t* labels, void* grad, int N, int C, long* correct) {
  float* ws = N > 4 ? static_cast<float*>(scratch(LOSS_WS, (size_t)loss_workspace_floats(N) * 4)) : nullptr;
  static unsigned* tickets = nullptr;  // zeroed once; every launch leaves them zeroed
  if (N > 4 && !tickets) {
    tickets = static_cast<unsigned*>(scratch(TICKETS, 64 * 4));
    HOST_HIP_CHECK(hipMemset(tickets, 0, 64 * 4));
  }
  char* out = static_cast<char*>(scratch(LOSS_OUT, 16));
  float* loss = reinterpret_cast<float*>(out);
  int* corr = reinterpret_cast<int*>(out + 8);
  loss_fused(kBF16, pred, nullptr, labels, grad, loss, corr, N, C, 1, 1e-15f, 1.0f, ws, N > 4 ? tickets : nullptr,
             S);
  char host[16];
  HOST_HIP_CHECK(hipMemcpy(host, out, 16, hipMemcpyDeviceToHost));
  float l;
  int c;
  std::memcpy(&l, host, 4);
  std::memcpy(&c, host + 8, 4);
  if (correct) *correct = c;
  return l;
}

void adam(float* p, const float* g, float* m, float* v, void* shadow, long n, float lr, float b1, float b2, float eps,
          float bc1, float bc2, float wd, bool decoupled) {
  adam_step(p, g, m, v, static_cast<bf16*>(shadow), n, lr, b1, b2, eps, bc1, bc2, wd, decoupled ? 1 : 0, nullptr, S);
}

void sgd(float* p, const float* g, float* vel, void* shadow, long n, float lr, float momentum) {
  sgd_step(p, g, vel, static_cast<bf16*>(shadow), n, lr, momentum, nullptr, S);
}

}  // namespace gpu_ops
}  // namespace dcnn
