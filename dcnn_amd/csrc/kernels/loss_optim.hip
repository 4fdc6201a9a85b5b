// Fused loss (+gradient +accuracy) and flat-buffer optimizer kernels.
//
// Reference: K37/K38 (src/nn/loss_impl/cuda/loss_ops.cu:18-376: separate loss / grad kernels,
// cudaMallocAsync + two-stage reduce + D2H + stream sync per call), K41 accuracy
// (src/utils/accuracy_impl/cuda/accuracy.cu:15-115: cudaMalloc per call, default stream),
// K39/K40 Adam/SGD (one launch PER parameter tensor).
// Here: ONE kernel computes loss, gradient and the correct-count per batch (one wave per
// sample row, device-side scalars, no host sync, graph-capturable); optimizers run ONE
// launch over the flat fp32 master buffer and refresh the bf16 shadow copy used by the
// MFMA kernels in the same pass.
#include "common.h"
#include "api.h"

namespace dcnn {

enum LossType { kCE = 0, kSoftmaxCE = 1, kLogSoftmaxCE = 2, kMSE = 3, kMAE = 4, kHuber = 5 };

// One wave per sample row (4 rows per workgroup). Each row's loss and hit are written to a
// workspace; the workgroups then take a ticket and the last one sums the N row values in a
// fixed pairwise order (agent release / acquire around the ticket): the loss is bit-reproducible
// with no float atomics and no memset of the outputs.
template <typename T>
__device__ __forceinline__ void loss_row(const T* __restrict__ pred, const float* __restrict__ target,
                                         const int64_t* __restrict__ labels, T* __restrict__ grad, int row, int N,
                                         int C, int type, float param, float gscale, int lane, float* lsum_out,
                                         int* hit) {
  const T* p = pred + (long)row * C;
  auto tgt = [&](int c) -> float {
    if (labels) return (int64_t)c == labels[row] ? 1.f : 0.f;
    return target[(long)row * C + c];
  };
  // argmax of prediction and of target (first max wins)
  float pm = -INFINITY, tm = -INFINITY;
  int pi = 0x7fffffff, ti = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    const float v = to_f(p[c]), t = tgt(c);
    if (v > pm) { pm = v; pi = c; }
    if (t > tm) { tm = t; ti = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float pv = __shfl_xor(pm, o, 64), tv = __shfl_xor(tm, o, 64);
    const int pj = __shfl_xor(pi, o, 64), tj = __shfl_xor(ti, o, 64);
    if (pv > pm || (pv == pm && pj < pi)) { pm = pv; pi = pj; }
    if (tv > tm || (tv == tm && tj < ti)) { tm = tv; ti = tj; }
  }
  const float invN = 1.f / (float)N, invNC = 1.f / ((float)N * (float)C);
  // gradient scale: gscale = 1 / world under data parallelism (the gradient average folded into
  // the loss gradient, so no separate pass scales it)
  const float ginvN = invN * gscale, ginvNC = invNC * gscale;
  float lsum = 0.f;
  if (type == kSoftmaxCE || type == kLogSoftmaxCE) {
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += __expf(to_f(p[c]) - pm);
    s = wave_sum(s);
    const float lse = pm + __logf(s);
    // loss uses the first class whose target > 0.5 (loss_ops.cpp semantics)
    int hot = 0x7fffffff;
    for (int c = lane; c < C; c += 64) if (tgt(c) > 0.5f && c < hot) hot = c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hot = min(hot, __shfl_xor(hot, o, 64));
    if (hot < C) lsum = (lse - to_f(p[hot])) * invN;
    if (grad) {
      const float inv_s = 1.f / s;
      for (int c = lane; c < C; c += 64)
        grad[(long)row * C + c] = from_f<T>((__expf(to_f(p[c]) - pm) * inv_s - tgt(c)) * ginvN);
    }
  } else if (type == kCE) {
    int hot = 0x7fffffff;
    for (int c = lane; c < C; c += 64) if (tgt(c) > 0.5f && c < hot) hot = c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hot = min(hot, __shfl_xor(hot, o, 64));
    if (hot < C) {
      const float v = fminf(fmaxf(to_f(p[hot]), param), 1.f - param);
      lsum = -__logf(v) * invN;
    }
    if (grad)
      for (int c = lane; c < C; c += 64)
        grad[(long)row * C + c] = from_f<T>((to_f(p[c]) - tgt(c)) * ginvN);
  } else {
    for (int c = lane; c < C; c += 64) {
      const float d = to_f(p[c]) - tgt(c), ad = fabsf(d);
      float l, g;
      if (type == kMSE) { l = d * d; g = 2.f * d * ginvNC; }
      else if (type == kMAE) { l = ad; g = d > 0.f ? ginvNC : -ginvNC; }
      else {
        if (ad <= param) { l = 0.5f * d * d; g = d * ginvNC; }
        else { l = param * ad - 0.5f * param * param; g = (d > 0.f ? param : -param) * ginvNC; }
      }
      lsum += l;
      if (grad) grad[(long)row * C + c] = from_f<T>(g);
    }
    lsum = wave_sum(lsum) * invNC;
  }
  *lsum_out += lsum;
  *hit += (pi == ti) ? 1 : 0;
}

template <typename T>
__global__ void __launch_bounds__(256) loss_kernel(const T* __restrict__ pred, const float* __restrict__ target,
                                                   const int64_t* __restrict__ labels, T* __restrict__ grad,
                                                   float* __restrict__ loss_out, int* __restrict__ correct, int N,
                                                   int C, int type, float param, float gscale,
                                                   float* __restrict__ rowv, unsigned* __restrict__ ticket) {
  __shared__ float sl[256];
  __shared__ int sc[256];
  __shared__ int last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  float lsum = 0.f;
  int hits = 0;
  if (row < N) loss_row<T>(pred, target, labels, grad, row, N, C, type, param, gscale, lane, &lsum, &hits);
  if (gridDim.x == 1) {
    if (lane == 0) { sl[w] = lsum; sc[w] = hits; }
    __syncthreads();
    if (threadIdx.x == 0) {
      *loss_out = (sl[0] + sl[1]) + (sl[2] + sl[3]);
      if (correct) *correct = sc[0] + sc[1] + sc[2] + sc[3];
    }
    return;
  }
  if (lane == 0 && row < N) {
    rowv[row] = lsum;
    reinterpret_cast<int*>(rowv + N)[row] = hits;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  // last workgroup: thread t sums rows t, t + 256, ... in order, then a fixed LDS tree
  float l = 0.f;
  int h = 0;
  for (int r = threadIdx.x; r < N; r += 256) { l += rowv[r]; h += reinterpret_cast<const int*>(rowv + N)[r]; }
  sl[threadIdx.x] = l;
  sc[threadIdx.x] = h;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) { sl[threadIdx.x] += sl[threadIdx.x + o]; sc[threadIdx.x] += sc[threadIdx.x + o]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *loss_out = sl[0];
    if (correct) *correct = sc[0];
    *ticket = 0u;  // ready for the next loss on this stream
  }
}

int loss_workspace_floats(int N) { return 2 * N; }

void loss_fused(int dt, const void* pred, const float* target, const int64_t* labels, void* grad, float* loss_out,
                int* correct, int N, int C, int type, float param, float gscale, float* ws, unsigned* ticket,
                hipStream_t s) {
  const int blocks = (N + 3) / 4;
  if (blocks > 1 && (!ws || !ticket)) throw std::runtime_error("loss_fused: workspace required");
  if (dt == 0)
    hipLaunchKernelGGL(loss_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)pred, target, labels,
                       (float*)grad, loss_out, correct, N, C, type, param, gscale, ws, ticket);
  else
    hipLaunchKernelGGL(loss_kernel<bf16>, dim3(blocks), dim3(256), 0, s, (const bf16*)pred, target, labels,
                       (bf16*)grad, loss_out, correct, N, C, type, param, gscale, ws, ticket);
  DCNN_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------
// Adam / AdamW over the flat master buffer (+ bf16 shadow refresh). Semantics of
// src/nn/optimizers_impl/cuda/adam_kernels.cu:17-57: bias-corrected, epsilon after sqrt,
// L2 variant adds wd*lr*param to the update, AdamW decays the parameter first.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float adam1(float& p, float g, float& m, float& v, float lr, float b1, float b2, float eps,
                                       float bc1, float bc2, float wd, int decoupled) {
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  float upd = lr * (m / bc1) / (sqrtf(v / bc2) + eps);
  if (wd > 0.f) {
    if (decoupled) p -= wd * lr * p;
    else upd += wd * lr * p;
  }
  p -= upd;
  return p;
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, bf16* __restrict__ shadow, long n, float lr, float b1, float b2,
                            float eps, float bc1, float bc2, float wd, int decoupled,
                            const float* __restrict__ hyper) {
  // hyper (optional, device memory): {lr, bc1, bc2} so a captured hipGraph replays with the
  // current step's values without re-capture.
  if (hyper) { lr = hyper[0]; bc1 = hyper[1]; bc2 = hyper[2]; }
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i], gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i], vv = reinterpret_cast<float4*>(v)[i];
    adam1(pp.x, gg.x, mm.x, vv.x, lr, b1, b2, eps, bc1, bc2, wd, decoupled);
    adam1(pp.y, gg.y, mm.y, vv.y, lr, b1, b2, eps, bc1, bc2, wd, decoupled);
    adam1(pp.z, gg.z, mm.z, vv.z, lr, b1, b2, eps, bc1, bc2, wd, decoupled);
    adam1(pp.w, gg.w, mm.w, vv.w, lr, b1, b2, eps, bc1, bc2, wd, decoupled);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (shadow) {
      bf16x4 b = {(bf16)pp.x, (bf16)pp.y, (bf16)pp.z, (bf16)pp.w};
      reinterpret_cast<bf16x4*>(shadow)[i] = b;
    }
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam1(pp, g[i], mm, vv, lr, b1, b2, eps, bc1, bc2, wd, decoupled);
    p[i] = pp; m[i] = mm; v[i] = vv;
    if (shadow) shadow[i] = (bf16)pp;
  }
}

__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ vel,
                           bf16* __restrict__ shadow, long n, float lr, float mom, const float* __restrict__ hyper) {
  if (hyper) lr = hyper[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float pp = p[i];
    if (vel) {  // v = mu*v - lr*g ; p += v   (sgd_kernels.cu:27)
      const float vv = mom * vel[i] - lr * g[i];
      vel[i] = vv;
      pp += vv;
    } else {
      pp -= lr * g[i];
    }
    p[i] = pp;
    if (shadow) shadow[i] = (bf16)pp;
  }
}

void adam_step(float* p, const float* g, float* m, float* v, bf16* shadow, long n, float lr, float b1, float b2,
               float eps, float bc1, float bc2, float wd, int decoupled, const float* hyper, hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1, 256, 4096)), dim3(256), 0, s, p, g, m, v, shadow, n, lr, b1,
                     b2, eps, bc1, bc2, wd, decoupled, hyper);
  DCNN_LAUNCH_CHECK();
}

// Adam step scalars on the device: t += 1, bc1 = 1 - b1^t, bc2 = 1 - b2^t (hyper = {lr, bc1, bc2, t}).
// Captured in the step graph ahead of adam_kernel, so a replay needs no host upload at all.
__global__ void adam_scalars_kernel(float* hyper, float b1, float b2) {
  if (threadIdx.x == 0) {
    const float t = hyper[3] + 1.f;
    hyper[3] = t;
    hyper[1] = 1.f - powf(b1, t);
    hyper[2] = 1.f - powf(b2, t);
  }
}

void adam_scalars(float* hyper, float b1, float b2, hipStream_t s) {
  hipLaunchKernelGGL(adam_scalars_kernel, dim3(1), dim3(64), 0, s, hyper, b1, b2);
  DCNN_LAUNCH_CHECK();
}

void sgd_step(float* p, const float* g, float* vel, bf16* shadow, long n, float lr, float mom, const float* hyper,
              hipStream_t s) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, p, g, vel, shadow, n, lr, mom, hyper);
  DCNN_LAUNCH_CHECK();
}

}  // namespace dcnn
