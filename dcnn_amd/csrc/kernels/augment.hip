// Device-side batch assembly for the HBM-resident data plane (data/device_loader.py): gather the
// batch's samples from a dataset kept in device memory (uint8 or fp32, NCHW per sample), run the
// reference's augmentation chain on each image, write the model's fp32 NCHW input and the labels.
//
// The reference augments every sample on the host, op by op (include/data_augmentation/
// augmentation.hpp:114, random_crop.hpp:11, cutout.hpp:11, ...), and copies the batch to the GPU.
// At ~80k images/s per MI355X (~650k per node) an 8-core host cannot keep up; here the dataset
// (Tiny-ImageNet: 1.2 GB as uint8) lives in HBM and one launch per batch does the whole chain:
//
//  * one workgroup per sample; the image is staged in LDS as fp32 (C*H*W <= 16384 floats = 64 KB,
//    two buffers for the geometric ops), so every op of the chain is an LDS pass and the op order
//    is exactly the reference's (crop after flip, clamp after brightness, ...);
//  * randomness is counter-based (splitmix64 of (seed, sample index, op, draw)): no RNG state, the
//    same sample in the same epoch gets the same augmentation at any batch size or position, and
//    the host reference (tests/test_device_loader.py) reproduces every draw;
//  * the semantics of each op are the host backend's (csrc/native/data.cpp apply_one): flips,
//    brightness / contrast / gaussian noise with [0, 1] clamping, random crop as a shifted window
//    with zero fill, cutout, bilinear rotation about the centre with zero fill, normalisation.
#include "api.h"
#include "common.h"

namespace dcnn {

namespace {

__device__ __forceinline__ unsigned long long aug_mix(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// uniform in [0, 1) with 24 bits: draw `d` of op `k` for sample `s`
__device__ __forceinline__ float aug_uniform(unsigned long long seed, long s, int k, unsigned d) {
  const unsigned long long h =
      aug_mix(seed ^ aug_mix((unsigned long long)s * 0x100000001B3ull + ((unsigned long long)k << 32) + d));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float clamp01f(float v) { return fminf(fmaxf(v, 0.f), 1.f); }

}  // namespace

__global__ void __launch_bounds__(256) augment_batch_kernel(AugBatchArgs p) {
  extern __shared__ __attribute__((aligned(16))) float img[];
  const int b = blockIdx.x;
  const int C = p.C, H = p.H, W = p.W, HW = H * W, n = C * HW;
  float* cur = img;
  float* alt = img + n;
  const long s = p.idx[b];
  if (threadIdx.x == 0 && p.labels_out) p.labels_out[b] = p.labels[s];
  // ---- gather (uint8 / 255 or fp32)
  if (p.src_u8) {
    const unsigned char* src = reinterpret_cast<const unsigned char*>(p.src) + (size_t)s * n;
    for (int i = threadIdx.x; i < n; i += 256) cur[i] = (float)src[i] * (1.0f / 255.0f);
  } else {
    const float* src = reinterpret_cast<const float*>(p.src) + (size_t)s * n;
    for (int i = threadIdx.x; i < n; i += 256) cur[i] = src[i];
  }
  __syncthreads();
  for (int k = 0; k < p.nops; ++k) {
    const AugOpDev op = p.ops[k];
    if (op.kind == AUG_NORMALIZE) {  // always applied
      for (int i = threadIdx.x; i < n; i += 256) {
        const int c = i / HW;
        cur[i] = (cur[i] - op.a[c < 3 ? c : 0]) / op.a[3 + (c < 3 ? c : 0)];
      }
      __syncthreads();
      continue;
    }
    if (aug_uniform(p.seed, s, k, 0) >= op.p) continue;  // (uniform over the workgroup: no divergence)
    bool swap = false;
    switch (op.kind) {
      case AUG_HFLIP:
        for (int i = threadIdx.x; i < n; i += 256) {
          const int x = i % W;
          alt[i] = cur[i - x + (W - 1 - x)];
        }
        swap = true;
        break;
      case AUG_VFLIP:
        for (int i = threadIdx.x; i < n; i += 256) {
          const int c = i / HW, y = (i - c * HW) / W, x = i % W;
          alt[i] = cur[c * HW + (H - 1 - y) * W + x];
        }
        swap = true;
        break;
      case AUG_BRIGHTNESS: {
        const float f = -op.a[0] + 2.f * op.a[0] * aug_uniform(p.seed, s, k, 1);
        for (int i = threadIdx.x; i < n; i += 256) cur[i] = clamp01f(cur[i] + f);
        break;
      }
      case AUG_CONTRAST: {
        const float f = 1.f - op.a[0] + 2.f * op.a[0] * aug_uniform(p.seed, s, k, 1);
        for (int i = threadIdx.x; i < n; i += 256) cur[i] = clamp01f(cur[i] * f);
        break;
      }
      case AUG_NOISE:
        for (int i = threadIdx.x; i < n; i += 256) {
          // Box-Muller from two per-pixel draws
          const float u1 = fmaxf(aug_uniform(p.seed, s, k, 2 + 2u * (unsigned)i), 1e-7f);
          const float u2 = aug_uniform(p.seed, s, k, 3 + 2u * (unsigned)i);
          const float g = sqrtf(-2.f * logf(u1)) * cosf(6.28318530717958647f * u2);
          cur[i] = clamp01f(cur[i] + op.a[0] * g);
        }
        break;
      case AUG_CROP: {
        const int pad = (int)op.a[0], span = 2 * pad + 1;
        const int sx = min((int)(aug_uniform(p.seed, s, k, 1) * span), span - 1) - pad;
        const int sy = min((int)(aug_uniform(p.seed, s, k, 2) * span), span - 1) - pad;
        for (int i = threadIdx.x; i < n; i += 256) {
          const int c = i / HW, y = (i - c * HW) / W, x = i % W;
          const int yy = y + sy, xx = x + sx;
          alt[i] = (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0.f : cur[c * HW + yy * W + xx];
        }
        swap = true;
        break;
      }
      case AUG_CUTOUT: {
        const int sz = (int)op.a[0];
        const int nx = max(0, W - sz) + 1, ny = max(0, H - sz) + 1;
        const int x0 = min((int)(aug_uniform(p.seed, s, k, 1) * nx), nx - 1);
        const int y0 = min((int)(aug_uniform(p.seed, s, k, 2) * ny), ny - 1);
        for (int i = threadIdx.x; i < n; i += 256) {
          const int c = i / HW, y = (i - c * HW) / W, x = i % W;
          (void)c;
          if (x >= x0 && x < x0 + sz && y >= y0 && y < y0 + sz) cur[i] = 0.f;
        }
        break;
      }
      case AUG_ROTATION: {
        const float ang = (-op.a[0] + 2.f * op.a[0] * aug_uniform(p.seed, s, k, 1)) * 3.14159265358979f / 180.f;
        const float ca = cosf(ang), sa = sinf(ang), cx = W / 2.f, cy = H / 2.f;
        for (int i = threadIdx.x; i < n; i += 256) {
          const int c = i / HW, y = (i - c * HW) / W, x = i % W;
          const float fx0 = (x - cx) * ca - (y - cy) * sa + cx, fy0 = (x - cx) * sa + (y - cy) * ca + cy;
          const int x1 = (int)floorf(fx0), y1 = (int)floorf(fy0);
          const float fx = fx0 - x1, fy = fy0 - y1;
          const float* q = cur + c * HW;
          auto at = [&](int yy, int xx) { return (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0.f : q[yy * W + xx]; };
          alt[i] = (1 - fx) * (1 - fy) * at(y1, x1) + fx * (1 - fy) * at(y1, x1 + 1) + (1 - fx) * fy * at(y1 + 1, x1) +
                   fx * fy * at(y1 + 1, x1 + 1);
        }
        swap = true;
        break;
      }
      default:
        break;
    }
    __syncthreads();
    if (swap) {
      float* t = cur;
      cur = alt;
      alt = t;
    }
  }
  // ---- out: fp32 NCHW, 16-byte stores where the row allows
  float* out = p.out + (size_t)b * n;
  if ((n & 3) == 0) {
    for (int i = threadIdx.x * 4; i < n; i += 1024)
      *reinterpret_cast<float4*>(out + i) = *reinterpret_cast<const float4*>(cur + i);
  } else {
    for (int i = threadIdx.x; i < n; i += 256) out[i] = cur[i];
  }
}

bool augment_batch_supported(int C, int H, int W) { return C >= 1 && C * H * W <= kAugMaxFloats; }

void augment_batch(const AugBatchArgs& a, hipStream_t s) {
  if (!augment_batch_supported(a.C, a.H, a.W)) throw std::runtime_error("augment_batch: image too large for LDS");
  if (a.nops < 0 || a.nops > kAugMaxOps) throw std::runtime_error("augment_batch: too many ops");
  if (a.B <= 0) return;
  const int lds = 2 * a.C * a.H * a.W * 4;
  static bool attr = false;
  if (!attr) {
    DCNN_HIP_CHECK(hipFuncSetAttribute((const void*)augment_batch_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       2 * kAugMaxFloats * 4));
    attr = true;
  }
  hipLaunchKernelGGL(augment_batch_kernel, dim3(a.B), dim3(256), lds, s, a);
  DCNN_LAUNCH_CHECK();
}

}  // namespace dcnn
