// GPU backend of the C++ host API: the HIP/CDNA4 kernel library (csrc/kernels/*.hip) driven
// from C++ — bf16 NHWC activations, fp32 master parameters, bf16 operand shadows.
//
// Convolution routing (the same kernels and the same rules as the Python front end's main
// routes, ops/hip.py): 3x3 stride-1 'same' convs and their data gradients on the persistent halo
// kernel (hconv / hconv3, split-K on small grids), their weight gradients on the halo wgrad
// (hwgrad); 1x1 convs on the streaming kernel (g1s); everything else on the gathered MFMA GEMM
// (gemm_g2 forward, the stride-phase-grouped gemm_g2 data gradient, gemm_t2 weight gradient);
// odd channel counts on the generic implicit GEMM (gemm_nt / gemm_tn). BatchNorm runs on the
// deterministic slab statistics, the losses and the optimizers on the fused kernels. Work goes to
// the null stream in order; workspaces are grow-only device buffers reused across calls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
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
namespace {
// Caching device allocator: freed blocks go to a per-(device, size class) free list and are handed
// out again instead of hipFree / hipMalloc per tensor (hipFree waits for the whole device, so a
// step that releases its temporaries would otherwise serialise host and GPU at every op). All host
// API work is on the null stream, in order, so a block released by the host while a queued
// kernel still reads it is only reused by work queued after that kernel. Size classes are
// quarter-power-of-two steps (at most 25% slack); on an out-of-memory the cached blocks are
// released and the allocation retried.
// A graph's private blocks: everything allocated while it captured (gpu::Graph).
struct CapturePool {
  std::map<std::pair<int, size_t>, std::vector<void*>> free_blocks;
  std::vector<void*> owned;
};
struct BlockPool {
  std::mutex mu;
  std::map<std::pair<int, size_t>, std::vector<void*>> free_blocks;
  std::unordered_map<void*, std::pair<int, size_t>> owner;  // block -> (device, class bytes)
  std::unordered_map<void*, CapturePool*> graph_owned;      // block -> the graph it belongs to
  size_t cached = 0;
};
BlockPool& pool() {
  static BlockPool* p = new BlockPool;  // never destroyed: tensors may outlive static teardown
  return *p;
}
thread_local CapturePool* t_capture = nullptr;  // the pool of the graph this thread is capturing
size_t size_class(size_t n) {
  if (n <= 512) return 512;
  int lg = 63 - __builtin_clzll((unsigned long long)(n - 1));  // 2^lg < n <= 2^(lg + 1)
  const size_t step = (size_t)1 << (lg - 1);                   // quarter of 2^(lg + 1)
  return (n + step - 1) / step * step;
}
void release_cached(BlockPool& bp) {
  HOST_HIP_CHECK(hipDeviceSynchronize());
  for (auto& kv : bp.free_blocks)
    for (void* p : kv.second) {
      bp.owner.erase(p);
      (void)hipFree(p);
    }
  bp.free_blocks.clear();
  bp.cached = 0;
}
}  // namespace

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
void set_device(int dev) { HOST_HIP_CHECK(hipSetDevice(dev)); }
void* alloc(size_t nbytes) {
  int dev = 0;
  HOST_HIP_CHECK(hipGetDevice(&dev));
  const size_t cls = size_class(nbytes);
  BlockPool& bp = pool();
  std::lock_guard<std::mutex> g(bp.mu);
  CapturePool* cp = t_capture;
  if (cp) {  // a capturing graph first reuses its own freed blocks
    auto it = cp->free_blocks.find({dev, cls});
    if (it != cp->free_blocks.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      return p;
    }
  }
  void* p = nullptr;
  auto it = bp.free_blocks.find({dev, cls});
  if (it != bp.free_blocks.end() && !it->second.empty()) {
    p = it->second.back();
    it->second.pop_back();
    bp.cached -= cls;
  } else {
    const hipError_t e = hipMalloc(&p, cls);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      if (cp) throw std::runtime_error(std::string("gpu::alloc: hipMalloc failed while capturing a graph: ") +
                                       hipGetErrorString(e));
      release_cached(bp);
      HOST_HIP_CHECK(hipMalloc(&p, cls));
    }
    bp.owner[p] = {dev, cls};
  }
  if (cp) {
    bp.graph_owned[p] = cp;
    cp->owned.push_back(p);
  }
  return p;
}
void free(void* p) {
  if (p == nullptr) return;
  BlockPool& bp = pool();
  std::lock_guard<std::mutex> g(bp.mu);
  auto it = bp.owner.find(p);
  if (it == bp.owner.end()) {
    (void)hipFree(p);
    return;
  }
  auto gi = bp.graph_owned.find(p);
  if (gi != bp.graph_owned.end()) {  // a graph's block stays the graph's
    gi->second->free_blocks[it->second].push_back(p);
    return;
  }
  bp.free_blocks[it->second].push_back(p);
  bp.cached += it->second.second;
}
size_t cached_bytes() {
  BlockPool& bp = pool();
  std::lock_guard<std::mutex> g(bp.mu);
  return bp.cached;
}
void empty_cache() {
  BlockPool& bp = pool();
  std::lock_guard<std::mutex> g(bp.mu);
  release_cached(bp);
}
// ---- flows (streams) and events
namespace {
thread_local hipStream_t t_flow = nullptr;      // set_flow() override
thread_local hipStream_t t_default[64] = {};    // the thread's default flow per device
}  // namespace
Flow flow() {
  if (t_flow) return t_flow;
  int dev = 0;
  HOST_HIP_CHECK(hipGetDevice(&dev));
  if (!t_default[dev]) HOST_HIP_CHECK(hipStreamCreate(&t_default[dev]));  // (blocking: ordered with the null stream)
  return t_default[dev];
}
void set_flow(Flow f) { t_flow = static_cast<hipStream_t>(f); }
Flow flow_create() {
  hipStream_t s = nullptr;
  HOST_HIP_CHECK(hipStreamCreate(&s));
  return s;
}
void flow_destroy(Flow f) {
  if (f) (void)hipStreamDestroy(static_cast<hipStream_t>(f));
}
void flow_synchronize(Flow f) { HOST_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(f ? f : flow()))); }
Event event_create() {
  hipEvent_t e = nullptr;
  HOST_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return e;
}
void event_destroy(Event e) {
  if (e) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
}
void event_record(Event e, Flow f) {
  HOST_HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(e), static_cast<hipStream_t>(f ? f : flow())));
}
void flow_wait(Flow f, Event e) {
  HOST_HIP_CHECK(hipStreamWaitEvent(static_cast<hipStream_t>(f ? f : flow()), static_cast<hipEvent_t>(e), 0));
}
void event_synchronize(Event e) { HOST_HIP_CHECK(hipEventSynchronize(static_cast<hipEvent_t>(e))); }

void copy(void* dst, const void* src, size_t nbytes, int kind) {
  static const hipMemcpyKind k[] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice};
  hipStream_t s = static_cast<hipStream_t>(flow());
  HOST_HIP_CHECK(hipMemcpyAsync(dst, src, nbytes, k[kind], s));
  // host <-> device: the host buffer is usable when this returns (and a D2H sees the flow's work)
  if (kind != 2) {
    if (Graph::capturing()) throw std::runtime_error("gpu::copy: a host copy inside a graph capture");
    HOST_HIP_CHECK(hipStreamSynchronize(s));
  }
}
void copy2_d2d(void* d0, const void* s0, size_t n0, void* d1, const void* s1, size_t n1) {
  copy_pair(d0, s0, (long)n0, d1, s1, (long)n1, static_cast<hipStream_t>(flow()));
}
void zero(void* p, size_t nbytes) { HOST_HIP_CHECK(hipMemsetAsync(p, 0, nbytes, static_cast<hipStream_t>(flow()))); }
void synchronize() { HOST_HIP_CHECK(hipDeviceSynchronize()); }

// ---- graphs
bool Graph::capturing() { return t_capture != nullptr; }
void Graph::begin() {
  if (t_capture) throw std::runtime_error("gpu::Graph: nested capture");
  if (exec_) throw std::runtime_error("gpu::Graph: already captured");
  flow_ = flow();
  auto* cp = new CapturePool;
  pool_ = cp;
  // a previous eager step's work must not be captured into (or race with) the graph
  HOST_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(flow_)));
  // relaxed: a block the capture needs beyond the cached ones comes from hipMalloc, which the
  // stricter modes refuse while a capture is open (the allocation is not stream work)
  HOST_HIP_CHECK(hipStreamBeginCapture(static_cast<hipStream_t>(flow_), hipStreamCaptureModeRelaxed));
  t_capture = cp;
}
void Graph::end() {
  if (t_capture != pool_) throw std::runtime_error("gpu::Graph: end() without begin()");
  t_capture = nullptr;
  hipGraph_t g = nullptr;
  HOST_HIP_CHECK(hipStreamEndCapture(static_cast<hipStream_t>(flow_), &g));
  graph_ = g;
  hipGraphExec_t ex = nullptr;
  HOST_HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  exec_ = ex;
}
void Graph::replay() {
  if (!exec_) throw std::runtime_error("gpu::Graph: replay before capture");
  HOST_HIP_CHECK(hipGraphLaunch(static_cast<hipGraphExec_t>(exec_), static_cast<hipStream_t>(flow())));
}
Graph::~Graph() {
  if (t_capture == pool_ && pool_) {  // destroyed mid-capture (an exception): end the capture
    t_capture = nullptr;
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(static_cast<hipStream_t>(flow_), &g);
    if (g) (void)hipGraphDestroy(g);
    (void)hipGetLastError();
  }
  if (exec_ || graph_) (void)hipDeviceSynchronize();  // no replay in flight uses the blocks below
  if (exec_) (void)hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec_));
  if (graph_) (void)hipGraphDestroy(static_cast<hipGraph_t>(graph_));
  if (auto* cp = static_cast<CapturePool*>(pool_)) {
    BlockPool& bp = pool();
    std::lock_guard<std::mutex> g(bp.mu);
    // the graph's blocks return to the shared cache (blocks still held by live tensors come back
    // there when those are freed)
    std::unordered_map<void*, bool> is_free;
    for (auto& kv : cp->free_blocks)
      for (void* p : kv.second) is_free[p] = true;
    for (void* p : cp->owned) {
      bp.graph_owned.erase(p);
      if (is_free.count(p)) {
        auto o = bp.owner.find(p);
        bp.free_blocks[o->second].push_back(p);
        bp.cached += o->second.second;
      }
    }
    delete cp;
  }
}

// Inter-process buffers (pipeline transport "ipc"): a whole hipMalloc allocation (IPC exports the
// base of an allocation, so these never come from the caching pool) and its 64-byte handle.
void* ipc_alloc(size_t nbytes, void* handle_out) {
  static_assert(sizeof(hipIpcMemHandle_t) == kIpcHandleBytes, "IPC handle size");
  void* p = nullptr;
  HOST_HIP_CHECK(hipMalloc(&p, nbytes));
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(p);
    throw std::runtime_error("hipIpcGetMemHandle failed (the host must allow dmabuf IPC)");
  }
  std::memcpy(handle_out, &h, sizeof h);
  return p;
}
void ipc_free(void* p) {
  if (p != nullptr) (void)hipFree(p);
}
void* ipc_open(const void* handle) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof h);
  void* p = nullptr;
  HOST_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return p;
}
void ipc_close(void* p) {
  if (p != nullptr) (void)hipIpcCloseMemHandle(p);
}
Event ipc_event_create(void* handle_out) {
  static_assert(sizeof(hipIpcEventHandle_t) == kIpcHandleBytes, "IPC event handle size");
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventInterprocess) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  hipIpcEventHandle_t h;
  if (hipIpcGetEventHandle(&h, e) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipEventDestroy(e);
    return nullptr;
  }
  std::memcpy(handle_out, &h, sizeof h);
  return e;
}
Event ipc_event_open(const void* handle) {
  hipIpcEventHandle_t h;
  std::memcpy(&h, handle, sizeof h);
  hipEvent_t e = nullptr;
  HOST_HIP_CHECK(hipIpcOpenEventHandle(&e, h));
  return e;
}
bool stream_values_supported() {
  static const bool ok = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return v != 0;
  }();
  return ok;
}
void flow_write_u32(void* p, uint32_t v) {
  HOST_HIP_CHECK(hipStreamWriteValue32(static_cast<hipStream_t>(flow()), p, v, 0));
}
void flow_wait_u32_geq(void* p, uint32_t v) {
  HOST_HIP_CHECK(hipStreamWaitValue32(static_cast<hipStream_t>(flow()), p, v, hipStreamWaitValueGte, 0xffffffffu));
}
}  // namespace gpu

namespace gpu_ops {
namespace {
constexpr int kPlain = 0, kConvFwd = 1, kConvDgrad = 2;
constexpr int kBF16 = 1;
// the calling thread's current flow (gpu::flow()): every launch of the host API goes there
inline hipStream_t cur() { return static_cast<hipStream_t>(gpu::flow()); }

// grow-only workspace per purpose
enum Slot { W_T = 0, SLAB, BSLAB, STAT_SLAB, STAT_SUMS, STAT_PART, LOSS_WS, LOSS_OUT, TICKETS, HPART, HTICKETS, GN_AFF,
            FWD_STATS, BWD_STATS, FWD_STATS2, STAT_SLAB2, STAT_SUMS2, STAT_PART2, NSLOTS };
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
  hipLaunchKernelGGL(transpose16_kernel, grid, dim3(32, 8), 0, cur(), static_cast<const uint16_t*>(in),
                     static_cast<uint16_t*>(out), rows, cols);
  HOST_HIP_CHECK(hipGetLastError());
}

PoolGeom geom(const PoolShape& p) { return PoolGeom{p.N, p.H, p.W, p.C, p.OH, p.OW, p.KH, p.KW, p.SH, p.SW, p.PH, p.PW}; }

// ---- residual join / masks on bf16 (8 elements per thread when aligned)
__global__ void add_bf16_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, bf16* __restrict__ y, long n,
                                int relu) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = (float)a[i] + (float)b[i];
    if (relu) v = fmaxf(v, 0.f);
    y[i] = (bf16)v;
  }
}
__global__ void relu_mask_bf16_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ yv, bf16* __restrict__ dx,
                                      long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dx[i] = (float)yv[i] > 0.f ? dy[i] : (bf16)0.f;
}
int grid_of(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

// ---- op recording (DCNN_RECORD_OPS=<file>): one JSON line per conv call with its geometry, the
// epilogue options and the routing decision, so tests/test_gpu_cpp_geometry.py replays exactly the
// calls a production step makes (through the C ABI, capi.cpp) against fp32 PyTorch
FILE* rec_file() {
  static FILE* f = [] {
    const char* p = std::getenv("DCNN_RECORD_OPS");
    return p && *p ? std::fopen(p, "a") : nullptr;
  }();
  return f;
}
void rec(const char* op, const ConvShape& s, int route, std::initializer_list<std::pair<const char*, int>> flags) {
  FILE* f = rec_file();
  if (!f) return;
  std::fprintf(f, "{\"op\": \"%s\", \"shape\": [%d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %d, %d], \"route\": %d", op,
               s.N, s.C, s.H, s.W, s.Co, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, s.OH, s.OW, route);
  for (const auto& kv : flags) std::fprintf(f, ", \"%s\": %d", kv.first, kv.second);
  std::fprintf(f, "}\n");
  std::fflush(f);
}
// test-only fault injection (capi.cpp dcnn_c_set_fault): bit 0 drops the fused BatchNorm
// backward's ReLU mask operand in conv_dgrad (the geometry test must then fail)
int g_fault = [] {  // (DCNN_TEST_FAULT=<bits>: the same faults for a whole test process)
  const char* v = std::getenv("DCNN_TEST_FAULT");
  return v && *v ? std::atoi(v) : 0;
}();

// split-K workspace of a halo conv: (partials, zeroed ticket words) — the kernel leaves them zeroed
void hconv_workspace(HConvArgs& a) {
  a.splits = hconv_splits(a.NB, a.H, a.W, a.Cs, a.N, a.ntaps);
  a.part = nullptr;
  a.tickets = nullptr;
  if (a.splits <= 1) {
    a.splits = 1;
    return;
  }
  const long tiles = hconv_tiles(a.NB, a.H, a.W, a.Cs, a.N, a.ntaps);
  a.part = static_cast<float*>(scratch(HPART, (size_t)tiles * a.splits * hconv_tile_elems(a.NB, a.H, a.W, a.Cs, a.N,
                                                                                          a.ntaps) * 4));
  static size_t zeroed = 0;  // ticket words zeroed so far (grown only; left zeroed by every launch)
  const size_t need = (size_t)tiles * 64 * 4;
  a.tickets = static_cast<unsigned*>(scratch(HTICKETS, need));
  if (zeroed < need) {
    HOST_HIP_CHECK(hipMemsetAsync(a.tickets, 0, need, cur()));
    zeroed = need;
  }
}

// gathered-GEMM argument block (gemm2.hip) for a forward conv
G2Args g2_fwd_args(const void* x, const void* w, void* y, const float* bias, const ConvShape& s) {
  G2Args a{};
  a.A = static_cast<const bf16*>(x);
  a.B = static_cast<const bf16*>(w);
  a.C = static_cast<bf16*>(y);
  a.a_bytes = (unsigned)((long)s.N * s.H * s.W * s.C * 2);
  a.b_bytes = (unsigned)((long)s.Co * s.KH * s.KW * s.C * 2);
  a.M = s.N * s.OH * s.OW;
  a.N = s.Co;
  a.Cs = s.C;
  a.H = s.H; a.W = s.W; a.GH = s.OH; a.GW = s.OW; a.SY = s.SH; a.SX = s.SW;
  int t = 0;
  for (int ky = 0; ky < s.KH; ++ky)
    for (int kx = 0; kx < s.KW; ++kx, ++t) {
      const int dy = ky - s.PH, dx = kx - s.PW;
      a.tap_dy[t] = dy; a.tap_dx[t] = dx; a.tap_srcoff[t] = (dy * s.W + dx) * s.C; a.tap_b[t] = (ky * s.KW + kx) * s.C;
    }
  a.ntaps = t;
  a.ldb = s.KH * s.KW * s.C;
  a.ldc = s.Co;
  a.OH = s.OH; a.OW = s.OW; a.OSY = 1; a.OSX = 1; a.ORY = 0; a.ORX = 0;
  a.bias = bias;
  return a;
}

// SecondaryStats scope: forward conv statistics go to the second slab workspace
thread_local bool t_secondary = false;
inline Slot fwd_stats_slot() { return t_secondary ? FWD_STATS2 : FWD_STATS; }

ConvRouteGeom route_geom(const ConvShape& s, int g1s_mode) {
  return ConvRouteGeom{s.N, s.C, s.H, s.W, s.Co, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, s.OH, s.OW, g1s_mode};
}

// Weight-gradient split-K partials: while a backward is open (begin/end_deferred_reduce) every
// slab is a buffer of its own, queued, and summed into its gradient by ONE batched launch at the
// end of the backward (multi_splitk_reduce, kMaxRed slabs per launch) instead of one reduce per
// layer; outside it, the shared workspace and an immediate reduce. (Like the scratch workspaces,
// the queue is process state: one thread drives a process's GPU backend — the trainer, or a
// pipeline stage's event loop.)
struct PendingRed {
  Tensor slab;
  float* out;
  long n;
  int splits;
};
std::vector<PendingRed> g_pending;
bool g_defer = false;
size_t g_pending_bytes = 0;
void launch_pending();
// queued slab bytes that trigger a batched reduce before the backward ends (DCNN_REDUCE_FLUSH_MB;
// 0: only at the end): the earlier slabs are then read back while more of them are still in the
// 256 MB Infinity Cache, and their buffers return to the allocator sooner. Same box, two
// alternating reps per value (tools/gpu/pool2_check.sh), ResNet-18 b256 / ResNet-50 b32 img/s:
// end only 90.68k-90.84k / 8050-8066, 48 MB 90.38k-90.50k / 8076-8096, 96 MB 90.77k-90.89k /
// 8100-8115, 160 MB 89.35k-89.86k / 8079-8092, 256 MB 89.84k-89.87k / 8004-8030.
size_t reduce_flush_bytes() {
  static const size_t v = [] {
    const char* e = std::getenv("DCNN_REDUCE_FLUSH_MB");
    return (size_t)((e ? std::atof(e) : 96.0) * (1 << 20));
  }();
  return v;
}

float* wgrad_slab(Slot slot, size_t bytes, Tensor& hold) {
  if (!g_defer) return static_cast<float*>(scratch(slot, bytes));
  int dev = 0;
  HOST_HIP_CHECK(hipGetDevice(&dev));
  hold = Tensor::empty({(int64_t)((bytes + 3) / 4)}, DType::F32, Device::gpu(dev));
  return hold.ptr<float>();
}

void wgrad_reduce(const Tensor& hold, const Tensor& bhold, const float* slab, float* gw, long n, const float* bslab,
                  float* gb, long nb, int splits) {
  if (g_defer) {
    g_pending.push_back({hold, gw, n, splits});
    if (gb) g_pending.push_back({bhold, gb, nb, splits});
    g_pending_bytes += (size_t)n * splits * 4 + (gb ? (size_t)nb * splits * 4 : 0);
    if (reduce_flush_bytes() && g_pending_bytes >= reduce_flush_bytes()) launch_pending();
    return;
  }
  if (gb)
    splitk_reduce2(slab, gw, n, bslab, gb, nb, splits, 1, cur());
  else
    splitk_reduce(slab, gw, n, splits, 1, cur());
}
}  // namespace

void begin_deferred_reduce() { g_defer = true; }
void set_fault(int f) { g_fault = f; }
void flush_deferred_reduce() {
  const bool on = g_defer;
  end_deferred_reduce();
  g_defer = on;
}
void end_deferred_reduce() {
  launch_pending();
  g_defer = false;
}

namespace {
void launch_pending() {
  for (size_t b = 0; b < g_pending.size(); b += kMaxRed) {
    MultiRed t{};
    t.count = (int)std::min(g_pending.size() - b, (size_t)kMaxRed);
    for (int k = 0; k < t.count; ++k) {
      const PendingRed& e = g_pending[b + k];
      t.e[k].slab = e.slab.ptr<float>();
      t.e[k].out = e.out;
      t.e[k].n = e.n;
      t.e[k].splits = e.splits;
    }
    multi_splitk_reduce(t, cur());
  }
  g_pending.clear();  // (the slabs return to the caching allocator, reused only by later work)
  g_pending_bytes = 0;
}
}  // namespace

void input_to_nhwc(const float* x, void* y, int N, int C, int HW) { nchw_to_nhwc(kBF16, x, y, N, C, HW, cur()); }
void nhwc_to_nchw(const void* x, void* y, int N, int HW, int C) { transpose16(x, y, N, HW, C); }
void nchw_to_nhwc_bf16(const void* x, void* y, int N, int HW, int C) { transpose16(x, y, N, C, HW); }
void cast_bf16(const float* x, void* y, long n) { cast_f32_bf16(x, static_cast<bf16*>(y), n, cur()); }
void zero(void* p, long nbytes) { zero_bytes(p, nbytes, cur()); }

const float* conv_fwd(const void* x, const void* w, const float* bias, void* y, const ConvShape& s, int* stat_rows) {
  const long xb = (long)s.N * s.H * s.W * s.C * 2, wb = (long)s.Co * s.KH * s.KW * s.C * 2;
  const bool want = stat_rows != nullptr;
  if (want) *stat_rows = 0;
  auto slab_of = [&](int rows) {
    *stat_rows = rows;
    return static_cast<float*>(scratch(fwd_stats_slot(), (size_t)rows * 3 * s.Co * 4));
  };
  const int M = s.N * s.OH * s.OW;
  // the shared routing table (conv_route.cpp): the same kernels as the Python front end
  const int route = conv_fwd_route(route_geom(s, want ? 1 : 0));
  rec("fwd", s, route, {{"bias", bias != nullptr}, {"stats", want}});
  if (route == ROUTE_HALO && xb < (1l << 31)) {
    HConvArgs a{};
    a.A = static_cast<const bf16*>(x); a.B = static_cast<const bf16*>(w); a.C = static_cast<bf16*>(y);
    a.a_bytes = (unsigned)xb; a.b_bytes = (unsigned)wb;
    a.NB = s.N; a.H = s.H; a.W = s.W; a.Cs = s.C; a.N = s.Co; a.ldb = s.KH * s.KW * s.C; a.ntaps = s.KH * s.KW;
    for (int t = 0; t < a.ntaps; ++t) {
      a.tap_dy[t] = t / s.KW - s.PH; a.tap_dx[t] = t % s.KW - s.PW; a.tap_b[t] = t * s.C;
    }
    a.bias = bias;
    if (want) a.stats = slab_of(hconv_stat_rows(s.N, s.H, s.W, s.C, s.Co, a.ntaps, 0));
    hconv_workspace(a);
    hconv(a, cur());
    return a.stats;
  }
  if (route == ROUTE_G1S) {
    float* st = want ? slab_of(g1s_rows(M, s.Co, s.C, 1)) : nullptr;
    g1s(static_cast<const bf16*>(x), static_cast<const bf16*>(w), static_cast<bf16*>(y), M, s.Co, s.C, s.H, s.W, s.OH,
        s.OW, s.SH, bias, nullptr, st, 0, nullptr, 0, BnbArgs{}, want ? 1 : 0, cur());
    return st;
  }
  if (route != ROUTE_GENERIC && xb < (1l << 31) && wb < (1l << 31)) {
    G2Args a = g2_fwd_args(x, w, y, bias, s);
    if (want) a.stats = slab_of(gemm_g2_stat_rows(M, s.Co));
    gemm_g2(a, cur());
    return a.stats;
  }
  const int K = s.KH * s.KW * s.C;
  float* st = want ? slab_of(gemm_nt_stat_rows(M, s.Co)) : nullptr;
  NtArgs a{static_cast<const bf16*>(x), static_cast<const bf16*>(w), y, M, s.Co, K, 0, K, s.Co,
           kConvFwd, s.N, s.H, s.W, s.C, s.OH, s.OW, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, bias, nullptr, st, 0, 0};
  gemm_nt(a, cur());
  return st;
}

void weight_transpose(const void* w, void* wt, int Co, int T, int C) {
  conv_weight_transpose(kBF16, w, static_cast<bf16*>(wt), Co, T, C, cur());
}
void multi_weight_transpose(const int64_t* table, int n, long max_tiles) {
  dcnn::multi_weight_transpose(table, n, max_tiles, cur());
}

const float* conv_dgrad(const void* dy, const void* w, void* dx, const ConvShape& s, const void* residual,
                        bool w_transposed, const BnbOperands* bnb, int* bnb_rows) {
  const int T = s.KH * s.KW, K = T * s.Co;
  if (bnb_rows) *bnb_rows = 0;
  BnbArgs ba{};
  if (bnb) {
    ba.y = (g_fault & 1) ? nullptr : static_cast<const bf16*>(bnb->y);
    ba.x = static_cast<const bf16*>(bnb->x);
    ba.mean = bnb->mean;
    ba.istd = bnb->istd;
    // (the fault drops the mask either way)
    static const bool mask_x_env = [] {
      const char* v = std::getenv("DCNN_BNB_MASK_X");
      return !(v && v[0] == '0');
    }();
    if (bnb->mask_from_x && bnb->y && mask_x_env && !(g_fault & 1)) {
      ba.mask_x = 1;
      ba.gamma = bnb->gamma;
      ba.beta = bnb->beta;
    }
  }
  auto slab_of = [&](int rows) {
    *bnb_rows = rows;
    return static_cast<float*>(scratch(BWD_STATS, (size_t)rows * 2 * s.C * 4));
  };
  const bf16* wt = static_cast<const bf16*>(w);
  if (!w_transposed) {
    bf16* t = static_cast<bf16*>(scratch(W_T, (size_t)s.Co * T * s.C * 2));
    conv_weight_transpose(kBF16, w, t, s.Co, T, s.C, cur());  // [Co][T][C] -> [C][T][Co]
    wt = t;
  }
  const long dyb = (long)s.N * s.OH * s.OW * s.Co * 2, wtb = (long)s.C * T * s.Co * 2;
  // shared routing table (conv_route.cpp); g1s mode 2: the streaming dgrad with the BN epilogue
  const int route = conv_dgrad_route(route_geom(s, bnb ? 2 : 0));
  rec("dgrad", s, route, {{"residual", residual != nullptr}, {"w_t", w_transposed}, {"bnb", bnb != nullptr},
                         {"bnb_mask", bnb != nullptr && bnb->y != nullptr}});
  if (route == ROUTE_HALO && dyb < (1l << 31)) {
    // transposed conv of a stride-1 'same' conv: tap (ky, kx) reads dy at (PH - ky, PW - kx)
    HConvArgs a{};
    a.A = static_cast<const bf16*>(dy); a.B = wt; a.C = static_cast<bf16*>(dx);
    a.a_bytes = (unsigned)dyb; a.b_bytes = (unsigned)wtb;
    a.NB = s.N; a.H = s.OH; a.W = s.OW; a.Cs = s.Co; a.N = s.C; a.ldb = T * s.Co; a.ntaps = T;
    for (int t = 0; t < T; ++t) {
      const int ky = t / s.KW, kx = t % s.KW;
      a.tap_dy[t] = s.PH - ky; a.tap_dx[t] = s.PW - kx; a.tap_b[t] = t * s.Co;
    }
    a.residual = static_cast<const bf16*>(residual);
    if (bnb) {
      a.bnb = ba;
      a.stats = slab_of(hconv_stat_rows(s.N, s.OH, s.OW, s.Co, s.C, T, 0));
    }
    hconv_workspace(a);
    hconv(a, cur());
    return a.stats;
  }
  if (route == ROUTE_G1S) {  // streaming 1x1 data gradient
    const int M = s.N * s.H * s.W;
    float* st = bnb ? slab_of(g1s_rows(M, s.C, s.Co, 2)) : nullptr;
    g1s(static_cast<const bf16*>(dy), wt, static_cast<bf16*>(dx), M, s.C, s.Co, s.H, s.W, s.H, s.W, 1, nullptr,
        static_cast<const bf16*>(residual), st, 0, nullptr, 0, bnb ? ba : BnbArgs{}, bnb ? 2 : 0, cur());
    return st;
  }
  if (route != ROUTE_GENERIC && dyb < (1l << 31) && wtb < (1l << 31)) {
    // stride-phase decomposition: output phase (ry, rx) is a dense GEMM over the taps reaching
    // it; all phases are row classes of ONE grouped launch (phases no tap reaches write zeros)
    struct Cls { int ry, rx, GH, GW, t0, nt; };
    std::vector<Cls> cls;
    G2Args a{};
    int nt = 0;
    bool uniform = true;
    for (int ry = 0; ry < s.SH; ++ry)
      for (int rx = 0; rx < s.SW; ++rx) {
        const int GH = (s.H - ry + s.SH - 1) / s.SH, GW = (s.W - rx + s.SW - 1) / s.SW;
        if (GH <= 0 || GW <= 0) continue;
        Cls c{ry, rx, GH, GW, nt, 0};
        for (int ky = 0; ky < s.KH; ++ky) {
          if ((ry + s.PH - ky) % s.SH) continue;
          const int dyo = (ry + s.PH - ky) / s.SH;
          for (int kx = 0; kx < s.KW; ++kx) {
            if ((rx + s.PW - kx) % s.SW) continue;
            const int dxo = (rx + s.PW - kx) / s.SW;
            if (nt >= 64) throw std::runtime_error("conv_dgrad: more than 64 taps");
            a.tap_dy[nt] = dyo; a.tap_dx[nt] = dxo; a.tap_srcoff[nt] = (dyo * s.OW + dxo) * s.Co;
            a.tap_b[nt] = (ky * s.KW + kx) * s.Co;
            ++nt;
            ++c.nt;
          }
        }
        if (!cls.empty() && (c.GH != cls[0].GH || c.GW != cls[0].GW)) uniform = false;
        cls.push_back(c);
      }
    const long rows = (long)s.N * (cls.empty() ? 0 : cls[0].GH * cls[0].GW);
    if (uniform && !cls.empty() && cls.size() <= 4 && (cls.size() == 1 || rows % 128 == 0)) {
      a.A = static_cast<const bf16*>(dy); a.B = wt; a.C = static_cast<bf16*>(dx);
      a.a_bytes = (unsigned)dyb; a.b_bytes = (unsigned)wtb;
      a.M = (int)(rows * (long)cls.size()); a.N = s.C; a.Cs = s.Co;
      a.H = s.OH; a.W = s.OW; a.GH = cls[0].GH; a.GW = cls[0].GW; a.SY = 1; a.SX = 1;
      a.ntaps = nt; a.ldb = T * s.Co; a.ldc = s.C;
      a.OH = s.H; a.OW = s.W; a.OSY = s.SH; a.OSX = s.SW; a.ORY = cls[0].ry; a.ORX = cls[0].rx;
      a.residual = static_cast<const bf16*>(residual);
      if (cls.size() > 1) {
        a.ncls = (int)cls.size();
        a.cls_rows = (int)rows;
        for (size_t k = 0; k < cls.size(); ++k) {
          a.cls_t0[k] = cls[k].t0; a.cls_nt[k] = cls[k].nt; a.cls_ory[k] = cls[k].ry; a.cls_orx[k] = cls[k].rx;
        }
      }
      // the producing BatchNorm's mask + backward statistics in the epilogue when every stride
      // phase has taps (a zero-tap phase's rows are written by the fill path, not the MMA epilogue)
      bool all_taps = true;
      for (const Cls& c : cls) all_taps = all_taps && c.nt > 0;
      if (bnb && all_taps) {
        a.bnb = ba;
        a.stats = slab_of(gemm_g2_stat_rows(a.M, s.C));
      }
      gemm_g2(a, cur());
      return a.stats;
    }
  }
  NtArgs a{static_cast<const bf16*>(dy), wt, dx, s.N * s.H * s.W, s.C, K, 0, K, s.C, kConvDgrad, s.N, s.OH, s.OW,
           s.Co, s.H, s.W, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, nullptr, static_cast<const bf16*>(residual), nullptr,
           0, 0};
  gemm_nt(a, cur());
  return nullptr;
}

void conv_wgrad(const void* dy, const void* x, float* gw, float* gb, const ConvShape& s) {
  const int Ng = s.KH * s.KW * s.C, P = s.N * s.OH * s.OW;
  const long dyb = (long)P * s.Co * 2, xb = (long)s.N * s.H * s.W * s.C * 2;
  const int route = conv_wgrad_route(route_geom(s, -1));  // shared routing table (conv_route.cpp)
  rec("wgrad", s, route, {{"bias", gb != nullptr}, {"deferred", g_defer}});
  if (route == ROUTE_HALO) {
    const int splits = hwgrad_splits(s.N, s.H, s.W, s.C, s.Co);
    Tensor hold, bhold;
    float* slab = wgrad_slab(SLAB, (size_t)splits * s.Co * Ng * 4, hold);
    float* bslab = gb ? wgrad_slab(BSLAB, (size_t)splits * s.Co * 4, bhold) : nullptr;
    HWArgs a{};
    a.dY = static_cast<const bf16*>(dy); a.X = static_cast<const bf16*>(x); a.slab = slab; a.bias_slab = bslab;
    a.dy_bytes = (unsigned)dyb; a.x_bytes = (unsigned)xb;
    a.NB = s.N; a.H = s.H; a.W = s.W; a.Cs = s.C; a.Co = s.Co; a.ntaps = 9;
    for (int t = 0; t < 9; ++t) { a.tap_dy[t] = t / 3 - 1; a.tap_dx[t] = t % 3 - 1; }
    hwgrad(a, splits, cur());
    wgrad_reduce(hold, bhold, slab, gw, (long)s.Co * Ng, bslab, gb, s.Co, splits);
    return;
  }
  if (route == ROUTE_HALO_S2) {  // 3x3 stride 2: the stride-2 halo kernel (dY grid OH x OW)
    const int splits = hwgrad_s2_splits(s.N, s.OH, s.OW, s.C, s.Co);
    Tensor hold, bhold;
    float* slab = wgrad_slab(SLAB, (size_t)splits * s.Co * Ng * 4, hold);
    float* bslab = gb ? wgrad_slab(BSLAB, (size_t)splits * s.Co * 4, bhold) : nullptr;
    HWArgs a{};
    a.dY = static_cast<const bf16*>(dy); a.X = static_cast<const bf16*>(x); a.slab = slab; a.bias_slab = bslab;
    a.dy_bytes = (unsigned)dyb; a.x_bytes = (unsigned)xb;
    a.NB = s.N; a.H = s.OH; a.W = s.OW; a.Cs = s.C; a.Co = s.Co; a.ntaps = 9;
    hwgrad_s2(a, splits, cur());
    wgrad_reduce(hold, bhold, slab, gw, (long)s.Co * Ng, bslab, gb, s.Co, splits);
    return;
  }
  if ((route == ROUTE_GEMM_G2 || route == ROUTE_HALO_S2) && dyb < (1l << 31) && xb < (1l << 31) && P < (1 << 24)) {
    const int splits = gemm_t2_splits(s.Co, Ng, P);
    Tensor hold, bhold;
    float* slab = wgrad_slab(SLAB, (size_t)splits * s.Co * Ng * 4, hold);
    float* bslab = gb ? wgrad_slab(BSLAB, (size_t)splits * s.Co * 4, bhold) : nullptr;
    T2Args a{};
    a.dY = static_cast<const bf16*>(dy); a.X = static_cast<const bf16*>(x); a.slab = slab; a.bias_slab = bslab;
    a.a_bytes = (unsigned)dyb; a.b_bytes = (unsigned)xb;
    a.M = s.Co; a.N = Ng; a.P = P; a.ldy = s.Co; a.Cs = s.C; a.H = s.H; a.W = s.W; a.GH = s.OH; a.GW = s.OW;
    a.SY = s.SH; a.SX = s.SW;
    int t = 0;
    for (int ky = 0; ky < s.KH; ++ky)
      for (int kx = 0; kx < s.KW; ++kx, ++t) { a.tap_dy[t] = ky - s.PH; a.tap_dx[t] = kx - s.PW; }
    a.ntaps = t;
    gemm_t2(a, splits, cur());
    wgrad_reduce(hold, bhold, slab, gw, (long)s.Co * Ng, bslab, gb, s.Co, splits);
    return;
  }
  const int splits = gemm_tn_splits(s.Co, Ng, P);
  Tensor hold, bhold;
  float* slab = wgrad_slab(SLAB, (size_t)splits * s.Co * Ng * 4, hold);
  float* bslab = gb ? wgrad_slab(BSLAB, (size_t)splits * s.Co * 4, bhold) : nullptr;
  TnArgs a{static_cast<const bf16*>(dy), static_cast<const bf16*>(x), slab, bslab, s.Co, Ng, P, kConvFwd, s.N, s.H,
           s.W, s.C, s.OH, s.OW, s.KH, s.KW, s.SH, s.SW, s.PH, s.PW, 0, 0};
  gemm_tn(a, splits, cur());
  wgrad_reduce(hold, bhold, slab, gw, (long)s.Co * Ng, bslab, gb, s.Co, splits);
}

bool stem_ok(const ConvShape& s) {
  return s.KH == 3 && s.KW == 3 && s.SH == 1 && s.SW == 1 && s.PH == 1 && s.PW == 1 &&
         stem_supported(s.N, s.C, s.H, s.W, s.Co);
}

// weights / gradients: physical [Co][KH][KW][Ci] -> element strides of the logical (Co, Ci, ky, kx)
const float* stem_fwd(const float* x, const void* w, const float* bias, void* y, const ConvShape& s, int* stat_rows) {
  rec("stem_fwd", s, -1, {{"bias", bias != nullptr}, {"stats", stat_rows != nullptr}});
  StemArgs a{};
  a.x = x; a.w = w; a.w_bf16 = 1;
  a.ws[0] = 9l * s.C; a.ws[1] = 1; a.ws[2] = 3l * s.C; a.ws[3] = s.C;
  a.bias = bias; a.y = static_cast<bf16*>(y);
  a.N = s.N; a.Ci = s.C; a.H = s.H; a.W = s.W; a.Co = s.Co;
  if (stat_rows) {
    *stat_rows = stem_tiles_host(s.N, s.H, s.W);
    a.slab = static_cast<float*>(scratch(fwd_stats_slot(), (size_t)*stat_rows * 3 * s.Co * 4));
  }
  dcnn::stem_fwd(a, cur());
  return a.slab;
}

static void stem_wgrad_impl(const void* dy, const float* x, float* gw, float* gb, const ConvShape& s,
                            const StemBn* bn);

void stem_wgrad(const void* dy, const float* x, float* gw, float* gb, const ConvShape& s) {
  stem_wgrad_impl(dy, x, gw, gb, s, nullptr);
}

static std::pair<const float*, int> reduce_stats(int mode, const float* slab, int rows, int C);

void stem_wgrad_bn(const void* dy, const float* x, float* gw, float* gb, const ConvShape& s, const StemBn& bn) {
  stem_wgrad_impl(dy, x, gw, gb, s, &bn);
}

static void stem_wgrad_impl(const void* dy, const float* x, float* gw, float* gb, const ConvShape& s,
                            const StemBn* bn) {
  rec("stem_wgrad", s, -1, {{"bias", gb != nullptr}, {"deferred", g_defer}, {"bn", bn != nullptr}});
  std::pair<const float*, int> st{nullptr, 0};
  if (bn) st = reduce_stats(1, bn->slab, bn->rows, s.Co);  // (before the slab scratch below is taken)
  const int blocks = bn ? stem_wgrad_blocks_bnt(s.N, s.H, s.W) : stem_wgrad_blocks(s.N, s.H, s.W);
  const long n = 9l * s.C * s.Co;
  Tensor hold, bhold;
  float* slab = wgrad_slab(SLAB, (size_t)blocks * n * 4, hold);
  float* bslab = gb ? wgrad_slab(BSLAB, (size_t)blocks * s.Co * 4, bhold) : nullptr;
  StemArgs a{};
  a.x = x; a.dy = static_cast<const bf16*>(dy); a.slab = slab; a.bias_slab = bslab;
  a.gs[0] = 9l * s.C; a.gs[1] = 1; a.gs[2] = 3l * s.C; a.gs[3] = s.C;
  a.n_slab = n;
  a.N = s.N; a.Ci = s.C; a.H = s.H; a.W = s.W; a.Co = s.Co;
  if (bn) {
    a.bn_x = static_cast<const bf16*>(bn->x); a.bn_mean = bn->mean; a.bn_istd = bn->istd; a.bn_gamma = bn->gamma;
    a.bn_sums = st.first; a.bn_parts = st.second; a.bn_count = (float)((long)s.N * s.H * s.W);
    a.bn_dgamma = bn->dgamma; a.bn_dbeta = bn->dbeta; a.bn_eval = bn->train ? 0 : 1;
  }
  dcnn::stem_wgrad(a, blocks, cur());
  wgrad_reduce(hold, bhold, slab, gw, n, bslab, gb, s.Co, blocks);
}

void dense_fwd(const void* x, const void* w, const float* bias, void* y, int N, int In, int Out) {
  NtArgs a{static_cast<const bf16*>(x), static_cast<const bf16*>(w), y, N, Out, In, In, In, Out, kPlain, 0, 0, 0, 0,
           1, 1, 1, 1, 1, 1, 0, 0, bias, nullptr, nullptr, 0, 0};
  gemm_nt(a, cur());
}

void dense_dgrad(const void* dy, const void* w, void* dx, int N, int In, int Out) {
  bf16* wt = static_cast<bf16*>(scratch(W_T, (size_t)In * Out * 2));
  conv_weight_transpose(kBF16, w, wt, Out, 1, In, cur());  // [Out][In] -> [In][Out]
  NtArgs a{static_cast<const bf16*>(dy), wt, dx, N, In, Out, Out, Out, In, kPlain, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 0, 0,
           nullptr, nullptr, nullptr, 0, 0};
  gemm_nt(a, cur());
}

void dense_wgrad(const void* dy, const void* x, float* gw, float* gb, int N, int In, int Out) {
  const int splits = gemm_tn_splits(Out, In, N);
  Tensor hold, bhold;
  float* slab = wgrad_slab(SLAB, (size_t)splits * Out * In * 4, hold);
  float* bslab = gb ? wgrad_slab(BSLAB, (size_t)splits * Out * 4, bhold) : nullptr;
  TnArgs a{static_cast<const bf16*>(dy), static_cast<const bf16*>(x), slab, bslab, Out, In, N, kPlain, 0, 0, 0, 0, 1,
           1, 1, 1, 1, 1, 0, 0, In, 0};
  gemm_tn(a, splits, cur());
  wgrad_reduce(hold, bhold, slab, gw, (long)Out * In, bslab, gb, Out, splits);
}

// deterministic slab statistics: (pointer, parts) for bn_apply / bn_bwd_apply
static std::pair<const float*, int> reduce_stats(int mode, const float* slab, int rows, int C) {
  const int parts = bn_stat_parts(rows);
  float* sums = static_cast<float*>(scratch(STAT_SUMS, (size_t)2 * C * 4));
  float* part = parts > 1 ? static_cast<float*>(scratch(STAT_PART, (size_t)parts * 3 * C * 4)) : nullptr;
  bn_stat_reduce(mode, slab, rows, C, sums, part, nullptr, cur());
  return {parts > 1 ? part : sums, parts};
}

void bn_fwd(const void* x, void* y, long R, int C, const float* g, const float* b, float eps, bool train,
            float* rmean, float* rvar, float momentum, float* smean, float* sistd, bool relu, const void* residual) {
  if (!train) {
    bn_apply(kBF16, x, y, R, C, nullptr, 1, (float)R, g, b, eps, residual, relu ? 1 : 0, smean, sistd, rmean, rvar,
             momentum, 1, cur());
    return;
  }
  const int rows = bn_partial_rows(R, C);
  float* slab = static_cast<float*>(scratch(STAT_SLAB, (size_t)rows * 3 * C * 4));
  bn_partial(kBF16, x, nullptr, nullptr, nullptr, nullptr, nullptr, R, C, slab, 0, nullptr, cur());
  const auto st = reduce_stats(0, slab, rows, C);
  bn_apply(kBF16, x, y, R, C, st.first, st.second, (float)R, g, b, eps, residual, relu ? 1 : 0, smean, sistd, rmean,
           rvar, momentum, 0, cur());
}

void bn_fwd_slab(const void* x, void* y, long R, int C, const float* slab, int rows, const float* g, const float* b,
                 float eps, float* rmean, float* rvar, float momentum, float* smean, float* sistd, bool relu,
                 const void* residual) {
  const auto st = reduce_stats(0, slab, rows, C);
  bn_apply(kBF16, x, y, R, C, st.first, st.second, (float)R, g, b, eps, residual, relu ? 1 : 0, smean, sistd, rmean,
           rvar, momentum, 0, cur());
}

void bn_bwd_slab(const void* dy, const void* x, void* dx, long R, int C, const float* mean, const float* istd,
                 const float* g, float* dg, float* db, bool train, const float* slab, int rows) {
  const auto st = reduce_stats(1, slab, rows, C);
  bn_bwd_apply(kBF16, dy, nullptr, x, dx, R, C, mean, istd, g, st.first, st.second, (float)R, dg, db, train ? 0 : 1, cur());
}

void bn_bwd(const void* dy, const void* x, void* dx, long R, int C, const float* mean, const float* istd,
            const float* g, float* dg, float* db, bool train, const void* yout, void* dy_out) {
  const int rows = bn_partial_rows(R, C);
  float* slab = static_cast<float*>(scratch(STAT_SLAB, (size_t)rows * 2 * C * 4));
  bn_partial(kBF16, x, dy, yout, dy_out, mean, istd, R, C, slab, 1, nullptr, cur());
  const auto st = reduce_stats(1, slab, rows, C);
  bn_bwd_apply(kBF16, dy, yout, x, dx, R, C, mean, istd, g, st.first, st.second, (float)R, dg, db, train ? 0 : 1, cur());
}

SecondaryStats::SecondaryStats() { t_secondary = true; }
SecondaryStats::~SecondaryStats() { t_secondary = false; }

BnRaw bn_stats_raw(const void* x, long R, int C, const float* slab, int rows) {
  if (slab != nullptr && rows > 0) return BnRaw{slab, rows};
  const int n = bn_partial_rows(R, C);
  float* s = static_cast<float*>(scratch(STAT_SLAB2, (size_t)n * 3 * C * 4));
  bn_partial(kBF16, x, nullptr, nullptr, nullptr, nullptr, nullptr, R, C, s, 0, nullptr, cur());
  return BnRaw{s, n};
}

bool bn_dual_ok(long R, int C) { return bn_apply_dual_supported(R, C); }

// both statistics reduces of a pair in one launch: (pointer, parts) per side
static void reduce_pair(int mode, const float* slab_a, int rows_a, const float* slab_b, int rows_b, int C,
                        std::pair<const float*, int>& a, std::pair<const float*, int>& b) {
  const int pa = bn_stat_parts(rows_a), pb = bn_stat_parts(rows_b);
  float* sa = static_cast<float*>(scratch(STAT_SUMS, (size_t)2 * C * 4));
  float* sb = static_cast<float*>(scratch(STAT_SUMS2, (size_t)2 * C * 4));
  float* qa = pa > 1 ? static_cast<float*>(scratch(STAT_PART, (size_t)pa * 3 * C * 4)) : nullptr;
  float* qb = pb > 1 ? static_cast<float*>(scratch(STAT_PART2, (size_t)pb * 3 * C * 4)) : nullptr;
  bn_stat_reduce2(mode, slab_a, rows_a, sa, qa, slab_b, rows_b, sb, qb, C, cur());
  a = {pa > 1 ? qa : sa, pa};
  b = {pb > 1 ? qb : sb, pb};
}

void bn_fwd_dual(const BnFwdSide& a, const BnFwdSide& b, void* y, long R, int C, bool relu, bool train) {
  std::pair<const float*, int> sa{nullptr, 1}, sb{nullptr, 1};
  if (train) reduce_pair(0, a.raw.slab, a.raw.rows, b.raw.slab, b.raw.rows, C, sa, sb);
  auto side = [&](const BnFwdSide& s, const std::pair<const float*, int>& st) {
    return BnSide{s.x,     st.first, st.second, (float)R, s.g,        s.b,    s.eps,
                  s.smean, s.sistd,  s.rmean,   s.rvar,   s.momentum, train ? 0 : 1};
  };
  if (!bn_apply_dual(side(a, sa), side(b, sb), y, R, C, relu ? 1 : 0, cur()))
    throw std::runtime_error("bn_fwd_dual: unsupported shape");
}

void bn_bwd_dual(const void* dy, const BnBwdSides& a, const float* slab_a, int rows_a, const BnBwdSides& b, long R,
                 int C) {
  const int rows_b = bn_partial_rows(R, C);
  float* slab_b = static_cast<float*>(scratch(STAT_SLAB, (size_t)rows_b * 2 * C * 4));
  bn_partial(kBF16, b.x, dy, nullptr, nullptr, b.mean, b.istd, R, C, slab_b, 1, nullptr, cur());
  std::pair<const float*, int> sa, sb;
  reduce_pair(1, slab_a, rows_a, slab_b, rows_b, C, sa, sb);
  auto side = [&](const BnBwdSides& s, const std::pair<const float*, int>& st) {
    return BnBwdSide{s.x, s.dx, s.mean, s.istd, s.g, st.first, st.second, (float)R, s.dg, s.db};
  };
  if (!bn_bwd_apply_dual(dy, side(a, sa), side(b, sb), R, C, cur()))
    throw std::runtime_error("bn_bwd_dual: unsupported shape");
}

bool bn_relu_maxpool_ok(const PoolShape& p) {
  const PoolGeom g = geom(p);
  return dcnn::bn_relu_maxpool_supported(g) && dcnn::maxpool_bwd_bnb_supported(g);
}

void bn_relu_maxpool(const void* x, void* y, uint8_t* idx, const PoolShape& p, const float* slab, int rows,
                     const float* g, const float* b, float eps, float* rmean, float* rvar, float momentum,
                     float* smean, float* sistd) {
  const long R = (long)p.N * p.H * p.W;
  if (slab == nullptr || rows <= 0) {
    rows = bn_partial_rows(R, p.C);
    float* s = static_cast<float*>(scratch(STAT_SLAB, (size_t)rows * 3 * p.C * 4));
    bn_partial(kBF16, x, nullptr, nullptr, nullptr, nullptr, nullptr, R, p.C, s, 0, nullptr, cur());
    slab = s;
  }
  const auto st = reduce_stats(0, slab, rows, p.C);
  dcnn::bn_relu_maxpool(static_cast<const bf16*>(x), static_cast<bf16*>(y), idx, geom(p), st.first, st.second,
                        (float)R, g, b, eps, smean, sistd, rmean, rvar, momentum, cur());
}

const float* maxpool_bwd_bnb(const void* dy, const uint8_t* idx, const void* ypool, const void* x, const float* mean,
                             const float* istd, void* dx, const PoolShape& p, int* rows) {
  const PoolGeom g = geom(p);
  *rows = maxpool_bwd_bnb_rows(g);
  float* slab = static_cast<float*>(scratch(BWD_STATS, (size_t)*rows * 2 * p.C * 4));
  dcnn::maxpool_bwd_bnb(static_cast<const bf16*>(dy), idx, static_cast<const bf16*>(ypool),
                        static_cast<const bf16*>(x), mean, istd, static_cast<bf16*>(dx), g, slab, nullptr, cur());
  return slab;
}

void maxpool_fwd(const void* x, void* y, uint8_t* idx, const PoolShape& p) {
  if (p.KH * p.KW > 256) throw std::invalid_argument("maxpool: window larger than 256 taps");
  dcnn::maxpool_fwd(kBF16, x, y, idx, geom(p), cur());
}
void maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, const PoolShape& p) {
  dcnn::maxpool_bwd(kBF16, dy, idx, dx, geom(p), cur());
}
void avgpool_fwd(const void* x, void* y, const PoolShape& p) { dcnn::avgpool_fwd(kBF16, x, y, geom(p), cur()); }
void avgpool_bwd(const void* dy, void* dx, const PoolShape& p) { dcnn::avgpool_bwd(kBF16, dy, dx, geom(p), cur()); }

void act_fwd(int kind, const void* x, void* y, long n, float alpha) { dcnn::act_fwd(kBF16, x, y, n, kind, alpha, cur()); }
void act_bwd(int kind, const void* x, const void* dy, void* dx, long n, float alpha) {
  dcnn::act_bwd(kBF16, x, dy, dx, n, kind, alpha, cur());
}

// the fused loss kernels leave {loss (fp32), -, correct (int32)} in the LOSS_OUT slot; eager calls
// read it back, inside a graph capture the value stays on the device (loss_device())
double read_loss(const char* out, long* correct) {
  if (gpu::Graph::capturing()) {
    if (correct) *correct = -1;
    return std::nan("");
  }
  char host[16];
  hipStream_t s = cur();
  HOST_HIP_CHECK(hipMemcpyAsync(host, out, 16, hipMemcpyDeviceToHost, s));
  HOST_HIP_CHECK(hipStreamSynchronize(s));
  float l;
  int c;
  std::memcpy(&l, host, 4);
  std::memcpy(&c, host + 8, 4);
  if (correct) *correct = c;
  return l;
}

double softmax_ce(const void* pred, const int64_t* labels, void* grad, int N, int C, long* correct) {
  float* ws = N > 4 ? static_cast<float*>(scratch(LOSS_WS, (size_t)loss_workspace_floats(N) * 4)) : nullptr;
  static unsigned* tickets = nullptr;  // zeroed once; every launch leaves them zeroed
  if (N > 4 && !tickets) {
    tickets = static_cast<unsigned*>(scratch(TICKETS, 64 * 4));
    HOST_HIP_CHECK(hipMemsetAsync(tickets, 0, 64 * 4, cur()));
  }
  char* out = static_cast<char*>(scratch(LOSS_OUT, 16));
  float* loss = reinterpret_cast<float*>(out);
  int* corr = reinterpret_cast<int*>(out + 8);
  loss_fused(kBF16, pred, nullptr, labels, grad, loss, corr, N, C, 1, 1e-15f, 1.0f, ws, N > 4 ? tickets : nullptr,
             cur());
  return read_loss(out, correct);
}

double loss(int kind, const void* pred, const float* target, const int64_t* labels, void* grad, int N, int C,
            float param, long* correct, float grad_scale) {
  loss_launch(kind, pred, target, labels, grad, N, C, param, grad_scale);
  return read_last_loss(correct);
}

double read_last_loss(long* correct) { return read_loss(static_cast<const char*>(scratch(LOSS_OUT, 16)), correct); }

void loss_launch(int kind, const void* pred, const float* target, const int64_t* labels, void* grad, int N, int C,
                 float param, float grad_scale) {
  float* ws = N > 4 ? static_cast<float*>(scratch(LOSS_WS, (size_t)loss_workspace_floats(N) * 4)) : nullptr;
  static unsigned* tickets = nullptr;
  if (N > 4 && !tickets) {
    tickets = static_cast<unsigned*>(scratch(TICKETS, 64 * 4));
    HOST_HIP_CHECK(hipMemsetAsync(tickets, 0, 64 * 4, cur()));
  }
  char* out = static_cast<char*>(scratch(LOSS_OUT, 16));
  loss_fused(kBF16, pred, target, labels, grad, reinterpret_cast<float*>(out), reinterpret_cast<int*>(out + 8), N, C,
             kind, param, grad_scale, ws, N > 4 ? tickets : nullptr, cur());
}

void groupnorm_fwd(const void* x, void* y, int N, int HW, int C, int G, const float* g, const float* b, float eps,
                   float* smean, float* sistd) {
  gn_fwd(kBF16, x, y, N, HW, C, G, g, b, eps, smean, sistd, cur());
}

void groupnorm_bwd(const void* dy, const void* x, void* dx, int N, int HW, int C, int G, const float* g,
                   const float* mean, const float* istd, float* dg, float* db) {
  float* aff = static_cast<float*>(scratch(GN_AFF, (size_t)N * 2 * C * 4));  // per-image affine partials
  gn_bwd(kBF16, dy, x, dx, N, HW, C, G, g, mean, istd, dg, db, aff, cur());
}

void softmax_fwd(const void* x, void* y, long rows, int C) { softmax_rows(kBF16, x, y, rows, C, cur()); }
void softmax_bwd(const void* y, const void* dy, void* dx, long rows, int C) {
  softmax_rows_bwd(kBF16, y, dy, dx, rows, C, cur());
}
void dropout(const void* x, void* y, long n, float p, uint64_t seed) { dcnn::dropout(kBF16, x, y, n, p, seed, nullptr, cur()); }

void add(const void* a, const void* b, void* y, long n, bool relu) {
  hipLaunchKernelGGL(add_bf16_kernel, dim3(grid_of(n)), dim3(256), 0, cur(), static_cast<const bf16*>(a),
                     static_cast<const bf16*>(b), static_cast<bf16*>(y), n, relu ? 1 : 0);
  HOST_HIP_CHECK(hipGetLastError());
}

void relu_mask(const void* dy, const void* y, void* dx, long n) {
  hipLaunchKernelGGL(relu_mask_bf16_kernel, dim3(grid_of(n)), dim3(256), 0, cur(), static_cast<const bf16*>(dy),
                     static_cast<const bf16*>(y), static_cast<bf16*>(dx), n);
  HOST_HIP_CHECK(hipGetLastError());
}

void adam(float* p, const float* g, float* m, float* v, void* shadow, long n, float lr, float b1, float b2, float eps,
          float bc1, float bc2, float wd, bool decoupled) {
  adam_step(p, g, m, v, static_cast<bf16*>(shadow), n, lr, b1, b2, eps, bc1, bc2, wd, decoupled ? 1 : 0, nullptr, cur());
}

const void* loss_device() { return scratch(LOSS_OUT, 16); }

void adam_hyper_step(float* hyper, float b1, float b2) { adam_scalars(hyper, b1, b2, cur()); }
void adam_dev(float* p, const float* g, float* m, float* v, void* shadow, long n, float b1, float b2, float eps,
              float wd, bool decoupled, const float* hyper) {
  adam_step(p, g, m, v, static_cast<bf16*>(shadow), n, 0.f, b1, b2, eps, 1.f, 1.f, wd, decoupled ? 1 : 0, hyper, cur());
}

void sgd(float* p, const float* g, float* vel, void* shadow, long n, float lr, float momentum) {
  sgd_step(p, g, vel, static_cast<bf16*>(shadow), n, lr, momentum, nullptr, cur());
}

}  // namespace gpu_ops
}  // namespace dcnn
