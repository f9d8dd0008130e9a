// Deterministic mode (TDL_DETERMINISTIC=1 / det_set; SURVEY §5.2 "deterministic-mode runs compared
// bit-wise across 2 launches").
//
// The fast paths reduce across workgroups with fp32 atomics (BN statistics and backward sums,
// per-image / per-row loss terms): the sum is exact up to rounding but its order — and therefore
// the last bits — depends on workgroup timing, so two runs of the same step differ by a few ulps
// and training trajectories drift apart.  In deterministic mode every such reduction writes one
// partial row per workgroup into a slab and `slab_sum_kernel` adds the rows in index order
// (out += Σ_b slab[b]); conv-epilogue BN statistics are computed by the (slab-reduced) BN
// statistics pass instead, and the consumer-dgrad / pooling fusions of the BN-backward sums are
// turned off so the BN backward reduces itself.  Everything else (split-K weight gradients, bias
// column sums, depthwise weight gradients) already reduces fixed slabs in order.
//
// Scope: the bf16 GPU path.  Slabs are per stream (the side-stream weight gradients run
// concurrently with the compute stream) and grow on demand.  Growth is not allowed inside a
// HIP-graph capture (no allocation on the capturing thread): Trainer.capture runs its warm-up
// steps on the capture stream itself, so the slabs exist at their final size.  A slab a capture
// has baked into a graph is never freed — a later growth of that stream's slab retires it.
#include "common.h"
#include "kernels.h"

#include <map>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace tdl {

static int g_det_override = -1;

int deterministic() {
  static const int m = [] {
    const char* e = getenv("TDL_DETERMINISTIC");
    return e ? atoi(e) : 0;
  }();
  return g_det_override >= 0 ? g_det_override : m;
}

void det_set(int on) { g_det_override = on; }

namespace {

struct Slab {
  float* p = nullptr;
  size_t cap = 0;
  bool captured = false;  // referenced by a captured graph: retire instead of free
};
std::mutex g_slab_mu;
std::map<hipStream_t, Slab> g_slabs;
std::vector<float*> g_retired;  // slabs of captured graphs (live as long as the process)

__global__ void slab_sum_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                int rows, long n, long row_stride) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += slab[r * row_stride + i];
  out[i] += s;
}

}  // namespace

float* det_slab(size_t floats, hipStream_t st) {
  std::lock_guard<std::mutex> g(g_slab_mu);
  Slab& s = g_slabs[st];
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(st, &cap);
  if (floats > s.cap) {
    if (cap != hipStreamCaptureStatusNone)
      throw std::runtime_error("deterministic mode: slab growth inside a HIP-graph capture "
                               "(run the warm-up steps on the capture stream, as "
                               "Trainer.capture does, or capture without TDL_DETERMINISTIC)");
    if (s.p) {
      (void)hipStreamSynchronize(st);
      if (s.captured)
        g_retired.push_back(s.p);
      else
        (void)hipFree(s.p);
      s.captured = false;
    }
    s.cap = std::max<size_t>(floats, (size_t)1 << 20);
    if (hipMalloc((void**)&s.p, s.cap * sizeof(float)) != hipSuccess)
      throw std::runtime_error("deterministic mode: slab allocation failed");
  }
  if (cap != hipStreamCaptureStatusNone) s.captured = true;
  return s.p;
}

void slab_sum_launch(const float* slab, float* out, int rows, long n, long row_stride,
                     hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, slab,
                     out, rows, n, row_stride);
}

}  // namespace tdl
