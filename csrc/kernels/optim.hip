// Fused optimizer updates over the flat parameter buffers (models/params.py): one launch updates
// the whole model — fp32 master, fp32 slots, bf16 compute copy — reading the data-parallel
// gradient scale and a per-64-element weight-decay flag.  float4 vectorised (offsets of every
// parameter are 64-element aligned, the buffer length is a multiple of 64).  An optional device
// scalar multiplies the learning rate (HIP-graph replays: the host writes the step's lr there
// instead of baking it into the captured kernel arguments).
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

constexpr int NT = 256;

__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                           bf16_t* __restrict__ lowp, const uint8_t* __restrict__ flags, long n4,
                           float lr, const float* __restrict__ lr_scale, float mu, float wd,
                           float gs, int nesterov) {
  if (lr_scale) lr *= *lr_scale;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
    const float d = flags[(i * 4) >> 6] ? wd : 0.f;
    float4 pv = ((float4*)p)[i];
    const float4 gv = ((const float4*)g)[i];
    float4 mv = ((float4*)m)[i];
    float pa[4] = {pv.x, pv.y, pv.z, pv.w};
    const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
    float ma[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gg = ga[j] * gs + d * pa[j];
      ma[j] = mu * ma[j] + gg;
      pa[j] -= lr * (nesterov ? gg + mu * ma[j] : ma[j]);
    }
    ((float4*)p)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    ((float4*)m)[i] = make_float4(ma[0], ma[1], ma[2], ma[3]);
    if (lowp) ((uint2*)lowp)[i] = make_uint2(pack2(pa[0], pa[1]), pack2(pa[2], pa[3]));
  }
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, bf16_t* __restrict__ lowp,
                            const uint8_t* __restrict__ flags, long n4, float lr_t,
                            const float* __restrict__ lr_scale, float b1, float b2, float eps,
                            float wd, float gs) {
  if (lr_scale) lr_t *= *lr_scale;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
    const float d = flags[(i * 4) >> 6] ? wd : 0.f;
    float4 pv = ((float4*)p)[i];
    const float4 gv = ((const float4*)g)[i];
    float4 mv = ((float4*)m)[i];
    float4 vv = ((float4*)v)[i];
    float pa[4] = {pv.x, pv.y, pv.z, pv.w};
    const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
    float ma[4] = {mv.x, mv.y, mv.z, mv.w};
    float va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gg = ga[j] * gs + d * pa[j];
      ma[j] = b1 * ma[j] + (1.f - b1) * gg;
      va[j] = b2 * va[j] + (1.f - b2) * gg * gg;
      pa[j] -= lr_t * ma[j] / (sqrtf(va[j]) + eps);
    }
    ((float4*)p)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    ((float4*)m)[i] = make_float4(ma[0], ma[1], ma[2], ma[3]);
    ((float4*)v)[i] = make_float4(va[0], va[1], va[2], va[3]);
    if (lowp) ((uint2*)lowp)[i] = make_uint2(pack2(pa[0], pa[1]), pack2(pa[2], pa[3]));
  }
}

inline int blocks_for(long n) { return (int)std::min<long>(2048, std::max<long>(1, (n + NT - 1) / NT)); }

}  // namespace

void sgd_momentum_launch(float* p, const float* g, float* mom, bf16_t* lowp, const uint8_t* flags,
                         long n, float lr, const float* lr_scale, float mu, float wd, float gscale,
                         bool nesterov, hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(blocks_for(n / 4)), dim3(NT), 0, st, p, g, mom, lowp, flags,
                     n / 4, lr, lr_scale, mu, wd, gscale, nesterov ? 1 : 0);
}

void adam_launch(float* p, const float* g, float* m, float* v, bf16_t* lowp, const uint8_t* flags,
                 long n, float lr_t, const float* lr_scale, float b1, float b2, float eps, float wd,
                 float gscale, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n / 4)), dim3(NT), 0, st, p, g, m, v, lowp, flags,
                     n / 4, lr_t, lr_scale, b1, b2, eps, wd, gscale);
}

}  // namespace tdl
