// Losses and metrics:
//  * softmax cross-entropy — one workgroup per row: max, Σexp, loss and (softmax − q)/N in one
//    kernel (the gradient is produced in the forward pass; backward only rescales it);
//  * binary Lovász hinge per image (reference core/losses.py:5-92) — one 1024-thread workgroup per
//    image: errors → LDS bitonic sort (descending, index tie-break like tf.nn.top_k) of up to
//    16384 (key, index) pairs (96 KB of the 160 KB LDS) → gather labels → block scans for the
//    Jaccard gradient → loss and ∂loss/∂logit scattered back to pixel order;
//    Images above 16384 pixels (any input_shape beyond 128×128) take the multi-pass path: the
//    same bitonic network over the whole padded row in global memory — a local LDS pass sorts
//    16384-element chunks, each later merge stage runs its strides ≥ 16384 as global
//    compare-exchange passes and the rest in one LDS pass per chunk — then one workgroup per
//    image walks the sorted row in 4096-element chunks with a carried block scan;
//  * segmentation metrics per image (reference core/metric.py): TP/FP/FN/TN block counts → IoU
//    threshold score and pixel accuracy.
#include "common.h"
#include "kernels.h"

namespace tdl {
namespace {

__device__ __forceinline__ float ld(const void* p, bool bf, long i) {
  return bf ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}

__device__ __forceinline__ float ld_label(const void* p, int kind, long i) {
  switch (kind) {
    case 0: return ((const float*)p)[i];
    case 1: return (float)((const uint8_t*)p)[i];
    case 2: return (float)((const int64_t*)p)[i];
    case 3: return bf2f(((const bf16_t*)p)[i]);
    default: return (float)((const int32_t*)p)[i];
  }
}

template <int NTH>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NTH / 64; ++i) t += sh[i];
  return t;
}

template <int NTH>
__device__ __forceinline__ float block_max(float v, float* sh) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NTH / 64; ++i) t = fmaxf(t, sh[i]);
  return t;
}

__global__ void __launch_bounds__(256) softmax_xent_kernel(const void* __restrict__ logits, int bf,
                                                           const int64_t* __restrict__ labels,
                                                           float* __restrict__ loss,
                                                           void* __restrict__ grad, int N, int K,
                                                           float eps, float* __restrict__ slab) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const long base = (long)row * K;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < K; i += 256) mx = fmaxf(mx, ld(logits, bf, base + i));
  mx = block_max<256>(mx, sh);
  float se = 0.f, sx = 0.f;
  for (int i = threadIdx.x; i < K; i += 256) {
    const float v = ld(logits, bf, base + i);
    se += __expf(v - mx);
    sx += v;
  }
  se = block_sum<256>(se, sh);
  sx = block_sum<256>(sx, sh);
  const float lse = mx + __logf(se);
  const int lab = (int)labels[row];
  const float xl = ld(logits, bf, base + lab);
  const float on = 1.f - eps, off = eps / K;
  // loss = lse − Σ q·x,  q = on·onehot + off
  const float l = lse - on * xl - off * sx;
  const float invN = 1.f / N;
  for (int i = threadIdx.x; i < K; i += 256) {
    const float v = ld(logits, bf, base + i);
    const float p = __expf(v - lse);
    const float g = (p - off - (i == lab ? on : 0.f)) * invN;
    if (bf)
      ((bf16_t*)grad)[base + i] = f2bf(g);
    else
      ((float*)grad)[base + i] = g;
  }
  if (threadIdx.x == 0) {
    if (slab) slab[row] = l * invN;  // deterministic mode: summed in row order (det.hip)
    else atomicAdd(loss, l * invN);
  }
}

// Forward-only classification head for evaluation / prediction (no gradient): per row the
// softmax probabilities (optional, fp32), and with labels the summed cross-entropy and the count
// of rows whose argmax (first maximal index, like torch.argmax) is the label.  One workgroup per
// row; deterministic mode sums the per-row terms in row order.
__global__ void __launch_bounds__(256) softmax_eval_kernel(const void* __restrict__ logits, int bf,
                                                           const int64_t* __restrict__ labels,
                                                           float* __restrict__ loss_sum,
                                                           float* __restrict__ correct,
                                                           float* __restrict__ probs, int N, int K,
                                                           float* __restrict__ slab) {
  __shared__ float sh[4];
  __shared__ int shi[4];
  const int row = blockIdx.x;
  const long base = (long)row * K;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < K; i += 256) mx = fmaxf(mx, ld(logits, bf, base + i));
  mx = block_max<256>(mx, sh);
  float se = 0.f;
  int first = K;
  for (int i = threadIdx.x; i < K; i += 256) {
    const float v = ld(logits, bf, base + i);
    se += __expf(v - mx);
    if (v == mx && i < first) first = i;
  }
  se = block_sum<256>(se, sh);
  // block minimum of the first maximal index
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o, 64));
  if ((threadIdx.x & 63) == 0) shi[threadIdx.x >> 6] = first;
  __syncthreads();
  first = min(min(shi[0], shi[1]), min(shi[2], shi[3]));
  const float lse = mx + __logf(se);
  if (probs) {
    for (int i = threadIdx.x; i < K; i += 256) probs[base + i] = __expf(ld(logits, bf, base + i) - lse);
  }
  if (labels && threadIdx.x == 0) {
    const int lab = (int)labels[row];
    const float l = lse - ld(logits, bf, base + lab);
    const float c = first == lab ? 1.f : 0.f;
    if (slab) {
      slab[row] = l;
      slab[N + row] = c;
    } else {
      if (loss_sum) atomicAdd(loss_sum, l);
      if (correct) atomicAdd(correct, c);
    }
  }
}

// --------------------------------------------------------------------------------------------
// Lovász hinge
// --------------------------------------------------------------------------------------------
constexpr int LV_THREADS = 1024;
constexpr int LV_MAXP = 16384;

__global__ void __launch_bounds__(LV_THREADS) lovasz_kernel(const void* __restrict__ logits, int bf,
                                                            const void* __restrict__ labels,
                                                            int lkind, float* __restrict__ loss,
                                                            float* __restrict__ grad, int B,
                                                            int P, float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) char lsm[];
  float* key = (float*)lsm;                        // LV_MAXP floats (errors, later scan values)
  uint16_t* idx = (uint16_t*)(key + LV_MAXP);      // LV_MAXP indices
  float* part = (float*)(idx + LV_MAXP);           // LV_THREADS partials + spare
  const int img = blockIdx.x;
  const long base = (long)img * P;
  int Pp = 1;
  while (Pp < P) Pp <<= 1;
  const int tid = threadIdx.x;
  // errors = 1 − logit·sign; padding = −inf (sorts last)
  for (int i = tid; i < Pp; i += LV_THREADS) {
    if (i < P) {
      const float lab = ld_label(labels, lkind, base + i);
      const float sgn = 2.f * (lab > 0.5f ? 1.f : 0.f) - 1.f;
      const float e = 1.f - ld(logits, bf, base + i) * sgn;
      // a NaN error (diverged logits) sorts first as +inf: a NaN compares false both ways and
      // would let the −inf padding entries (index ≥ P) move into the first P positions
      key[i] = e == e ? e : INFINITY;
    } else {
      key[i] = -INFINITY;
    }
    idx[i] = (uint16_t)i;
  }
  __syncthreads();
  // bitonic sort, descending by key, ascending index on ties
  for (int size = 2; size <= Pp; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < Pp / 2; t += LV_THREADS) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const float ka = key[lo], kb = key[hi];
        const int ia = idx[lo], ib = idx[hi];
        // "a before b" in descending order
        const bool a_first = (ka > kb) || (ka == kb && ia < ib);
        const bool swap = desc ? !a_first : a_first;
        if (swap) {
          key[lo] = kb;
          key[hi] = ka;
          idx[lo] = (uint16_t)ib;
          idx[hi] = (uint16_t)ia;
        }
      }
      __syncthreads();
    }
  }
  // per-thread contiguous segments for the scans
  const int seg = (P + LV_THREADS - 1) / LV_THREADS;
  const int s0 = tid * seg, s1 = min(P, s0 + seg);
  float gts_local = 0.f;
  for (int i = s0; i < s1; ++i) gts_local += ld_label(labels, lkind, base + idx[i]) > 0.5f ? 1.f : 0.f;
  part[tid] = gts_local;
  __syncthreads();
  // exclusive block scan of the 1024 per-thread counts: wave scans + scan of the 16 wave totals
  float& gts_total = part[LV_THREADS];
  float* wtot = part + LV_THREADS + 4;  // 16 wave totals
  {
    const int lane = tid & 63, w = tid >> 6;
    float v = gts_local, incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    float before = 0.f, all = 0.f;
    for (int i = 0; i < LV_THREADS / 64; ++i) {
      const float t = wtot[i];
      if (i < w) before += t;
      all += t;
    }
    part[tid] = before + incl - v;
    if (tid == 0) gts_total = all;
    __syncthreads();
  }
  const float gts = gts_total;
  // walk the segment: cumulative gt and (1-gt) at position i (inclusive)
  float cum_gt = part[tid];
  float loss_local = 0.f;
  // jaccard at i-1 needed for the difference: compute at s0-1 first
  float prev_j = 0.f;
  if (s0 > 0 && s0 < P) {
    const float cg = cum_gt;                        // inclusive cumsum at s0-1
    const float cng = (float)s0 - cg;
    prev_j = 1.f - (gts - cg) / (gts + cng);
  }
  for (int i = s0; i < s1; ++i) {
    const int pix = min((int)idx[i], P - 1);  // (never a padding index: see the key init)
    const float g = ld_label(labels, lkind, base + pix) > 0.5f ? 1.f : 0.f;
    cum_gt += g;
    const float cng = (float)(i + 1) - cum_gt;
    const float jac = 1.f - (gts - cum_gt) / (gts + cng);
    const float gr = (i == 0) ? jac : jac - prev_j;
    prev_j = jac;
    const float e = key[i];
    if (e > 0.f) loss_local += e * gr;
    const float sgn = 2.f * g - 1.f;
    grad[base + pix] = (e > 0.f ? -sgn * gr : 0.f) / (float)B;
  }
  float* red = part + LV_THREADS + 4 + LV_THREADS / 64;
  const float tot = block_sum<LV_THREADS>(loss_local, red);
  if (tid == 0) {
    if (slab) slab[img] = tot / (float)B;
    else atomicAdd(loss, tot / (float)B);
  }
}

// ---- multi-pass Lovász hinge for P > LV_MAXP ------------------------------------------------
constexpr int LVG_CHUNK = 16384;  // elements per LDS pass (1024 threads, 128 KB of LDS)

__device__ __forceinline__ bool lv_before(float ka, int ia, float kb, int ib) {
  return (ka > kb) || (ka == kb && ia < ib);  // descending key, ascending index on ties
}

__global__ void __launch_bounds__(256) lovasz_init_kernel(const void* __restrict__ logits, int bf,
                                                          const void* __restrict__ labels,
                                                          int lkind, float* __restrict__ key,
                                                          int* __restrict__ idx, int P, int Pp) {
  const long img = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Pp) return;
  float k = -INFINITY;
  if (i < P) {
    const float lab = ld_label(labels, lkind, img * P + i);
    const float sgn = lab > 0.5f ? 1.f : -1.f;
    k = 1.f - ld(logits, bf, img * P + i) * sgn;
    if (k != k) k = INFINITY;  // NaN sorts first (see lovasz_kernel)
  }
  key[img * Pp + i] = k;
  idx[img * Pp + i] = i;
}

// one (size, stride) step of the bitonic network, stride ≥ LVG_CHUNK: one pair per thread
__global__ void __launch_bounds__(256) lovasz_bitonic_global_kernel(float* __restrict__ key,
                                                                    int* __restrict__ idx, int Pp,
                                                                    int size, int stride) {
  const long row = (long)blockIdx.y * Pp;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= Pp / 2) return;
  const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
  const bool desc = (lo & size) == 0;
  const float ka = key[row + lo], kb = key[row + hi];
  const int ia = idx[row + lo], ib = idx[row + hi];
  const bool a_first = lv_before(ka, ia, kb, ib);
  if (desc ? !a_first : a_first) {
    key[row + lo] = kb;
    key[row + hi] = ka;
    idx[row + lo] = ib;
    idx[row + hi] = ia;
  }
}

// every step with stride < LVG_CHUNK of the merge stages size_lo … size_hi (doubling), on one
// LDS-resident chunk; the direction of a pair follows its position in the whole row
__global__ void __launch_bounds__(LV_THREADS) lovasz_bitonic_local_kernel(float* __restrict__ key,
                                                                          int* __restrict__ idx,
                                                                          int Pp, int size_lo,
                                                                          int size_hi) {
  extern __shared__ __attribute__((aligned(16))) char lsm[];
  float* k = (float*)lsm;
  int* ix = (int*)(k + LVG_CHUNK);
  const long row = (long)blockIdx.y * Pp;
  const int c0 = blockIdx.x * LVG_CHUNK;
  const int tid = threadIdx.x;
  for (int i = tid; i < LVG_CHUNK; i += LV_THREADS) {
    k[i] = key[row + c0 + i];
    ix[i] = idx[row + c0 + i];
  }
  __syncthreads();
  for (int size = size_lo; size <= size_hi; size <<= 1) {
    for (int stride = min(size, LVG_CHUNK) >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < LVG_CHUNK / 2; t += LV_THREADS) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const bool desc = ((c0 + lo) & size) == 0;
        const float ka = k[lo], kb = k[hi];
        const int ia = ix[lo], ib = ix[hi];
        const bool a_first = lv_before(ka, ia, kb, ib);
        if (desc ? !a_first : a_first) {
          k[lo] = kb;
          k[hi] = ka;
          ix[lo] = ib;
          ix[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < LVG_CHUNK; i += LV_THREADS) {
    key[row + c0 + i] = k[i];
    idx[row + c0 + i] = ix[i];
  }
}

// Jaccard-gradient walk over the sorted row: 4096-element chunks (4 per thread), block scan of
// the ground-truth counts with a carry between chunks
__global__ void __launch_bounds__(LV_THREADS) lovasz_scan_kernel(const void* __restrict__ labels,
                                                                 int lkind,
                                                                 const float* __restrict__ key,
                                                                 const int* __restrict__ idx,
                                                                 float* __restrict__ loss,
                                                                 float* __restrict__ grad, int B,
                                                                 int P, int Pp,
                                                                 float* __restrict__ slab) {
  __shared__ float wtot[LV_THREADS / 64];
  __shared__ float red[LV_THREADS / 64 + 4];
  const long img = blockIdx.x;
  const long lbase = img * P, kbase = img * Pp;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int PER = 4, STEP = LV_THREADS * PER;
  float gl = 0.f;
  for (int i = tid; i < P; i += LV_THREADS) gl += ld_label(labels, lkind, lbase + i) > 0.5f ? 1.f : 0.f;
  const float gts = block_sum<LV_THREADS>(gl, red);
  float carry = 0.f, loss_local = 0.f;
  for (int start = 0; start < P; start += STEP) {
    const int i0 = start + tid * PER;
    float g[PER];
    int pix[PER];
    float mine = 0.f;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = i0 + j;
      pix[j] = i < P ? min(idx[kbase + i], P - 1) : 0;  // never a padding index
      g[j] = i < P && ld_label(labels, lkind, lbase + pix[j]) > 0.5f ? 1.f : 0.f;
      mine += g[j];
    }
    float incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    __syncthreads();  // wtot reuse across chunks
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    float before = 0.f, all = 0.f;
#pragma unroll
    for (int q = 0; q < LV_THREADS / 64; ++q) {
      const float t = wtot[q];
      if (q < w) before += t;
      all += t;
    }
    float cum = carry + before + incl - mine;  // inclusive count before element i0
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = i0 + j;
      if (i >= P) break;
      const float cprev = cum;
      cum += g[j];
      const float jac = 1.f - (gts - cum) / (gts + ((float)(i + 1) - cum));
      float gr = jac;
      if (i > 0) gr -= 1.f - (gts - cprev) / (gts + ((float)i - cprev));
      const float e = key[kbase + i];
      if (e > 0.f) loss_local += e * gr;
      grad[lbase + pix[j]] = (e > 0.f ? -(2.f * g[j] - 1.f) * gr : 0.f) / (float)B;
    }
    carry += all;
  }
  const float tot = block_sum<LV_THREADS>(loss_local, red);
  if (tid == 0) {
    if (slab) slab[img] = tot / (float)B;
    else atomicAdd(loss, tot / (float)B);
  }
}

__global__ void __launch_bounds__(256) seg_metrics_kernel(const void* __restrict__ labels, int lkind,
                                                          const float* __restrict__ pred,
                                                          float* __restrict__ score,
                                                          float* __restrict__ acc, int P,
                                                          int kaggle) {
  __shared__ float sh[4];
  const long base = (long)blockIdx.x * P;
  float tp = 0, fp = 0, fn = 0, tn = 0;
  for (int i = threadIdx.x; i < P; i += 256) {
    const bool l = ld_label(labels, lkind, base + i) > 0.5f;
    const bool p = pred[base + i] > 0.5f;
    tp += (l && p);
    fp += (!l && p);
    fn += (l && !p);
    tn += (!l && !p);
  }
  tp = block_sum<256>(tp, sh);
  fp = block_sum<256>(fp, sh);
  fn = block_sum<256>(fn, sh);
  tn = block_sum<256>(tn, sh);
  if (threadIdx.x == 0) {
    const float den = tp + fp + fn;
    const float iou = den > 0.f ? tp / den : 1.f;
    float s = 0.f;
    for (int t = 0; t < 10; ++t) {
      const float th = 0.5f + 0.05f * t;
      const float hit = iou > th ? 1.f : 0.f;
      s += kaggle ? hit : iou * hit;
    }
    score[blockIdx.x] = s / 10.f;
    acc[blockIdx.x] = (tp + tn) / (float)P;
  }
}

}  // namespace

void softmax_xent_launch(const void* logits, bool bf16, const int64_t* labels, float* loss,
                         void* grad, int N, int K, float smoothing, hipStream_t st) {
  float* slab = deterministic() ? det_slab((size_t)N, st) : nullptr;
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(N), dim3(256), 0, st, logits, bf16 ? 1 : 0, labels,
                     loss, grad, N, K, smoothing, slab);
  if (slab) slab_sum_launch(slab, loss, N, 1, 1, st);
}

void softmax_eval_launch(const void* logits, bool bf16, const int64_t* labels, float* loss_sum,
                         float* correct, float* probs, int N, int K, hipStream_t st) {
  float* slab = (labels && deterministic()) ? det_slab((size_t)2 * N, st) : nullptr;
  hipLaunchKernelGGL(softmax_eval_kernel, dim3(N), dim3(256), 0, st, logits, bf16 ? 1 : 0, labels,
                     loss_sum, correct, probs, N, K, slab);
  if (slab) {
    if (loss_sum) slab_sum_launch(slab, loss_sum, N, 1, 1, st);
    if (correct) slab_sum_launch(slab + N, correct, N, 1, 1, st);
  }
}

void lovasz_hinge_launch(const void* logits, bool logits_bf16, const void* labels, int label_kind,
                         float* loss, float* grad, int B, int P, hipStream_t st) {
  const size_t lds = LV_MAXP * 4 + LV_MAXP * 2 + LV_THREADS * 4 + 256;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)lovasz_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    attr_set = true;
  }
  float* slab = deterministic() ? det_slab((size_t)B, st) : nullptr;
  hipLaunchKernelGGL(lovasz_kernel, dim3(B), dim3(LV_THREADS), lds, st, logits,
                     logits_bf16 ? 1 : 0, labels, label_kind, loss, grad, B, P, slab);
  if (slab) slab_sum_launch(slab, loss, B, 1, 1, st);
}

int lovasz_padded_len(int P) {
  int Pp = LVG_CHUNK;
  while (Pp < P) Pp <<= 1;
  return Pp;
}

void lovasz_hinge_large_launch(const void* logits, bool logits_bf16, const void* labels,
                               int label_kind, float* loss, float* grad, float* key, int* idx, int B,
                               int P, hipStream_t st) {
  const int Pp = lovasz_padded_len(P);
  const size_t lds = (size_t)LVG_CHUNK * 8;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)lovasz_bitonic_local_kernel,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(lovasz_init_kernel, dim3(Pp / 256, B), dim3(256), 0, st, logits,
                     logits_bf16 ? 1 : 0, labels, label_kind, key, idx, P, Pp);
  const dim3 lgrid(Pp / LVG_CHUNK, B), ggrid(Pp / 2 / 256, B);
  hipLaunchKernelGGL(lovasz_bitonic_local_kernel, lgrid, dim3(LV_THREADS), lds, st, key, idx, Pp,
                     2, LVG_CHUNK);
  for (int size = 2 * LVG_CHUNK; size <= Pp; size <<= 1) {
    for (int stride = size >> 1; stride >= LVG_CHUNK; stride >>= 1)
      hipLaunchKernelGGL(lovasz_bitonic_global_kernel, ggrid, dim3(256), 0, st, key, idx, Pp, size,
                         stride);
    hipLaunchKernelGGL(lovasz_bitonic_local_kernel, lgrid, dim3(LV_THREADS), lds, st, key, idx, Pp,
                       size, size);
  }
  float* slab = deterministic() ? det_slab((size_t)B, st) : nullptr;
  hipLaunchKernelGGL(lovasz_scan_kernel, dim3(B), dim3(LV_THREADS), 0, st, labels, label_kind, key,
                     idx, loss, grad, B, P, Pp, slab);
  if (slab) slab_sum_launch(slab, loss, B, 1, 1, st);
}

void seg_metrics_launch(const void* labels, int label_kind, const float* pred, float* score,
                        float* acc, int B, int P, bool kaggle, hipStream_t st) {
  hipLaunchKernelGGL(seg_metrics_kernel, dim3(B), dim3(256), 0, st, labels, label_kind, pred, score,
                     acc, P, kaggle ? 1 : 0);
}

}  // namespace tdl
