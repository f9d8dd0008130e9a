// Depthwise k×k convolution (depth multiplier 1), NHWC bf16, weights [R][S][C] bf16, fp32 grads.
// Memory-bound: each lane owns one 16-B channel vector (8 channels) of one output (fwd) or input
// (dgrad) pixel; wgrad keeps R·S·8 fp32 partial sums per lane over a pixel range, reduces them
// through LDS and issues one contiguous atomic row per workgroup.  Scalar variants handle
// C % 8 != 0 (e.g. the single-channel Laplacian of the preprocessing).
#include "conv_common.h"

namespace tdl {
namespace {
using convk::OOB;
using convk::bload16;
using convk::make_rsrc;
using convk::rsrc_t;
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int NT = 256;
inline int blocks_for(long n) { return (int)std::min<long>(8192, std::max<long>(1, (n + NT - 1) / NT)); }

// ReLU on 8 packed bf16 values: clear every half whose sign bit is set
__device__ __forceinline__ uint32_t relu2(uint32_t v) {
  return v & ~(((v >> 15) & 0x00010001u) * 0xFFFFu);
}
__device__ __forceinline__ uint4 relu8(uint4 v) {
  return make_uint4(relu2(v.x), relu2(v.y), relu2(v.z), relu2(v.w));
}
// dx · [x > 0] for the fused input ReLU's backward
__device__ __forceinline__ void mask_pos(float* acc, const bf16_t* xp) {
  float xv[8];
  unpack8(*(const uint4*)xp, xv);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = xv[j] > 0.f ? acc[j] : 0.f;
}

// residual-gradient join: acc += dadd (8 channels)
__device__ __forceinline__ void add8(float* acc, const bf16_t* p) {
  float v[8];
  unpack8(*(const uint4*)p, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] += v[j];
}

template <int V>
__device__ __forceinline__ void ldv(const bf16_t* p, float* f) {
  if constexpr (V == 8) unpack8(*(const uint4*)p, f);
  else f[0] = bf2f(*p);
}

template <int V>
__device__ __forceinline__ void stv(bf16_t* p, const float* f) {
  if constexpr (V == 8) *(uint4*)p = pack8(f);
  else *p = f2bf(f[0]);
}

template <int V>
__global__ void dw_fwd_kernel(DwArgs a) {
  const int cv = a.C / V;
  const long total = (long)a.N * a.Ho * a.Wo * cv;
  for (long t = blockIdx.x * (long)NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    const int c = (int)(t % cv) * V;
    long p = t / cv;
    const int wo = (int)(p % a.Wo);
    p /= a.Wo;
    const int ho = (int)(p % a.Ho);
    const int n = (int)(p / a.Ho);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = a.bias ? a.bias[c + j] : 0.f;
    for (int r = 0; r < a.R; ++r) {
      const int hi = ho * a.sh - a.ph + r * a.dh;
      if ((unsigned)hi >= (unsigned)a.H) continue;
      for (int s = 0; s < a.S; ++s) {
        const int wi = wo * a.sw - a.pw + s * a.dwl;
        if ((unsigned)wi >= (unsigned)a.W) continue;
        float xv[V], wv[V];
        ldv<V>(a.x + (((long)n * a.H + hi) * a.W + wi) * a.C + c, xv);
        ldv<V>(a.w + ((long)r * a.S + s) * a.C + c, wv);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += xv[j] * wv[j];
      }
    }
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] = fmaxf(acc[j], 0.f);
    }
    stv<V>(a.out + (((long)n * a.Ho + ho) * a.Wo + wo) * a.C + c, acc);
  }
}

template <int V>
__global__ void dw_dgrad_kernel(DwArgs a) {
  const int cv = a.C / V;
  const long total = (long)a.N * a.H * a.W * cv;
  for (long t = blockIdx.x * (long)NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    const int c = (int)(t % cv) * V;
    long p = t / cv;
    const int w = (int)(p % a.W);
    p /= a.W;
    const int h = (int)(p % a.H);
    const int n = (int)(p / a.H);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int r = 0; r < a.R; ++r) {
      int th = h + a.ph - r * a.dh;
      if (th < 0 || th % a.sh) continue;
      th /= a.sh;
      if (th >= a.Ho) continue;
      for (int s = 0; s < a.S; ++s) {
        int tw = w + a.pw - s * a.dwl;
        if (tw < 0 || tw % a.sw) continue;
        tw /= a.sw;
        if (tw >= a.Wo) continue;
        float gv[V], wv[V];
        ldv<V>(a.dy + (((long)n * a.Ho + th) * a.Wo + tw) * a.C + c, gv);
        ldv<V>(a.w + ((long)r * a.S + s) * a.C + c, wv);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += gv[j] * wv[j];
      }
    }
    const long o = (((long)n * a.H + h) * a.W + w) * a.C + c;
    if (a.dadd) {
      float d[V];
      ldv<V>(a.dadd + o, d);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += d[j];
    }
    stv<V>(a.out + o, acc);
  }
}

// wgrad: block = (pixel range) × (channel vectors); lane owns one channel vector for all R·S taps
template <int V, int RS>
__global__ void __launch_bounds__(NT) dw_wgrad_kernel(DwArgs a, long pix_per_block) {
  const int cv = a.C / V;
  const int lanes_c = min(cv, NT);
  const int rpp = NT / lanes_c;  // pixel lanes per pass
  const int t = threadIdx.x;
  const int cvi = t % lanes_c + blockIdx.y * lanes_c;
  const int pl = t / lanes_c;
  const long P = (long)a.N * a.Ho * a.Wo;
  const long p0 = blockIdx.x * pix_per_block, p1 = min(P, p0 + pix_per_block);
  float acc[RS][V];
  float db[V];
#pragma unroll
  for (int k = 0; k < RS; ++k)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[k][j] = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) db[j] = 0.f;
  const bool active = pl < rpp && cvi < cv;
  const int rsa = a.R * a.S;
  const int c = cvi * V;
  if (active) {
    for (long p = p0 + pl; p < p1; p += rpp) {
      const int wo = (int)(p % a.Wo);
      const long q = p / a.Wo;
      const int ho = (int)(q % a.Ho);
      const int n = (int)(q / a.Ho);
      float gv[V];
      ldv<V>(a.dy + p * a.C + c, gv);
#pragma unroll
      for (int j = 0; j < V; ++j) db[j] += gv[j];
#pragma unroll
      for (int k = 0; k < RS; ++k) {
        if (k >= rsa) break;
        const int r = k / a.S, s = k - (k / a.S) * a.S;
        const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dwl;
        if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) continue;
        float xv[V];
        ldv<V>(a.x + (((long)n * a.H + hi) * a.W + wi) * a.C + c, xv);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[k][j] += gv[j] * xv[j];
      }
    }
  }
  // reduce across pixel lanes through LDS, one tap at a time
  __shared__ float red[NT][V + 1];
#pragma unroll
  for (int k = 0; k <= RS; ++k) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if constexpr (true) red[t][j] = (k < RS) ? acc[k < RS ? k : 0][j] : db[j];
    }
    __syncthreads();
    for (int o = t; o < lanes_c * V; o += NT) {
      const int lc = o / V, j = o % V;
      const int cc = (lc + blockIdx.y * lanes_c) * V + j;
      if (lc + blockIdx.y * lanes_c < cv) {
        float s = 0.f;
        for (int r = 0; r < rpp; ++r) s += red[r * lanes_c + lc][j];
        if (k < rsa)
          atomicAdd(a.dw + (long)k * a.C + cc, s);
        else if (k == RS && a.db)
          atomicAdd(a.db + cc, s);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Row-oriented kernels for C % 8 == 0 (the model path).  A workgroup owns one output row (fwd) /
// input row (dgrad) of one channel group: lane = (channel vector, pixel lane), so the R·S filter
// taps of the lane's 8 channels live in registers for the whole row and there is no per-pixel
// index division (the generic kernels above divide 64-bit indices per element).
// ---------------------------------------------------------------------------------------------
struct RowGeom {
  int lanes_c, rpp;  // channel-vector lanes per group, pixel lanes
};
inline RowGeom row_geom(int cv) {
  RowGeom g;
  g.lanes_c = std::min(cv, NT);
  g.rpp = std::max(1, NT / g.lanes_c);
  return g;
}

template <int RS>
__global__ void __launch_bounds__(NT) dw_fwd_rows(DwArgs a, int lanes_c, int rpp) {
  const int cv = a.C / 8;
  const int t = threadIdx.x, lc = t % lanes_c, pl = t / lanes_c;
  const int cvi = lc + blockIdx.y * lanes_c;
  if (pl >= rpp || cvi >= cv) return;
  const int c = cvi * 8;
  const int row = blockIdx.x, n = row / a.Ho, ho = row - n * a.Ho;
  float wv[RS][8], bias[8];
#pragma unroll
  for (int k = 0; k < RS; ++k) unpack8(*(const uint4*)(a.w + (long)k * a.C + c), wv[k]);
#pragma unroll
  for (int j = 0; j < 8; ++j) bias[j] = a.bias ? a.bias[c + j] : 0.f;
  const bf16_t* xn = a.x + (long)n * a.H * a.W * a.C + c;
  bf16_t* yrow = a.out + ((long)row * a.Wo) * a.C + c;
  for (int wo = pl; wo < a.Wo; wo += rpp) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = bias[j];
#pragma unroll
    for (int k = 0; k < RS; ++k) {
      const int r = k / a.S, s = k - r * a.S;
      const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dwl;
      if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) continue;
      float xv[8];
      uint4 xr = *(const uint4*)(xn + ((long)hi * a.W + wi) * a.C);
      if (a.relu_in) xr = relu8(xr);
      unpack8(xr, xv);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += xv[j] * wv[k][j];
    }
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j], 0.f);
    }
    *(uint4*)(yrow + (long)wo * a.C) = pack8(acc);
  }
}

template <int RS>
__global__ void __launch_bounds__(NT) dw_dgrad_rows(DwArgs a, int lanes_c, int rpp) {
  const int cv = a.C / 8;
  const int t = threadIdx.x, lc = t % lanes_c, pl = t / lanes_c;
  const int cvi = lc + blockIdx.y * lanes_c;
  if (pl >= rpp || cvi >= cv) return;
  const int c = cvi * 8;
  const int row = blockIdx.x, n = row / a.H, h = row - n * a.H;
  float wv[RS][8];
#pragma unroll
  for (int k = 0; k < RS; ++k) unpack8(*(const uint4*)(a.w + (long)k * a.C + c), wv[k]);
  const bf16_t* gn = a.dy + (long)n * a.Ho * a.Wo * a.C + c;
  bf16_t* xrow = a.out + ((long)row * a.W) * a.C + c;
  for (int w = pl; w < a.W; w += rpp) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int k = 0; k < RS; ++k) {
      const int r = k / a.S, s = k - r * a.S;
      int th = h + a.ph - r * a.dh, tw = w + a.pw - s * a.dwl;
      if (th < 0 || tw < 0) continue;
      if (a.sh > 1) {
        if (th % a.sh) continue;
        th /= a.sh;
      }
      if (a.sw > 1) {
        if (tw % a.sw) continue;
        tw /= a.sw;
      }
      if (th >= a.Ho || tw >= a.Wo) continue;
      float gv[8];
      unpack8(*(const uint4*)(gn + ((long)th * a.Wo + tw) * a.C), gv);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += gv[j] * wv[k][j];
    }
    if (a.mask_x) mask_pos(acc, a.mask_x + ((long)row * a.W + w) * a.C + c);
    if (a.dadd) add8(acc, a.dadd + ((long)row * a.W + w) * a.C + c);
    *(uint4*)(xrow + (long)w * a.C) = pack8(acc);
  }
}

// Stride-2 3×3 input gradient (Xception's strided separable convs, dilation 1): the forward reads
// x[2t − p + r], so dx row h = 2m − p takes dy rows m (tap 0) and m−1 (tap 2) and row h+1 takes
// dy row m (tap 1) — likewise for columns.  A lane owns one 2×2 dx block × 8 channels: it reads the
// 2×2 dy window (rows m−1, m × columns n−1, n) once and does the 9 FMAs of the 4 outputs (4 + 2 +
// 2 + 1 taps), no parity tests or divisions per pixel.  Loads are range-checked buffer loads
// (outside the image → zeros) issued together; the row kernel's per-tap branches around loads
// serialised them (4 dgrads, 1.78 ms of the Xception-41 b128 step,
// profiles/r04_xception41_b128_fold_step_breakdown.txt).
__global__ void __launch_bounds__(NT) dw_dgrad_s2_kernel(const bf16_t* __restrict__ dy,
                                                         const bf16_t* __restrict__ wt,
                                                         bf16_t* __restrict__ dx,
                                                         const bf16_t* __restrict__ mask_x,
                                                         const bf16_t* __restrict__ dadd, int N,
                                                         int H, int W, int C, int Ho, int Wo,
                                                         int ph, int pw, int MG, int NG) {
  const int cv = C / 8;
  const long total = (long)N * MG * NG * cv;
  const rsrc_t rdy = make_rsrc(dy, (uint32_t)((long)N * Ho * Wo * C * 2));
  for (long t = blockIdx.x * (long)NT + threadIdx.x; t < total; t += (long)gridDim.x * NT) {
    const int c = (int)(t % cv) * 8;
    long q = t / cv;
    const int ng = (int)(q % NG);
    q /= NG;
    const int mg = (int)(q % MG);
    const int n = (int)(q / MG);
    // dx rows h0 = 2·mg − ph (even u = h + ph), h0 + 1; columns w0 = 2·ng − pw, w0 + 1
    const int h0 = 2 * mg - ph, w0 = 2 * ng - pw;
    auto off = [&](int tm, int tn) -> uint32_t {
      return ((unsigned)tm < (unsigned)Ho && (unsigned)tn < (unsigned)Wo)
                 ? (uint32_t)((((long)n * Ho + tm) * Wo + tn) * C + c) * 2u
                 : OOB;
    };
    const uint4 g11 = bload16(rdy, off(mg, ng)), g10 = bload16(rdy, off(mg, ng - 1));
    const uint4 g01 = bload16(rdy, off(mg - 1, ng)), g00 = bload16(rdy, off(mg - 1, ng - 1));
    float w9[9][8];
#pragma unroll
    for (int k = 0; k < 9; ++k) unpack8(*(const uint4*)(wt + (long)k * C + c), w9[k]);
    float a11[8], a10[8], a01[8], a00[8];
    unpack8(g11, a11);
    unpack8(g10, a10);
    unpack8(g01, a01);
    unpack8(g00, a00);
    float o[4][8];  // (h0,w0) (h0,w1) (h1,w0) (h1,w1)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[0][j] = a11[j] * w9[0][j] + a10[j] * w9[2][j] + a01[j] * w9[6][j] + a00[j] * w9[8][j];
      o[1][j] = a11[j] * w9[1][j] + a01[j] * w9[7][j];
      o[2][j] = a11[j] * w9[3][j] + a10[j] * w9[5][j];
      o[3][j] = a11[j] * w9[4][j];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int h = h0 + (e >> 1), w = w0 + (e & 1);
      if ((unsigned)h >= (unsigned)H || (unsigned)w >= (unsigned)W) continue;
      const long p = (((long)n * H + h) * W + w) * C + c;
      if (mask_x) mask_pos(o[e], mask_x + p);
      if (dadd) add8(o[e], dadd + p);
      *(uint4*)(dx + p) = pack8(o[e]);
    }
  }
}

// wgrad: workgroup = a range of output rows × one channel group; R·S·8 (+8 bias) fp32 partials per
// lane, combined over pixel lanes in LDS and written as this workgroup's slab row — no atomics
// (the generic kernel's per-block atomics all hit the same R·S·C addresses); the slabs are then
// summed by the split-K reduction kernel.
template <int RS>
__global__ void __launch_bounds__(NT) dw_wgrad_rows(DwArgs a, int lanes_c, int rpp,
                                                    int rows_per_block, float* ws_w, float* ws_b) {
  const int cv = a.C / 8;
  const int t = threadIdx.x, lc = t % lanes_c, pl = t / lanes_c;
  const int cvi = lc + blockIdx.y * lanes_c;
  const bool active = pl < rpp && cvi < cv;
  const int c = cvi * 8;
  const int rows = a.N * a.Ho;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  float acc[RS][8], db[8];
#pragma unroll
  for (int k = 0; k < RS; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) db[j] = 0.f;
  if (active) {
    for (int row = r0; row < r1; ++row) {
      const int n = row / a.Ho, ho = row - n * a.Ho;
      const bf16_t* grow = a.dy + ((long)row * a.Wo) * a.C + c;
      const bf16_t* xn = a.x + (long)n * a.H * a.W * a.C + c;
      for (int wo = pl; wo < a.Wo; wo += rpp) {
        float gv[8];
        unpack8(*(const uint4*)(grow + (long)wo * a.C), gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) db[j] += gv[j];
#pragma unroll
        for (int k = 0; k < RS; ++k) {
          const int r = k / a.S, s = k - r * a.S;
          const int hi = ho * a.sh - a.ph + r * a.dh, wi = wo * a.sw - a.pw + s * a.dwl;
          if ((unsigned)hi >= (unsigned)a.H || (unsigned)wi >= (unsigned)a.W) continue;
          float xv[8];
          uint4 xr = *(const uint4*)(xn + ((long)hi * a.W + wi) * a.C);
          if (a.relu_in) xr = relu8(xr);
          unpack8(xr, xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[k][j] += gv[j] * xv[j];
        }
      }
    }
  }
  __shared__ float red[NT][9];
  const long slab_w = (long)blockIdx.x * RS * a.C, slab_b = (long)blockIdx.x * a.C;
#pragma unroll
  for (int k = 0; k <= RS; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[t][j] = (k < RS) ? acc[k < RS ? k : 0][j] : db[j];
    __syncthreads();
    if (pl == 0 && cvi < cv) {
      float sum[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) sum[j] = 0.f;
      for (int q = 0; q < rpp; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) sum[j] += red[q * lanes_c + lc][j];
      float* dst = (k < RS) ? ws_w + slab_w + (long)k * a.C + c : ws_b + slab_b + c;
      *(float4*)dst = make_float4(sum[0], sum[1], sum[2], sum[3]);
      *(float4*)(dst + 4) = make_float4(sum[4], sum[5], sum[6], sum[7]);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Sliding-window kernels for the common 3×3 / stride 1 / dilation 1 case (Xception's separable
// convs, the preprocessing Laplacian's shape class).  The row kernels above load all 9 taps of
// every output pixel from the cache hierarchy (9 × 16 B per 16 B written: L1/TA-bound at ≈1/3
// of HBM bandwidth).  Here a lane walks a CONTIGUOUS run of output columns and keeps the 3×3
// input window in registers (packed bf16): each step loads only the 3 vectors of the new input
// column.  One kernel serves the forward and, with the filter rotated 180° (FLIP) and the
// complementary padding, the stride-1 dgrad:
//   out[h, w] = Σ_{r,s} in[h − P_h + r, w − P_w + s] · W[r, s]
// (dgrad: in = dy, P = 2 − pad, W[r, s] = w[2 − r, 2 − s]).
// ---------------------------------------------------------------------------------------------
template <bool FLIP>
__global__ void __launch_bounds__(NT) dw_slide_kernel(const bf16_t* __restrict__ in,
                                                      const bf16_t* __restrict__ wt,
                                                      const float* __restrict__ bias,
                                                      bf16_t* __restrict__ out, int Hi, int Wi,
                                                      int Ho, int Wo, int C, int Ph, int Pw,
                                                      int relu, int lanes_c, int rpp, int seg,
                                                      int relu_in,
                                                      const bf16_t* __restrict__ mask_x,
                                                      const bf16_t* __restrict__ dadd) {
  const int cv = C / 8;
  const int t = threadIdx.x, lc = t % lanes_c, pl = t / lanes_c;
  const int cvi = lc + blockIdx.y * lanes_c;
  if (pl >= rpp || cvi >= cv) return;
  const int c = cvi * 8;
  const int row = blockIdx.x, n = row / Ho, ho = row - n * Ho;
  const int w0 = pl * seg, w1 = min(Wo, w0 + seg);
  if (w0 >= w1) return;
  float wv[9][8], b[8];
#pragma unroll
  for (int k = 0; k < 9; ++k) unpack8(*(const uint4*)(wt + (long)(FLIP ? 8 - k : k) * C + c), wv[k]);
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = bias ? bias[c + j] : 0.f;
  const bf16_t* base = in + (long)n * Hi * Wi * C + c;
  int hi[3];
  bool hv[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    hi[r] = ho - Ph + r;
    hv[r] = (unsigned)hi[r] < (unsigned)Hi;
  }
  auto col = [&](int r, int wi) -> uint4 {
    if (!hv[r] || (unsigned)wi >= (unsigned)Wi) return make_uint4(0, 0, 0, 0);
    const uint4 v = *(const uint4*)(base + ((long)hi[r] * Wi + wi) * C);
    return relu_in ? relu8(v) : v;
  };
  // (no software prefetch here: the extra column pushes the kernel to 178 VGPRs and 2 waves per
  // SIMD, measured slower than 3 waves without it; the wgrad kernel below does gain from it)
  uint4 win[3][3];  // [row][column], packed bf16
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    win[r][1] = col(r, w0 - Pw);
    win[r][2] = col(r, w0 - Pw + 1);
  }
  bf16_t* orow = out + ((long)row * Wo) * C + c;
  for (int w = w0; w < w1; ++w) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      win[r][0] = win[r][1];
      win[r][1] = win[r][2];
      win[r][2] = col(r, w - Pw + 2);
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = b[j];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        float xv[8];
        unpack8(win[r][s], xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += xv[j] * wv[r * 3 + s][j];
      }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaxf(acc[j], 0.f);
    }
    if (mask_x) mask_pos(acc, mask_x + ((long)row * Wo + w) * C + c);
    if (dadd) add8(acc, dadd + ((long)row * Wo + w) * C + c);
    *(uint4*)(orow + (long)w * C) = pack8(acc);
  }
}

// The same sliding window with 4 channels per lane (8-B vectors) and the next column prefetched
// one step ahead: half the registers of the 8-channel kernel (≈ 70 VGPRs → ≥ 6 waves per SIMD)
// and a load in flight under every step's FMAs, so more bytes are in flight per CU; the block is
// sized to the active lanes (channel vectors × pixel lanes rounded up to a wave).
__device__ __forceinline__ void unpack4(const uint2& v, float* f) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 lo_hi(uint32_t v) {  // two bf16 → two fp32
  f32x2 r;
  r.x = __uint_as_float(v << 16);
  r.y = __uint_as_float(v & 0xffff0000u);
  return r;
}

template <bool FLIP>
__global__ void __launch_bounds__(NT) dw_slide4_kernel(const bf16_t* __restrict__ in,
                                                       const bf16_t* __restrict__ wt,
                                                       const float* __restrict__ bias,
                                                       bf16_t* __restrict__ out, int Hi, int Wi,
                                                       int Ho, int Wo, int C, int Ph, int Pw,
                                                       int relu, int lanes_c, int rpp, int seg,
                                                       int relu_in,
                                                       const bf16_t* __restrict__ mask_x,
                                                       const bf16_t* __restrict__ dadd) {
  // The window is kept unpacked (fp32 pairs), so a step converts only its new column, and the
  // FMAs run as packed fp32 pairs (v_pk_fma_f32).  (Measured alternatives, Xception-41 b128:
  // columns prefetched in blocks of 4 — 141 VGPRs, 3 waves — 2394 img/s; XCD-aware row order
  // 2471; both vs 2488 for this form.)
  const int cv = C / 4;
  const int t = threadIdx.x, lc = t % lanes_c, pb = t / lanes_c;
  const int cvi = lc + blockIdx.y * lanes_c;
  if (pb >= rpp || cvi >= cv) return;
  const int pl = blockIdx.z * rpp + pb;  // pixel lane of the row (blockIdx.z: lane group)
  const int c = cvi * 4;
  const int row = blockIdx.x, n = row / Ho, ho = row - n * Ho;
  const int w0 = pl * seg, w1 = min(Wo, w0 + seg);
  if (w0 >= w1) return;
  f32x2 wv[9][2], b[2];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const uint2 q = *(const uint2*)(wt + (long)(FLIP ? 8 - k : k) * C + c);
    wv[k][0] = lo_hi(q.x);
    wv[k][1] = lo_hi(q.y);
  }
  b[0] = bias ? f32x2{bias[c], bias[c + 1]} : f32x2{0.f, 0.f};
  b[1] = bias ? f32x2{bias[c + 2], bias[c + 3]} : f32x2{0.f, 0.f};
  const bf16_t* base = in + (long)n * Hi * Wi * C + c;
  int hi[3];
  bool hv[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    hi[r] = ho - Ph + r;
    hv[r] = (unsigned)hi[r] < (unsigned)Hi;
  }
  auto col = [&](int r, int wi) -> uint2 {
    if (!hv[r] || (unsigned)wi >= (unsigned)Wi) return make_uint2(0, 0);
    const uint2 v = *(const uint2*)(base + ((long)hi[r] * Wi + wi) * C);
    return relu_in ? make_uint2(relu2(v.x), relu2(v.y)) : v;
  };
  f32x2 win[3][3][2];  // [row][column][channel pair], fp32
  uint2 nxt[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const uint2 a1 = col(r, w0 - Pw), a2 = col(r, w0 - Pw + 1);
    win[r][1][0] = lo_hi(a1.x);
    win[r][1][1] = lo_hi(a1.y);
    win[r][2][0] = lo_hi(a2.x);
    win[r][2][1] = lo_hi(a2.y);
    nxt[r] = col(r, w0 - Pw + 2);
  }
  bf16_t* orow = out + ((long)row * Wo) * C + c;
#pragma unroll 3
  for (int w = w0; w < w1; ++w) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        win[r][0][h] = win[r][1][h];
        win[r][1][h] = win[r][2][h];
      }
      win[r][2][0] = lo_hi(nxt[r].x);
      win[r][2][1] = lo_hi(nxt[r].y);
      nxt[r] = col(r, w - Pw + 3);  // next step's column, in flight under this step's FMAs
    }
    f32x2 acc[2] = {b[0], b[1]};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          acc[h] = __builtin_elementwise_fma(win[r][s2][h], wv[r * 3 + s2][h], acc[h]);
    float o[4] = {acc[0].x, acc[0].y, acc[1].x, acc[1].y};
    if (relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    if (mask_x) {
      const uint2 m = *(const uint2*)(mask_x + ((long)row * Wo + w) * C + c);
      const f32x2 m0 = lo_hi(m.x), m1 = lo_hi(m.y);
      o[0] = m0.x > 0.f ? o[0] : 0.f;
      o[1] = m0.y > 0.f ? o[1] : 0.f;
      o[2] = m1.x > 0.f ? o[2] : 0.f;
      o[3] = m1.y > 0.f ? o[3] : 0.f;
    }
    if (dadd) {
      const uint2 d = *(const uint2*)(dadd + ((long)row * Wo + w) * C + c);
      const f32x2 d0 = lo_hi(d.x), d1 = lo_hi(d.y);
      o[0] += d0.x;
      o[1] += d0.y;
      o[2] += d1.x;
      o[3] += d1.y;
    }
    *(uint2*)(orow + (long)w * C) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
  }
}

// LDS-tiled depthwise 3×3 stride 1: a workgroup stages its (TR+2)×(TW+2) input pixels × 64
// channels once (LDS-DMA; with tiles up to the 64 KiB LDS bound ≈1.1–1.2× the tile's own bytes
// incl. halo), then every lane (4 channels × one output column) slides down the TR rows reading
// its 3×3 window from LDS.
// The register-window kernels above re-fetch each input row for 3 output-row workgroups from the
// fabric (PMC: 3.2× the input bytes); here the re-reads are LDS reads.
constexpr int DT_TW = 32, DT_CH = 64;

__device__ __forceinline__ void unpack4x2(const uint2& v, f32x2* f) {
  f[0] = lo_hi(v.x);
  f[1] = lo_hi(v.y);
}
__device__ __forceinline__ uint2 relu4(uint2 v) { return make_uint2(relu2(v.x), relu2(v.y)); }

constexpr int DT_NT = 512;  // tile-kernel workgroup cap (16 channel lanes × ≤ 32 columns)

// Stage one output tile's (tr+2)×(tw+2)-pixel × 64-channel input halo in LDS and (AFF) apply the
// folded input BN + ReLU to it in place — shared by the forward / input-gradient tile kernel and
// the weight-gradient tile kernel.
template <bool AFF>
__device__ __forceinline__ void dw_stage_tile(uint4* tile, const bf16_t* __restrict__ src, int Hi,
                                              int Wi, int C, int ih0, int iw0, int pitch,
                                              int chunks, int cg0, int t,
                                              const float* __restrict__ aff, int aff_ld) {
  // (ih0, iw0): the input pixel of the halo's top-left corner (may be negative: padding)
  // staging: LDS-DMA, one 1-KiB piece (64 lanes × 16 B, lane-linear in LDS) per wave instruction;
  // padding / ragged chunks read past the range-checked descriptor (zeros).  No per-chunk branch
  // around a load, so the pieces stream back-to-back instead of one latency each.
  {
    const rsrc_t rs = make_rsrc(src, (uint32_t)((long)Hi * Wi * C * 2));
    const int nwv = blockDim.x >> 6, ln = t & 63;
    for (int j = t >> 6; j * 64 < chunks; j += nwv) {
      const int i = j * 64 + ln, k = i & 7, pix = i >> 3;
      const int r = pix / pitch, cc = pix - r * pitch;
      const int hi = ih0 + r, wi = iw0 + cc, ch = cg0 + k * 8;
      const bool ok = i < chunks && (unsigned)hi < (unsigned)Hi && (unsigned)wi < (unsigned)Wi &&
                      ch < C;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)((char*)tile + j * 1024), 16,
                                               ok ? (uint32_t)(((hi * Wi + wi) * C + ch) * 2) : OOB,
                                               0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if constexpr (AFF) {
    // the input BN + ReLU folded in: u = relu(a·z + b), rounded to bf16 as the BN's apply pass
    // would store it, in place on the staged tile; out-of-image pixels keep the DMA's zeros (the
    // padding is zero in u, not relu(b))
    const int ch = cg0 + (t & 7) * 8;  // blockDim.x % 64 == 0: a thread's chunks share one group
    if (ch < C) {
      // (the coefficients are loaded per tile through a pointer the compiler cannot prove
      // invariant: hoisted out of the tile loop they held 16 VGPRs across the whole computation
      // and the kernel spilled at its 128-register budget)
      const float* ap = aff + ch;
      asm volatile("" : "+v"(ap));
      const float4 a0 = *(const float4*)ap, a1 = *(const float4*)(ap + 4);
      const float4 b0 = *(const float4*)(ap + aff_ld), b1 = *(const float4*)(ap + aff_ld + 4);
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      for (int i = t; i < chunks; i += blockDim.x) {
        const int pix = i >> 3, r = pix / pitch, cc = pix - r * pitch;
        const int hi = ih0 + r, wi = iw0 + cc;
        if ((unsigned)hi < (unsigned)Hi && (unsigned)wi < (unsigned)Wi) {
          float v[8];
          unpack8(tile[i], v);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = fmaxf(fmaf(v[j], av[j], bv[j]), 0.f);
          tile[i] = pack8(v);
        }
      }
    }
    __syncthreads();
  }
}

template <bool FLIP, bool RIN, bool AFF = false, int ST = 1>
__global__ void __launch_bounds__(DT_NT, 4) dw_tile_kernel(const bf16_t* __restrict__ in,
                                                        const bf16_t* __restrict__ wt,
                                                        const float* __restrict__ bias,
                                                        bf16_t* __restrict__ out, int Hi, int Wi,
                                                        int Ho, int Wo, int C, int Ph, int Pw,
                                                        int relu, int tr, int tw, int rg,
                                                        int tiles_h, int tiles_w,
                                                        const bf16_t* __restrict__ mask_x,
                                                        float* __restrict__ stats,
                                                        const bf16_t* __restrict__ bn_x, int ntiles,
                                                        const bf16_t* __restrict__ dadd,
                                                        const float* __restrict__ aff, int aff_ld) {
  // stats (optional, fp32 [2][C], accumulated): BN sums of the stored bf16 outputs — (Σy, Σy²)
  // for the BN that normalises this forward's output, or (Σg, Σg·bn_x) with bn_x the input of
  // the BN whose output gradient this dgrad produces (bn.hip red_raw) — so that BN skips its
  // separate reduce pass
  // tile: tr × tw output pixels (runtime: tw ≤ DT_TW, tr bounded by LDS, balanced splits); lanes:
  // 16 channel lanes (4 channels each) × tw column lanes × rg row groups (each slides over
  // ⌈tr / rg⌉ rows).  Four channels per lane keep the sliding window + taps at 72 fp32 registers
  // (8 per lane needed ≈170 VGPRs: 2 waves per SIMD, too few to hide the halo DMA latency).
  // A workgroup walks tiles blockIdx.x, +gridDim.x, … < ntiles (one tile per workgroup unless
  // the launcher caps the grid — with statistics, so each workgroup flushes its sums once).
  extern __shared__ uint4 tile[];  // dw_tile_smem(): the launch's halo tile (whole DMA pieces)
  const uint2* tile2 = (const uint2*)tile;
  const int t = threadIdx.x;
  const int cl = t & 15, rest = t >> 4, cg0 = blockIdx.y * DT_CH;
  float ss[4], sq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ss[j] = sq[j] = 0.f;
  for (int tb = blockIdx.x; tb < ntiles; tb += gridDim.x) {
  if (tb != (int)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
  int b = tb;
  const int tx = b % tiles_w;
  b /= tiles_w;
  const int ty = b % tiles_h;
  const int n = b / tiles_h;
  static_assert(ST == 1 || (ST == 2 && !FLIP), "stride 2: forward only");
  const int h0 = ty * tr, w0 = tx * tw;
  // the halo: (tr−1)·ST + 3 input rows × (tw−1)·ST + 3 columns
  const int pitch = (tw - 1) * ST + 3, chunks = ((tr - 1) * ST + 3) * pitch * 8;
  const bf16_t* src = in + (long)n * Hi * Wi * C;
  dw_stage_tile<!FLIP && AFF>(tile, src, Hi, Wi, C, h0 * ST - Ph, w0 * ST - Pw, pitch, chunks, cg0,
                              t, aff, aff_ld);
  const int pw = rest % tw, g = rest / tw;
  const int w = w0 + pw, c = cg0 + cl * 4;
  const int rpg = (tr + rg - 1) / rg, r0 = g * rpg;
  const int r1 = min(min(tr, r0 + rpg), Ho - h0);
  const bool active = !(g >= rg || w >= Wo || c >= C || r0 >= r1);
  // the fused input ReLU (RIN) is applied on the LDS read (the DMA stages raw values); a pixel's
  // 64 channels are 16 uint2 slots, this lane's 4 channels slot cl
  auto ldt = [&](int pix) { const uint2 v = tile2[pix * 16 + cl]; return RIN ? relu4(v) : v; };
  if (active) {
  f32x2 wv[9][2], bb[2];
#pragma unroll
  for (int k = 0; k < 9; ++k) unpack4x2(*(const uint2*)(wt + (long)(FLIP ? 8 - k : k) * C + c), wv[k]);
#pragma unroll
  for (int q = 0; q < 2; ++q)
    bb[q] = bias ? f32x2{bias[c + 2 * q], bias[c + 2 * q + 1]} : f32x2{0.f, 0.f};
  f32x2 win[3][3][2];
  const int pc = pw * ST;  // this lane's window columns pc … pc+2 of the halo
  if constexpr (ST == 1) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) unpack4x2(ldt((r0 + r) * pitch + pc + s2), win[r + 1][s2]);
  } else {
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) unpack4x2(ldt(r0 * ST * pitch + pc + s2), win[2][s2]);
  }
  for (int h = r0; h < r1; ++h) {
    // slide the window down to output row h (input rows h·ST … h·ST+2)
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) {
      if constexpr (ST == 1) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          win[0][s2][q] = win[1][s2][q];
          win[1][s2][q] = win[2][s2][q];
        }
        unpack4x2(ldt((h + 2) * pitch + pc + s2), win[2][s2]);
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) win[0][s2][q] = win[2][s2][q];
        unpack4x2(ldt((h * ST + 1) * pitch + pc + s2), win[1][s2]);
        unpack4x2(ldt((h * ST + 2) * pitch + pc + s2), win[2][s2]);
      }
    }
    f32x2 acc[2] = {bb[0], bb[1]};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2)
#pragma unroll
        for (int q = 0; q < 2; ++q)
          acc[q] = __builtin_elementwise_fma(win[r][s2][q], wv[r * 3 + s2][q], acc[q]);
    float o[4] = {acc[0].x, acc[0].y, acc[1].x, acc[1].y};
    if (relu) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    const long op = (((long)n * Ho + h0 + h) * Wo + w) * C + c;
    uint2 xb = make_uint2(0, 0);
    if constexpr (FLIP && AFF) {
      // folded input BN + ReLU: dx · [a·bn_x + b > 0] (bn_x = the BN input the forward staged)
      xb = *(const uint2*)(bn_x + op);
      const float* ap = aff + c;  // (re-read per row, not hoisted: see the forward's transform)
      asm volatile("" : "+v"(ap));
      const float4 ma = *(const float4*)ap, mb = *(const float4*)(ap + aff_ld);
      const f32x2 x0 = lo_hi(xb.x), x1 = lo_hi(xb.y);
      o[0] = fmaf(x0.x, ma.x, mb.x) > 0.f ? o[0] : 0.f;
      o[1] = fmaf(x0.y, ma.y, mb.y) > 0.f ? o[1] : 0.f;
      o[2] = fmaf(x1.x, ma.z, mb.z) > 0.f ? o[2] : 0.f;
      o[3] = fmaf(x1.y, ma.w, mb.w) > 0.f ? o[3] : 0.f;
    } else if (mask_x) {  // dx · [x > 0] for the fused input ReLU's backward
      const uint2 xm = *(const uint2*)(mask_x + op);
      const f32x2 x0 = lo_hi(xm.x), x1 = lo_hi(xm.y);
      o[0] = x0.x > 0.f ? o[0] : 0.f;
      o[1] = x0.y > 0.f ? o[1] : 0.f;
      o[2] = x1.x > 0.f ? o[2] : 0.f;
      o[3] = x1.y > 0.f ? o[3] : 0.f;
    }
    if (dadd) {  // residual-gradient join
      const uint2 d = *(const uint2*)(dadd + op);
      const f32x2 d0 = lo_hi(d.x), d1 = lo_hi(d.y);
      o[0] += d0.x;
      o[1] += d0.y;
      o[2] += d1.x;
      o[3] += d1.y;
    }
    const uint2 packed = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
    *(uint2*)(out + op) = packed;
    if (stats) {
      const f32x2 q0 = lo_hi(packed.x), q1 = lo_hi(packed.y);  // the stored bf16 values
      const float q[4] = {q0.x, q0.y, q1.x, q1.y};
      if (bn_x) {
        if constexpr (!(FLIP && AFF)) xb = *(const uint2*)(bn_x + op);
        const f32x2 x0 = lo_hi(xb.x), x1 = lo_hi(xb.y);
        const float xv[4] = {x0.x, x0.y, x1.x, x1.y};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ss[j] += q[j];
          sq[j] = fmaf(q[j], xv[j], sq[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ss[j] += q[j];
          sq[j] = fmaf(q[j], q[j], sq[j]);
        }
      }
    }
  }
  }
  }  // tiles
  if (stats) {
    // workgroup reduction over the lanes of each of the 64 channels (the LDS tile is free now),
    // then one atomic pair per channel
    __syncthreads();
    // layout [2][L lanes][64 channels]: a lane's 4 channels are one 16-B store and the summing
    // threads read consecutive channels (no bank conflicts either way)
    float* red = (float*)tile;
    const int L = blockDim.x >> 4;  // lanes per channel lane (≤ 32)
    *(float4*)(red + rest * 64 + cl * 4) = make_float4(ss[0], ss[1], ss[2], ss[3]);
    *(float4*)(red + (L + rest) * 64 + cl * 4) = make_float4(sq[0], sq[1], sq[2], sq[3]);
    __syncthreads();
    for (int o = t; o < 128; o += blockDim.x) {  // (64-thread workgroups for tiny images)
      const int which = o >> 6, ch = o & 63;
      float v = 0.f;
      for (int i = 0; i < L; ++i) v += red[(which * L + i) * 64 + ch];
      if (cg0 + ch < C) atomicAdd(stats + which * C + cg0 + ch, v);
    }
  }
}

// Weight gradient on the tile machinery: a workgroup walks output tiles (blockIdx.x, +gridDim.x,
// …), stages each tile's input halo in LDS exactly as the forward does (RIN: input ReLU on the LDS
// read; AFF: the folded BN + ReLU applied to the staged tile), and every lane (4 channels × one
// output column) slides down its rows with the 3×3 window in fp32 registers, accumulating
// dW[tap] += window[tap] · dy (18 packed FMAs per output row; dy read once, straight from global).
// Per workgroup one partial per (tap, channel): shuffles over the 4 column lanes of a wave that
// share a channel lane, then the waves through LDS, written to slab blockIdx.x (the caller's
// split-K reduce sums the slabs).  The sliding-window kernel below unpacks its packed window
// 9× per output (144 VALU per 8 channels per output vs ≈30 per 4 here).
template <bool RIN, bool AFF, int ST = 1>
__global__ void __launch_bounds__(DT_NT, 4) dw_wgrad_tile_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, int Hi, int Wi, int Ho, int Wo,
    int C, int Ph, int Pw, int tr, int tw, int rg, int tiles_h, int tiles_w, int ntiles,
    const float* __restrict__ aff, int aff_ld, float* __restrict__ ws_w, float* __restrict__ ws_b) {
  extern __shared__ uint4 tile[];
  const uint2* tile2 = (const uint2*)tile;
  const int t = threadIdx.x;
  const int cl = t & 15, rest = t >> 4, cg0 = blockIdx.y * DT_CH;
  f32x2 acc[9][2], dsum[2];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k][0] = acc[k][1] = f32x2{0.f, 0.f};
  dsum[0] = dsum[1] = f32x2{0.f, 0.f};
  for (int tb = blockIdx.x; tb < ntiles; tb += gridDim.x) {
    if (tb != (int)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
    int b = tb;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int n = b / tiles_h;
    const int h0 = ty * tr, w0 = tx * tw;
    const int pitch = (tw - 1) * ST + 3, chunks = ((tr - 1) * ST + 3) * pitch * 8;
    dw_stage_tile<AFF>(tile, x + (long)n * Hi * Wi * C, Hi, Wi, C, h0 * ST - Ph, w0 * ST - Pw, pitch,
                       chunks, cg0, t, aff, aff_ld);
    const int pw = rest % tw, g = rest / tw;
    const int w = w0 + pw, c = cg0 + cl * 4;
    const int rpg = (tr + rg - 1) / rg, r0 = g * rpg;
    const int r1 = min(min(tr, r0 + rpg), Ho - h0);
    if (g >= rg || w >= Wo || c >= C || r0 >= r1) continue;
    auto ldt = [&](int pix) { const uint2 v = tile2[pix * 16 + cl]; return RIN ? relu4(v) : v; };
    f32x2 win[3][3][2];
    const int pc = pw * ST;
    if constexpr (ST == 1) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) unpack4x2(ldt((r0 + r) * pitch + pc + s2), win[r + 1][s2]);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) unpack4x2(ldt(r0 * ST * pitch + pc + s2), win[2][s2]);
    }
    const bf16_t* gp = dy + (((long)n * Ho + h0) * Wo + w) * C + c;
    for (int h = r0; h < r1; ++h) {
      const uint2 gv = *(const uint2*)(gp + (long)h * Wo * C);
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        if constexpr (ST == 1) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            win[0][s2][q] = win[1][s2][q];
            win[1][s2][q] = win[2][s2][q];
          }
          unpack4x2(ldt((h + 2) * pitch + pc + s2), win[2][s2]);
        } else {
#pragma unroll
          for (int q = 0; q < 2; ++q) win[0][s2][q] = win[2][s2][q];
          unpack4x2(ldt((h * ST + 1) * pitch + pc + s2), win[1][s2]);
          unpack4x2(ldt((h * ST + 2) * pitch + pc + s2), win[2][s2]);
        }
      }
      f32x2 gf[2];
      unpack4x2(gv, gf);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            acc[r * 3 + s2][q] = __builtin_elementwise_fma(win[r][s2][q], gf[q], acc[r * 3 + s2][q]);
      dsum[0] = dsum[0] + gf[0];
      dsum[1] = dsum[1] + gf[1];
    }
  }
  // reduce over the lanes that share a channel lane: within a wave the 4 column lanes t, t^16,
  // t^32, t^48, then the waves through LDS (the staged tile is dead: reuse its space)
  __syncthreads();
  float* red = (float*)tile;  // [waves][16 channel lanes][40]
  const int wv = t >> 6, lane = t & 63, nwv = blockDim.x >> 6;
  float v[40];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    v[k * 4 + 0] = acc[k][0].x;
    v[k * 4 + 1] = acc[k][0].y;
    v[k * 4 + 2] = acc[k][1].x;
    v[k * 4 + 3] = acc[k][1].y;
  }
  v[36] = dsum[0].x;
  v[37] = dsum[0].y;
  v[38] = dsum[1].x;
  v[39] = dsum[1].y;
#pragma unroll
  for (int j = 0; j < 40; ++j) {
    v[j] += __shfl_xor(v[j], 16, 64);
    v[j] += __shfl_xor(v[j], 32, 64);
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 40; ++j) red[(wv * 16 + lane) * 40 + j] = v[j];
  }
  __syncthreads();
  const long slab = blockIdx.x;
  for (int i = t; i < 16 * 40; i += blockDim.x) {
    const int l = i / 40, j = i - l * 40;
    float sum = 0.f;
    for (int q = 0; q < nwv; ++q) sum += red[(q * 16 + l) * 40 + j];
    const int c = cg0 + l * 4 + (j & 3);
    if (c >= C) continue;
    if (j < 36)
      ws_w[(slab * 9 + (j >> 2)) * C + c] = sum;
    else if (ws_b)
      ws_b[slab * C + c] = sum;
  }
}

// tile-kernel grid (x): every tile its own workgroup, except with fused statistics — then
// ≈ TDL_DW_STAT_WG workgroups in all, each walking several tiles and flushing its sums once
// (one atomic pair per channel per workgroup instead of per tile)
int dw_tile_grid(int ntiles, int C, bool stats) {
  if (!stats) return ntiles;
  static const int target = [] {
    const char* e = getenv("TDL_DW_STAT_WG");
    return e ? std::max(1, atoi(e)) : 2048;
  }();
  const int cg = cdiv(C, DT_CH);
  return std::max(1, std::min(ntiles, cdiv(target, cg)));
}

// balanced tiling of an Ho × Wo output: tw ≤ 32 columns, tr as tall as the LDS bound allows,
// rg = 32 / tw row groups (≤ 16 · 32 = 512 threads)
struct DwTileGeom {
  int tr, tw, rg, th, twn, nt, st;
  // 1-KiB DMA pieces of the (tr−1)·st+3 × (tw−1)·st+3-pixel × 64-channel input halo
  long pieces() const { return cdiv(((tr - 1) * st + 3) * ((tw - 1) * st + 3) * 8, 64); }
};
DwTileGeom dw_tile_geom(int Ho, int Wo, int st = 1) {
  // rows per tile: as many as the 64 KiB LDS bound below allows (TDL_DW_TR caps it; 8 was the
  // round-4 default — Xception b128 shapes 10–14 % faster with taller tiles: fewer halo re-reads
  // per output, and the workgroups per CU are LDS-bound either way, dev/tools/dw_micro.py)
  static const int tr_max = [] {
    const char* e = getenv("TDL_DW_TR");
    return e ? std::max(1, std::min(32, atoi(e))) : 32;
  }();
  DwTileGeom g;
  g.st = st;
  g.twn = cdiv(Wo, DT_TW / st);  // stride 2: ≤ 16 output columns (33 input columns) per tile
  g.tw = cdiv(Wo, g.twn);
  g.th = cdiv(Ho, tr_max);
  g.tr = cdiv(Ho, g.th);
  // the halo tile within the 64 KiB of dynamic LDS a launch gets without an attribute
  while (g.tr > 1 && g.pieces() * 1024 > 65536) {
    ++g.th;
    g.tr = cdiv(Ho, g.th);
  }
  g.rg = std::max(1, std::min(DT_TW / g.tw, g.tr));
  g.nt = cdiv(16 * g.tw * g.rg, 64) * 64;
  return g;
}

// dynamic LDS of a tile launch: the (tr+2)×(tw+2)×64-channel halo in whole 1-KiB DMA pieces (or
// the statistics reduction's 128 × lanes floats) — sized to the launch, not the largest tile, so
// small-image layers fit more workgroups per CU (56 KiB for a whole 19×19 image)
size_t dw_tile_smem(const DwTileGeom& g, bool stats) {
  const size_t halo = (size_t)g.pieces() * 1024;
  const size_t red = stats ? (size_t)128 * (g.nt / 16) * 4 : 0;
  return std::max(halo, red);
}

// wgrad with the same sliding window over x: a lane walks a contiguous run of output columns of
// each of its workgroup's rows; per output pixel one dy vector + the 3 vectors of the new x column.
__global__ void __launch_bounds__(NT) dw_wgrad_slide(DwArgs a, int lanes_c, int rpp, int seg,
                                                     int rows_per_block, float* ws_w, float* ws_b) {
  const int cv = a.C / 8;
  const int t = threadIdx.x, lc = t % lanes_c, pl = t / lanes_c;
  const int cvi = lc + blockIdx.y * lanes_c;
  const bool active = pl < rpp && cvi < cv;
  const int c = cvi * 8;
  const int rows = a.N * a.Ho;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  const int w0 = pl * seg, w1 = min(a.Wo, w0 + seg);
  float acc[9][8], db[8];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) db[j] = 0.f;
  float av[8], bv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) av[j] = bv[j] = 0.f;
  if (active && a.aff) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      av[j] = a.aff[c + j];
      bv[j] = a.aff[a.aff_ld + c + j];
    }
  }
  if (active && w0 < w1) {
    for (int row = r0; row < r1; ++row) {
      const int n = row / a.Ho, ho = row - n * a.Ho;
      const bf16_t* grow = a.dy + ((long)row * a.Wo) * a.C + c;
      const bf16_t* xn = a.x + (long)n * a.H * a.W * a.C + c;
      int hi[3];
      bool hv[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        hi[r] = ho - a.ph + r;
        hv[r] = (unsigned)hi[r] < (unsigned)a.H;
      }
      auto col = [&](int r, int wi) -> uint4 {
        if (!hv[r] || (unsigned)wi >= (unsigned)a.W) return make_uint4(0, 0, 0, 0);
        const uint4 v = *(const uint4*)(xn + ((long)hi[r] * a.W + wi) * a.C);
        if (a.aff) {  // folded input BN + ReLU (bf16-rounded as the forward's staged u)
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], av[j], bv[j]), 0.f);
          return pack8(f);
        }
        return a.relu_in ? relu8(v) : v;
      };
      uint4 win[3][3], nxt[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        win[r][1] = col(r, w0 - a.pw);
        win[r][2] = col(r, w0 - a.pw + 1);
        nxt[r] = col(r, w0 - a.pw + 2);
      }
      uint4 gnext = *(const uint4*)(grow + (long)w0 * a.C);
      for (int wo = w0; wo < w1; ++wo) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          win[r][0] = win[r][1];
          win[r][1] = win[r][2];
          win[r][2] = nxt[r];
        }
        const uint4 gcur = gnext;
        if (wo + 1 < w1) {  // next column's x and dy loads in flight under this column's FMAs
#pragma unroll
          for (int r = 0; r < 3; ++r) nxt[r] = col(r, wo - a.pw + 3);
          gnext = *(const uint4*)(grow + (long)(wo + 1) * a.C);
        }
        float gv[8];
        unpack8(gcur, gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) db[j] += gv[j];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            float xv[8];
            unpack8(win[r][s], xv);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[r * 3 + s][j] += gv[j] * xv[j];
          }
      }
    }
  }
  __shared__ float red[NT][9];
  const long slab_w = (long)blockIdx.x * 9 * a.C, slab_b = (long)blockIdx.x * a.C;
#pragma unroll
  for (int k = 0; k <= 9; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[t][j] = (k < 9) ? acc[k < 9 ? k : 0][j] : db[j];
    __syncthreads();
    if (pl == 0 && cvi < cv) {
      float sum[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) sum[j] = 0.f;
      for (int q = 0; q < rpp; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) sum[j] += red[q * lanes_c + lc][j];
      float* dst = (k < 9) ? ws_w + slab_w + (long)k * a.C + c : ws_b + slab_b + c;
      *(float4*)dst = make_float4(sum[0], sum[1], sum[2], sum[3]);
      *(float4*)(dst + 4) = make_float4(sum[4], sum[5], sum[6], sum[7]);
    }
    __syncthreads();
  }
}

// the sliding-window path: 3×3, stride 1, dilation 1, C % 8 == 0, and the padding keeps every
// window inside [−2, W + 1] (0 ≤ pad ≤ 2)
bool slide_ok(const DwArgs& a) {
  return a.C % 8 == 0 && a.R == 3 && a.S == 3 && a.sh == 1 && a.sw == 1 && a.dh == 1 &&
         a.dwl == 1 && a.ph >= 0 && a.ph <= 2 && a.pw >= 0 && a.pw <= 2 &&
         getenv("TDL_DW_SLIDE_OFF") == nullptr;
}

// lanes: channel vectors × pixel lanes; each pixel lane owns ⌈W / rpp⌉ consecutive columns
struct SlideGeom {
  int lanes_c, rpp, seg;
};
// LDS-tiled kernel (default; TDL_DW_TILE=0 falls back to the sliding-window kernels)
bool dw_tile() {
  static const int v = [] {
    const char* e = getenv("TDL_DW_TILE");
    return e ? atoi(e) : 1;
  }();
  return v != 0;
}
// the tile kernel's DMA offsets are 32-bit bytes within one image
bool dw_tile_fits(long h, long w, long c) { return h * w * c * 2 < (1L << 31) - 64; }
// stride-2 3×3 on the tile kernels (forward, weight gradient); TDL_DW_S2_TILE=0: the row kernels
// (read per call: dev/tools/dw_micro.py A/Bs in-process)
bool s2_tile_ok(const DwArgs& a) {
  const char* e = getenv("TDL_DW_S2_TILE");
  return (e == nullptr || atoi(e) != 0) && a.C % 8 == 0 && a.R == 3 && a.S == 3 && a.sh == 2 &&
         a.sw == 2 && a.dh == 1 && a.dwl == 1 && a.ph >= 0 && a.ph <= 2 && a.pw >= 0 &&
         a.pw <= 2 && dw_tile() && dw_tile_fits(a.H, a.W, a.C);
}

// 4-channel sliding kernel (default; TDL_DW_VEC=8 selects the 8-channel one)
bool slide4() {
  static const int v = [] {
    const char* e = getenv("TDL_DW_VEC");
    return e ? atoi(e) : 4;
  }();
  return v == 4;
}

// 4-channel kernel: TDL_DW_SEG > 0 spreads a row's pixel lanes over blockIdx.z so that each
// lane's run is ≈ that many columns.  Default 0 (one block's lanes per row): measured on
// Xception-41, runs of 2 / 4 / 8 columns lose to whole-row runs (2278 / 2402 / 2448 vs 2489
// img/s) — the 2 warm-up columns each run loads cost more than the shorter dependency chain.
struct Slide4Geom {
  int lanes_c, rpp, seg, gz, nt;
};
Slide4Geom slide4_geom(int cv, int W) {
  static const int target = [] {
    const char* e = getenv("TDL_DW_SEG");
    return e ? atoi(e) : 0;
  }();
  Slide4Geom g;
  g.lanes_c = std::min(cv, NT);
  g.rpp = std::max(1, std::min(NT / g.lanes_c, W));
  const int lanes = target > 0 ? std::max(1, cdiv(W, target)) : g.rpp;
  g.gz = std::max(1, cdiv(lanes, g.rpp));
  g.rpp = cdiv(lanes, g.gz);
  g.seg = cdiv(W, g.rpp * g.gz);
  g.nt = cdiv(g.lanes_c * g.rpp, 64) * 64;
  return g;
}

SlideGeom slide_geom(int cv, int W) {
  SlideGeom g;
  g.lanes_c = std::min(cv, NT);
  g.rpp = std::max(1, std::min(NT / g.lanes_c, W));
  g.seg = cdiv(W, g.rpp);
  g.rpp = cdiv(W, g.seg);
  return g;
}

template <int V>
void wgrad_dispatch(const DwArgs& a, hipStream_t st) {
  const int cv = a.C / V;
  const int lanes_c = std::min(cv, NT);
  const int rpp = NT / lanes_c;
  const long P = (long)a.N * a.Ho * a.Wo;
  long blocks = std::min<long>(1024, std::max<long>(1, P / (rpp * 8)));
  const long ppb = (P + blocks - 1) / blocks;
  blocks = (P + ppb - 1) / ppb;
  dim3 grid((unsigned)blocks, (unsigned)((cv + lanes_c - 1) / lanes_c));
  const int RS = a.R * a.S;
  if (RS == 9)
    hipLaunchKernelGGL((dw_wgrad_kernel<V, 9>), grid, dim3(NT), 0, st, a, ppb);
  else if (RS == 1)
    hipLaunchKernelGGL((dw_wgrad_kernel<V, 1>), grid, dim3(NT), 0, st, a, ppb);
  else if (RS <= 25 && V == 1)
    hipLaunchKernelGGL((dw_wgrad_kernel<1, 25>), grid, dim3(NT), 0, st, a, ppb);
  else if (V == 1)
    hipLaunchKernelGGL((dw_wgrad_kernel<1, 49>), grid, dim3(NT), 0, st, a, ppb);
}

}  // namespace

// the kernels that implement DwArgs::aff: stride-1 3×3 on the LDS tile kernels (fwd / dgrad) and
// the sliding weight-gradient kernel
bool dwconv_aff_ok(const DwArgs& a) {
  return slide_ok(a) && dw_tile() && dw_tile_fits(a.H, a.W, a.C) &&
         dw_tile_fits(a.Ho, a.Wo, a.C) && dwconv_wgrad_slabs(a) > 0;
}

bool dwconv_fwd_launch(const DwArgs& a, hipStream_t st) {
  const long outs = (long)a.N * a.Ho * a.Wo * a.C;
  if (slide_ok(a) && dw_tile() && dw_tile_fits(a.H, a.W, a.C)) {
    const DwTileGeom g = dw_tile_geom(a.Ho, a.Wo);
    const int ntiles = a.N * g.th * g.twn;
    dim3 grid((unsigned)dw_tile_grid(ntiles, a.C, a.stats != nullptr), (unsigned)cdiv(a.C, DT_CH));
    auto kern = a.aff ? dw_tile_kernel<false, false, true>
                : a.relu_in ? dw_tile_kernel<false, true> : dw_tile_kernel<false, false>;
    hipLaunchKernelGGL(kern, grid, dim3(g.nt), dw_tile_smem(g, a.stats != nullptr),
                       st, a.x, a.w, a.bias, a.out,
                       a.H, a.W, a.Ho, a.Wo, a.C, a.ph, a.pw, a.relu, g.tr, g.tw, g.rg, g.th,
                       g.twn, (const bf16_t*)nullptr, a.stats, (const bf16_t*)nullptr,
                       ntiles, (const bf16_t*)nullptr, a.aff, a.aff_ld);
    return a.stats != nullptr;
  } else if (slide_ok(a) && slide4()) {
    const Slide4Geom g = slide4_geom(a.C / 4, a.Wo);
    dim3 grid((unsigned)(a.N * a.Ho), (unsigned)cdiv(a.C / 4, g.lanes_c), (unsigned)g.gz);
    hipLaunchKernelGGL(dw_slide4_kernel<false>, grid, dim3(g.nt), 0, st, a.x, a.w, a.bias, a.out,
                       a.H, a.W, a.Ho, a.Wo, a.C, a.ph, a.pw, a.relu, g.lanes_c, g.rpp, g.seg,
                       a.relu_in, (const bf16_t*)nullptr, (const bf16_t*)nullptr);
  } else if (slide_ok(a)) {
    const SlideGeom g = slide_geom(a.C / 8, a.Wo);
    dim3 grid((unsigned)(a.N * a.Ho), (unsigned)cdiv(a.C / 8, g.lanes_c));
    hipLaunchKernelGGL(dw_slide_kernel<false>, grid, dim3(NT), 0, st, a.x, a.w, a.bias, a.out, a.H,
                       a.W, a.Ho, a.Wo, a.C, a.ph, a.pw, a.relu, g.lanes_c, g.rpp, g.seg, a.relu_in,
                       (const bf16_t*)nullptr, (const bf16_t*)nullptr);
  } else if (s2_tile_ok(a) && !a.aff) {
    const DwTileGeom g = dw_tile_geom(a.Ho, a.Wo, 2);
    const int ntiles = a.N * g.th * g.twn;
    dim3 grid((unsigned)dw_tile_grid(ntiles, a.C, a.stats != nullptr), (unsigned)cdiv(a.C, DT_CH));
    auto kern = a.relu_in ? dw_tile_kernel<false, true, false, 2> : dw_tile_kernel<false, false, false, 2>;
    hipLaunchKernelGGL(kern, grid, dim3(g.nt), dw_tile_smem(g, a.stats != nullptr),
                       st, a.x, a.w, a.bias, a.out,
                       a.H, a.W, a.Ho, a.Wo, a.C, a.ph, a.pw, a.relu, g.tr, g.tw, g.rg, g.th,
                       g.twn, (const bf16_t*)nullptr, a.stats, (const bf16_t*)nullptr,
                       ntiles, (const bf16_t*)nullptr, (const float*)nullptr, 0);
    return a.stats != nullptr;
  } else if (a.C % 8 == 0 && a.R * a.S == 9) {
    const RowGeom g = row_geom(a.C / 8);
    dim3 grid((unsigned)(a.N * a.Ho), (unsigned)cdiv(a.C / 8, g.lanes_c));
    hipLaunchKernelGGL(dw_fwd_rows<9>, grid, dim3(NT), 0, st, a, g.lanes_c, g.rpp);
  } else if (a.C % 8 == 0) {
    hipLaunchKernelGGL(dw_fwd_kernel<8>, dim3(blocks_for(outs / 8)), dim3(NT), 0, st, a);
  } else {
    hipLaunchKernelGGL(dw_fwd_kernel<1>, dim3(blocks_for(outs)), dim3(NT), 0, st, a);
  }
  return false;
}

bool dwconv_dgrad_launch(const DwArgs& a, hipStream_t st) {
  const long ins = (long)a.N * a.H * a.W * a.C;
  if (slide_ok(a) && dw_tile() && dw_tile_fits(a.Ho, a.Wo, a.C)) {  // stride-1 dgrad = fwd of dy, rotated filter, padding 2 − p
    const DwTileGeom g = dw_tile_geom(a.H, a.W);
    const int ntiles = a.N * g.th * g.twn;
    dim3 grid((unsigned)dw_tile_grid(ntiles, a.C, a.stats != nullptr), (unsigned)cdiv(a.C, DT_CH));
    auto kern = a.aff ? dw_tile_kernel<true, false, true> : dw_tile_kernel<true, false>;
    hipLaunchKernelGGL(kern, grid, dim3(g.nt),
                       dw_tile_smem(g, a.stats != nullptr), st, a.dy, a.w, nullptr, a.out,
                       a.Ho, a.Wo, a.H, a.W, a.C, 2 - a.ph, 2 - a.pw, 0, g.tr, g.tw, g.rg, g.th,
                       g.twn, a.mask_x, a.stats, a.bn_x, ntiles, a.dadd, a.aff, a.aff_ld);
    return a.stats != nullptr;
  } else if (slide_ok(a) && slide4()) {  // stride-1 dgrad = fwd of dy, rotated filter, padding 2 − p
    const Slide4Geom g = slide4_geom(a.C / 4, a.W);
    dim3 grid((unsigned)(a.N * a.H), (unsigned)cdiv(a.C / 4, g.lanes_c), (unsigned)g.gz);
    hipLaunchKernelGGL(dw_slide4_kernel<true>, grid, dim3(g.nt), 0, st, a.dy, a.w, nullptr, a.out,
                       a.Ho, a.Wo, a.H, a.W, a.C, 2 - a.ph, 2 - a.pw, 0, g.lanes_c, g.rpp, g.seg,
                       0, a.mask_x, a.dadd);
  } else if (slide_ok(a)) {  // stride-1 dgrad = forward of dy with the rotated filter, padding 2 − p
    const SlideGeom g = slide_geom(a.C / 8, a.W);
    dim3 grid((unsigned)(a.N * a.H), (unsigned)cdiv(a.C / 8, g.lanes_c));
    hipLaunchKernelGGL(dw_slide_kernel<true>, grid, dim3(NT), 0, st, a.dy, a.w, nullptr, a.out,
                       a.Ho, a.Wo, a.H, a.W, a.C, 2 - a.ph, 2 - a.pw, 0, g.lanes_c, g.rpp, g.seg, 0,
                       a.mask_x, a.dadd);
  } else if (a.C % 8 == 0 && a.R == 3 && a.S == 3 && a.sh == 2 && a.sw == 2 && a.dh == 1 &&
             a.dwl == 1 && a.ph >= 0 && a.pw >= 0 && a.ph <= 2 && a.pw <= 2 &&
             (long)a.N * a.Ho * a.Wo * a.C * 2 < (1L << 31) - 64 &&
             getenv("TDL_DW_S2_OFF") == nullptr) {
    // stride-2 3×3: one lane per 2×2 dx block (groups cover rows −ph … H−1 and columns −pw … W−1)
    const int MG = (a.H + a.ph + 1) / 2, NG = (a.W + a.pw + 1) / 2;
    const long work = (long)a.N * MG * NG * (a.C / 8);
    hipLaunchKernelGGL(dw_dgrad_s2_kernel, dim3((unsigned)std::min<long>(65536, cdiv(work, NT))),
                       dim3(NT), 0, st, a.dy, a.w, a.out, a.mask_x, a.dadd, a.N, a.H, a.W, a.C,
                       a.Ho, a.Wo, a.ph, a.pw, MG, NG);
  } else if (a.C % 8 == 0 && a.R * a.S == 9) {
    const RowGeom g = row_geom(a.C / 8);
    dim3 grid((unsigned)(a.N * a.H), (unsigned)cdiv(a.C / 8, g.lanes_c));
    hipLaunchKernelGGL(dw_dgrad_rows<9>, grid, dim3(NT), 0, st, a, g.lanes_c, g.rpp);
  } else if (a.C % 8 == 0) {
    hipLaunchKernelGGL(dw_dgrad_kernel<8>, dim3(blocks_for(ins / 8)), dim3(NT), 0, st, a);
  } else {
    hipLaunchKernelGGL(dw_dgrad_kernel<1>, dim3(blocks_for(ins)), dim3(NT), 0, st, a);
  }
  return false;
}

// slab rows for the row-oriented wgrad (0: generic atomic kernel)
// the tile weight gradient (stride-1 3×3, like the forward tile kernel; TDL_DW_WG_TILE=0: the
// sliding-window kernel): one slab per workgroup, ≈2048 workgroups
namespace {
bool dw_wgrad_tile_ok(const DwArgs& a) {
  const char* e = getenv("TDL_DW_WG_TILE");  // (read per call: dev/tools/dw_micro.py A/Bs in-process)
  const bool on = e == nullptr || atoi(e) != 0;
  return on && ((slide_ok(a) && dw_tile() && dw_tile_fits(a.H, a.W, a.C) &&
                 dw_tile_fits(a.Ho, a.Wo, a.C)) ||
                (s2_tile_ok(a) && !a.aff));
}
int dw_wgrad_tile_grid(const DwArgs& a) {
  const DwTileGeom g = dw_tile_geom(a.Ho, a.Wo, a.sh);
  const int ntiles = a.N * g.th * g.twn;
  return std::max(1, std::min(ntiles, cdiv(2048, cdiv(a.C, DT_CH))));
}
}  // namespace

int dwconv_wgrad_slabs(const DwArgs& a) {
  if (!(a.C % 8 == 0 && a.R * a.S == 9)) return 0;
  if (dw_wgrad_tile_ok(a)) return dw_wgrad_tile_grid(a);
  const int rows = a.N * a.Ho;
  const RowGeom g = row_geom(a.C / 8);
  const int groups = cdiv(a.C / 8, g.lanes_c);
  const int target = std::max(1, 1024 / groups);  // ≈4 workgroups per CU
  const int rpb = std::max(1, cdiv(rows, target));
  return cdiv(rows, rpb);
}

void dwconv_wgrad_launch(const DwArgs& a, float* ws, hipStream_t st) {
  if (a.R * a.S > 49) return;  // host checks reject this
  const int slabs = dwconv_wgrad_slabs(a);
  if (slabs > 0 && ws != nullptr) {
    const RowGeom g = row_geom(a.C / 8);
    const int rows = a.N * a.Ho;
    const int rpb = cdiv(rows, slabs);
    dim3 grid((unsigned)slabs, (unsigned)cdiv(a.C / 8, g.lanes_c));
    float* ws_w = ws;
    float* ws_b = ws + (long)slabs * 9 * a.C;
    if (dw_wgrad_tile_ok(a)) {
      const DwTileGeom tg = dw_tile_geom(a.Ho, a.Wo, a.sh);
      const int ntiles = a.N * tg.th * tg.twn;
      const size_t smem = std::max(dw_tile_smem(tg, false), (size_t)(tg.nt / 64) * 16 * 40 * 4);
      auto k = a.sh == 2 ? (a.relu_in ? dw_wgrad_tile_kernel<true, false, 2>
                                      : dw_wgrad_tile_kernel<false, false, 2>)
               : a.aff ? dw_wgrad_tile_kernel<false, true>
               : a.relu_in ? dw_wgrad_tile_kernel<true, false> : dw_wgrad_tile_kernel<false, false>;
      hipLaunchKernelGGL(k, dim3((unsigned)slabs, (unsigned)cdiv(a.C, DT_CH)), dim3(tg.nt), smem, st,
                         a.x, a.dy, a.H, a.W, a.Ho, a.Wo, a.C, a.ph, a.pw, tg.tr, tg.tw, tg.rg,
                         tg.th, tg.twn, ntiles, a.aff, a.aff_ld, ws_w, a.db ? ws_b : nullptr);
    } else if (slide_ok(a)) {
      const SlideGeom sg = slide_geom(a.C / 8, a.Wo);
      hipLaunchKernelGGL(dw_wgrad_slide, grid, dim3(NT), 0, st, a, sg.lanes_c, sg.rpp, sg.seg, rpb,
                         ws_w, ws_b);
    } else {
      hipLaunchKernelGGL(dw_wgrad_rows<9>, grid, dim3(NT), 0, st, a, g.lanes_c, g.rpp, rpb, ws_w,
                         ws_b);
    }
    splitk_reduce_launch(ws_w, a.dw, 9L * a.C, slabs, a.accum != 0, st);
    if (a.db) splitk_reduce_launch(ws_b, a.db, a.C, slabs, a.accum != 0, st);
    return;
  }
  if (!a.accum) {  // the atomic kernels accumulate: overwrite = clear first
    (void)hipMemsetAsync(a.dw, 0, sizeof(float) * a.R * a.S * a.C, st);
    if (a.db) (void)hipMemsetAsync(a.db, 0, sizeof(float) * a.C, st);
  }
  if (a.C % 8 == 0 && (a.R * a.S == 9 || a.R * a.S == 1))
    wgrad_dispatch<8>(a, st);
  else
    wgrad_dispatch<1>(a, st);
}

}  // namespace tdl
