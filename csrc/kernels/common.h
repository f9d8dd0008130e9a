// Shared device helpers for the gfx950 (CDNA4, wave64) kernels of tensorflowdistributedlearning_amd.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

namespace tdl {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even; keeps NaN a NaN (hipcc lowers the cast to v_cvt_pk_bf16_f32)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// two floats → packed bf16 pair (round-to-nearest-even) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  const bf16x2 h = __builtin_convertvector((f32x2){a, b}, bf16x2);
  return __builtin_bit_cast(uint32_t, h);
}

// ReLU of a packed bf16 pair in one v_pk_max_i16: a bf16 is negative iff its int16 bit pattern
// is (−0 → +0; a NaN with the sign bit set → 0)
__device__ __forceinline__ uint32_t relu_pk_bf16(uint32_t v) {
  const s16x2 x = __builtin_bit_cast(s16x2, v);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, (s16x2){0, 0}));
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// element-type-generic 8-vector / scalar access (bf16 storage or the fp32 path): kernels that are
// pure data movement (pooling, upsample) are templated on the storage type through these
__device__ __forceinline__ void load8(const bf16_t* p, float* f) { unpack8(*(const uint4*)p, f); }
__device__ __forceinline__ void load8(const float* p, float* f) {
  const float4 a = ((const float4*)p)[0], b = ((const float4*)p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void store8(bf16_t* p, const float* f) { *(uint4*)p = pack8(f); }
__device__ __forceinline__ void store8(float* p, const float* f) {
  ((float4*)p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  ((float4*)p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}
__device__ __forceinline__ float load1(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float load1(const float* p) { return *p; }
__device__ __forceinline__ void store1(bf16_t* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void store1(float* p, float v) { *p = v; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Device-side |x|max for fp8 scaling.  A single float hit by one atomic per wave serialises in
// L2 (~10 ns each: 8k waves ≈ 90 µs), so a "slot" is AMAX_SPREAD partial maxima 256 B apart
// (different L2 channels); each workgroup reduces in LDS and issues one atomicMax to the partial
// blockIdx % AMAX_SPREAD.  Readers max the partials (one load per lane).  A delayed-scaling ring
// is 3 slots: read slot p (previous call), accumulate into p+1, clear p+2 for the next call.

// all threads of the block must call it (contains __syncthreads); v ≥ 0
__device__ __forceinline__ void amax_publish(float* slot, float v) {
  __shared__ float red[16];
  v = wave_max(v);
  const int nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = red[0];
    for (int w = 1; w < nw; ++w) b = fmaxf(b, red[w]);
    if (b > 0.f)
      atomicMax((unsigned int*)(slot + (blockIdx.x % AMAX_SPREAD) * AMAX_STRIDE), __float_as_uint(b));
  }
}

__device__ __forceinline__ float amax_read(const float* slot) {
  const int l = threadIdx.x & 63;
  return wave_max(l < AMAX_SPREAD ? slot[l * AMAX_STRIDE] : 0.f);
}

__device__ __forceinline__ void amax_clear(float* slot) {
  if (blockIdx.x == 0 && threadIdx.x < AMAX_SPREAD) slot[threadIdx.x * AMAX_STRIDE] = 0.f;
}

// XCD-aware bijective remap of a linear workgroup id (MI355X: 8 XCDs, blocks dealt round robin;
// give each XCD a contiguous range of tiles so neighbouring tiles share an L2) — guide §5.5 T1.
__device__ __forceinline__ int xcd_remap(int id, int nwg) {
  if (nwg < 16) return id;
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = id % 8, local = id / 8;
  const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + local;
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace tdl
