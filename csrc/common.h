// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of the edge split-inference framework.
// Everything here assumes wave64 and bf16 storage as raw 16-bit words.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define EDGE_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;   // MFMA A/B fragment (4 VGPRs)
typedef __attribute__((ext_vector_type(4))) float f32x4_t;      // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16_t;    // 32x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;     // packed-f32 VALU operands (v_pk_mul/add/fma_f32)

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// ---- fp32 execution by split-bf16 MFMA ("x6") -------------------------------------------------------------
// x = x0 + x1 + x2 exactly, each a bf16 (8 significant bits; the residual after two round-to-nearest steps has at
// most 8 significant bits left).  A product x*y is then sum_{i+j<=2} xi*yj up to terms of relative size 2^-27,
// below fp32's own rounding (2^-24), and every bf16 x bf16 product is exact in the fp32 MFMA accumulator.
// The six terms are a K-concatenation, so an ordinary bf16 MFMA GEMM over K' = 6K computes the fp32-accurate
// product with the K-blocks  A' = [a2 | a0 | a1 | a1 | a0 | a0],  B' = [b0 | b2 | b1 | b0 | b1 | b0]
// (the small terms first: they are accumulated before the large ones).  Weights are stored as B' [N, 6K]; an
// activation is stored once per plane, [a0 | a1 | a2] ([rows, 3K], half the bytes of A'), and the GEMM's A loader
// reads K-block j of A' from plane x6_aplane(j) (x6_acol).
constexpr int X6_TERMS = 6;
__device__ __forceinline__ void split3(float x, float& p0, float& p1, float& p2) {
  p0 = (float)(__bf16)x;
  const float r = x - p0;
  p1 = (float)(__bf16)r;
  p2 = (float)(__bf16)(r - p1);
}
// column of the 3-plane activation row holding column kp of A' (K = plane width; K-blocks never straddle a K-tile)
__device__ __forceinline__ int x6_acol(int kp, int K) {
  const int j = kp / K;                          // A' block 0..5, planes 2 0 1 1 0 0
  return ((0x1102 >> (4 * j)) & 3) * K + (kp - j * K);
}
// Store 4 consecutive values v[0..3] at column `col` of an X6 activation row (plane width K): three 8-byte stores.
__device__ __forceinline__ void store_x6_4(bf16_t* __restrict__ row, int K, int col, const float (&v)[4]) {
  float p[3][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split3(v[e], p[0][e], p[1][e], p[2][e]);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    u32x2_t w;
    w[0] = pack_bf2(p[i][0], p[i][1]);
    w[1] = pack_bf2(p[i][2], p[i][3]);
    *(u32x2_t*)(row + i * (size_t)K + col) = w;
  }
}
// 8 consecutive values: three 16-byte stores.
__device__ __forceinline__ void store_x6_8(bf16_t* __restrict__ row, int K, int col, const float (&v)[8]) {
  float p[3][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) split3(v[e], p[0][e], p[1][e], p[2][e]);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    u32x4_t w;
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = pack_bf2(p[i][2 * e], p[i][2 * e + 1]);
    *(u32x4_t*)(row + i * (size_t)K + col) = w;
  }
}

// silu(x) = x / (1 + e^-x) on the hardware transcendentals (v_exp_f32, v_rcp_f32, ~1 ulp): a plain '/' compiles
// to the IEEE division sequence (2 v_div_scale + v_div_fmas + v_div_fixup + v_rcp + FMAs), which made the
// SwiGLU epilogue of the gate/up GEMM cost ~20 VALU per output.  Saturates correctly: e^-x = inf -> 0.
__device__ __forceinline__ float fast_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float fast_silu(float x) { return x * fast_sigmoid(x); }

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

// Block-wide sum for blockDim.x == NT (multiple of 64).  `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  // global -> LDS DMA, 16 B per lane; LDS destination = wave-uniform base + lane*16.
  __builtin_amdgcn_global_load_lds(gsrc, LDS_PTR(lds_wave_base), 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Bijective XCD-aware remap of a linear workgroup id (8 XCDs): consecutive logical ids land on one XCD.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

#define HIP_RET(expr)                       \
  do {                                      \
    hipError_t _e = (expr);                 \
    if (_e != hipSuccess) return (int)_e;   \
  } while (0)
