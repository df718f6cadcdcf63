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

// x = x0 + x1 + x2 exactly, each a bf16 (8 significant bits): the split-bf16 products of the fp32 attention kernel
// (attention_f32.hip x6_dot: the six plane products with i + j <= 2, exact to 2^-27 relative).
__device__ __forceinline__ void split3(float x, float& p0, float& p1, float& p2) {
  p0 = (float)(__bf16)x;
  const float r = x - p0;
  p1 = (float)(__bf16)r;
  p2 = (float)(__bf16)(r - p1);
}

// ---- fp32 GEMMs by split-fp16 MFMA ("h3") ---------------------------------------------------------------
// A GEMM operand is scaled by a power of two s (exact) and split into two fp16 planes, s x = hi + lo with
// hi = fp16(s x) (11 significant bits) and lo = fp16(s x - hi) (the residual, exact in fp32; 11 more bits).  The
// fp32 product is then hi_a hi_b + hi_a lo_b + lo_a hi_b (the dropped lo_a lo_b is 2^-22 relative and the residual
// rounding 2^-23: measured error below the CPU fp32 GEMM's own, tools/h3_error.py), and every fp16 x fp16 product
// is exact in the fp32 MFMA accumulator.  The three terms are a K-concatenation, so an ordinary fp16 MFMA GEMM over
// K' = 3K computes it with the K-blocks  A' = [a_lo | a_hi | a_hi],  B' = [b_hi | b_lo | b_hi]  (small terms
// first), at the bf16/fp16 matrix-core rate - half the MFMAs of a three-plane bf16 split (six products).  The
// epilogue multiplies by alpha = 1 / (s_a s_b).  The scales keep every plane inside the fp16 range: the model
// derives s_a per GEMM input from a bound on |x| that holds for any input (models/model.py h3 scales: RMSNorm /
// LayerNorm outputs, attention outputs and SwiGLU / GELU outputs are bounded by the weights), s_b from max |w|.
// Weights are stored as B' [N, 3K]; an activation once per plane, [hi | lo] ([rows, 2K]), and the GEMM's A loader
// reads K-block j of A' from plane (1 0 0)[j] (h3_acol).  A weight that is exact in fp16 after scaling (b_lo = 0: a
// bf16 or fp16 checkpoint, as the HF Qwen2 / Pythia releases) needs only the two products a_lo b_hi + a_hi b_hi,
// the K' = 2K GEMM on B' = [b_hi | b_hi] (the same result: the third term is exactly zero).
typedef uint16_t f16_t;   // fp16 storage as raw 16-bit words
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;
__device__ __forceinline__ void split2h(float x, float& hi, float& lo) {
  hi = (float)(_Float16)x;
  lo = (float)(_Float16)(x - hi);
}
__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
  return __builtin_bit_cast(uint32_t, f16x2_t{(_Float16)a, (_Float16)b});
}
// split2h of a value pair as packed planes: H = [hi(x0) | hi(x1)] by v_cvt_pk_f16_f32, L = [lo(x0) | lo(x1)] with
// lo = f16(x - hi) straight from the fp32 value and the f16 hi half by v_fma_mixlo_f16 / v_fma_mixhi_f16 (x - hi is
// exact, one RNE to f16): bit-identical to split2h + pack_h2 in 3 VALU instead of 5-6.  The asm's operands are the
// fp32 inputs and the convert's result; the convert reads the inputs first, so any MFMA -> VALU hazard on them is
// resolved by the compiler-visible instruction before the asm issues.
__device__ __forceinline__ u32x2_t split2h_pk(float x0, float x1) {   // -> {H, L}
  const uint32_t H = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{x0, x1}, f16x2_t));
  uint32_t L;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(L) : "v"(x0), "v"(H), "v"(x1));
  return u32x2_t{H, L};
}
// column of the 2-plane activation row holding column kp of A' (K = plane width; K-blocks never straddle a K-tile)
__device__ __forceinline__ int h3_acol(int kp, int K) {
  const int j = kp / K;                          // A' block 0..2: planes lo hi hi
  return (j == 0 ? K : 0) + (kp - j * K);
}
// Store s * v[0..3] at column `col` of an h3 activation row (plane width K): two 8-byte stores.
// Nontemporal store (global_store ... nt) for the large streamed outputs that overflow the 256 MB Infinity Cache
// anyway (the SwiGLU planes: 637 MB per bench GEMM): measured 2 % faster than plain stores on the power-limited
// gate/up GEMM (profiles/history/r05/gemm_epilogue/probe_store_policy.log), bit-identical.
template <class T>
__device__ __forceinline__ void store_nt(T* p, const T& v) {
  __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void store_h3_4(f16_t* __restrict__ row, int K, int col, const float (&v)[4], float s) {
  const float x0 = v[0] * s, x1 = v[1] * s, x2 = v[2] * s, x3 = v[3] * s;
  const u32x2_t t0 = split2h_pk(x0, x1), t1 = split2h_pk(x2, x3);
  *(u32x2_t*)(row + col) = u32x2_t{t0[0], t1[0]};
  *(u32x2_t*)(row + (size_t)K + col) = u32x2_t{t0[1], t1[1]};
}
// 8 consecutive values: two 16-byte stores.
__device__ __forceinline__ void store_h3_8(f16_t* __restrict__ row, int K, int col, const float (&v)[8], float s) {
  u32x4_t wh, wl;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const u32x2_t t = split2h_pk(v[2 * e] * s, v[2 * e + 1] * s);
    wh[e] = t[0];
    wl[e] = t[1];
  }
  *(u32x4_t*)(row + col) = wh;
  *(u32x4_t*)(row + (size_t)K + col) = wl;
}

// T21-style store widening for the swapped 16x16 MFMA layout: lane group g = lane>>4 holds 4 consecutive
// columns g*4.. of a 16-column group.  v_permlane16_swap exchanges rows 1,3 of `lo` with rows 0,2 of `hi`,
// so for two groups (lo, hi) lanes g=0/2 end with 8 consecutive columns of `lo` and lanes g=1/3 with 8 of `hi`:
// one 16-byte store per lane at column offset (g&1)*16 + (g>>1)*8 of the 32-column pair (was two 8-byte stores).
__device__ __forceinline__ u32x4_t pair_swap16(u32x2_t lo, u32x2_t hi) {
  const auto r0 = __builtin_amdgcn_permlane16_swap(lo[0], hi[0], false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(lo[1], hi[1], false, false);
  return u32x4_t{r0[0], r1[0], r0[1], r1[1]};
}
__device__ __forceinline__ int pair_col(int g) { return (g & 1) * 16 + (g >> 1) * 8; }
// max over lanes l, l ^ 16 and l ^ 32 without LDS: v_permlane16_swap / v_permlane32_swap of a value with itself give
// every lane the pair (x_l, x_partner) in some order (a __shfl_xor is a ds_bpermute plus index arithmetic)
__device__ __forceinline__ float xor_max16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor_max32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
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
