// Memory-bound row kernels: embedding gather, RMSNorm, LayerNorm (single and dual-output), with an
// optional row-gather so the final norm runs only on the rows that are scored (K1, K3, K9 of SURVEY §2.4).
// One wave64 per row, 16-byte vector loads (8 bf16 per lane per chunk), fp32 statistics.
#include "common.h"

template <int NCH>
__device__ __forceinline__ void load_row(const bf16_t* __restrict__ src, int H, float (&v)[NCH][8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < H) {
      u32x4_t w = *(const u32x4_t*)(src + col);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[c][2 * j] = bf_lo(w[j]); v[c][2 * j + 1] = bf_hi(w[j]); }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
}

template <int NCH>
__device__ __forceinline__ void store_row(bf16_t* __restrict__ dst, int H, const float (&v)[NCH][8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < H) {
      u32x4_t w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = pack_bf2(v[c][2 * j], v[c][2 * j + 1]);
      *(u32x4_t*)(dst + col) = w;
    }
  }
}

template <int NCH>
__device__ __forceinline__ void load_vec(const bf16_t* __restrict__ p, int H, float (&v)[NCH][8]) { load_row<NCH>(p, H, v); }

// ---------------------------------------------------------------------------------------------
template <int NCH>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      bf16_t* __restrict__ y, const int* __restrict__ rows, int R,
                                                      int H, float eps) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int src_row = rows ? rows[r] : r;
  float v[NCH][8], g[NCH][8];
  load_row<NCH>(x + (size_t)src_row * H, H, v);
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)H + eps);
  load_vec<NCH>(w, H, g);
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // HF: (x * rsqrt(var+eps)).to(bf16) then * weight  -> round twice like the reference.
      const float n = bf2f(f2bf(v[c][j] * rs));
      v[c][j] = n * g[c][j];
    }
  store_row<NCH>(y + (size_t)r * H, H, v);
}

template <int NCH, bool DUAL>
__global__ __launch_bounds__(256) void layernorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w1,
                                                        const bf16_t* __restrict__ b1, const bf16_t* __restrict__ w2,
                                                        const bf16_t* __restrict__ b2, bf16_t* __restrict__ y1,
                                                        bf16_t* __restrict__ y2, const int* __restrict__ rows, int R,
                                                        int H, float eps) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int src_row = rows ? rows[r] : r;
  float v[NCH][8], g[NCH][8], b[NCH][8], o[NCH][8];
  load_row<NCH>(x + (size_t)src_row * H, H, v);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[c][j];
  const float mean = wave_sum(s) / (float)H;
  const int lane = threadIdx.x & 63;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const bool ok = (c * 64 + lane) * 8 < H;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[c][j] - mean;
      v[c][j] = d;
      ss += ok ? d * d : 0.f;
    }
  }
  const float rs = rsqrtf(wave_sum(ss) / (float)H + eps);
  load_vec<NCH>(w1, H, g);
  load_vec<NCH>(b1, H, b);
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[c][j] = v[c][j] * rs * g[c][j] + b[c][j];
  store_row<NCH>(y1 + (size_t)r * H, H, o);
  if (DUAL) {
    load_vec<NCH>(w2, H, g);
    load_vec<NCH>(b2, H, b);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[c][j] = v[c][j] * rs * g[c][j] + b[c][j];
    store_row<NCH>(y2 + (size_t)r * H, H, o);
  }
}

__global__ __launch_bounds__(256) void embedding_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ table,
                                                        bf16_t* __restrict__ out, int T, int H, int V) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= T) return;
  int64_t id = ids[r];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const u32x4_t* src = (const u32x4_t*)(table + (size_t)id * H);
  u32x4_t* dst = (u32x4_t*)(out + (size_t)r * H);
  for (int c = threadIdx.x & 63; c < H / 8; c += 64) dst[c] = src[c];
}

// ---------------------------------------------------------------------------------------------
#define DISPATCH_NCH(H, ...)                       \
  do {                                             \
    const int _nch = ((H) / 8 + 63) / 64;          \
    if (_nch <= 1) { constexpr int NCH = 1; __VA_ARGS__; } \
    else if (_nch <= 2) { constexpr int NCH = 2; __VA_ARGS__; } \
    else if (_nch <= 4) { constexpr int NCH = 4; __VA_ARGS__; } \
    else if (_nch <= 8) { constexpr int NCH = 8; __VA_ARGS__; } \
    else return (int)hipErrorInvalidValue;        \
  } while (0)

EDGE_API int edge_rmsnorm(const void* x, const void* w, void* y, const int* rows, int R, int H, float eps,
                          hipStream_t st) {
  if (H % 8 || R <= 0) return R == 0 ? 0 : (int)hipErrorInvalidValue;
  dim3 grid((R + 3) / 4);
  DISPATCH_NCH(H, rmsnorm_kernel<NCH><<<grid, 256, 0, st>>>((const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, rows, R,
                                                           H, eps));
  return (int)hipGetLastError();
}

EDGE_API int edge_layernorm(const void* x, const void* w1, const void* b1, const void* w2, const void* b2, void* y1,
                            void* y2, const int* rows, int R, int H, float eps, hipStream_t st) {
  if (H % 8 || R <= 0) return R == 0 ? 0 : (int)hipErrorInvalidValue;
  dim3 grid((R + 3) / 4);
  if (y2) {
    DISPATCH_NCH(H, (layernorm_kernel<NCH, true><<<grid, 256, 0, st>>>(
                        (const bf16_t*)x, (const bf16_t*)w1, (const bf16_t*)b1, (const bf16_t*)w2, (const bf16_t*)b2,
                        (bf16_t*)y1, (bf16_t*)y2, rows, R, H, eps)));
  } else {
    DISPATCH_NCH(H, (layernorm_kernel<NCH, false><<<grid, 256, 0, st>>>(
                        (const bf16_t*)x, (const bf16_t*)w1, (const bf16_t*)b1, nullptr, nullptr, (bf16_t*)y1,
                        nullptr, rows, R, H, eps)));
  }
  return (int)hipGetLastError();
}

EDGE_API int edge_embedding(const int64_t* ids, const void* table, void* out, int T, int H, int V, hipStream_t st) {
  if (H % 8) return (int)hipErrorInvalidValue;
  if (T <= 0) return 0;
  embedding_kernel<<<(T + 3) / 4, 256, 0, st>>>(ids, (const bf16_t*)table, (bf16_t*)out, T, H, V);
  return (int)hipGetLastError();
}

// Per-row sum of squares in 64-column slabs: ssq[r, s] = sum_{c in slab s} x[r, c]^2 (the partial layout the
// residual GEMM epilogues produce; consumed by the fused-RMSNorm GEMMs).  Wave per row.
template <int NCH>
__global__ __launch_bounds__(256) void row_ssq_kernel(const bf16_t* __restrict__ x, float* __restrict__ ssq, int R,
                                                      int H) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  float v[NCH][8];
  load_row<NCH>(x + (size_t)r * H, H, v);
  const int P = H / 64;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[c][j] * v[c][j];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    const int slab = c * 8 + (lane >> 3);
    if ((lane & 7) == 0 && slab < P) ssq[(size_t)r * P + slab] = s;
  }
}

EDGE_API int edge_row_ssq(const void* x, float* ssq, int R, int H, hipStream_t st) {
  if (H % 64) return (int)hipErrorInvalidValue;
  if (R <= 0) return 0;
  DISPATCH_NCH(H, row_ssq_kernel<NCH><<<(R + 3) / 4, 256, 0, st>>>((const bf16_t*)x, ssq, R, H));
  return (int)hipGetLastError();
}

// rscale[r] = rsqrt(sum_p ssq[r, p] / H + eps): the per-row RMSNorm factor from the slab partials.
__global__ __launch_bounds__(256) void row_rscale_kernel(const float* __restrict__ ssq, float* __restrict__ rs, int R,
                                                         int P, int H, float eps, const float* __restrict__ mul) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= R) return;
  const float* p = ssq + (size_t)r * P;
  float s = 0.f;
  for (int i = 0; i < P; ++i) s += p[i];
  const float v = rsqrtf(s / (float)H + eps);
  rs[r] = mul ? v * mul[r] : v;
}

EDGE_API int edge_row_rscale(const float* ssq, float* rs, int R, int P, int H, float eps, hipStream_t st) {
  if (R <= 0) return 0;
  row_rscale_kernel<<<(R + 255) / 256, 256, 0, st>>>(ssq, rs, R, P, H, eps, nullptr);
  return (int)hipGetLastError();
}

// rs[r] = rsqrt(sum_p ssq[r, p] / H + eps) * mul[r]: the consumer row scale of the fp32 fused RMSNorm (mul = the
// producer's 1 / p_m, gemm.hip EPI_F32_RESID_NP)
EDGE_API int edge_row_rscale_mul(const float* ssq, const float* mul, float* rs, int R, int P, int H, float eps,
                                 hipStream_t st) {
  if (R <= 0) return 0;
  if (!mul) return (int)hipErrorInvalidValue;
  row_rscale_kernel<<<(R + 255) / 256, 256, 0, st>>>(ssq, rs, R, P, H, eps, mul);
  return (int)hipGetLastError();
}

// =============================================================================================
// fp32 execution mode: fp32 activations in, fp32 statistics, and GEMM-input outputs written as 2-plane h3 split-fp16
// activations [R, 2H] at scale s (common.h) that the fp32-mode GEMMs consume (s = 0: plain fp32 [R, H] instead).
template <int NCH>
__device__ __forceinline__ void load_row_f32(const float* __restrict__ src, int H, float (&v)[NCH][8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < H) {
      const f32x4_t a = *(const f32x4_t*)(src + col), b = *(const f32x4_t*)(src + col + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[c][j] = a[j]; v[c][4 + j] = b[j]; }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
}

template <int NCH>
__device__ __forceinline__ void store_row_f32_or_h3(void* __restrict__ dst, int H, const float (&v)[NCH][8],
                                                    float h3s) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col >= H) continue;
    if (h3s > 0.f) {
      store_h3_8((f16_t*)dst, H, col, v[c], h3s);
    } else {
      float* d = (float*)dst + col;
      *(f32x4_t*)d = f32x4_t{v[c][0], v[c][1], v[c][2], v[c][3]};
      *(f32x4_t*)(d + 4) = f32x4_t{v[c][4], v[c][5], v[c][6], v[c][7]};
    }
  }
}

__device__ __forceinline__ void* out_row(void* y, size_t r, int H, float h3s) {
  return h3s > 0.f ? (void*)((f16_t*)y + r * 2 * (size_t)H) : (void*)((float*)y + r * (size_t)H);
}

// HF Qwen2RMSNorm in fp32: y = w * (x * rsqrt(mean(x^2) + eps)).
template <int NCH>
__global__ __launch_bounds__(256) void rmsnorm_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          void* __restrict__ y, const int* __restrict__ rows, int R,
                                                          int H, float eps, float h3s, float* __restrict__ rstd_out) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int src_row = rows ? rows[r] : r;
  float v[NCH][8], g[NCH][8];
  load_row_f32<NCH>(x + (size_t)src_row * H, H, v);
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) ss = fmaf(v[c][j], v[c][j], ss);
  ss = wave_sum(ss);
  const float rs = 1.f / sqrtf(ss / (float)H + eps);
  if (rstd_out && (threadIdx.x & 63) == 0) rstd_out[r] = rs;   // the normaliser itself (AttnLRP saves it detached)
  load_row_f32<NCH>(w, H, g);
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[c][j] = g[c][j] * (v[c][j] * rs);
  store_row_f32_or_h3<NCH>(out_row(y, r, H, h3s), H, v, h3s);
}

template <int NCH, bool DUAL>
__global__ __launch_bounds__(256) void layernorm_f32_kernel(const float* __restrict__ x, const float* __restrict__ w1,
                                                            const float* __restrict__ b1, const float* __restrict__ w2,
                                                            const float* __restrict__ b2, void* __restrict__ y1,
                                                            void* __restrict__ y2, const int* __restrict__ rows, int R,
                                                            int H, float eps, float h3s1, float h3s2) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int src_row = rows ? rows[r] : r;
  const int lane = threadIdx.x & 63;
  float v[NCH][8], g[NCH][8], b[NCH][8], o[NCH][8];
  load_row_f32<NCH>(x + (size_t)src_row * H, H, v);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[c][j];
  const float mean = wave_sum(s) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const bool ok = (c * 64 + lane) * 8 < H;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[c][j] - mean;
      v[c][j] = d;
      ss += ok ? d * d : 0.f;
    }
  }
  const float rs = 1.f / sqrtf(wave_sum(ss) / (float)H + eps);
  load_row_f32<NCH>(w1, H, g);
  load_row_f32<NCH>(b1, H, b);
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[c][j] = fmaf(v[c][j] * rs, g[c][j], b[c][j]);
  store_row_f32_or_h3<NCH>(out_row(y1, r, H, h3s1), H, o, h3s1);
  if (DUAL) {
    load_row_f32<NCH>(w2, H, g);
    load_row_f32<NCH>(b2, H, b);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[c][j] = fmaf(v[c][j] * rs, g[c][j], b[c][j]);
    store_row_f32_or_h3<NCH>(out_row(y2, r, H, h3s2), H, o, h3s2);
  }
}

// fp32 [R, H] (rows optionally gathered) -> 2-plane h3 activation [R, 2H] at scale s
template <int NCH>
__global__ __launch_bounds__(256) void split_h3_kernel(const float* __restrict__ x, f16_t* __restrict__ y,
                                                       const int* __restrict__ rows, int R, int H, float s) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  float v[NCH][8];
  load_row_f32<NCH>(x + (size_t)(rows ? rows[r] : r) * H, H, v);
  store_row_f32_or_h3<NCH>(y + (size_t)r * 2 * H, H, v, s);
}

__global__ __launch_bounds__(256) void embedding_f32_kernel(const int64_t* __restrict__ ids,
                                                            const float* __restrict__ table, float* __restrict__ out,
                                                            int T, int H, int V) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= T) return;
  int64_t id = ids[r];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const f32x4_t* src = (const f32x4_t*)(table + (size_t)id * H);
  f32x4_t* dst = (f32x4_t*)(out + (size_t)r * H);
  for (int c = threadIdx.x & 63; c < H / 4; c += 64) dst[c] = src[c];
}

// h3_scale > 0: output as a 2-plane h3 activation [R, 2H] at that scale; 0: fp32 [R, H]
EDGE_API int edge_rmsnorm_f32(const float* x, const float* w, void* y, const int* rows, int R, int H, float eps,
                              float h3_scale, hipStream_t st) {
  if (H % 8 || R <= 0 || h3_scale < 0.f) return R == 0 ? 0 : (int)hipErrorInvalidValue;
  dim3 grid((R + 3) / 4);
  DISPATCH_NCH(H, rmsnorm_f32_kernel<NCH><<<grid, 256, 0, st>>>(x, w, y, rows, R, H, eps, h3_scale, nullptr));
  return (int)hipGetLastError();
}

// edge_rmsnorm_f32 that also writes the row normalisers rsqrt(mean(x^2) + eps) to rstd [R]
EDGE_API int edge_rmsnorm_f32_rstd(const float* x, const float* w, void* y, const int* rows, int R, int H, float eps,
                                   float h3_scale, float* rstd, hipStream_t st) {
  if (H % 8 || R <= 0 || h3_scale < 0.f || !rstd) return R == 0 ? 0 : (int)hipErrorInvalidValue;
  dim3 grid((R + 3) / 4);
  DISPATCH_NCH(H, rmsnorm_f32_kernel<NCH><<<grid, 256, 0, st>>>(x, w, y, rows, R, H, eps, h3_scale, rstd));
  return (int)hipGetLastError();
}

EDGE_API int edge_layernorm_f32(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                                void* y1, void* y2, const int* rows, int R, int H, float eps, float h3_scale1,
                                float h3_scale2, hipStream_t st) {
  if (H % 8 || R <= 0 || h3_scale1 < 0.f || h3_scale2 < 0.f) return R == 0 ? 0 : (int)hipErrorInvalidValue;
  dim3 grid((R + 3) / 4);
  if (y2) {
    DISPATCH_NCH(H, (layernorm_f32_kernel<NCH, true><<<grid, 256, 0, st>>>(x, w1, b1, w2, b2, y1, y2, rows, R, H, eps,
                                                                           h3_scale1, h3_scale2)));
  } else {
    DISPATCH_NCH(H, (layernorm_f32_kernel<NCH, false><<<grid, 256, 0, st>>>(x, w1, b1, nullptr, nullptr, y1, nullptr,
                                                                            rows, R, H, eps, h3_scale1, 0.f)));
  }
  return (int)hipGetLastError();
}

EDGE_API int edge_split_h3(const float* x, void* y, const int* rows, int R, int H, float s, hipStream_t st) {
  if (H % 8 || R <= 0 || !(s > 0.f)) return R == 0 ? 0 : (int)hipErrorInvalidValue;
  DISPATCH_NCH(H, split_h3_kernel<NCH><<<(R + 3) / 4, 256, 0, st>>>(x, (f16_t*)y, rows, R, H, s));
  return (int)hipGetLastError();
}

EDGE_API int edge_embedding_f32(const int64_t* ids, const float* table, float* out, int T, int H, int V,
                                hipStream_t st) {
  if (H % 4) return (int)hipErrorInvalidValue;
  if (T <= 0) return 0;
  embedding_f32_kernel<<<(T + 3) / 4, 256, 0, st>>>(ids, table, out, T, H, V);
  return (int)hipGetLastError();
}
