// fp32 causal GQA attention for head_dim 64 and the fp32 token-importance scorers, the
// attention half of the framework's fp32 execution mode (the reference evaluates its models in fp32:
// Experiments/Qwen2-0.5B/qwen_layer_wise.py:17, Experiments/Pythia-70M/pythia_model.py:25 load without a dtype).
//
// Matrix work runs on the gfx950 f32 matrix cores, v_mfma_f32_16x16x4_f32: exact fp32 products and fp32
// accumulation (the GEMMs of the same mode use the split-bf16 X6 scheme instead, see common.h; attention is ~3 %
// of the FLOPs at S = 512 and takes the f32 instruction, which needs no operand splitting).
//
//   flash_attn_fwd_f32 : O = softmax(Q K^T) V, online softmax, optional row LSE; O written as fp32 rows or
//                        directly in the X6 layout the O-projection GEMM consumes.
//   attn_lastrow_f32   : P[S-1, :] per head.
//   attn_colsum_f32    : sum_i P[i, j] per head from Q, K and the row LSE (second sweep, key block outer).
//
// Layouts as the bf16 kernels (attention.hip): q [B,Hq,S,64] (RoPE applied, pre-scaled), k [B,Hkv,S,64],
// vt [B,Hkv,64,s_pad] (V^T, zero padded), o [B*S, Hq*64] (fp32) or [B*S, 3*Hq*64] (3-plane X6).
//
// 16x16x4 f32 MFMA operand layout: lane l supplies A[m = l&15][k = l>>4] and B[k = l>>4][n = l&15]; the result
// D[m][n] sits in lane l, register r at m = 4(l>>4) + r, n = l&15.  The contraction index k of MFMA number kk is
// mapped to d = 16(l>>4) + kk, so a lane's 16 operands of a row are 16 CONSECUTIVE floats (four ds_read_b128).
//   S^T = K Q^T : A = K rows (m = key), B = Q^T -> lane holds 4 consecutive keys of ONE query row (row max is
//                 in-lane + 2 shuffles; the row's P values are the B operand of P.V without any data movement)
//   O^T += V^T P^T : MFMA (kt, r) contracts keys {16kt + 4g + r}; A = V^T rows (m = d) read as one ds_read_b128
//                 of 4 consecutive keys per (d-tile, key-subtile).
// LDS image: rows of 256 B (64 fp32), 16-byte chunk c of row r stored at c ^ hsw(r & 15), hsw(r) =
// 4*[0,2,3,1][(r>>2)&3] + (r&3).  A ds_read_b128 is serviced in 16-lane groups ({0-3,12-15,20-27}, ...); the
// K reads (row l&15, chunk 4g+s) and the V^T reads (row l&15, chunk 4kt+g) of each group then hit 16 distinct
// 16-byte bank slots.
#include "common.h"

namespace {
constexpr int FKT = 64;            // keys per tile
constexpr int FTILE = 64 * 256;    // 64 rows x 256 B
constexpr float FLOG2E = 1.4426950408889634f;
constexpr float FTAU = 8.f;

__device__ __forceinline__ int hsw(int r) {
  const int R = (r >> 2) & 3;
  const int a = (R >> 1) | (((R ^ (R >> 1)) & 1) << 1);  // [0,2,3,1]
  return (a << 2) | (r & 3);
}

// Stage a 64-row x 64-float tile: 16 wave-instructions of 1 KiB (4 rows each), 4 per wave.
__device__ __forceinline__ void stage_f32(const float* __restrict__ base, size_t row_stride, int row0, int row_max,
                                          int col0, char* lds, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = i * 4 + wave;
    const int r = blk * 4 + (lane >> 4);
    const int c = (lane & 15) ^ hsw(r);
    int gr = row0 + r;
    gr = gr < row_max ? gr : row_max - 1;
    glds16(base + (size_t)gr * row_stride + col0 + c * 4, lds + blk * 1024);
  }
}

__device__ __forceinline__ f32x4_t lds_chunk(const char* lds, int row, int chunk) {
  return *(const f32x4_t*)(lds + row * 256 + ((chunk ^ hsw(row)) << 4));
}

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <bool MASK>
__device__ __forceinline__ void f32_tile(const char* lk, const char* lv, const float (&qf)[16], f32x4_t (&oacc)[4],
                                         float& m2, float& l_run, int kb, int qrow, int S, int g, int ql) {
  f32x4_t st[4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    const int row = kt * 16 + ql;
    f32x4_t kf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) kf[s] = lds_chunk(lk, row, 4 * g + s);
    st[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) st[kt] = mfma4(kf[kk >> 2][kk & 3], qf[kk], st[kt]);
  }
  if constexpr (MASK) {
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb * FKT + kt * 16 + 4 * g + r;
        if (key > qrow || key >= S) st[kt][r] = -INFINITY;
      }
  }
  float mloc = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, st[kt][r]);
  mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
  mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
  const float mc = mloc * FLOG2E;
  if (__builtin_amdgcn_ballot_w64(mc > m2 + FTAU)) {  // wave-uniform lazy rescale (p <= 2^TAU otherwise)
    const float mn = fmaxf(m2, mc);
    const float alpha = exp2f(m2 - mn);              // m2 = -inf on the first tile -> 0
    m2 = mn;
    l_run *= alpha;
#pragma unroll
    for (int d = 0; d < 4; ++d) oacc[d] *= alpha;
  }
  float ps = 0.f;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = exp2f(fmaf(st[kt][r], FLOG2E, -m2));
      st[kt][r] = p;
      ps += p;
    }
  l_run += ps;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int row = dt * 16 + ql;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const f32x4_t vf = lds_chunk(lv, row, 4 * kt + g);
#pragma unroll
      for (int r = 0; r < 4; ++r) oacc[dt] = mfma4(vf[r], st[kt][r], oacc[dt]);
    }
  }
}
}  // namespace

// One workgroup = 4 waves = 64 query rows of one (window, head); each wave owns 16 rows.  K / V^T tiles of 64
// keys are DMA'd to LDS (global_load_lds, swizzled source) and double-buffered; XCD-aware block order as the bf16
// v2 kernel: the query blocks and heads of one (window, kv head) group run on one XCD, heavy blocks first.
template <bool X6OUT>
__global__ __launch_bounds__(256, 2) void flash_attn_fwd_f32_kernel(const float* __restrict__ q,
                                                                   const float* __restrict__ k,
                                                                   const float* __restrict__ vt, void* __restrict__ o,
                                                                   float* __restrict__ lse,
                                                                   const float* __restrict__ n_rows, int B, int Hq,
                                                                   int Hkv, int S, int s_pad) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, ql = lane & 15;
  const int nqb = (S + 63) / 64;
  const int G = Hq / Hkv, NG = B * Hkv;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int cnt = (NG - xcd + 7) >> 3;
  const int per_qb = cnt * G;
  if (j >= per_qb * nqb) return;
  const int qb = nqb - 1 - j / per_qb;
  const int rem = j - (nqb - 1 - qb) * per_qb;
  const int grp = xcd + 8 * (rem / G);
  const int b = grp / Hkv, hk = grp - b * Hkv, h = hk * G + rem % G;
  if (n_rows && qb * 64 + 63 < S - 1 - (int)n_rows[b]) return;  // scored-rows mode (last layer)

  const float* qh = q + ((size_t)b * Hq + h) * S * 64;
  const float* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const float* vh = vt + ((size_t)b * Hkv + hk) * 64 * (size_t)s_pad;

  const int q0 = qb * 64 + wave * 16;
  const int qrow = q0 + ql;
  const int qld = qrow < S ? qrow : S - 1;
  float qf[16];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const f32x4_t v = *(const f32x4_t*)(qh + (size_t)qld * 64 + 16 * g + 4 * s);
#pragma unroll
    for (int e = 0; e < 4; ++e) qf[4 * s + e] = v[e];
  }
  f32x4_t oacc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) oacc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m2 = -INFINITY, l_run = 0.f;

  const int nkb = qb + 1;
  const int kmax = (q0 + 15) / FKT;  // last key tile this wave needs (wave-uniform)
  stage_f32(kh, 64, 0, S, 0, smem, wave, lane);
  stage_f32(vh, s_pad, 0, 64, 0, smem + FTILE, wave, lane);
  for (int kb = 0; kb < nkb; ++kb) {
    wait_vmcnt0();
    __syncthreads();  // tile kb landed for every wave; every wave's reads of tile kb-1 retired
    if (kb + 1 < nkb) {
      char* nx = smem + ((kb + 1) & 1) * 2 * FTILE;
      stage_f32(kh, 64, (kb + 1) * FKT, S, 0, nx, wave, lane);
      stage_f32(vh, s_pad, 0, 64, (kb + 1) * FKT, nx + FTILE, wave, lane);
    }
    if (kb > kmax) continue;
    const char* cur = smem + (kb & 1) * 2 * FTILE;
    if (kb * FKT + FKT - 1 <= q0 && kb * FKT + FKT - 1 < S)
      f32_tile<false>(cur, cur + FTILE, qf, oacc, m2, l_run, kb, qrow, S, g, ql);
    else
      f32_tile<true>(cur, cur + FTILE, qf, oacc, m2, l_run, kb, qrow, S, g, ql);
  }

  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  if (qrow < S) {
    const float inv = 1.f / l_run;
    const int W = Hq * 64;
    if constexpr (X6OUT) {
      bf16_t* orow = (bf16_t*)o + ((size_t)b * S + qrow) * (size_t)(3 * W);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float v[4] = {oacc[dt][0] * inv, oacc[dt][1] * inv, oacc[dt][2] * inv, oacc[dt][3] * inv};
        store_x6_4(orow, W, h * 64 + dt * 16 + 4 * g, v);
      }
    } else {
      float* orow = (float*)o + ((size_t)b * S + qrow) * (size_t)W + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) *(f32x4_t*)(orow + dt * 16 + 4 * g) = oacc[dt] * inv;
    }
    if (lse && g == 0) lse[((size_t)b * Hq + h) * S + qrow] = m2 * 0.6931471805599453f + logf(l_run);
  }
}

// Last-row probabilities: one workgroup per (b, h); P[S-1, j] = softmax_j(q_{S-1} . k_j), fp32 throughout.
__global__ __launch_bounds__(256) void attn_lastrow_f32_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                               float* __restrict__ out, int Hq, int Hkv, int S) {
  extern __shared__ float sc[];  // S scores
  __shared__ float qv[64];
  __shared__ float red[4];
  const int bh = blockIdx.x, b = bh / Hq, h = bh - b * Hq, hk = h / (Hq / Hkv);
  const float* qr = q + (((size_t)b * Hq + h) * S + (S - 1)) * 64;
  const float* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  if (threadIdx.x < 64) qv[threadIdx.x] = qr[threadIdx.x];
  __syncthreads();
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < S; j += 256) {
    const f32x4_t* kr = (const f32x4_t*)(kh + (size_t)j * 64);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const f32x4_t w = kr[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) s = fmaf(qv[c * 4 + e], w[e], s);
    }
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max<256>(mx, red);
  float sum = 0.f;
  for (int j = threadIdx.x; j < S; j += 256) {
    const float p = expf(sc[j] - mx);
    sc[j] = p;
    sum += p;
  }
  sum = block_sum<256>(sum, red);
  const float inv = 1.f / sum;
  float* orow = out + (size_t)bh * S;
  for (int j = threadIdx.x; j < S; j += 256) orow[j] = sc[j] * inv;
}

// Column sums of P for one (b, h, 64-key block): sum over query rows i >= key of exp(q_i . k_j - lse_i).
// S = Q K^T with the key on the MFMA column: lane holds key 16ni + (lane&15) for query rows 4g + r, so the
// column sum over a 16-row tile is lane-local; waves split the query tiles, LDS combines them.
__global__ __launch_bounds__(256) void attn_colsum_f32_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                              const float* __restrict__ lse, float* __restrict__ out,
                                                              int B, int Hq, int Hkv, int S) {
  __shared__ float part[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int nkb = (S + 63) / 64;
  const int kb = blockIdx.x % nkb;
  const int bh = blockIdx.x / nkb, b = bh / Hq, h = bh - b * Hq, hk = h / (Hq / Hkv);
  const float* qh = q + ((size_t)b * Hq + h) * S * 64;
  const float* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const float* lh = lse + ((size_t)b * Hq + h) * S;

  float kf[4][16];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    int key = kb * 64 + ni * 16 + cl;
    key = key < S ? key : S - 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f32x4_t v = *(const f32x4_t*)(kh + (size_t)key * 64 + 16 * g + 4 * s);
#pragma unroll
      for (int e = 0; e < 4; ++e) kf[ni][4 * s + e] = v[e];
    }
  }
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  for (int qt = kb * 4 + wave; qt * 16 < S; qt += 4) {
    const int qa = qt * 16 + cl;
    const int qla = qa < S ? qa : S - 1;
    float qf[16];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f32x4_t v = *(const f32x4_t*)(qh + (size_t)qla * 64 + 16 * g + 4 * s);
#pragma unroll
      for (int e = 0; e < 4; ++e) qf[4 * s + e] = v[e];
    }
    float lrow[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qi = qt * 16 + g * 4 + r;
      lrow[r] = qi < S ? lh[qi] : INFINITY;
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      f32x4_t s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) s = mfma4(qf[kk], kf[ni][kk], s);
      const int key = kb * 64 + ni * 16 + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = qt * 16 + g * 4 + r;
        csum[ni] += (qi >= key && qi < S) ? expf(s[r] - lrow[r]) : 0.f;
      }
    }
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    float v = csum[ni];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (g == 0) part[wave][ni * 16 + cl] = v;
  }
  __syncthreads();
  if (tid < 64) {
    const int key = kb * 64 + tid;
    if (key < S) out[((size_t)b * Hq + h) * S + key] = (part[0][tid] + part[1][tid]) + (part[2][tid] + part[3][tid]);
  }
}

// out_x6 != 0: O as a 3-plane X6 activation [B*S, 3*Hq*64] (bf16 planes) for the O-projection; else fp32
// [B*S, Hq*64].
EDGE_API int edge_flash_attn_fwd_f32(const float* q, const float* k, const float* vt, void* o, float* lse,
                                     const float* n_rows, int B, int Hq, int Hkv, int S, int s_pad, int out_x6,
                                     hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv || s_pad % 64 || s_pad < S) return (int)hipErrorInvalidValue;
  const int G = Hq / Hkv, maxcnt = (B * Hkv + 7) / 8;
  const dim3 grid(8 * maxcnt * G * ((S + 63) / 64));
  if (out_x6)
    hipLaunchKernelGGL(flash_attn_fwd_f32_kernel<true>, grid, dim3(256), 4 * FTILE, st, q, k, vt, o, lse, n_rows, B,
                       Hq, Hkv, S, s_pad);
  else
    hipLaunchKernelGGL(flash_attn_fwd_f32_kernel<false>, grid, dim3(256), 4 * FTILE, st, q, k, vt, o, lse, n_rows, B,
                       Hq, Hkv, S, s_pad);
  return (int)hipGetLastError();
}

EDGE_API int edge_attn_lastrow_f32(const float* q, const float* k, float* out, int B, int Hq, int Hkv, int S,
                                   hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv || S > 16384) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(attn_lastrow_f32_kernel, dim3(B * Hq), dim3(256), S * sizeof(float), st, q, k, out, Hq, Hkv, S);
  return (int)hipGetLastError();
}

EDGE_API int edge_attn_colsum_f32(const float* q, const float* k, const float* lse, float* out, int B, int Hq, int Hkv,
                                  int S, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv) return (int)hipErrorInvalidValue;
  const int nkb = (S + 63) / 64;
  hipLaunchKernelGGL(attn_colsum_f32_kernel, dim3(B * Hq * nkb), dim3(256), 0, st, q, k, lse, out, B, Hq, Hkv, S);
  return (int)hipGetLastError();
}
