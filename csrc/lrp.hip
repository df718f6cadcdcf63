// AttnLRP relevance backward for the offline head-relevance calibration (reference C8,
// Experiments/Relevance/main.py:84-103 with lxt's efficient AttnLRP rules).
//
// The relevance pass is "Input x modified Gradient": a backward pass through the frozen model in which
//   * the two attention matmuls (Q K^T and A V) and the gate*up product use the uniform rule (each operand
//     gets half of the plain gradient),
//   * SiLU uses the identity rule (backward multiplies by silu(g)/g = sigmoid(g)),
//   * the norms are linear in x with the normaliser detached,
//   * the softmax uses its plain gradient.
// Only input gradients are needed (weights are frozen), so the backward of every linear layer is one GEMM
// with the transposed weight (csrc/gemm.hip) and the per-layer residual/row-scale epilogue.  This file holds
// the non-GEMM parts:
//
//   lrp_attn_delta : D[b,h,i] = sum_j A_ij dA_ij = 0.5 dO_i . O_i (uniform rule on A V); per-(window, head)
//                    relevance rel[b,h] = sum_i D[b,h,i] - the quantity the reference hook sums over S x S
//                    (sum_{ij} A * dA).  No S x S tensor exists anywhere.
//   lrp_attn_dkdv  : dK, dV partials for one (window, q head, 64-key block) over the causal query tiles:
//                    P recomputed from Q K^T and the forward LSE, dA = 0.5 dO V^T, dS = P (dA - D),
//                    dV = 0.5 P^T dO, dK = 0.5 dS^T Q.  The GQA group sum is fused into lrp_rope_pack.
//   lrp_attn_dq    : dQ = 0.5 dS K for one (window, q head, 64-query block) over its causal key tiles.
//                    dK/dV and dQ are separate sweeps: no atomics, deterministic.
//   lrp_rope_pack  : inverse RoPE (transpose rotation) + q scaling, scatter dQ/dK/dV into the token-major
//                    d[q|k|v] operand of the QKV input-gradient GEMM.
//   swiglu_il / lrp_swiglu_bwd : forward SiLU(g)*u and its LRP backward on the interleaved gate|up layout
//                    (IL_BLOCK = 16 columns of gate, then 16 of up).
//   lrp_gelu_bwd / lrp_ln_bwd : GPT-NeoX rules (GELU identity rule; LayerNorm with detached variance).
//
// MFMA: v_mfma_f32_16x16x32_bf16 everywhere.  Lane l holds A[row = l&15][k = 8(l>>4)..+7],
// B[k = 8(l>>4)..+7][col = l&15] and C[row = 4(l>>4)+r][col = l&15].  Products whose K dimension is the
// token axis reuse the lane-local probabilities of two 16-token sub-tiles as the A (or B) operand, with the
// token order permuted as kappa(g, j) = 16(j>>2) + 4g + (j&3); the other operand is read in the same order from
// the row-major LDS tile by the hardware-transposing ds_read_b64_tr_b16 (no transposed copy is staged).
#include "common.h"

namespace {
// Row-major 32 x 64 bf16 tiles, 128-byte rows, 16-byte chunks XOR-swizzled by tsw(row): conflict-free for the
// staging writes, the b128 row-fragment reads and the transposed reads (the same map as csrc/lrp_f32.hip x6sw).
// History: the first version padded the rows (144 B) and staged a transposed [64][40] copy with 2-byte writes that
// were 8-way bank conflicts.
__device__ __forceinline__ int tsw(int r) { return (((r >> 1) & 1) << 1) | ((((r >> 1) ^ (r >> 2)) & 1) << 2); }

__device__ __forceinline__ bf16x8_t ld_row_frag(const bf16_t* t, int row, int col) {
  return *(const bf16x8_t*)(t + row * 64 + (((col >> 3) ^ tsw(row)) << 3));
}

// B (or A) operand over the permuted token axis for columns 16 dt .. + 15: lane (cl, g) gets column 16 dt + cl of
// tokens kappa(g, 0..7) = 4g .. 4g + 3, 16 + 4g .. + 3, two ds_read_b64_tr_b16 (lane 4q + p of a 16-lane group
// addresses token row q of the 4-row block, columns 4p .. 4p + 3; every lane of the wave executes it).
typedef short s4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8_t ld_t_frag(const bf16_t* t, int dt, int g, int cl) {
  typedef __attribute__((address_space(3))) s4_t lds_s4;
  const int q = cl >> 2, p = cl & 3, ch = 2 * dt + (p >> 1);
  const int r0 = 4 * g + q, r1 = 16 + 4 * g + q;
  const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(t + r0 * 64 + ((ch ^ tsw(r0)) << 3) + (p & 1) * 4));
  const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(t + r1 * 64 + ((ch ^ tsw(r1)) << 3) + (p & 1) * 4));
  const short __attribute__((ext_vector_type(8))) v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

// 32 rows x 64 bf16 (row stride `ld` elements, rows clamped to < nrows): one 16-byte chunk per thread, loaded into
// a register (a tile ahead) and stored into the swizzled row-major tile.
__device__ __forceinline__ u32x4_t load32(const bf16_t* __restrict__ src, size_t ld, int row0, int nrows) {
  const int t = threadIdx.x, r = t >> 3, c = (t & 7) * 8;
  const int gr = row0 + r;
  return gr < nrows ? *(const u32x4_t*)(src + (size_t)gr * ld + c) : u32x4_t{0u, 0u, 0u, 0u};
}
__device__ __forceinline__ void store32(const u32x4_t& v, bf16_t* tr) {
  const int t = threadIdx.x, r = t >> 3;
  *(u32x4_t*)(tr + r * 64 + (((t & 7) ^ tsw(r)) << 3)) = v;
}

__device__ __forceinline__ bf16x8_t pack8(const f32x4_t& a, const f32x4_t& b) {
  bf16x8_t f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    f[r] = (__bf16)a[r];
    f[4 + r] = (__bf16)b[r];
  }
  return f;
}
}  // namespace

// ---------------------------------------------------------------------------------------------
// D and per-(window, head) relevance.  o, dO token-major [B*S, Hq*64]; D [B,Hq,S]; rel [B,Hq].
__global__ __launch_bounds__(256) void lrp_attn_delta_kernel(const bf16_t* __restrict__ o,
                                                             const bf16_t* __restrict__ dO, float* __restrict__ D,
                                                             float* __restrict__ rel, int Hq, int S) {
  // 8 lanes per token row (8 consecutive values each: every load instruction reads 8 whole 128-byte rows), the row's
  // dot product reduced over its 8 lanes by xor shuffles
  __shared__ float red[4];
  const int bh = blockIdx.x, b = bh / Hq, h = bh - b * Hq;
  const int sub = threadIdx.x & 7, r0 = threadIdx.x >> 3;
  float tot = 0.f;
  for (int i = r0; i < S; i += 32) {
    const size_t off = ((size_t)b * S + i) * (size_t)(Hq * 64) + h * 64 + sub * 8;
    const u32x4_t a = *(const u32x4_t*)(o + off), d = *(const u32x4_t*)(dO + off);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) s += bf_lo(a[e]) * bf_lo(d[e]) + bf_hi(a[e]) * bf_hi(d[e]);
#pragma unroll
    for (int x = 1; x < 8; x <<= 1) s += __shfl_xor(s, x, 64);
    s *= 0.5f;
    if (sub == 0) {
      D[(size_t)bh * S + i] = s;
      tot += s;
    }
  }
  tot = block_sum<256>(tot, red);
  if (threadIdx.x == 0) rel[bh] = tot;
}

// ---------------------------------------------------------------------------------------------
// dK, dV partials per q head.  q [B,Hq,S,64] (pre-scaled), k, v [B,Hkv,S,64], dO token-major,
// lse/D [B,Hq,S] -> dk, dv fp32 [B,Hq,S,64] (the GQA group sum happens in lrp_rope_pack).  Workgroup =
// (b, q head, 64-key block): 7x the workgroups of a per-kv-head sweep; wave w owns keys kb*64+16w..+15.
__global__ __launch_bounds__(256) void lrp_attn_dkdv_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                            const bf16_t* __restrict__ v,
                                                            const bf16_t* __restrict__ dO,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ D, float* __restrict__ dk,
                                                            float* __restrict__ dv, int B, int Hq, int Hkv, int S) {
  __shared__ __attribute__((aligned(16))) bf16_t sQ[32 * 64];
  __shared__ __attribute__((aligned(16))) bf16_t sO[32 * 64];
  __shared__ float sL[32], sD[32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int nkb = (S + 63) / 64;
  const int kb = blockIdx.x / (B * Hq);                // lightest (last) key blocks last: kb ascending = heavy first
  const int bh = blockIdx.x % (B * Hq), b = bh / Hq, h = bh - b * Hq, hk = h / (Hq / Hkv);
  const int key = kb * 64 + wave * 16 + cl;          // this lane's key (B-operand column / A-operand row)
  const int keyc = key < S ? key : S - 1;
  const int wkey_max = kb * 64 + __builtin_amdgcn_readfirstlane(wave) * 16 + 15;   // the wave's last key (scalar)
  const bf16_t* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const bf16_t* vh = v + ((size_t)b * Hkv + hk) * S * 64;
  bf16x8_t kB[2], vB[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    kB[ks] = *(const bf16x8_t*)(kh + (size_t)keyc * 64 + ks * 32 + g * 8);
    vB[ks] = *(const bf16x8_t*)(vh + (size_t)keyc * 64 + ks * 32 + g * 8);
  }
  f32x4_t dka[4], dva[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dka[d] = dva[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  (void)nkb;

  const int q_first = (kb * 64) & ~31;
  {
    const bf16_t* qh = q + ((size_t)b * Hq + h) * S * 64;
    const bf16_t* doh = dO + (size_t)b * S * (Hq * 64) + h * 64;
    const float* lh = lse + ((size_t)b * Hq + h) * S;
    const float* dh = D + ((size_t)b * Hq + h) * S;
    u32x4_t nq = load32(qh, 64, q_first, S), no = load32(doh, (size_t)Hq * 64, q_first, S);
    float nl = INFINITY, nd = 0.f;
    if (tid < 32 && q_first + tid < S) nl = lh[q_first + tid], nd = dh[q_first + tid];
    for (int q0 = q_first; q0 < S; q0 += 32) {
      __syncthreads();
      store32(nq, sQ);
      store32(no, sO);
      if (tid < 32) sL[tid] = nl, sD[tid] = nd;
      if (q0 + 32 < S) {   // the next tile's values under this tile's MFMAs
        nq = load32(qh, 64, q0 + 32, S);
        no = load32(doh, (size_t)Hq * 64, q0 + 32, S);
        if (tid < 32) {
          const int qi = q0 + 32 + tid;
          nl = qi < S ? lh[qi] : INFINITY;
          nd = qi < S ? dh[qi] : 0.f;
        }
      }
      __syncthreads();
      f32x4_t p[2], ds[2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x4_t s = {0.f, 0.f, 0.f, 0.f}, da = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(sQ, sub * 16 + cl, ks * 32 + g * 8), kB[ks], s,
                                                       0, 0, 0);
          da = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(sO, sub * 16 + cl, ks * 32 + g * 8), vB[ks], da,
                                                        0, 0, 0);
        }
        // s[r] = score(query = q0 + sub*16 + 4g + r, key); no masking on tiles wholly below this wave's keys
        if (q0 >= wkey_max && q0 + 32 <= S && wkey_max < S) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ql = sub * 16 + g * 4 + r;
            const float pr = __expf(s[r] - sL[ql]);
            p[sub][r] = pr;
            ds[sub][r] = pr * (0.5f * da[r] - sD[ql]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ql = sub * 16 + g * 4 + r;
            const int qi = q0 + ql;
            const bool ok = qi < S && key <= qi && key < S;
            const float pr = ok ? __expf(s[r] - sL[ql]) : 0.f;
            p[sub][r] = pr;
            ds[sub][r] = pr * (0.5f * da[r] - sD[ql]);
          }
        }
      }
      const bf16x8_t pf = pack8(p[0], p[1]);
      const bf16x8_t dsf = pack8(ds[0], ds[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dva[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, ld_t_frag(sO, dt, g, cl), dva[dt], 0, 0, 0);
        dka[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dsf, ld_t_frag(sQ, dt, g, cl), dka[dt], 0, 0, 0);
      }
    }
  }
  // C[row = key 4g + r of this wave][col = d 16dt + cl]
  float* dkh = dk + ((size_t)b * Hq + h) * S * 64;
  float* dvh = dv + ((size_t)b * Hq + h) * S * 64;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kr = kb * 64 + wave * 16 + g * 4 + r;
    if (kr < S) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dkh[(size_t)kr * 64 + dt * 16 + cl] = 0.5f * dka[dt][r];
        dvh[(size_t)kr * 64 + dt * 16 + cl] = 0.5f * dva[dt][r];
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// dQ.  Workgroup = (b, h, 64-query block); wave w owns queries qb*64 + 16w .. +15 (lane column cl).
// S^T = K Q^T and dA^T = V dO^T keep the query on the lane, so dQ^T = K^T dS^T takes dS^T lane-locally.
__global__ __launch_bounds__(256) void lrp_attn_dq_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                          const bf16_t* __restrict__ v, const bf16_t* __restrict__ dO,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ D, float* __restrict__ dq,
                                                          int B, int Hq, int Hkv, int S) {
  __shared__ __attribute__((aligned(16))) bf16_t sK[32 * 64];
  __shared__ __attribute__((aligned(16))) bf16_t sV[32 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int nqb = (S + 63) / 64;
  const int qb = nqb - 1 - blockIdx.x / (B * Hq);          // heaviest query blocks first
  const int bh = blockIdx.x % (B * Hq), b = bh / Hq, h = bh - b * Hq, hk = h / (Hq / Hkv);
  const int qi = qb * 64 + wave * 16 + cl;
  const int qic = qi < S ? qi : S - 1;
  const int wq_min = qb * 64 + __builtin_amdgcn_readfirstlane(wave) * 16;   // the wave's first query (scalar)
  const bf16_t* qh = q + ((size_t)b * Hq + h) * S * 64;
  const bf16_t* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const bf16_t* vh = v + ((size_t)b * Hkv + hk) * S * 64;
  const bf16_t* dorow = dO + ((size_t)b * S + qic) * (size_t)(Hq * 64) + h * 64;
  bf16x8_t qB[2], oB[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    qB[ks] = *(const bf16x8_t*)(qh + (size_t)qic * 64 + ks * 32 + g * 8);
    oB[ks] = *(const bf16x8_t*)(dorow + ks * 32 + g * 8);
  }
  const float lq = lse[((size_t)b * Hq + h) * S + qic];
  const float dq_ = D[((size_t)b * Hq + h) * S + qic];
  f32x4_t acc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) acc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int kend = min(S, qb * 64 + 64);
  u32x4_t nk = load32(kh, 64, 0, S), nv = load32(vh, 64, 0, S);
  for (int k0 = 0; k0 < kend; k0 += 32) {
    __syncthreads();
    store32(nk, sK);
    store32(nv, sV);
    if (k0 + 32 < kend) {   // the next key tile under this tile's MFMAs
      nk = load32(kh, 64, k0 + 32, S);
      nv = load32(vh, 64, k0 + 32, S);
    }
    __syncthreads();
    f32x4_t ds[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x4_t s = {0.f, 0.f, 0.f, 0.f}, da = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(sK, sub * 16 + cl, ks * 32 + g * 8), qB[ks], s, 0,
                                                     0, 0);
        da = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_row_frag(sV, sub * 16 + cl, ks * 32 + g * 8), oB[ks], da, 0,
                                                      0, 0);
      }
      // s[r] = score(key = k0 + sub*16 + 4g + r, query = qi); no masking on key tiles at or below this wave's queries
      if (k0 + 31 <= wq_min && wq_min + 15 < S) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[sub][r] = __expf(s[r] - lq) * (0.5f * da[r] - dq_);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kj = k0 + sub * 16 + g * 4 + r;
          const bool ok = qi < S && kj <= qi;
          const float pr = ok ? __expf(s[r] - lq) : 0.f;
          ds[sub][r] = pr * (0.5f * da[r] - dq_);
        }
      }
    }
    const bf16x8_t dsf = pack8(ds[0], ds[1]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
      acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_t_frag(sK, dt, g, cl), dsf, acc[dt], 0, 0, 0);
  }
  // acc[dt][r] = dQ^T[d = 16dt + 4g + r][query qi]
  if (qi < S) {
    float* o = dq + (((size_t)b * Hq + h) * S + qi) * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *(f32x4_t*)(o + dt * 16 + g * 4) = 0.5f * acc[dt];
  }
}

// ---------------------------------------------------------------------------------------------
// Inverse RoPE + q scale + GQA group sum of the dK/dV partials ([B,Hq,S,64] each) + scatter into
// token-major d[q|k|v] (bf16 [B*S, (Hq+2Hkv)*64]).
// Forward: r1 = x1 c - x2 s, r2 = x2 c + x1 s (first rot_dim dims).  Transpose: x1 = r1 c + r2 s,
// x2 = r2 c - r1 s.  One thread per (token, head, d).
__global__ __launch_bounds__(256) void lrp_rope_pack_kernel(const float* __restrict__ dq, const float* __restrict__ dk,
                                                            const float* __restrict__ dv,
                                                            const float* __restrict__ cosT,
                                                            const float* __restrict__ sinT, bf16_t* __restrict__ out,
                                                            int B, int S, int Hq, int Hkv, int rot_dim, float q_scale) {
  const int Ht = Hq + 2 * Hkv;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)B * S * Ht * 64;
  if (idx >= total) return;
  const int d = idx & 63;
  const size_t th = idx >> 6;
  const int hh = th % Ht;
  const size_t t = th / Ht;
  const int b = t / S, s = t - (size_t)b * S;
  const float* src;
  float scale = 1.f;
  bool rope = true;
  const int G = Hq / Hkv;
  int ng = 1;
  if (hh < Hq) {
    src = dq + (((size_t)b * Hq + hh) * S + s) * 64;
    scale = q_scale;
  } else if (hh < Hq + Hkv) {
    src = dk + (((size_t)b * Hq + (hh - Hq) * G) * S + s) * 64;
    ng = G;
  } else {
    src = dv + (((size_t)b * Hq + (hh - Hq - Hkv) * G) * S + s) * 64;
    ng = G;
    rope = false;
  }
  // dk / dv: sum of the per-q-head partials of the GQA group (head stride S*64)
  const int half = rot_dim >> 1;
  const int dp = (!rope || d >= rot_dim) ? d : (d < half ? d + half : d - half);
  float x0 = 0.f, xp = 0.f;
  for (int gi = 0; gi < ng; ++gi) {
    x0 += src[(size_t)gi * S * 64 + d];
    xp += src[(size_t)gi * S * 64 + dp];
  }
  float val;
  if (!rope || d >= rot_dim) {
    val = x0;
  } else if (d < half) {
    const float c = cosT[(size_t)s * half + d], sn = sinT[(size_t)s * half + d];
    val = x0 * c + xp * sn;
  } else {
    const int j = d - half;
    const float c = cosT[(size_t)s * half + j], sn = sinT[(size_t)s * half + j];
    val = x0 * c - xp * sn;
  }
  out[idx] = f2bf(val * scale);
}

// ---------------------------------------------------------------------------------------------
// Interleaved gate|up (blocks of 16 columns): a = silu(g) * u  and the LRP backward
//   dg = 0.5 dm u sigmoid(g)  (uniform rule on g*u, identity rule on SiLU),  du = 0.5 dm silu(g).
// One thread per 8 consecutive columns of one 16-column block: 16-byte loads and stores.
__global__ __launch_bounds__(256) void swiglu_il_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ a,
                                                        size_t n8, int I) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n8) return;
  const int I8 = I >> 3;
  const size_t t = idx / I8;
  const int c = (int)(idx - t * I8) * 8, blk = c >> 4, e = c & 15;
  const bf16_t* row = gu + t * (size_t)(2 * I) + blk * 32 + e;
  const u32x4_t gv = *(const u32x4_t*)row, uv = *(const u32x4_t*)(row + 16);
  u32x4_t o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float g0 = bf_lo(gv[i]), g1 = bf_hi(gv[i]);
    o[i] = pack_bf2(fast_silu(g0) * bf_lo(uv[i]), fast_silu(g1) * bf_hi(uv[i]));
  }
  *(u32x4_t*)(a + t * (size_t)I + c) = o;
}

__global__ __launch_bounds__(256) void lrp_swiglu_bwd_kernel(const bf16_t* __restrict__ dm,
                                                             const bf16_t* __restrict__ gu, bf16_t* __restrict__ dgu,
                                                             size_t n8, int I) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n8) return;
  const int I8 = I >> 3;
  const size_t t = idx / I8;
  const int c = (int)(idx - t * I8) * 8, blk = c >> 4, e = c & 15;
  const size_t off = t * (size_t)(2 * I) + blk * 32 + e;
  const u32x4_t gv = *(const u32x4_t*)(gu + off), uv = *(const u32x4_t*)(gu + off + 16);
  const u32x4_t mv = *(const u32x4_t*)(dm + t * (size_t)I + c);
  u32x4_t og, ou;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float g0 = bf_lo(gv[i]), g1 = bf_hi(gv[i]);
    const float s0 = fast_sigmoid(g0), s1 = fast_sigmoid(g1);
    const float m0 = 0.5f * bf_lo(mv[i]), m1 = 0.5f * bf_hi(mv[i]);
    og[i] = pack_bf2(m0 * bf_lo(uv[i]) * s0, m1 * bf_hi(uv[i]) * s1);
    ou[i] = pack_bf2(m0 * g0 * s0, m1 * g1 * s1);
  }
  *(u32x4_t*)(dgu + off) = og;
  *(u32x4_t*)(dgu + off + 16) = ou;
}

// GELU identity rule: dx = dy * gelu(a)/a (0.5 at a = 0).  a = pre-activation (bf16), in place on dy.
__global__ __launch_bounds__(256) void lrp_gelu_bwd_kernel(bf16_t* __restrict__ dy, const bf16_t* __restrict__ a,
                                                           size_t n) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n) return;
  const float x = bf2f(a[idx]);
  const float gel = 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  const float ratio = fabsf(x) > 1e-6f ? gel / x : 0.5f;
  dy[idx] = f2bf(bf2f(dy[idx]) * ratio);
}

// LayerNorm with detached variance (mean NOT detached): y = (x - mean x) * rstd * w + b.
// dx = gc - mean(gc), gc = dy * rstd * w.  out = resid + dx1 (+ dx2 for the second norm of the dual).
// One wave per row.  rstd [R] fp32.
__global__ __launch_bounds__(256) void lrp_ln_bwd_kernel(const bf16_t* __restrict__ dy1, const float* __restrict__ rs1,
                                                         const bf16_t* __restrict__ w1,
                                                         const bf16_t* __restrict__ dy2, const float* __restrict__ rs2,
                                                         const bf16_t* __restrict__ w2,
                                                         const bf16_t* __restrict__ resid, bf16_t* __restrict__ out,
                                                         int R, int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const size_t base = (size_t)row * H;
  const float r1 = rs1[row], r2 = dy2 ? rs2[row] : 0.f;
  float m1 = 0.f, m2 = 0.f;
  for (int c = lane; c < H; c += 64) {
    m1 += bf2f(dy1[base + c]) * r1 * bf2f(w1[c]);
    if (dy2) m2 += bf2f(dy2[base + c]) * r2 * bf2f(w2[c]);
  }
  m1 = wave_sum(m1) / H;
  m2 = wave_sum(m2) / H;
  for (int c = lane; c < H; c += 64) {
    float v = bf2f(resid[base + c]) + bf2f(dy1[base + c]) * r1 * bf2f(w1[c]) - m1;
    if (dy2) v += bf2f(dy2[base + c]) * r2 * bf2f(w2[c]) - m2;
    out[base + c] = f2bf(v);
  }
}

// LayerNorm statistics (for the rules above): rstd of (x - mean) per row.
__global__ __launch_bounds__(256) void ln_rstd_kernel(const bf16_t* __restrict__ x, float* __restrict__ rstd, int R,
                                                      int H, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const size_t base = (size_t)row * H;
  float s = 0.f;
  for (int c = lane; c < H; c += 64) s += bf2f(x[base + c]);
  const float mu = wave_sum(s) / H;
  float v = 0.f;
  for (int c = lane; c < H; c += 64) {
    const float d = bf2f(x[base + c]) - mu;
    v += d * d;
  }
  v = wave_sum(v) / H;
  if (lane == 0) rstd[row] = rsqrtf(v + eps);
}

// ---------------------------------------------------------------------------------------------
static inline unsigned nblk(size_t n) { return (unsigned)((n + 255) / 256); }

EDGE_API int edge_lrp_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dO,
                               const float* lse, float* D, float* rel, float* dq, float* dk, float* dv, int B, int Hq,
                               int Hkv, int S, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv) return (int)hipErrorInvalidValue;
  const int nb = (S + 63) / 64;
  lrp_attn_delta_kernel<<<B * Hq, 256, 0, st>>>((const bf16_t*)o, (const bf16_t*)dO, D, rel, Hq, S);
  lrp_attn_dkdv_kernel<<<B * Hq * nb, 256, 0, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                      (const bf16_t*)dO, lse, D, dk, dv, B, Hq, Hkv, S);
  lrp_attn_dq_kernel<<<B * Hq * nb, 256, 0, st>>>((const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                                                   (const bf16_t*)dO, lse, D, dq, B, Hq, Hkv, S);
  return (int)hipGetLastError();
}

EDGE_API int edge_lrp_rope_pack(const float* dq, const float* dk, const float* dv, const float* cosT,
                                const float* sinT, void* out, int B, int S, int Hq, int Hkv, int rot_dim,
                                float q_scale, hipStream_t st) {
  const size_t n = (size_t)B * S * (Hq + 2 * Hkv) * 64;
  if (!n) return 0;
  if (rot_dim > 64 || rot_dim % 2) return (int)hipErrorInvalidValue;
  lrp_rope_pack_kernel<<<nblk(n), 256, 0, st>>>(dq, dk, dv, cosT, sinT, (bf16_t*)out, B, S, Hq, Hkv, rot_dim,
                                                 q_scale);
  return (int)hipGetLastError();
}

EDGE_API int edge_swiglu_il(const void* gu, void* a, long long T, int I, hipStream_t st) {
  const size_t n8 = (size_t)T * I / 8;
  if (!n8) return 0;
  if (I % 16) return (int)hipErrorInvalidValue;
  swiglu_il_kernel<<<nblk(n8), 256, 0, st>>>((const bf16_t*)gu, (bf16_t*)a, n8, I);
  return (int)hipGetLastError();
}

EDGE_API int edge_lrp_swiglu_bwd(const void* dm, const void* gu, void* dgu, long long T, int I, hipStream_t st) {
  const size_t n8 = (size_t)T * I / 8;
  if (!n8) return 0;
  if (I % 16) return (int)hipErrorInvalidValue;
  lrp_swiglu_bwd_kernel<<<nblk(n8), 256, 0, st>>>((const bf16_t*)dm, (const bf16_t*)gu, (bf16_t*)dgu, n8, I);
  return (int)hipGetLastError();
}

EDGE_API int edge_lrp_gelu_bwd(void* dy, const void* a, long long n, hipStream_t st) {
  if (n <= 0) return 0;
  lrp_gelu_bwd_kernel<<<nblk(n), 256, 0, st>>>((bf16_t*)dy, (const bf16_t*)a, (size_t)n);
  return (int)hipGetLastError();
}

EDGE_API int edge_lrp_ln_bwd(const void* dy1, const float* rs1, const void* w1, const void* dy2, const float* rs2,
                             const void* w2, const void* resid, void* out, int R, int H, hipStream_t st) {
  if (R <= 0) return 0;
  lrp_ln_bwd_kernel<<<(R + 3) / 4, 256, 0, st>>>((const bf16_t*)dy1, rs1, (const bf16_t*)w1, (const bf16_t*)dy2,
                                                 rs2, (const bf16_t*)w2, (const bf16_t*)resid, (bf16_t*)out, R, H);
  return (int)hipGetLastError();
}

EDGE_API int edge_ln_rstd(const void* x, float* rstd, int R, int H, float eps, hipStream_t st) {
  if (R <= 0) return 0;
  ln_rstd_kernel<<<(R + 3) / 4, 256, 0, st>>>((const bf16_t*)x, rstd, R, H, eps);
  return (int)hipGetLastError();
}
