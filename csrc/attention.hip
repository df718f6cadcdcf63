// Causal GQA attention for head_dim 64 on gfx950 MFMA, plus the token-importance scorers of the
// reference:
//
//   flash_attn_fwd : O = softmax(Q K^T) V with online softmax, never materialising S x S; optional
//                    per-row LSE output (input of the column-sum scorer): mask-free interior tiles, exp2 + lazy
//                    rescale, 3-stage ring, XCD-aware order, two query tiles per wave.
//   attn_lastrow   : P[S-1, :] per head  -> "last_row" importance (Qwen2-0.5B/main.py:80-86).
//   attn_colsum    : sum_i P[i, j] per head, recomputed from Q, K and the LSE (FA-backward style sweep,
//                    key block outer / query tiles inner) -> "regular_importance", "weighted_importance",
//                    "aggregate_till" (Qwen2-0.5B/main.py:46-92).
//   head_combine   : out[b, j] (+)= scale * sum_h w[h] * x[b, h, j].
//
// Layouts: q [B,Hq,S,64] (RoPE applied, pre-scaled by 1/sqrt(64)), k [B,Hkv,S,64], vt [B,Hkv,64,S_pad]
// (V transposed, zero padded to a multiple of 64 keys), o [B*S, Hq*64] token-major.
//
// Forward structure: one workgroup = 4 waves = 64 query rows of one head; each wave owns 16 rows. K and
// V^T tiles of 64 keys are staged to LDS by global_load_lds (XOR-swizzled source), double-buffered and
// shared by the 4 waves. S^T = K.Q^T is computed with the key on the MFMA row so each lane holds 16
// scores of ONE query row: the row max is 15 fmax + 2 shuffles, the P fragment for the P.V MFMA is the
// lane's own registers (keys permuted identically in the V^T operand), and the O^T accumulator keeps
// the query on the lane so the alpha rescale is lane-local.
#include "common.h"

namespace {
constexpr int KT = 64;                // keys per tile
constexpr int TILE = KT * 128;        // 64 rows x 128 B
__device__ __forceinline__ int aswz(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void stage64(const bf16_t* __restrict__ base, size_t row_stride, int row0, int row_max,
                                        int col0, char* lds, int wave, int lane) {
  // 8 wave-instructions of 1 KiB (8 rows x 128 B) per 64x64 bf16 tile; 2 per wave.
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = i * 4 + wave;
    const int r = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ aswz(r);
    int gr = row0 + r;
    gr = gr < row_max ? gr : row_max - 1;
    glds16(base + (size_t)gr * row_stride + col0 + c * 8, lds + blk * 1024);
  }
}
}  // namespace

// ---------------------------------------------------------------------------------------------
// Forward tile body (round 1 measured a plain one-tile-per-wave loop at ≈210 VALU per wave per 64-key tile against
// 16 MFMAs, with a 1-tile load lead that left every tile waiting on L2/MALL):
//   * masking only on the diagonal tile (kb == qb is the only tile with keys > query or keys >= S);
//     interior tiles run a mask-free body;
//   * exp2 domain: p = exp2(fma(s, log2e, -m2)) (one FMA + one v_exp per score);
//   * lazy rescaling: the running max moves only when a row's tile max exceeds it by more than TAU = 8
//     (log2 units, wave-uniform decision), so the alpha rescale of O and l is skipped on most tiles and
//     p stays <= 2^8 (exact in fp32, representable in bf16);
//   * a 3-stage K/V ring: tile kb+2 is issued while tile kb is computed (vmcnt(4) keeps tile kb+1 in
//     flight across the barrier);
//   * XCD-aware block order: the query blocks and heads of one (window, kv head) group run on one XCD,
//     so its K/V tiles are fetched into that XCD's L2 once; heavy (late) query blocks are dispatched first.
namespace {
constexpr float LOG2E = 1.4426950408889634f;
constexpr float TAU = 8.f;
constexpr int NST = 3;

}  // namespace

// ---------------------------------------------------------------------------------------------
// The forward: TWO 16-row query tiles per wave (128 query rows per workgroup).
// One tile per wave reads 16 ds_read_b128 (8 K + 8 V^T fragments) per 16 MFMAs per wave and tile: at 3 waves per SIMD that
// alone asks ~250 B/clk/CU of the LDS array (peak 256).  Here every K and V^T fragment feeds both row tiles,
// so the reads per MFMA halve.  Each wave runs the key tiles up to its own last row (wave-uniform skip of
// the tile past the diagonal) and masks exactly one tile; softmax state is per row tile.
namespace {
template <bool MASK>
__device__ __forceinline__ void fa3_tile(const char* lk, const char* lv, const bf16x8_t (&qf)[2][2],
                                         f32x4_t (&oacc)[2][4], float (&m2)[2], float (&l_run)[2], int kb, int q0,
                                         int S, int g, int ql) {
  f32x4_t st[2][4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    st[0][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    st[1][ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int r = 32 * (ni >> 1) + 8 * (ql >> 2) + 4 * (ni & 1) + (ql & 3);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8_t kf = *(const bf16x8_t*)(lk + r * 128 + (((ks * 4 + g) ^ aswz(r)) << 4));
      st[0][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[0][ks], st[0][ni], 0, 0, 0);
      st[1][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[1][ks], st[1][ni], 0, 0, 0);
    }
  }
  bf16x8_t pf[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if constexpr (MASK) {
      const int qrow = q0 + t * 16 + ql;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb * KT + 32 * (ni >> 1) + 8 * g + 4 * (ni & 1) + r;
          if (key > qrow || key >= S) st[t][ni][r] = -INFINITY;
        }
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, st[t][ni][r]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float mc = mloc * LOG2E;
    if (__builtin_amdgcn_ballot_w64(mc > m2[t] + TAU)) {   // wave-uniform: rescale every row of tile t exactly
      const float mn = fmaxf(m2[t], mc);
      const float alpha = __builtin_amdgcn_exp2f(m2[t] - mn);
      m2[t] = mn;
      l_run[t] *= alpha;
#pragma unroll
      for (int d = 0; d < 4; ++d) oacc[t][d] *= alpha;
    }
    float ps = 0.f;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(st[t][ni][r], LOG2E, -m2[t]));
        ps += p;
        pf[t][ni >> 1][(ni & 1) * 4 + r] = (__bf16)p;
      }
    l_run[t] += ps;
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const int row = dt * 16 + ql;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8_t vf = *(const bf16x8_t*)(lv + row * 128 + (((ks * 4 + g) ^ aswz(row)) << 4));
      oacc[0][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[0][ks], oacc[0][dt], 0, 0, 0);
      oacc[1][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[1][ks], oacc[1][dt], 0, 0, 0);
    }
  }
}
}  // namespace

template <int OCC>
__global__ __launch_bounds__(256, OCC) void flash_attn_fwd3_kernel(const bf16_t* __restrict__ q,
                                                                 const bf16_t* __restrict__ k,
                                                                 const bf16_t* __restrict__ vt,
                                                                 bf16_t* __restrict__ o, float* __restrict__ lse,
                                                                 const float* __restrict__ n_rows,
                                                                 int B, int Hq, int Hkv, int S, int s_pad) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, ql = lane & 15;
  const int nqb = (S + 127) / 128;
  const int G = Hq / Hkv, NG = B * Hkv;
  // XCD-aware order: XCD `xcd` owns (window, kv head) groups xcd, xcd+8, ...; heavy query blocks first
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int cnt = (NG - xcd + 7) >> 3;
  const int per_qb = cnt * G;
  if (j >= per_qb * nqb) return;
  const int qb = nqb - 1 - j / per_qb;
  const int rem = j - (nqb - 1 - qb) * per_qb;
  const int grp = xcd + 8 * (rem / G);
  const int b = grp / Hkv, hk = grp - b * Hkv, h = hk * G + rem % G;
  if (n_rows && qb * 128 + 127 < S - 1 - (int)n_rows[b]) return;  // scored-rows mode (last layer)

  const bf16_t* qh = q + ((size_t)b * Hq + h) * S * 64;
  const bf16_t* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const bf16_t* vh = vt + ((size_t)b * Hkv + hk) * 64 * (size_t)s_pad;

  const int q0 = qb * 128 + wave * 32;  // this wave's rows: q0 + 16 t + ql
  bf16x8_t qf[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int qrow = q0 + t * 16 + ql;
    const int qld = qrow < S ? qrow : S - 1;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[t][ks] = *(const bf16x8_t*)(qh + (size_t)qld * 64 + ks * 32 + g * 8);
  }
  f32x4_t oacc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int d = 0; d < 4; ++d) oacc[t][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m2[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};

  const int nkb = min(2 * qb + 2, (S + KT - 1) / KT);
  const int kmax = (q0 + 31) / KT;  // last key tile this wave needs (wave-uniform)
  stage64(kh, 64, 0, S, 0, smem, wave, lane);
  stage64(vh, s_pad, 0, 64, 0, smem + TILE, wave, lane);
  if (nkb > 1) {
    stage64(kh, 64, KT, S, 0, smem + 2 * TILE, wave, lane);
    stage64(vh, s_pad, 0, 64, KT, smem + 3 * TILE, wave, lane);
  }
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kb + 2 < nkb) {
      char* nx = smem + ((kb + 2) % NST) * 2 * TILE;
      stage64(kh, 64, (kb + 2) * KT, S, 0, nx, wave, lane);
      stage64(vh, s_pad, 0, 64, (kb + 2) * KT, nx + TILE, wave, lane);
    }
    if (kb > kmax) continue;  // every key of this tile is past this wave's rows
    const char* cur = smem + (kb % NST) * 2 * TILE;
    if (kb * KT + KT - 1 <= q0 && kb * KT + KT - 1 < S)
      fa3_tile<false>(cur, cur + TILE, qf, oacc, m2, l_run, kb, q0, S, g, ql);
    else
      fa3_tile<true>(cur, cur + TILE, qf, oacc, m2, l_run, kb, q0, S, g, ql);
  }

#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float l = l_run[t];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const int qrow = q0 + t * 16 + ql;
    if (qrow < S) {
      const float inv = __builtin_amdgcn_rcpf(l);
      bf16_t* orow = o + ((size_t)b * S + qrow) * (size_t)(Hq * 64) + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        u32x2_t w;
        w[0] = pack_bf2(oacc[t][dt][0] * inv, oacc[t][dt][1] * inv);
        w[1] = pack_bf2(oacc[t][dt][2] * inv, oacc[t][dt][3] * inv);
        *(u32x2_t*)(orow + dt * 16 + g * 4) = w;
      }
      if (lse && g == 0) lse[((size_t)b * Hq + h) * S + qrow] = m2[t] * 0.6931471805599453f + logf(l);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Last-row probabilities: one workgroup per (b, h); P[S-1, j] = softmax_j(q_{S-1} . k_j).
__global__ __launch_bounds__(256) void attn_lastrow_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                           float* __restrict__ out, int Hq, int Hkv, int S) {
  extern __shared__ float sc[];  // S scores
  __shared__ float qv[64];
  __shared__ float red[4];
  const int bh = blockIdx.x, b = bh / Hq, h = bh - b * Hq, hk = h / (Hq / Hkv);
  const bf16_t* qr = q + (((size_t)b * Hq + h) * S + (S - 1)) * 64;
  const bf16_t* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  if (threadIdx.x < 64) qv[threadIdx.x] = bf2f(qr[threadIdx.x]);
  __syncthreads();
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < S; j += 256) {
    const u32x4_t* kr = (const u32x4_t*)(kh + (size_t)j * 64);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const u32x4_t w = kr[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) s += qv[c * 8 + 2 * e] * bf_lo(w[e]) + qv[c * 8 + 2 * e + 1] * bf_hi(w[e]);
    }
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = block_max<256>(mx, red);
  float sum = 0.f;
  for (int j = threadIdx.x; j < S; j += 256) {
    const float p = __expf(sc[j] - mx);
    sc[j] = p;
    sum += p;
  }
  sum = block_sum<256>(sum, red);
  const float inv = 1.f / sum;
  float* orow = out + (size_t)bh * S;
  for (int j = threadIdx.x; j < S; j += 256) orow[j] = sc[j] * inv;
}

// ---------------------------------------------------------------------------------------------
// Column sums of P for one (b, h, 64-key block): sum over query rows i >= key of exp(q_i.k_j - lse_i).
// D = Q K^T with the key on the MFMA column: lane holds key (lane&15)+16ni for query rows 4g+r, so the
// column sum over a 16-row tile is 4 lane-local adds; waves split the query tiles, LDS combines them.
__global__ __launch_bounds__(256) void attn_colsum_kernel(const bf16_t* __restrict__ q, const bf16_t* __restrict__ k,
                                                          const float* __restrict__ lse, float* __restrict__ out,
                                                          int B, int Hq, int Hkv, int S) {
  __shared__ float part[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int nkb = (S + 63) / 64;
  const int kb = blockIdx.x % nkb;
  const int bh = blockIdx.x / nkb, b = bh / Hq, h = bh - b * Hq, hk = h / (Hq / Hkv);
  const bf16_t* qh = q + ((size_t)b * Hq + h) * S * 64;
  const bf16_t* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const float* lh = lse + ((size_t)b * Hq + h) * S;

  bf16x8_t kf[4][2];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    int key = kb * 64 + ni * 16 + cl;
    key = key < S ? key : S - 1;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) kf[ni][ks] = *(const bf16x8_t*)(kh + (size_t)key * 64 + ks * 32 + g * 8);
  }
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  // query tiles of 16 rows starting at the first row that can see this key block
  for (int qt = kb * 4 + wave; qt * 16 < S; qt += 4) {
    const int qa = qt * 16 + cl;            // row this lane loads for the A operand
    const int qla = qa < S ? qa : S - 1;
    bf16x8_t qf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[ks] = *(const bf16x8_t*)(qh + (size_t)qla * 64 + ks * 32 + g * 8);
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
      for (int ks = 0; ks < 2; ++ks) s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf[ni][ks], s, 0, 0, 0);
      const int key = kb * 64 + ni * 16 + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = qt * 16 + g * 4 + r;
        csum[ni] += (qi >= key && qi < S) ? __expf(s[r] - lrow[r]) : 0.f;
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
    if (key < S) out[((size_t)b * Hq + h) * S + key] = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
  }
}

// out[b, j] = beta * out[b, j] + scale * sum_h w[h] * x[b, h, j]   (w == nullptr -> all ones)
__global__ __launch_bounds__(256) void head_combine_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           float* __restrict__ out, int B, int Hq, int S, float scale,
                                                           float beta) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * S) return;
  const int b = idx / S, j = idx - b * S;
  float acc = 0.f;
  for (int h = 0; h < Hq; ++h) acc += (w ? w[h] : 1.f) * x[((size_t)b * Hq + h) * S + j];
  out[idx] = (beta != 0.f ? beta * out[idx] : 0.f) + scale * acc;
}

// n_rows (nullable, [B] fp32): per-window count of scored rows (the last n_rows[b]+1 positions); query
// blocks entirely before them are skipped (their O rows are left unwritten).
EDGE_API int edge_flash_attn_fwd(const void* q, const void* k, const void* vt, void* o, float* lse, const float* n_rows,
                                 int B, int Hq, int Hkv, int S, int s_pad, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv || s_pad % 64 || s_pad < S) return (int)hipErrorInvalidValue;
  // 3 workgroups per CU (58.5 us at the bench shape, against 70.5 for the one-tile-per-wave kernel)
  const int G = Hq / Hkv, maxcnt = (B * Hkv + 7) / 8;
  const dim3 grid(8 * maxcnt * G * ((S + 127) / 128));
  hipLaunchKernelGGL(flash_attn_fwd3_kernel<3>, grid, dim3(256), 2 * NST * TILE, st, (const bf16_t*)q,
                     (const bf16_t*)k, (const bf16_t*)vt, (bf16_t*)o, lse, n_rows, B, Hq, Hkv, S, s_pad);
  return (int)hipGetLastError();
}

EDGE_API int edge_attn_lastrow(const void* q, const void* k, float* out, int B, int Hq, int Hkv, int S,
                               hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv || S > 16384) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(attn_lastrow_kernel, dim3(B * Hq), dim3(256), S * sizeof(float), st, (const bf16_t*)q,
                     (const bf16_t*)k, out, Hq, Hkv, S);
  return (int)hipGetLastError();
}

EDGE_API int edge_attn_colsum(const void* q, const void* k, const float* lse, float* out, int B, int Hq, int Hkv,
                              int S, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv) return (int)hipErrorInvalidValue;
  const int nkb = (S + 63) / 64;
  hipLaunchKernelGGL(attn_colsum_kernel, dim3(B * Hq * nkb), dim3(256), 0, st, (const bf16_t*)q, (const bf16_t*)k,
                     lse, out, B, Hq, Hkv, S);
  return (int)hipGetLastError();
}

EDGE_API int edge_head_combine(const float* x, const float* w, float* out, int B, int Hq, int S, float scale,
                               float beta, hipStream_t st) {
  if (B * S <= 0) return 0;
  head_combine_kernel<<<(B * S + 255) / 256, 256, 0, st>>>(x, w, out, B, Hq, S, scale, beta);
  return (int)hipGetLastError();
}
