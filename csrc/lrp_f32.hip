// AttnLRP relevance backward at the reference's precision (fp32; SURVEY §2.4 K17, reference C8:
// Experiments/Relevance/main.py:84-103, normalisation :111-118).
//
// The bf16 engine (lrp.hip) stores every operand in bf16.  This file is its fp32 counterpart, built around the
// fp32 execution mode of the forward (csrc/common.h "h3"): every GEMM of the backward pass - the input gradients
// through the frozen projections, with the transposed weights - runs on the same split-fp16 matrix-core GEMM as
// the forward (csrc/gemm.hip EPI_F32*), and the non-GEMM parts are here, in fp32:
//
//   lrp_attn_delta_f32  D[b,h,i] = 0.5 dO_i . O_i (uniform rule on A V) and the per-(window, head) relevance
//                       rel[b,h] = sum_i D[b,h,i] = sum_{ij} A_ij dA_ij - the reference hook's quantity.
//   lrp_attn_dkdv_h3    dK, dV per (window, q head or kv-head group, 64-key block): P recomputed from Q K^T and the
//                       forward LSE, dA = 0.5 dO V^T, dS = P (dA - D), dV = 0.5 P^T dO, dK = 0.5 dS^T Q.
//   lrp_attn_dq_h3      dQ = 0.5 dS K per (window, q head, 64-query block).  Separate sweeps: no atomics.
//                       Products on scaled two-fp16-plane splits (three products).
//   *_h3 rule kernels   the LRP rules whose output feeds a backward GEMM (SwiGLU / GELU identity rule with the
//                       uniform product rule, inverse RoPE + GQA sum) write it directly as an h3 activation with a
//                       per-row power-of-two scale: gradients have no a-priori bound, so each row is scaled to put
//                       its own max |value| just below 2^15 (fp16 planes can never overflow) and the GEMM's
//                       per-row epilogue scale multiplies by the inverse (exact: powers of two), times an optional
//                       per-row factor (the detached norm's rstd).
//   split_h3_dyn        the same per-row-scaled split for a plain fp32 gradient (the residual stream).
//   swiglu_h3 / gelu_h3 forward activations from the saved fp32 pre-activations to the down / proj GEMM input.
//   row_rstd_f32, lrp_ln_bwd_f32, group_absprod   detached-norm statistics, the LayerNorm rule, and the
//                       channel-group relevance sum |x dx| of the boundary codec's bit allocation.
//
// f32 MFMA 16x16x4: lane l holds A[row = l&15][k = l>>4], B[k = l>>4][col = l&15], C[row = 4(l>>4)+r][col = l&15].
// The 64-wide reductions over the head dimension use the order d(s, g) = 16(s>>2) + 4g + (s&3) for step s and
// k-slot g, so a lane's four consecutive steps read four consecutive floats (one 16-byte LDS read); the reductions
// over tokens use the lane-local probabilities with k-slot g <-> token 4g + kk (the bf16 kernels' trick).
#include "common.h"

namespace {
constexpr int LDF = 68;   // LDS row stride (floats) of the staged 64-wide tiles

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Stage 64 rows x 64 floats (row stride `ld` floats; rows >= nrows zero-filled) into an LDS tile [64][LDF].
__device__ __forceinline__ void stage64(const float* __restrict__ src, size_t ld, int row0, int nrows, float* t) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = threadIdx.x + it * 256, r = idx >> 4, c = (idx & 15) * 4;
    const int gr = row0 + r;
    f32x4_t v = {0.f, 0.f, 0.f, 0.f};
    if (gr < nrows) v = *(const f32x4_t*)(src + (size_t)gr * ld + c);
    *(f32x4_t*)(t + r * LDF + c) = v;
  }
}

// Power-of-two row scale: s = 2^(15 - E) with max = m 2^E, m in [0.5, 1): s * max < 2^15.  Returns s, sets inv = 1/s.
__device__ __forceinline__ float row_pow2_scale(float mx, float& inv) {
  if (!(mx > 0.f) || !isfinite(mx)) {
    inv = 1.f;
    return 1.f;
  }
  int e;
  (void)frexpf(mx, &e);
  const int sh = 15 - e;
  inv = ldexpf(1.f, -sh);
  return ldexpf(1.f, sh);
}

__device__ __forceinline__ float sigmoid_f32(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float gelu_f32(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_ratio(float x) { return fabsf(x) > 1e-6f ? gelu_f32(x) / x : 0.5f; }
}  // namespace

// ---------------------------------------------------------------------------------------------
// D and per-(window, head) relevance.  o, dO token-major fp32 [B*S, Hq*64]; D [B,Hq,S]; rel [B,Hq].
__global__ __launch_bounds__(256) void lrp_attn_delta_f32_kernel(const float* __restrict__ o,
                                                                 const float* __restrict__ dO, float* __restrict__ D,
                                                                 float* __restrict__ rel, int Hq, int S,
                                                                 float* __restrict__ dmax) {
  // 16 lanes per token row (4 consecutive values each: every load instruction reads 4 whole 256-byte rows), the
  // row's dot product reduced over its 16 lanes by xor shuffles
  __shared__ float red[4];
  const int bh = blockIdx.x, b = bh / Hq, h = bh - b * Hq;
  const int sub = threadIdx.x & 15, r0 = threadIdx.x >> 4;
  float tot = 0.f, mx = 0.f;
  for (int i = r0; i < S; i += 16) {
    const size_t off = ((size_t)b * S + i) * (size_t)(Hq * 64) + h * 64 + sub * 4;
    const f32x4_t a = *(const f32x4_t*)(o + off), d = *(const f32x4_t*)(dO + off);
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(d[0]), fabsf(d[1])), fmaxf(fabsf(d[2]), fabsf(d[3]))));
    float s = fmaf(a[0], d[0], fmaf(a[1], d[1], fmaf(a[2], d[2], a[3] * d[3])));
#pragma unroll
    for (int x = 1; x < 16; x <<= 1) s += __shfl_xor(s, x, 64);
    s *= 0.5f;
    if (sub == 0) {
      D[(size_t)bh * S + i] = s;
      tot += s;
    }
  }
  tot = block_sum<256>(tot, red);
  if (threadIdx.x == 0) rel[bh] = tot;
  if (dmax) {   // (uniform branch: every thread takes part in the reduction)
    __syncthreads();
    mx = block_max<256>(mx, red);
    if (threadIdx.x == 0) dmax[bh] = mx;
  }
}

// ---------------------------------------------------------------------------------------------
// The dK / dV and dQ sweeps on scaled fp16 planes ("h3", the forward attention's scheme): every operand - q, k, v,
// dO, and the in-register P and dS - is scaled by a power of two and split into two fp16 planes, and each product is
// the three plane products lo x hi + hi x lo + hi x hi on v_mfma_f32_16x16x32_f16.  The scales keep every plane inside
// the fp16 range:
//   q, k, v  sq, sk, sv: the forward attention's model bounds (s |x| <= 2^15, models/model.py h3 scales)
//   dO       so = 2^(15 - E) from the max |dO| over the kv head's q heads (the delta kernel's per-head maxima)
//   P        sp = 2^14 (P <= 1)
//   dS       sd = so sv 2^-21: |dS| <= |P| (|dA| / 2 + |D|) <= 64 max|dO| max|v| < 2^15 / sd
// Values far below their scale keep an absolute error of ~2^-25 / s (fp16's subnormal step): ~2^-40 relative to the
// largest value of the same operand.  Round 4's form split every operand into three bf16 planes instead (six
// products, no scales, fp32's exponent range on every element): 1.34x the time of these sweeps
// (profiles/history/r05/lrp_attn_h3/probe.log), removed.
//
// 16x16x32 fragments: lane l holds A[row l&15][k 8(l>>4)+j] and B[k 8(l>>4)+j][col l&15], C[row 4(l>>4)+r][col l&15].
// A score tile computed with the query (dkdv) or the key (dq) on the C rows puts 4 rows of a 16-row block on a lane;
// two such blocks give the lane the 8 k-slots of a 32-deep reduction over those rows, in the order
// slot 8g + j <-> row perm(g, j) = (j < 4 ? 4g + j : 16 + 4g + j - 4): the probabilities / dS are then the lane's own
// A / B fragments, and the other operand is read from its row-major LDS image in that row order by transposing reads
// (ds_read_b64_tr_b16).  A 32 x 64 tile is staged row-major only ([32][64] per plane, 16-byte chunks swizzled):
// thread t owns the row pair 2 rp, 2 rp + 1 and columns 4 c4 .. +3 (tile_own): two 16-byte global loads (tile_load,
// issued a tile ahead so their latency hides under the previous tile's MFMAs) and one 8-byte write per row and plane.
namespace {
// 16-byte chunk swizzle of the row-major images (128-byte rows): conflict-free for the b64 staging writes, the b128
// row-fragment reads and the ds_read_b64_tr_b16 transposed reads alike (searched over the XOR maps of the row bits
// with the bank model of MI355X_MICROARCH §LDS; the plain (r >> 1) & 7 is 2-way on the writes and the tr reads)
__device__ __forceinline__ int tile_sw(int r) { return (((r >> 1) & 1) << 1) | ((((r >> 1) ^ (r >> 2)) & 1) << 2); }
typedef short s4_t __attribute__((ext_vector_type(4)));
struct TileRegs { f32x4_t v[2]; };
__device__ __forceinline__ void tile_own(int t, int& r, int& c4) {
  const int w = t >> 6, l = t & 63, q = (l >> 3) & 3;
  r = 2 * (2 * w + (q & 1) + 8 * (q >> 1));
  c4 = (l & 7) + 8 * (l >> 5);
}
__device__ __forceinline__ void tile_load(const float* __restrict__ src, size_t ld, int row0, int nrows, TileRegs& R) {
  int r, c4;
  tile_own(threadIdx.x, r, c4);
  const int c = 4 * c4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int gr = row0 + r + i;
    R.v[i] = gr < nrows ? *(const f32x4_t*)(src + (size_t)gr * ld + c) : f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
}
constexpr int H3P = 32 * 64 * 2;   // one fp16 plane of a 32 x 64 tile (bytes)
__device__ __forceinline__ f32x4_t mfma_f16r(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                0, 0, 0);
}
__device__ __forceinline__ f32x4_t h3dot(const bf16x8_t (&a)[2], const bf16x8_t (&b)[2], f32x4_t c) {
  c = mfma_f16r(a[1], b[0], c);
  c = mfma_f16r(a[0], b[1], c);
  return mfma_f16r(a[0], b[0], c);
}
// s * v[0..7] as the two fp16 planes of one fragment
__device__ __forceinline__ void split_frag_s(const float (&v)[8], float s, bf16x8_t (&p)[2]) {
  u32x4_t H, L;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const u32x2_t t = split2h_pk(v[2 * e] * s, v[2 * e + 1] * s);
    H[e] = t[0];
    L[e] = t[1];
  }
  p[0] = __builtin_bit_cast(bf16x8_t, H);
  p[1] = __builtin_bit_cast(bf16x8_t, L);
}
// the staged tile's two fp16 planes of s * x
__device__ __forceinline__ void h3_store(const TileRegs& R, char* rm, float s) {
  int r, c4;
  tile_own(threadIdx.x, r, c4);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const u32x2_t t0 = split2h_pk(R.v[i][0] * s, R.v[i][1] * s), t1 = split2h_pk(R.v[i][2] * s, R.v[i][3] * s);
    const int row = r + i;
    const int off = row * 128 + (((c4 >> 1) ^ tile_sw(row)) << 4) + (c4 & 1) * 8;
    *(u32x2_t*)(rm + off) = u32x2_t{t0[0], t1[0]};
    *(u32x2_t*)(rm + H3P + off) = u32x2_t{t0[1], t1[1]};
  }
}
__device__ __forceinline__ void rm_frags_h(const char* img, int row, int chunk, bf16x8_t (&f)[2]) {
#pragma unroll
  for (int pl = 0; pl < 2; ++pl) f[pl] = *(const bf16x8_t*)(img + pl * H3P + row * 128 + ((chunk ^ tile_sw(row)) << 4));
}
__device__ __forceinline__ void tr_frags_h(const char* img, int dt, int g, int cl, bf16x8_t (&f)[2]) {
  const int q = cl >> 2, p = cl & 3, ch = 2 * dt + (p >> 1);
  const int r0 = 4 * g + q, r1 = 16 + 4 * g + q;
  const int o0 = r0 * 128 + ((ch ^ tile_sw(r0)) << 4) + (p & 1) * 8;
  const int o1 = r1 * 128 + ((ch ^ tile_sw(r1)) << 4) + (p & 1) * 8;
#pragma unroll
  for (int pl = 0; pl < 2; ++pl) {
    typedef __attribute__((address_space(3))) s4_t lds_s4;
    const s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + pl * H3P + o0));
    const s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + pl * H3P + o1));
    const short __attribute__((ext_vector_type(8))) v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    f[pl] = __builtin_bit_cast(bf16x8_t, v);
  }
}
__device__ __forceinline__ void row_frags_h(const float* __restrict__ rowp, bf16x8_t (&f)[2][2], int g, float s) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const f32x4_t a = *(const f32x4_t*)(rowp + 32 * ks + 8 * g);
    const f32x4_t b = *(const f32x4_t*)(rowp + 32 * ks + 8 * g + 4);
    const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    split_frag_s(v, s, f[ks]);
  }
}
// the dO scale of kv head hk of window b: 2^(15 - E) for the max over its G q heads' max |dO| = m 2^E
__device__ __forceinline__ float dO_scale(const float* __restrict__ dmax, int b, int Hq, int hk, int G) {
  float mx = 0.f;
  for (int j = 0; j < G; ++j) mx = fmaxf(mx, dmax[(size_t)b * Hq + hk * G + j]);
  float inv;
  return row_pow2_scale(mx, inv);
}
}  // namespace

template <bool GS>
__global__ __launch_bounds__(256) void lrp_attn_dkdv_h3_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                               const float* __restrict__ v,
                                                               const float* __restrict__ dO,
                                                               const float* __restrict__ lse,
                                                               const float* __restrict__ D,
                                                               const float* __restrict__ dmax, float* __restrict__ dk,
                                                               float* __restrict__ dv, int B, int Hq, int Hkv, int S,
                                                               float sq, float sk, float sv) {
  // double-buffered tiles: tile it + 1 is staged while tile it is computed, one barrier per tile
  __shared__ __attribute__((aligned(16))) char sQ[2][2 * H3P], sO[2][2 * H3P];
  __shared__ float sL[2][32], sD[2][32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int G = Hq / Hkv, HH = GS ? Hkv : Hq, NH = GS ? G : 1;
  const int kb = blockIdx.x / (B * HH);
  const int bh = blockIdx.x % (B * HH), b = bh / HH, hx = bh - b * HH;
  const int hk = GS ? hx : hx / G, h0 = GS ? hx * G : hx;
  const int key = kb * 64 + wave * 16 + cl;
  const int keyc = key < S ? key : S - 1;
  const int wkey_max = kb * 64 + __builtin_amdgcn_readfirstlane(wave) * 16 + 15;
  const float so = dO_scale(dmax, b, Hq, hk, G);
  const float sp = 16384.f, sd = so * sv * 0x1p-21f;
  // P = 2^(sc c1 - lse log2 e), dS = P (da c2 - D): the product scales folded into c1, c2
  const float c1 = 1.4426950408889634f / (sq * sk), c2 = 0.5f / (so * sv);
  bf16x8_t kf[2][2], vf[2][2];
  row_frags_h(k + (((size_t)b * Hkv + hk) * S + keyc) * 64, kf, g, sk);
  row_frags_h(v + (((size_t)b * Hkv + hk) * S + keyc) * 64, vf, g, sv);
  f32x4_t dka[4], dva[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dka[d] = dva[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int ntile = (S - kb * 64 + 31) / 32, nit = NH * ntile;
  TileRegs rq, ro;
  float nl = INFINITY, nd = 0.f;
  auto fetch = [&](int it) {
    const int hh = h0 + it / ntile, q0 = kb * 64 + 32 * (it % ntile);
    tile_load(q + ((size_t)b * Hq + hh) * S * 64, 64, q0, S, rq);
    tile_load(dO + (size_t)b * S * (Hq * 64) + hh * 64, (size_t)Hq * 64, q0, S, ro);
    if (tid < 32) {
      const int qi = q0 + tid;
      nl = qi < S ? lse[((size_t)b * Hq + hh) * S + qi] * 1.4426950408889634f : INFINITY;
      nd = qi < S ? D[((size_t)b * Hq + hh) * S + qi] : 0.f;
    }
  };
  auto stage = [&](int buf) {
    h3_store(rq, sQ[buf], sq);
    h3_store(ro, sO[buf], so);
    if (tid < 32) sL[buf][tid] = nl, sD[buf][tid] = nd;
  };
  fetch(0);
  stage(0);
  if (nit > 1) fetch(1);
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int q0 = kb * 64 + 32 * (it % ntile), cb = it & 1;
    const char* bQ = sQ[cb];
    const char* bO = sO[cb];
    const float* bL = sL[cb];
    const float* bD = sD[cb];
    float pv[8], dsv[8];
    const bool full = q0 >= wkey_max && q0 + 32 <= S && wkey_max < S;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x4_t sc = {0.f, 0.f, 0.f, 0.f}, da = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t qa[2], oa[2];
        rm_frags_h(bQ, sub * 16 + cl, 4 * ks + g, qa);
        rm_frags_h(bO, sub * 16 + cl, 4 * ks + g, oa);
        sc = h3dot(qa, kf[ks], sc);
        da = h3dot(oa, vf[ks], da);
      }
      if (full) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = sub * 16 + 4 * g + r;
          const float pr = __builtin_amdgcn_exp2f(fmaf(sc[r], c1, -bL[ql]));
          pv[4 * sub + r] = pr;
          dsv[4 * sub + r] = pr * fmaf(da[r], c2, -bD[ql]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = sub * 16 + 4 * g + r, qi = q0 + ql;
          const bool ok = qi < S && key <= qi && key < S;
          const float pr = ok ? __builtin_amdgcn_exp2f(fmaf(sc[r], c1, -bL[ql])) : 0.f;
          pv[4 * sub + r] = pr;
          dsv[4 * sub + r] = pr * fmaf(da[r], c2, -bD[ql]);
        }
      }
    }
    bf16x8_t pf[2], dsf[2];
    split_frag_s(pv, sp, pf);
    split_frag_s(dsv, sd, dsf);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x8_t ob[2], qb[2];
      tr_frags_h(bO, dt, g, cl, ob);
      tr_frags_h(bQ, dt, g, cl, qb);
      dva[dt] = h3dot(pf, ob, dva[dt]);
      dka[dt] = h3dot(dsf, qb, dka[dt]);
    }
    // stage tile it + 1 into the other buffer (its last readers finished before the previous barrier) and fetch
    // tile it + 2 into the registers the staging just consumed
    if (it + 1 < nit) {
      stage(cb ^ 1);
      if (it + 2 < nit) fetch(it + 2);
    }
    __syncthreads();
  }
  float* dkh = dk + ((size_t)b * HH + hx) * S * 64;
  float* dvh = dv + ((size_t)b * HH + hx) * S * 64;
  const float fk = 0.5f / (sd * sq), fv = 0.5f / (sp * so);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kr = kb * 64 + wave * 16 + g * 4 + r;
    if (kr < S) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dkh[(size_t)kr * 64 + dt * 16 + cl] = fk * dka[dt][r];
        dvh[(size_t)kr * 64 + dt * 16 + cl] = fv * dva[dt][r];
      }
    }
  }
}

__global__ __launch_bounds__(256) void lrp_attn_dq_h3_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                             const float* __restrict__ v, const float* __restrict__ dO,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ D,
                                                             const float* __restrict__ dmax, float* __restrict__ dq,
                                                             int B, int Hq, int Hkv, int S, float sq, float sk,
                                                             float sv) {
  __shared__ __attribute__((aligned(16))) char sK[2][2 * H3P], sV[2][2 * H3P];   // double-buffered, as dkdv
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int nqb = (S + 63) / 64;
  const int qb = nqb - 1 - blockIdx.x / (B * Hq);
  const int bh = blockIdx.x % (B * Hq), b = bh / Hq, h = bh - b * Hq, G = Hq / Hkv, hk = h / G;
  const int qi = qb * 64 + wave * 16 + cl;
  const int qic = qi < S ? qi : S - 1;
  const int wq_min = qb * 64 + __builtin_amdgcn_readfirstlane(wave) * 16;
  const float so = dO_scale(dmax, b, Hq, hk, G);
  const float sd = so * sv * 0x1p-21f;
  const float c1 = 1.4426950408889634f / (sq * sk), c2 = 0.5f / (so * sv);
  bf16x8_t qf[2][2], of[2][2];
  row_frags_h(q + (((size_t)b * Hq + h) * S + qic) * 64, qf, g, sq);
  row_frags_h(dO + ((size_t)b * S + qic) * (size_t)(Hq * 64) + h * 64, of, g, so);
  const float lq = lse[((size_t)b * Hq + h) * S + qic] * 1.4426950408889634f;
  const float dq_ = D[((size_t)b * Hq + h) * S + qic];
  const float* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const float* vh = v + ((size_t)b * Hkv + hk) * S * 64;
  f32x4_t acc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) acc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int kend = min(S, qb * 64 + 64);
  TileRegs rk, rv;
  auto fetch = [&](int k0) {
    tile_load(kh, 64, k0, S, rk);
    tile_load(vh, 64, k0, S, rv);
  };
  fetch(0);
  h3_store(rk, sK[0], sk);
  h3_store(rv, sV[0], sv);
  if (32 < kend) fetch(32);
  __syncthreads();
  for (int k0 = 0; k0 < kend; k0 += 32) {
    const int cb = (k0 >> 5) & 1;
    const char* bK = sK[cb];
    const char* bV = sV[cb];
    const bool full = k0 + 31 <= wq_min && wq_min + 15 < S;
    float dsv[8];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x4_t sc = {0.f, 0.f, 0.f, 0.f}, da = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t ka[2], va[2];
        rm_frags_h(bK, sub * 16 + cl, 4 * ks + g, ka);
        rm_frags_h(bV, sub * 16 + cl, 4 * ks + g, va);
        sc = h3dot(ka, qf[ks], sc);
        da = h3dot(va, of[ks], da);
      }
      if (full) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          dsv[4 * sub + r] = __builtin_amdgcn_exp2f(fmaf(sc[r], c1, -lq)) * fmaf(da[r], c2, -dq_);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kj = k0 + sub * 16 + 4 * g + r;
          const bool ok = qi < S && kj <= qi;
          const float pr = ok ? __builtin_amdgcn_exp2f(fmaf(sc[r], c1, -lq)) : 0.f;
          dsv[4 * sub + r] = pr * fmaf(da[r], c2, -dq_);
        }
      }
    }
    bf16x8_t dsf[2];
    split_frag_s(dsv, sd, dsf);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x8_t kt[2];
      tr_frags_h(bK, dt, g, cl, kt);
      acc[dt] = h3dot(kt, dsf, acc[dt]);
    }
    if (k0 + 32 < kend) {
      h3_store(rk, sK[cb ^ 1], sk);
      h3_store(rv, sV[cb ^ 1], sv);
      if (k0 + 64 < kend) fetch(k0 + 64);
    }
    __syncthreads();
  }
  if (qi < S) {
    const float f = 0.5f / (sk * sd);
    float* o = dq + (((size_t)b * Hq + h) * S + qi) * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *(f32x4_t*)(o + dt * 16 + g * 4) = f * acc[dt];
  }
}

// ---------------------------------------------------------------------------------------------
// Per-row power-of-two h3 split of rule outputs: a max pass and a store pass over the row.  For the model widths
// (rows up to 2048 / 8192 / 1024 values) a thread's values stay in registers between the two, so the row is read
// once; wider rows recompute them (template parameter 0).

// Inverse RoPE + q scale + GQA group sum of the dK/dV partials + scatter into the token-major d[q|k|v] row,
// as a per-row-scaled h3 activation out3 [B*S, 2W] (W = (Hq + 2Hkv) 64), rinv[row] = 1/s * post[row].
__device__ __forceinline__ float rope_pack_value(const float* __restrict__ dq, const float* __restrict__ dk,
                                                 const float* __restrict__ dv, const float* __restrict__ cosT,
                                                 const float* __restrict__ sinT, int b, int s, int c, int S, int Hq,
                                                 int Hkv, int rot_dim, float q_scale, int ksum) {
  const int hh = c >> 6, d = c & 63, G = Hq / Hkv;
  const float* src;
  float scale = 1.f;
  bool rope = true;
  int ng = 1;
  if (hh < Hq) {
    src = dq + (((size_t)b * Hq + hh) * S + s) * 64;
    scale = q_scale;
  } else if (hh < Hq + Hkv) {
    src = ksum ? dk + (((size_t)b * Hkv + (hh - Hq)) * S + s) * 64 : dk + (((size_t)b * Hq + (hh - Hq) * G) * S + s) * 64;
    ng = ksum ? 1 : G;
  } else {
    src = ksum ? dv + (((size_t)b * Hkv + (hh - Hq - Hkv)) * S + s) * 64
               : dv + (((size_t)b * Hq + (hh - Hq - Hkv) * G) * S + s) * 64;
    ng = ksum ? 1 : G;
    rope = false;
  }
  const int half = rot_dim >> 1;
  const bool rot = rope && d < rot_dim;
  const int dp = !rot ? d : (d < half ? d + half : d - half);
  float x0 = 0.f, xp = 0.f;
  for (int gi = 0; gi < ng; ++gi) {
    x0 += src[(size_t)gi * S * 64 + d];
    if (rot) xp += src[(size_t)gi * S * 64 + dp];
  }
  float val = x0;
  if (rot) {
    const int j = d < half ? d : d - half;
    const float cs = cosT[(size_t)s * half + j], sn = sinT[(size_t)s * half + j];
    val = d < half ? x0 * cs + xp * sn : x0 * cs - xp * sn;
  }
  return val * scale;
}

template <int NIT>   // NIT > 0: W <= 64 NIT, the row's values stay in registers between the max and the store
__global__ __launch_bounds__(256) void lrp_rope_pack_h3_kernel(const float* __restrict__ dq, const float* __restrict__ dk,
                                                               const float* __restrict__ dv,
                                                               const float* __restrict__ cosT,
                                                               const float* __restrict__ sinT, f16_t* __restrict__ out,
                                                               float* __restrict__ rinv,
                                                               const float* __restrict__ post, int B, int S, int Hq,
                                                               int Hkv, int rot_dim, float q_scale, int ksum) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * S) return;
  const int b = row / S, s = row - b * S, W = (Hq + 2 * Hkv) * 64;
  float mx = 0.f;
  float cache[NIT > 0 ? NIT : 1];
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int c = lane + 64 * it;
      cache[it] = c < W ? rope_pack_value(dq, dk, dv, cosT, sinT, b, s, c, S, Hq, Hkv, rot_dim, q_scale, ksum) : 0.f;
      mx = fmaxf(mx, fabsf(cache[it]));
    }
  } else {
    for (int c = lane; c < W; c += 64)
      mx = fmaxf(mx, fabsf(rope_pack_value(dq, dk, dv, cosT, sinT, b, s, c, S, Hq, Hkv, rot_dim, q_scale, ksum)));
  }
  mx = wave_max(mx);
  float inv;
  const float sc = row_pow2_scale(mx, inv);
  f16_t* o = out + (size_t)row * (2 * W);
  auto put = [&](int c, float v) {
    float hi, lo;
    split2h(sc * v, hi, lo);
    o[c] = __builtin_bit_cast(f16_t, (_Float16)hi);
    o[W + c] = __builtin_bit_cast(f16_t, (_Float16)lo);
  };
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int c = lane + 64 * it;
      if (c < W) put(c, cache[it]);
    }
  } else {
    for (int c = lane; c < W; c += 64)
      put(c, rope_pack_value(dq, dk, dv, cosT, sinT, b, s, c, S, Hq, Hkv, rot_dim, q_scale, ksum));
  }
  if (lane == 0) rinv[row] = inv * (post ? post[row] : 1.f);
}

// Same, 4 consecutive columns per lane (16-byte loads of the partials, the rotation partners and cos / sin; 8-byte
// plane stores): the rotated half-widths are multiples of 4 (rot_dim % 8 == 0), so a lane's 4 columns rotate
// together.  NIT = ceil(W / 256) groups of 4 columns per lane stay in registers between the row max and the stores.
template <int NIT>
__global__ __launch_bounds__(256) void lrp_rope_pack_h3_v4_kernel(const float* __restrict__ dq,
                                                                  const float* __restrict__ dk,
                                                                  const float* __restrict__ dv,
                                                                  const float* __restrict__ cosT,
                                                                  const float* __restrict__ sinT,
                                                                  f16_t* __restrict__ out, float* __restrict__ rinv,
                                                                  const float* __restrict__ post, int B, int S, int Hq,
                                                                  int Hkv, int rot_dim, float q_scale, int ksum) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * S) return;
  const int b = row / S, s = row - b * S, W = (Hq + 2 * Hkv) * 64, G = Hq / Hkv, half = rot_dim >> 1;
  float v[NIT][4];
  float mx = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = 4 * lane + 256 * it;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[it][e] = 0.f;
    if (c >= W) continue;
    const int hh = c >> 6, d = c & 63;
    const float* src;
    float scale = 1.f;
    bool rope = true;
    int ng = 1;
    if (hh < Hq) {
      src = dq + (((size_t)b * Hq + hh) * S + s) * 64;
      scale = q_scale;
    } else if (hh < Hq + Hkv) {
      src = ksum ? dk + (((size_t)b * Hkv + (hh - Hq)) * S + s) * 64
                 : dk + (((size_t)b * Hq + (hh - Hq) * G) * S + s) * 64;
      ng = ksum ? 1 : G;
    } else {
      src = ksum ? dv + (((size_t)b * Hkv + (hh - Hq - Hkv)) * S + s) * 64
                 : dv + (((size_t)b * Hq + (hh - Hq - Hkv) * G) * S + s) * 64;
      ng = ksum ? 1 : G;
      rope = false;
    }
    const bool rot = rope && d < rot_dim;
    const int dp = !rot ? d : (d < half ? d + half : d - half);
    f32x4_t x0 = {0.f, 0.f, 0.f, 0.f}, xp = {0.f, 0.f, 0.f, 0.f};
    for (int gi = 0; gi < ng; ++gi) {
      x0 += *(const f32x4_t*)(src + (size_t)gi * S * 64 + d);
      if (rot) xp += *(const f32x4_t*)(src + (size_t)gi * S * 64 + dp);
    }
    f32x4_t val = x0;
    if (rot) {
      const int j = d < half ? d : d - half;
      const f32x4_t cs = *(const f32x4_t*)(cosT + (size_t)s * half + j), sn = *(const f32x4_t*)(sinT + (size_t)s * half + j);
      val = d < half ? x0 * cs + xp * sn : x0 * cs - xp * sn;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[it][e] = val[e] * scale;
      mx = fmaxf(mx, fabsf(v[it][e]));
    }
  }
  mx = wave_max(mx);
  float inv;
  const float sc = row_pow2_scale(mx, inv);
  f16_t* o = out + (size_t)row * (2 * W);
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = 4 * lane + 256 * it;
    if (c < W) store_h3_4(o, W, c, v[it], sc);
  }
  if (lane == 0) rinv[row] = inv * (post ? post[row] : 1.f);
}

// Plain fp32 rows [R, K] -> per-row-scaled h3 activation [R, 2K] + rinv.  One wave per row, 4 values per access.
template <int NIT>   // NIT > 0: K <= 256 NIT, the row's values stay in registers (read once)
__global__ __launch_bounds__(256) void split_h3_dyn_kernel(const float* __restrict__ x, f16_t* __restrict__ out,
                                                           float* __restrict__ rinv, const float* __restrict__ post,
                                                           int R, int K) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const float* xr = x + (size_t)row * K;
  float mx = 0.f;
  f32x4_t cache[NIT > 0 ? NIT : 1];
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int c = lane * 4 + it * 256;
      if (c < K) {
        cache[it] = *(const f32x4_t*)(xr + c);
        const f32x4_t v = cache[it];
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      }
    }
  } else {
    for (int c = lane * 4; c < K; c += 256) {
      const f32x4_t v = *(const f32x4_t*)(xr + c);
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
  }
  mx = wave_max(mx);
  float inv;
  const float sc = row_pow2_scale(mx, inv);
  f16_t* o = out + (size_t)row * (2 * K);
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int c = lane * 4 + it * 256;
      if (c < K) {
        const float vv[4] = {cache[it][0], cache[it][1], cache[it][2], cache[it][3]};
        store_h3_4(o, K, c, vv, sc);
      }
    }
  } else {
    for (int c = lane * 4; c < K; c += 256) {
      const f32x4_t v = *(const f32x4_t*)(xr + c);
      const float vv[4] = {v[0], v[1], v[2], v[3]};
      store_h3_4(o, K, c, vv, sc);
    }
  }
  if (lane == 0) rinv[row] = inv * (post ? post[row] : 1.f);
}

// SwiGLU rule on the interleaved gate|up layout (blocks of 16 columns): dg = 0.5 dm u sigmoid(g) (uniform rule on g*u,
// identity rule on SiLU), du = 0.5 dm silu(g); output the interleaved d[gate|up] row [2I] as a per-row-scaled h3
// activation [T, 4I].  One workgroup per row, 8 columns of one 16-column block per thread and step.
__device__ __forceinline__ void swiglu_bwd8(const float* __restrict__ dmr, const float* __restrict__ gur, int c,
                                            float (&dg)[8], float (&du)[8]) {
  const int blk = c >> 4, e = c & 15;
  const float* gp = gur + blk * 32 + e;
#pragma unroll
  for (int i = 0; i < 8; i += 4) {
    const f32x4_t gv = *(const f32x4_t*)(gp + i), uv = *(const f32x4_t*)(gp + 16 + i);
    const f32x4_t mv = *(const f32x4_t*)(dmr + c + i);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float sg = sigmoid_f32(gv[t]), m = 0.5f * mv[t];
      dg[i + t] = m * uv[t] * sg;
      du[i + t] = m * gv[t] * sg;
    }
  }
}

template <int NIT>   // NIT > 0: a thread's <= NIT chunks of 8 columns stay in registers between the max and the store
__global__ __launch_bounds__(256) void lrp_swiglu_bwd_h3_kernel(const float* __restrict__ dm,
                                                                const float* __restrict__ gu, f16_t* __restrict__ out,
                                                                float* __restrict__ rinv,
                                                                const float* __restrict__ post, int I) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  const float* dmr = dm + (size_t)t * I;
  const float* gur = gu + (size_t)t * (2 * I);
  float mx = 0.f;
  float cg[NIT > 0 ? NIT : 1][8], cu[NIT > 0 ? NIT : 1][8];
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int c = (threadIdx.x + it * 256) * 8;
      if (c < I) {
        swiglu_bwd8(dmr, gur, c, cg[it], cu[it]);
#pragma unroll
        for (int i = 0; i < 8; ++i) mx = fmaxf(mx, fmaxf(fabsf(cg[it][i]), fabsf(cu[it][i])));
      }
    }
  } else {
    for (int c = threadIdx.x * 8; c < I; c += 256 * 8) {
      float dg[8], du[8];
      swiglu_bwd8(dmr, gur, c, dg, du);
#pragma unroll
      for (int i = 0; i < 8; ++i) mx = fmaxf(mx, fmaxf(fabsf(dg[i]), fabsf(du[i])));
    }
  }
  mx = block_max<256>(mx, red);
  float inv;
  const float sc = row_pow2_scale(mx, inv);
  const int W = 2 * I;
  f16_t* o = out + (size_t)t * (2 * W);
  if constexpr (NIT > 0) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int c = (threadIdx.x + it * 256) * 8;
      if (c < I) {
        const int col = (c >> 4) * 32 + (c & 15);
        store_h3_8(o, W, col, cg[it], sc);
        store_h3_8(o, W, col + 16, cu[it], sc);
      }
    }
  } else {
    for (int c = threadIdx.x * 8; c < I; c += 256 * 8) {
      float dg[8], du[8];
      swiglu_bwd8(dmr, gur, c, dg, du);
      const int col = (c >> 4) * 32 + (c & 15);
      store_h3_8(o, W, col, dg, sc);
      store_h3_8(o, W, col + 16, du, sc);
    }
  }
  if (threadIdx.x == 0) rinv[t] = inv * (post ? post[t] : 1.f);
}

// GELU identity rule on the fc output gradient (GPT-NeoX): dx = dy gelu(a)/a, as a per-row-scaled h3 activation.
__global__ __launch_bounds__(256) void lrp_gelu_bwd_h3_kernel(const float* __restrict__ dy, const float* __restrict__ a,
                                                              f16_t* __restrict__ out, float* __restrict__ rinv,
                                                              int I) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  const float* dr = dy + (size_t)t * I;
  const float* ar = a + (size_t)t * I;
  float mx = 0.f;
  for (int c = threadIdx.x; c < I; c += 256) mx = fmaxf(mx, fabsf(dr[c] * gelu_ratio(ar[c])));
  mx = block_max<256>(mx, red);
  float inv;
  const float sc = row_pow2_scale(mx, inv);
  f16_t* o = out + (size_t)t * (2 * I);
  for (int c = threadIdx.x; c < I; c += 256) {
    float hi, lo;
    split2h(sc * (dr[c] * gelu_ratio(ar[c])), hi, lo);
    o[c] = __builtin_bit_cast(f16_t, (_Float16)hi);
    o[I + c] = __builtin_bit_cast(f16_t, (_Float16)lo);
  }
  if (threadIdx.x == 0) rinv[t] = inv;
}

// Forward activations from saved fp32 pre-activations to the next GEMM's h3 input at the model's scale s:
// SwiGLU on the interleaved gate|up row [2I] -> [I] (act 0), GELU [I] -> [I] (act 1).
__global__ __launch_bounds__(256) void act_h3_kernel(const float* __restrict__ x, f16_t* __restrict__ out, size_t n4,
                                                     int I, int act, float s) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n4) return;
  const int I4 = I >> 2;
  const size_t t = idx / I4;
  const int c = (int)(idx - t * I4) * 4;
  float v[4];
  if (act == 0) {
    const float* gp = x + t * (size_t)(2 * I) + (c >> 4) * 32 + (c & 15);
    const f32x4_t gv = *(const f32x4_t*)gp, uv = *(const f32x4_t*)(gp + 16);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gv[e] * sigmoid_f32(gv[e]) * uv[e];
  } else {
    const f32x4_t xv = *(const f32x4_t*)(x + t * (size_t)I + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gelu_f32(xv[e]);
  }
  store_h3_4(out + t * (size_t)(2 * I), I, c, v, s);
}

// rstd per row: rsqrt(mean(x^2) + eps) (RMSNorm), or of the centred row (LayerNorm, center = 1).  One wave per row.
__global__ __launch_bounds__(256) void row_rstd_f32_kernel(const float* __restrict__ x, float* __restrict__ rstd, int R,
                                                           int H, float eps, int center) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const float* xr = x + (size_t)row * H;
  float mu = 0.f;
  if (center) {
    float s = 0.f;
    for (int c = lane; c < H; c += 64) s += xr[c];
    mu = wave_sum(s) / H;
  }
  float v = 0.f;
  for (int c = lane; c < H; c += 64) {
    const float d = xr[c] - mu;
    v = fmaf(d, d, v);
  }
  v = wave_sum(v) / H;
  if (lane == 0) rstd[row] = 1.f / sqrtf(v + eps);
}

// LayerNorm rule with detached variance (mean not detached), dual norm of one input (GPT-NeoX parallel residual):
// out = resid + (gc1 - mean gc1) + (gc2 - mean gc2), gc = dy * rstd * w.  fp32, one wave per row.
__global__ __launch_bounds__(256) void lrp_ln_bwd_f32_kernel(const float* __restrict__ dy1, const float* __restrict__ rs,
                                                             const float* __restrict__ w1,
                                                             const float* __restrict__ dy2,
                                                             const float* __restrict__ w2,
                                                             const float* __restrict__ resid, float* __restrict__ out,
                                                             int R, int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= R) return;
  const size_t base = (size_t)row * H;
  const float r = rs[row];
  float m1 = 0.f, m2 = 0.f;
  for (int c = lane; c < H; c += 64) {
    m1 += dy1[base + c] * r * w1[c];
    if (dy2) m2 += dy2[base + c] * r * w2[c];
  }
  m1 = wave_sum(m1) / H;
  m2 = wave_sum(m2) / H;
  for (int c = lane; c < H; c += 64) {
    float val = resid[base + c] + (dy1[base + c] * r * w1[c] - m1);
    if (dy2) val += dy2[base + c] * r * w2[c] - m2;
    out[base + c] = val;
  }
}

// Channel-group relevance of the residual stream: out[b * ob + g] = sum over the window's S tokens and the group's
// 64 channels of |x dx|.  One workgroup per (window, group); deterministic (no atomics).
// sens (optional): the group's quantization sensitivity sum over tokens t of max_c |x_tc|^2 * sum_c dx_tc^2 - the
// expected squared first-order output change of a max-abs quantizer of step max_c |x_tc| / qmax is that over 12 qmax^2
// (codec.wire.allocate_group_bits).  Wave w takes tokens w, w + 4, ...; its 64 lanes are the group's channels.
__global__ __launch_bounds__(256) void group_absprod_kernel(const float* __restrict__ x, const float* __restrict__ dx,
                                                            float* __restrict__ out, float* __restrict__ sens, int S,
                                                            int H, int G, int ob) {
  __shared__ float red[4];
  const int b = blockIdx.x / G, gi = blockIdx.x - b * G;
  const int c = threadIdx.x & 63;
  float acc = 0.f, sacc = 0.f;
  for (int s = threadIdx.x >> 6; s < S; s += 4) {
    const size_t off = ((size_t)b * S + s) * H + gi * 64 + c;
    const float xv = x[off], dv = dx[off];
    acc += fabsf(xv * dv);
    if (sens) {   // uniform branch: every lane of the wave takes part in the reductions
      float am = fabsf(xv), d2 = dv * dv;
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) {
        am = fmaxf(am, __shfl_xor(am, m, 64));
        d2 += __shfl_xor(d2, m, 64);
      }
      if (c == 0) sacc += am * am * d2;
    }
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) out[(size_t)b * ob + gi] = acc;
  if (sens) {
    __syncthreads();
    sacc = block_sum<256>(sacc, red);
    if (threadIdx.x == 0) sens[(size_t)b * ob + gi] = sacc;
  }
}

// ---------------------------------------------------------------------------------------------
static inline unsigned nblk(size_t n) { return (unsigned)((n + 255) / 256); }

// The h3-plane sweeps (lrp_attn_dkdv_h3 / dq_h3): q, k, v at the forward attention's plane scales sq, sk, sv (powers
// of two with s |x| <= 2^15); dmax [B * Hq] workspace (the per-head max |dO| the delta kernel writes).  gs: dk, dv as
// the GQA group sums [B, Hkv, S, 64], else per-q-head partials.
EDGE_API int edge_lrp_attn_bwd_h3(const float* q, const float* k, const float* v, const float* o, const float* dO,
                                  const float* lse, float* D, float* rel, float* dq, float* dk, float* dv, float* dmax,
                                  int B, int Hq, int Hkv, int S, int gs, float sq, float sk, float sv, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv || !dmax || !(sq > 0.f && sk > 0.f && sv > 0.f)) return (int)hipErrorInvalidValue;
  const int nb = (S + 63) / 64;
  lrp_attn_delta_f32_kernel<<<B * Hq, 256, 0, st>>>(o, dO, D, rel, Hq, S, dmax);
  if (gs)
    lrp_attn_dkdv_h3_kernel<true><<<B * Hkv * nb, 256, 0, st>>>(q, k, v, dO, lse, D, dmax, dk, dv, B, Hq, Hkv, S, sq,
                                                                 sk, sv);
  else
    lrp_attn_dkdv_h3_kernel<false><<<B * Hq * nb, 256, 0, st>>>(q, k, v, dO, lse, D, dmax, dk, dv, B, Hq, Hkv, S, sq,
                                                                 sk, sv);
  lrp_attn_dq_h3_kernel<<<B * Hq * nb, 256, 0, st>>>(q, k, v, dO, lse, D, dmax, dq, B, Hq, Hkv, S, sq, sk, sv);
  return (int)hipGetLastError();
}

static int rope_pack_h3(const float* dq, const float* dk, const float* dv, const float* cosT, const float* sinT,
                        void* out, float* rinv, const float* post, int B, int S, int Hq, int Hkv, int rot_dim,
                        float q_scale, int ksum, hipStream_t st) {
  const int R = B * S;
  if (R <= 0) return 0;
  if (rot_dim > 64 || rot_dim % 2 || Hkv <= 0 || Hq % Hkv) return (int)hipErrorInvalidValue;
  const int W = (Hq + 2 * Hkv) * 64;
  if (rot_dim % 8 == 0 && W <= 1280) {   // Qwen2-0.5B: W = 1152, 5 column groups per lane
    lrp_rope_pack_h3_v4_kernel<5><<<(R + 3) / 4, 256, 0, st>>>(dq, dk, dv, cosT, sinT, (f16_t*)out, rinv, post, B, S,
                                                                Hq, Hkv, rot_dim, q_scale, ksum);
  } else if (rot_dim % 8 == 0 && W <= 2048) {
    lrp_rope_pack_h3_v4_kernel<8><<<(R + 3) / 4, 256, 0, st>>>(dq, dk, dv, cosT, sinT, (f16_t*)out, rinv, post, B, S,
                                                                Hq, Hkv, rot_dim, q_scale, ksum);
  } else if (W <= 2048)
    lrp_rope_pack_h3_kernel<32><<<(R + 3) / 4, 256, 0, st>>>(dq, dk, dv, cosT, sinT, (f16_t*)out, rinv, post, B, S,
                                                              Hq, Hkv, rot_dim, q_scale, ksum);
  else
    lrp_rope_pack_h3_kernel<0><<<(R + 3) / 4, 256, 0, st>>>(dq, dk, dv, cosT, sinT, (f16_t*)out, rinv, post, B, S, Hq,
                                                             Hkv, rot_dim, q_scale, ksum);
  return (int)hipGetLastError();
}
EDGE_API int edge_lrp_rope_pack_h3(const float* dq, const float* dk, const float* dv, const float* cosT,
                                   const float* sinT, void* out, float* rinv, const float* post, int B, int S, int Hq,
                                   int Hkv, int rot_dim, float q_scale, hipStream_t st) {
  return rope_pack_h3(dq, dk, dv, cosT, sinT, out, rinv, post, B, S, Hq, Hkv, rot_dim, q_scale, 0, st);
}
// the same from dk, dv already summed over each GQA group ([B, Hkv, S, 64], edge_lrp_attn_bwd_h3 with gs)
EDGE_API int edge_lrp_rope_pack_h3_gs(const float* dq, const float* dk, const float* dv, const float* cosT,
                                      const float* sinT, void* out, float* rinv, const float* post, int B, int S,
                                      int Hq, int Hkv, int rot_dim, float q_scale, hipStream_t st) {
  return rope_pack_h3(dq, dk, dv, cosT, sinT, out, rinv, post, B, S, Hq, Hkv, rot_dim, q_scale, 1, st);
}

EDGE_API int edge_split_h3_dyn(const float* x, void* out, float* rinv, const float* post, int R, int K, hipStream_t st) {
  if (R <= 0) return 0;
  if (K % 4) return (int)hipErrorInvalidValue;
  if (K <= 1024)
    split_h3_dyn_kernel<4><<<(R + 3) / 4, 256, 0, st>>>(x, (f16_t*)out, rinv, post, R, K);
  else
    split_h3_dyn_kernel<0><<<(R + 3) / 4, 256, 0, st>>>(x, (f16_t*)out, rinv, post, R, K);
  return (int)hipGetLastError();
}

EDGE_API int edge_lrp_swiglu_bwd_h3(const float* dm, const float* gu, void* out, float* rinv, const float* post,
                                    int T, int I, hipStream_t st) {
  if (T <= 0) return 0;
  if (I % 16) return (int)hipErrorInvalidValue;
  if (I <= 3 * 2048)   // Qwen2-0.5B: I = 4864, three 8-column chunks per thread (the row read once)
    lrp_swiglu_bwd_h3_kernel<3><<<T, 256, 0, st>>>(dm, gu, (f16_t*)out, rinv, post, I);
  else
    lrp_swiglu_bwd_h3_kernel<0><<<T, 256, 0, st>>>(dm, gu, (f16_t*)out, rinv, post, I);
  return (int)hipGetLastError();
}

EDGE_API int edge_lrp_gelu_bwd_h3(const float* dy, const float* a, void* out, float* rinv, int T, int I,
                                  hipStream_t st) {
  if (T <= 0) return 0;
  lrp_gelu_bwd_h3_kernel<<<T, 256, 0, st>>>(dy, a, (f16_t*)out, rinv, I);
  return (int)hipGetLastError();
}

EDGE_API int edge_act_h3(const float* x, void* out, long long T, int I, int act, float s, hipStream_t st) {
  const size_t n4 = (size_t)T * I / 4;
  if (!n4) return 0;
  if ((act == 0 && I % 16) || I % 4 || act < 0 || act > 1 || !(s > 0.f)) return (int)hipErrorInvalidValue;
  act_h3_kernel<<<nblk(n4), 256, 0, st>>>(x, (f16_t*)out, n4, I, act, s);
  return (int)hipGetLastError();
}

EDGE_API int edge_row_rstd_f32(const float* x, float* rstd, int R, int H, float eps, int center, hipStream_t st) {
  if (R <= 0) return 0;
  row_rstd_f32_kernel<<<(R + 3) / 4, 256, 0, st>>>(x, rstd, R, H, eps, center);
  return (int)hipGetLastError();
}

EDGE_API int edge_lrp_ln_bwd_f32(const float* dy1, const float* rs, const float* w1, const float* dy2, const float* w2,
                                 const float* resid, float* out, int R, int H, hipStream_t st) {
  if (R <= 0) return 0;
  lrp_ln_bwd_f32_kernel<<<(R + 3) / 4, 256, 0, st>>>(dy1, rs, w1, dy2, w2, resid, out, R, H);
  return (int)hipGetLastError();
}

// out [B, >= H/64] (row stride out_stride): sum |x dx| per window and 64-channel group; sens (nullable, same layout):
// the quantization sensitivity of group_absprod_kernel
EDGE_API int edge_group_absprod(const float* x, const float* dx, float* out, float* sens, int B, int S, int H,
                                int out_stride, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (H % 64) return (int)hipErrorInvalidValue;
  const int G = H / 64;
  group_absprod_kernel<<<B * G, 256, 0, st>>>(x, dx, out, sens, S, H, G, out_stride);
  return (int)hipGetLastError();
}
