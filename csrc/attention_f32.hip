// fp32 causal GQA attention for head_dim 64 and the fp32 token-importance scorers, the
// attention half of the framework's fp32 execution mode (the reference evaluates its models in fp32:
// Experiments/Qwen2-0.5B/qwen_layer_wise.py:17, Experiments/Pythia-70M/pythia_model.py:25 load without a dtype).
//
// flash_attn_fwd_x6 runs the matrix work as split products on the matrix cores: scaled fp16 planes (h3, three products
// per fp32 product) or three bf16 planes (six products, common.h split3); 1.5x (bf16 planes) to 2.5x (fp16 planes) the
// round-1 kernel on the native v_mfma_f32_16x16x4_f32.  The exact-fp32 importance scorers below keep that MFMA.
//
//   flash_attn_fwd_x6  : O = softmax(Q K^T) V, online softmax, optional row LSE; O written as fp32 rows or
//                        directly in the h3 layout (common.h) the O-projection GEMM consumes.
//   attn_lastrow_f32   : P[S-1, :] per head.
//   attn_colsum_f32    : sum_i P[i, j] per head from Q, K and the row LSE (second sweep, key block outer).
//
// Layouts as the bf16 kernels (attention.hip): q [B,Hq,S,64] (RoPE applied, pre-scaled), k [B,Hkv,S,64],
// vt [B,Hkv,64,s_pad] (V^T, zero padded), o [B*S, Hq*64] (fp32) or [B*S, 2*Hq*64] (2-plane h3).
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
#include <cstdlib>

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

}  // namespace

// ---- split-bf16 ("x6") flash attention: the same fp32-accurate result on the bf16 matrix cores -------------------
// q, k, v and the probabilities are split into three bf16 planes (common.h split3) and every product is the sum of
// the six plane products a_i b_j with i + j <= 2 (v_mfma_f32_16x16x32_bf16; dropped terms 2^-27 relative, every
// bf16 x bf16 product exact in the fp32 accumulator): 96 bf16 MFMAs of 16 cycles per 16-query x 64-key tile against
// 128 f32 MFMAs of 32 cycles.  Same S^T = K Q^T / O^T += V^T P^T orientation as flash_attn_fwd_f32 (lane holds 4
// keys of one query; the probabilities are the lane's own P^T operand).  K and V^T tiles are read from global fp32
// into registers one tile ahead, split, and written to LDS as planes of 64 rows x 128 B (16-byte chunks swizzled by
// (row >> 1) & 7, the GEMM image); V^T keys are stored in the order the P^T operand holds them - within a 32-key
// block a lane's k-slots 8g..8g+7 are keys {4g..4g+3, 16+4g..16+4g+3} - so each A fragment is one ds_read_b128.
namespace {
constexpr int XPL = 64 * 128;                 // one bf16 plane of a 64 x 64 tile
__device__ __forceinline__ int xsw(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void split_frag(const float (&v)[8], bf16x8_t& a, bf16x8_t& b, bf16x8_t& c) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float p0, p1, p2;
    split3(v[e], p0, p1, p2);
    a[e] = (__bf16)p0;
    b[e] = (__bf16)p1;
    c[e] = (__bf16)p2;
  }
}
__device__ __forceinline__ bf16x8_t xfrag(const char* plane, int row, int chunk) {
  return *(const bf16x8_t*)(plane + row * 128 + ((chunk ^ xsw(row)) << 4));
}
__device__ __forceinline__ f32x4_t mfma_bf(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// the six plane products, small terms first
__device__ __forceinline__ f32x4_t x6_dot(const bf16x8_t (&a)[3], const bf16x8_t (&b)[3], f32x4_t c) {
  c = mfma_bf(a[2], b[0], c);
  c = mfma_bf(a[0], b[2], c);
  c = mfma_bf(a[1], b[1], c);
  c = mfma_bf(a[1], b[0], c);
  c = mfma_bf(a[0], b[1], c);
  return mfma_bf(a[0], b[0], c);
}
// h3 planes (common.h: [hi, lo] fp16 of the power-of-two scaled value, raw bits in a bf16x8_t): the three products
// a_lo b_hi + a_hi b_lo + a_hi b_hi on the fp16 matrix cores
__device__ __forceinline__ f32x4_t mfma_h(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                0, 0, 0);
}
__device__ __forceinline__ f32x4_t h3_dot(const bf16x8_t (&a)[2], const bf16x8_t (&b)[2], f32x4_t c) {
  c = mfma_h(a[1], b[0], c);
  c = mfma_h(a[0], b[1], c);
  return mfma_h(a[0], b[0], c);
}
// on value pairs: v_cvt_pk_f16_f32 for both planes, the residual on packed f32 (the same RNE splits as split2h)
__device__ __forceinline__ void split_frag_h(const float (&v)[8], float s, bf16x8_t& hi, bf16x8_t& lo) {
  u32x4_t H, L;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const f32x2_t x = f32x2_t{v[2 * e], v[2 * e + 1]} * f32x2_t{s, s};
    const f16x2_t h = __builtin_convertvector(x, f16x2_t);
    const f32x2_t r = x - __builtin_convertvector(h, f32x2_t);
    H[e] = __builtin_bit_cast(uint32_t, h);
    L[e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, f16x2_t));
  }
  hi = __builtin_bit_cast(bf16x8_t, H);
  lo = __builtin_bit_cast(bf16x8_t, L);
}
// the unscaled split of the probabilities (the loop's hot split): hi by v_cvt_pk_f16_f32, lo = f16(x - hi) by
// v_fma_mixlo_f16 / v_fma_mixhi_f16 straight from the fp32 value and the f16 hi half (x - hi is exact, one RNE to
// f16: the same bits as split_frag_h's convert-back / packed subtract / convert, in 3 instead of 5 VALU per pair;
// packed-f32 VALU beside MFMAs is the expensive kind).  Operands are VALU results (no MFMA -> asm hazard).
__device__ __forceinline__ uint32_t mix_lo2(float x0, float x1, uint32_t h) {
  uint32_t r;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %3, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(r) : "v"(x0), "v"(h), "v"(x1));
  return r;
}
// row max over the lane halves without fmaxf's sNaN canonicalisation (two v_max_f32 x, x per step; the scores are
// finite or -inf): the permlane swap's outputs are VALU results (no MFMA -> asm hazard)
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float xor_max16_raw(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_raw(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor_max32_raw(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_raw(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ void split_frag_h1(const float (&v)[8], bf16x8_t& hi, bf16x8_t& lo) {
  u32x4_t H, L;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    H[e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{v[2 * e], v[2 * e + 1]}, f16x2_t));
    L[e] = mix_lo2(v[2 * e], v[2 * e + 1], H[e]);
  }
  hi = __builtin_bit_cast(bf16x8_t, H);
  lo = __builtin_bit_cast(bf16x8_t, L);
}
// NPL planes of 8 values: three bf16 planes (x6) or two scaled fp16 planes (h3)
template <bool F16>
__device__ __forceinline__ void split_planes(const float (&v)[8], float s, bf16x8_t (&p)[F16 ? 2 : 3]) {
  if constexpr (F16) split_frag_h(v, s, p[0], p[1]);
  else split_frag(v, p[0], p[1], p[2]);
}
template <bool F16>
__device__ __forceinline__ f32x4_t plane_dot(const bf16x8_t (&a)[F16 ? 2 : 3], const bf16x8_t (&b)[F16 ? 2 : 3],
                                             f32x4_t c) {
  if constexpr (F16) return h3_dot(a, b, c);
  else return x6_dot(a, b, c);
}
}  // namespace

// NW waves of 16 query rows per workgroup (4: 64 rows, 8: 128 rows sharing each staged K / V^T tile).
// F16: the planes are the two scaled fp16 h3 planes (three fp16 MFMAs per product instead of six bf16): q, k and
// v are scaled by the powers of two sq, sk, sv (model bounds, so every plane stays in the fp16 range) and the
// probabilities by 2^(15 - TAU) (p <= 2^TAU under the lazy rescale); the scores are unscaled in the exp and the
// output in the final normalisation.
// KVP (with F16 and NW = 8): k / vt are not fp32 but the scaled fp16 h3 planes the QKV GEMM epilogue wrote
// (kp [B, Hkv, 2, S, 64], vp [B, Hkv, 2, 64, s_pad], V^T keys in the P^T operand order: gemm.hip kv_plane_pos); the
// K / V^T tiles are then staged by LDS DMA (global_load_lds, 16 bytes a lane, swizzle on the source address) into
// two buffers - no register staging, no per-tile split, one barrier per key tile, tile kb + 1 in flight while tile kb
// is computed.
// PRIO (8 waves, two per SIMD): waves NW/2 .. NW-1, the second-dispatched half and the arbitration loser of every
// segment, run at s_setprio 1 for the whole kernel (MI355X_MICROARCH "Two waves per SIMD", item 4).
template <bool H3OUT, int NW, bool F16, bool KVP = false, bool PRIO = false>
__global__ __launch_bounds__(NW * 64, 8 / NW) void flash_attn_fwd_x6_kernel(const float* __restrict__ q,
                                                                  const void* __restrict__ kin,
                                                                  const void* __restrict__ vtin, void* __restrict__ o,
                                                                  float* __restrict__ lse,
                                                                  const float* __restrict__ n_rows, int B, int Hq,
                                                                  int Hkv, int S, int s_pad, float h3s, float sq,
                                                                  float sk, float sv, float* __restrict__ o32) {
  // o32 (H3OUT, optional): O also as fp32 rows [B*S, Hq*64] (the AttnLRP forward saves it next to the planes)
  static_assert(!KVP || (F16 && NW == 8), "plane staging: h3 planes, 8 waves (8 KiB per DMA round)");
  constexpr int NPL = F16 ? 2 : 3;
  const float* __restrict__ k = (const float*)kin;
  const float* __restrict__ vt = (const float*)vtin;
  // probability scale 2^(15 - FTAU) of the fp16 planes, applied in the exp2 argument (the row sum l_run and the
  // probabilities carry it; the normalisation and the LSE take it out)
  constexpr float LSP = F16 ? 7.f : 0.f;
  static_assert(FTAU == 8.f, "LSP assumes p <= 2^8");
  extern __shared__ __attribute__((aligned(16))) char smem[];   // K planes (NPL x 8 KiB), V^T planes (NPL x 8 KiB)
  if constexpr (!F16) sq = sk = sv = 1.f;
  const float sc_log2 = FLOG2E / (sq * sk);   // score scale (natural log -> log2) of the scaled products
  // wave index in an SGPR: q0, kmax and the diagonal-tile test are wave-uniform scalars (scalar branches; with a VGPR
  // wave index the compiler if-converted the causal mask into every key tile)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            ql = lane & 15;
  if constexpr (PRIO) {
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  constexpr int QB = 16 * NW;          // query rows per workgroup
  const int nqb = (S + QB - 1) / QB;
  const int G = Hq / Hkv, NG = B * Hkv;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int cnt = (NG - xcd + 7) >> 3;
  const int per_qb = cnt * G;
  if (j >= per_qb * nqb) return;
  const int qb = nqb - 1 - j / per_qb;
  const int rem = j - (nqb - 1 - qb) * per_qb;
  const int grp = xcd + 8 * (rem / G);
  const int b = grp / Hkv, hk = grp - b * Hkv, h = hk * G + rem % G;
  if (n_rows && qb * QB + QB - 1 < S - 1 - (int)n_rows[b]) return;  // scored-rows mode (last layer)

  const float* qh = q + ((size_t)b * Hq + h) * S * 64;
  const float* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const float* vh = vt + ((size_t)b * Hkv + hk) * 64 * (size_t)s_pad;
  char* lk = smem;
  char* lv = smem + NPL * XPL;

  const int q0 = qb * QB + wave * 16;
  const int qrow = q0 + ql;
  const int qld = qrow < S ? qrow : S - 1;
  // Q^T operand planes: lane (query ql, g) holds d = 32 ks + 8g .. +7
  bf16x8_t qp[2][NPL];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    float v[8];
    const f32x4_t a = *(const f32x4_t*)(qh + (size_t)qld * 64 + 32 * ks + 8 * g);
    const f32x4_t c = *(const f32x4_t*)(qh + (size_t)qld * 64 + 32 * ks + 8 * g + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = c[e]; }
    split_planes<F16>(v, sq, qp[ks]);
  }
  f32x4_t oacc[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) oacc[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m2 = -INFINITY, l_run = 0.f;

  // staging: this lane's NF consecutive floats of K row / V^T row srow (64 rows over the NW waves)
  constexpr int NF = 64 * 64 / (NW * 64), LPR = 64 / NF;   // floats per lane, lanes per row
  const int srow = (wave * 64 + lane) / LPR, scol = (lane % LPR) * NF;
  f32x4_t kreg[NF / 4], vreg[NF / 4];
  auto load_tile = [&](int kb) {
    const int kr = min(kb * 64 + srow, S - 1);
    const float* kp = kh + (size_t)kr * 64 + scol;
    const float* vp = vh + (size_t)srow * s_pad + kb * 64 + scol;
#pragma unroll
    for (int i = 0; i < NF / 4; ++i) {
      kreg[i] = *(const f32x4_t*)(kp + 4 * i);
      vreg[i] = *(const f32x4_t*)(vp + 4 * i);
    }
  };
  auto write_tile = [&]() {
    // K row srow: d = scol .. + NF - 1 = chunks scol / 8 .. of each plane
#pragma unroll
    for (int hc = 0; hc < NF / 8; ++hc) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = kreg[2 * hc][e]; v[4 + e] = kreg[2 * hc + 1][e]; }
      bf16x8_t p[NPL];
      split_planes<F16>(v, sk, p);
      const int c = scol / 8 + hc;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) *(bf16x8_t*)(lk + pl * XPL + srow * 128 + ((c ^ xsw(srow)) << 4)) = p[pl];
    }
    // V^T row srow (= d): keys scol .. + NF - 1 in groups of 4; the group of keys 32 s + 16 hf + 4a .. +3 goes to
    // chunk 4 s + a, half hf
#pragma unroll
    for (int a4 = 0; a4 < NF / 4; ++a4) {
      const int key = scol + 4 * a4;
      const int sblk = key >> 5, hf = (key >> 4) & 1, a = (key >> 2) & 3;
      const int off = srow * 128 + (((4 * sblk + a) ^ xsw(srow)) << 4) + hf * 8;
      if constexpr (F16) {   // value pairs: v_cvt_pk_f16_f32 for both planes, the residual on packed f32
        u32x2_t H, L;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const f32x2_t x = f32x2_t{vreg[a4][2 * e], vreg[a4][2 * e + 1]} * f32x2_t{sv, sv};
          const f16x2_t h = __builtin_convertvector(x, f16x2_t);
          H[e] = __builtin_bit_cast(uint32_t, h);
          L[e] = __builtin_bit_cast(uint32_t, __builtin_convertvector(x - __builtin_convertvector(h, f32x2_t), f16x2_t));
        }
        *(u32x2_t*)(lv + 0 * XPL + off) = H;
        *(u32x2_t*)(lv + 1 * XPL + off) = L;
      } else {
        float p0[4], p1[4], p2[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split3(vreg[a4][e], p0[e], p1[e], p2[e]);
        *(u32x2_t*)(lv + 0 * XPL + off) = u32x2_t{pack_bf2(p0[0], p0[1]), pack_bf2(p0[2], p0[3])};
        *(u32x2_t*)(lv + 1 * XPL + off) = u32x2_t{pack_bf2(p1[0], p1[1]), pack_bf2(p1[2], p1[3])};
        *(u32x2_t*)(lv + 2 * XPL + off) = u32x2_t{pack_bf2(p2[0], p2[1]), pack_bf2(p2[2], p2[3])};
      }
    }
  };

  // KVP: DMA of key tile kb into buffer kb & 1 (4 plane tiles of 8 KiB: K hi, K lo, V^T hi, V^T lo); wave w stages
  // rows 8 w .. 8 w + 7 of each, lane -> (row 8 w + lane / 8, LDS chunk lane % 8 = global chunk (lane % 8) ^ xsw(row))
  const char* kph = (const char*)((const f16_t*)kin + ((size_t)b * Hkv + hk) * 2 * S * 64);
  const char* vph = (const char*)((const f16_t*)vtin + ((size_t)b * Hkv + hk) * 2 * 64 * (size_t)s_pad);
  const int drow = wave * 8 + (lane >> 3);
  const int dchunk = ((lane & 7) ^ xsw(drow)) << 4;
  auto dma_tile = [&](int kb) {
    char* buf = smem + (kb & 1) * 4 * XPL + wave * 1024;
    const size_t kr = (size_t)min(kb * 64 + drow, S - 1);
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      glds16(kph + ((size_t)pl * S + kr) * 128 + dchunk, buf + pl * XPL);
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      glds16(vph + (((size_t)pl * 64 + drow) * s_pad + kb * 64) * 2 + dchunk, buf + (2 + pl) * XPL);
  };

  const int nkb = min((qb + 1) * QB, S + 63) / 64;   // key tiles up to this block's last query row
  const int kmax = (q0 + 15) / 64;  // last key tile this wave needs (wave-uniform)
  if constexpr (KVP) dma_tile(0);
  else load_tile(0);
  for (int kb = 0; kb < nkb; ++kb) {
    if constexpr (KVP) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of tile kb landed
      __syncthreads();       // every wave's pieces landed; every wave's reads of tile kb - 1 (buffer (kb + 1) & 1) done
      if (kb + 1 < nkb) dma_tile(kb + 1);
      lk = smem + (kb & 1) * 4 * XPL;
      lv = lk + 2 * XPL;
    } else {
      __syncthreads();                 // every wave's reads of the previous tile retired
      write_tile();
      __syncthreads();                 // planes of tile kb visible
      if (kb + 1 < nkb) load_tile(kb + 1);
    }
    if (kb > kmax) continue;
    // S^T = K Q^T over the 4 key blocks of 16
    f32x4_t st[4];
    if constexpr (F16) {
      // product-major over the four independent key blocks (each accumulator sees h3_dot's product order, so the
      // scores are bit-identical to the block-major loop): consecutive MFMAs never wait on each other's result
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) st[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t kf[4][2];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int pl = 0; pl < 2; ++pl) kf[kt][pl] = xfrag(lk + pl * XPL, kt * 16 + ql, 4 * ks + g);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) st[kt] = mfma_h(kf[kt][1], qp[ks][0], st[kt]);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) st[kt] = mfma_h(kf[kt][0], qp[ks][1], st[kt]);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) st[kt] = mfma_h(kf[kt][0], qp[ks][0], st[kt]);
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const int row = kt * 16 + ql;
        st[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          bf16x8_t kf[NPL];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) kf[pl] = xfrag(lk + pl * XPL, row, 4 * ks + g);
          st[kt] = plane_dot<F16>(kf, qp[ks], st[kt]);
        }
      }
    }
    if (__builtin_expect(kb * 64 + 63 > q0 || kb * 64 + 63 >= S, 0)) {   // causal / sequence-end mask (scalar branch)
      // key kb 64 + 16 kt + 4 g + r is masked when 16 kt + r exceeds the lane's limit (one compare per value)
      const int lim = min(qrow, S - 1) - kb * 64 - 4 * g;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kt * 16 + r > lim) st[kt][r] = -INFINITY;
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) mloc = fmaxf(mloc, st[kt][r]);
    if constexpr (F16) mloc = xor_max32_raw(xor_max16_raw(mloc));
    else mloc = xor_max32(xor_max16(mloc));
    const float mc = mloc * sc_log2;
    if (__builtin_amdgcn_ballot_w64(mc > m2 + FTAU)) {  // wave-uniform lazy rescale
      const float mn = fmaxf(m2, mc);
      const float alpha = __builtin_amdgcn_exp2f(m2 - mn);   // v_exp_f32 (m2 = -inf -> 0)
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
        // v_exp_f32 without exp2f's denormal range reduction: p < 2^-126 of the row max does not matter
        const float pv = __builtin_amdgcn_exp2f(fmaf(st[kt][r], sc_log2, LSP - m2));
        st[kt][r] = pv;
        ps += pv;
      }
    l_run += ps;
    // O^T += V^T P^T: k-step s contracts the keys {32 s + 4g + r, 32 s + 16 + 4g + r}
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      float pv8[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) { pv8[r] = st[2 * sk][r]; pv8[4 + r] = st[2 * sk + 1][r]; }
      bf16x8_t pp[NPL];
      if constexpr (F16) {
        split_frag_h1(pv8, pp[0], pp[1]);
        bf16x8_t vf[4][2];   // product-major over the four d-blocks, as the scores above
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int pl = 0; pl < 2; ++pl) vf[dt][pl] = xfrag(lv + pl * XPL, dt * 16 + ql, 4 * sk + g);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) oacc[dt] = mfma_h(vf[dt][1], pp[0], oacc[dt]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) oacc[dt] = mfma_h(vf[dt][0], pp[1], oacc[dt]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) oacc[dt] = mfma_h(vf[dt][0], pp[0], oacc[dt]);
      } else {
        split_planes<F16>(pv8, 1.f, pp);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int row = dt * 16 + ql;
          bf16x8_t vf[NPL];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) vf[pl] = xfrag(lv + pl * XPL, row, 4 * sk + g);
          oacc[dt] = plane_dot<F16>(vf, pp, oacc[dt]);
        }
      }
    }
  }

  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  const float inv = 1.f / (l_run * sv);
  const int W = Hq * 64;
  u32x4_t oh[2], ol[2];
  if constexpr (H3OUT) {
    // h3 planes of O: the d-groups (0,1) and (2,3) pair-swapped (permlane16, partners share the query row) into 8
    // consecutive values per lane, one 16-byte store per plane and pair instead of two 8-byte ones
    u32x2_t hw[4], lw[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      float hi[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) hi[r] = oacc[dt][r] * inv * h3s;
      const u32x2_t t0 = split2h_pk(hi[0], hi[1]), t1 = split2h_pk(hi[2], hi[3]);
      hw[dt] = u32x2_t{t0[0], t1[0]};
      lw[dt] = u32x2_t{t0[1], t1[1]};
    }
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
      oh[q2] = pair_swap16(hw[2 * q2], hw[2 * q2 + 1]);
      ol[q2] = pair_swap16(lw[2 * q2], lw[2 * q2 + 1]);
    }
  }
  if (qrow < S) {
    if constexpr (H3OUT) {
      if (o32) {
        float* r32 = o32 + ((size_t)b * S + qrow) * (size_t)W + h * 64;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) *(f32x4_t*)(r32 + dt * 16 + 4 * g) = oacc[dt] * inv;
      }
      f16_t* orow = (f16_t*)o + ((size_t)b * S + qrow) * (size_t)(2 * W) + h * 64;
#pragma unroll
      for (int q2 = 0; q2 < 2; ++q2) {
        *(u32x4_t*)(orow + q2 * 32 + pair_col(g)) = oh[q2];
        *(u32x4_t*)(orow + W + q2 * 32 + pair_col(g)) = ol[q2];
      }
    } else {
      float* orow = (float*)o + ((size_t)b * S + qrow) * (size_t)W + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) *(f32x4_t*)(orow + dt * 16 + 4 * g) = oacc[dt] * inv;
    }
    if (lse && g == 0) lse[((size_t)b * Hq + h) * S + qrow] = (m2 - LSP) * 0.6931471805599453f + logf(l_run);
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

// ---- importance scorers on the split-plane matrix cores (the forward's h3 scheme) ----------------------------------
// Column sums of P for one (b, q head, 64-key block): sum over query rows i >= key of exp(q_i . k_j - lse_i).  The scores
// are the forward's: q and k as scaled fp16 h3 planes (powers of two sq, sk from the model's bounds), three fp16 MFMA
// products per score (v_mfma_f32_16x16x32_f16), so P is consistent with the LSE the forward wrote.  S = Q K^T keeps the
// key on the lane column: wave w owns keys kb*64 + 16w + (lane & 15), its K planes live in registers for the whole
// sweep, and the lane's 4 query rows per 16-row sub-tile are summed in-lane (two shuffles at the very end).  Query
// tiles of 64 rows (from the key block's diagonal to S) are split into planes once per workgroup and staged in LDS for
// all four waves; LSE in log2 units in LDS; the causal mask runs only on the diagonal tile; exp2 on v_exp_f32.
__global__ __launch_bounds__(256) void attn_colsum_h3_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                             const float* __restrict__ lse, float* __restrict__ out,
                                                             int B, int Hq, int Hkv, int S, float sq, float sk) {
  __shared__ __attribute__((aligned(16))) char lq[2 * XPL];   // Q hi / lo planes of the current 64-row tile
  __shared__ float l2[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            cl = lane & 15;
  const int kb = blockIdx.x / (B * Hq);                   // key block 0 (most causal queries) first
  const int bh = blockIdx.x - kb * (B * Hq), b = bh / Hq, h = bh - b * Hq, hk = h / (Hq / Hkv);
  const float* qh = q + ((size_t)b * Hq + h) * S * 64;
  const float* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const float* lh = lse + ((size_t)b * Hq + h) * S;
  const float sc_log2 = FLOG2E / (sq * sk);

  const int key = kb * 64 + wave * 16 + cl;
  const int kld = key < S ? key : S - 1;
  bf16x8_t kp[2][2];                      // B operand: K[key][d = 32 ks + 8g .. +7], hi / lo
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    float v[8];
    const f32x4_t a = *(const f32x4_t*)(kh + (size_t)kld * 64 + 32 * ks + 8 * g);
    const f32x4_t c = *(const f32x4_t*)(kh + (size_t)kld * 64 + 32 * ks + 8 * g + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = c[e]; }
    split_planes<true>(v, sk, kp[ks]);
  }
  // staging: 64 rows x 64 floats, 16 consecutive floats (two 8-float chunks) per thread
  const int srow = tid >> 2, scol = (tid & 3) * 16;
  f32x4_t qreg[4];
  auto load_tile = [&](int q0) {
    const int r = q0 + srow;
    if (r < S) {
#pragma unroll
      for (int i = 0; i < 4; ++i) qreg[i] = *(const f32x4_t*)(qh + (size_t)r * 64 + scol + 4 * i);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) qreg[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  };
  float csum = 0.f;
  const int qt0 = kb * 64;
  load_tile(qt0);
  for (int q0 = qt0; q0 < S; q0 += 64) {
    __syncthreads();                       // every wave's reads of the previous tile retired
#pragma unroll
    for (int hc = 0; hc < 2; ++hc) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = qreg[2 * hc][e]; v[4 + e] = qreg[2 * hc + 1][e]; }
      bf16x8_t p[2];
      split_planes<true>(v, sq, p);
      const int c = scol / 8 + hc;
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) *(bf16x8_t*)(lq + pl * XPL + srow * 128 + ((c ^ xsw(srow)) << 4)) = p[pl];
    }
    if (tid < 64) l2[tid] = q0 + tid < S ? lh[q0 + tid] * FLOG2E : INFINITY;
    __syncthreads();
    if (q0 + 64 < S) load_tile(q0 + 64);
    const bool diag = q0 == qt0;           // only the first query tile crosses the causal diagonal
#pragma unroll
    for (int sub = 0; sub < 4; ++sub) {
      f32x4_t st = {0.f, 0.f, 0.f, 0.f};
      const int row = sub * 16 + cl;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8_t qf[2];
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) qf[pl] = xfrag(lq + pl * XPL, row, 4 * ks + g);
        st = h3_dot(qf, kp[ks], st);
      }
      // st[r] = score(query q0 + sub*16 + 4g + r, key)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = sub * 16 + 4 * g + r;
        float pv = __builtin_amdgcn_exp2f(fmaf(st[r], sc_log2, -l2[ql]));
        if (diag && q0 + ql < key) pv = 0.f;
        csum += pv;
      }
    }
  }
  csum += __shfl_xor(csum, 16, 64);
  csum += __shfl_xor(csum, 32, 64);
  if (g == 0 && key < S) out[((size_t)b * Hq + h) * S + key] = csum;
}

// Last-row probabilities P[S-1, :] of the G = Hq / Hkv query heads of one (b, kv head) at once: the G last query rows
// are the MFMA A rows (up to 16), K the B columns, scores on the h3 planes as above; the G x S score rows go to LDS and a
// block softmax per head row finishes in fp32.
__global__ __launch_bounds__(256) void attn_lastrow_h3_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                              float* __restrict__ out, int Hq, int Hkv, int S,
                                                              float sq, float sk) {
  extern __shared__ float sc[];            // G x S scores
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int G = Hq / Hkv;
  const int bk = blockIdx.x, b = bk / Hkv, hk = bk - b * Hkv;
  const float* kh = k + ((size_t)b * Hkv + hk) * S * 64;
  const float inv_s = 1.f / (sq * sk);
  bf16x8_t qa[2][2];                       // A operand: row cl = head hk*G + cl (zero beyond G), d = 32 ks + 8g ..
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (cl < G) {
      const float* qr = q + (((size_t)b * Hq + hk * G + cl) * S + (S - 1)) * 64 + 32 * ks + 8 * g;
      const f32x4_t a = *(const f32x4_t*)qr, c = *(const f32x4_t*)(qr + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = c[e]; }
    }
    split_planes<true>(v, sq, qa[ks]);
  }
  for (int k0 = wave * 16; k0 < S; k0 += 64) {
    const int key = k0 + cl, kld = key < S ? key : S - 1;
    f32x4_t st = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      float v[8];
      const f32x4_t a = *(const f32x4_t*)(kh + (size_t)kld * 64 + 32 * ks + 8 * g);
      const f32x4_t c = *(const f32x4_t*)(kh + (size_t)kld * 64 + 32 * ks + 8 * g + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = c[e]; }
      bf16x8_t kf[2];
      split_planes<true>(v, sk, kf);
      st = h3_dot(qa[ks], kf, st);
    }
    // st[r] = score(head row 4g + r, key)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int hr = 4 * g + r;
      if (hr < G && key < S) sc[hr * S + key] = st[r] * inv_s;
    }
  }
  __syncthreads();
  for (int hr = 0; hr < G; ++hr) {
    float* row = sc + hr * S;
    float mx = -INFINITY;
    for (int j = tid; j < S; j += 256) mx = fmaxf(mx, row[j]);
    mx = block_max<256>(mx, red);
    float sum = 0.f;
    for (int j = tid; j < S; j += 256) {
      const float p = expf(row[j] - mx);
      row[j] = p;
      sum += p;
    }
    sum = block_sum<256>(sum, red);
    const float inv = 1.f / sum;
    float* orow = out + ((size_t)b * Hq + hk * G + hr) * S;
    for (int j = tid; j < S; j += 256) orow[j] = row[j] * inv;
  }
}

template <bool H3OUT>
static void launch_plane_attn(dim3 grid, hipStream_t st, const float* q, const void* kp, const void* vp, void* o,
                              float* lse, const float* n_rows, int B, int Hq, int Hkv, int S, int s_pad, float h3s,
                              float sq, float sk, float sv, float* o32) {
  static const bool prio = [] {   // EDGE_ATTN_PRIO=1: the younger wave half at s_setprio 1
    const char* e = getenv("EDGE_ATTN_PRIO");
    return e && e[0] == '1';
  }();
  if (prio)
    hipLaunchKernelGGL((flash_attn_fwd_x6_kernel<H3OUT, 8, true, true, true>), grid, dim3(512), 8 * XPL, st, q, kp, vp,
                       o, lse, n_rows, B, Hq, Hkv, S, s_pad, h3s, sq, sk, sv, o32);
  else
    hipLaunchKernelGGL((flash_attn_fwd_x6_kernel<H3OUT, 8, true, true>), grid, dim3(512), 8 * XPL, st, q, kp, vp, o,
                       lse, n_rows, B, Hq, Hkv, S, s_pad, h3s, sq, sk, sv, o32);
}

template <bool H3OUT, int NW, bool F16>
static void launch_split_attn(dim3 grid, hipStream_t st, const float* q, const float* k, const float* vt, void* o,
                              float* lse, const float* n_rows, int B, int Hq, int Hkv, int S, int s_pad, float h3s,
                              float sq, float sk, float sv) {
  hipLaunchKernelGGL((flash_attn_fwd_x6_kernel<H3OUT, NW, F16>), grid, dim3(NW * 64), (F16 ? 4 : 6) * XPL, st, q, k,
                     vt, o, lse, n_rows, B, Hq, Hkv, S, s_pad, h3s, sq, sk, sv, nullptr);
}

// out_h3_scale > 0: O as a 2-plane h3 activation [B*S, 2*Hq*64] (fp16 planes at that scale) for the O-projection;
// 0: fp32 [B*S, Hq*64].  sq, sk, sv > 0: the split-plane kernel runs on scaled fp16 planes (h3, three products; the
// caller guarantees s |x| <= 2^15 for q, k and v); 0: on three bf16 planes (six products).
EDGE_API int edge_flash_attn_fwd_f32(const float* q, const float* k, const float* vt, void* o, float* lse,
                                     const float* n_rows, int B, int Hq, int Hkv, int S, int s_pad, float out_h3_scale,
                                     float sq, float sk, float sv, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hq % Hkv || s_pad % 64 || s_pad < S || out_h3_scale < 0.f) return (int)hipErrorInvalidValue;
  const bool f16 = sq > 0.f;
  if (f16 && !(sk > 0.f && sv > 0.f)) return (int)hipErrorInvalidValue;
  const bool ho = out_h3_scale > 0.f;
  // 8 waves, 128 query rows per workgroup (the 4-wave / 64-row form measured slower)
  const int G = Hq / Hkv, maxcnt = (B * Hkv + 7) / 8;
  const dim3 gx(8 * maxcnt * G * ((S + 127) / 128));
  auto* fn = f16 ? (ho ? launch_split_attn<true, 8, true> : launch_split_attn<false, 8, true>)
                 : (ho ? launch_split_attn<true, 8, false> : launch_split_attn<false, 8, false>);
  fn(gx, st, q, k, vt, o, lse, n_rows, B, Hq, Hkv, S, s_pad, out_h3_scale, sq, sk, sv);
  return (int)hipGetLastError();
}

// fp32 attention from the K / V^T h3 planes of edge_gemm_qkv_rope_f32 (kp / vp at scales sk / sv; q fp32, split at
// sq): the KVP kernel.  Same arguments and outputs as edge_flash_attn_fwd_f32 otherwise; o32 (optional, with the h3
// output): O as fp32 rows too.
EDGE_API int edge_flash_attn_fwd_h3p(const float* q, const void* kp, const void* vp, void* o, float* lse,
                                    const float* n_rows, int B, int Hq, int Hkv, int S, int s_pad, float out_h3_scale,
                                    float sq, float sk, float sv, float* o32, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv || s_pad % 64 || s_pad < S || out_h3_scale < 0.f) return (int)hipErrorInvalidValue;
  if (!(sq > 0.f && sk > 0.f && sv > 0.f) || ((uintptr_t)kp & 15) || ((uintptr_t)vp & 15))
    return (int)hipErrorInvalidValue;
  const int G = Hq / Hkv, maxcnt = (B * Hkv + 7) / 8;
  const dim3 gx(8 * maxcnt * G * ((S + 127) / 128));
  if (o32 && !(out_h3_scale > 0.f)) return (int)hipErrorInvalidValue;
  (out_h3_scale > 0.f ? launch_plane_attn<true> : launch_plane_attn<false>)(gx, st, q, kp, vp, o, lse, n_rows, B, Hq,
                                                                            Hkv, S, s_pad, out_h3_scale, sq, sk, sv,
                                                                            o32);
  return (int)hipGetLastError();
}

// sq, sk > 0: scores on the scaled fp16 h3 planes (the forward's matrix-core scheme, the caller guarantees
// s |x| <= 2^15 for q and k); 0: the native f32-MFMA / scalar kernels (exact fp32 products).
EDGE_API int edge_attn_lastrow_f32(const float* q, const float* k, float* out, int B, int Hq, int Hkv, int S, float sq,
                                   float sk, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv || S > 16384) return (int)hipErrorInvalidValue;
  const int G = Hq / Hkv;
  if (sq > 0.f && sk > 0.f && G <= 16 && (size_t)G * S * sizeof(float) <= 60 * 1024) {
    hipLaunchKernelGGL(attn_lastrow_h3_kernel, dim3(B * Hkv), dim3(256), G * S * sizeof(float), st, q, k, out, Hq, Hkv,
                       S, sq, sk);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(attn_lastrow_f32_kernel, dim3(B * Hq), dim3(256), S * sizeof(float), st, q, k, out, Hq, Hkv, S);
  return (int)hipGetLastError();
}

EDGE_API int edge_attn_colsum_f32(const float* q, const float* k, const float* lse, float* out, int B, int Hq, int Hkv,
                                  int S, float sq, float sk, hipStream_t st) {
  if (B <= 0 || S <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv) return (int)hipErrorInvalidValue;
  const int nkb = (S + 63) / 64;
  if (sq > 0.f && sk > 0.f) {
    hipLaunchKernelGGL(attn_colsum_h3_kernel, dim3(B * Hq * nkb), dim3(256), 0, st, q, k, lse, out, B, Hq, Hkv, S, sq,
                       sk);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(attn_colsum_f32_kernel, dim3(B * Hq * nkb), dim3(256), 0, st, q, k, lse, out, B, Hq, Hkv, S);
  return (int)hipGetLastError();
}
