#include <type_traits>
// bf16 MFMA GEMM for gfx950 with fused epilogues: C[M,N] = epilogue(A[M,K] . B[N,K]^T).
//
// Both operands are K-contiguous (activations [T,K], nn.Linear weights [N,K]).  128x128 block tile,
// BK = 64, 4 waves (2x2), each wave a 64x64 sub-tile of 4x4 v_mfma_f32_16x16x32_bf16 accumulators.
// Tiles are staged global->LDS with 16-byte global_load_lds (LDS image lane-linear, the XOR swizzle is
// applied to the per-lane SOURCE address and to the ds_read_b128 address), double-buffered.
// The MFMA is issued "swapped" (weights as the A operand) so every lane owns 4 consecutive output
// columns of one row: epilogues are lane-local and stores are 8-byte vectors.
//
// Epilogues:
//   NONE, BIAS, RESID (+residual, may alias C), BIAS_RESID, BIAS_GELU, SWIGLU (gate/up interleaved in
//   16-row blocks -> silu(g)*u, output N/2 columns), QKV_ROPE (bias + RoPE + head-major q/k + V^T
//   scatter + q pre-scale: replaces three reference ops), LSE (LM head: per-row partial max/sum-exp and
//   target logit, logits are never written to memory).
#include "common.h"
#include <algorithm>
#include <cstdlib>
#include <cstring>

enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_RESID = 2, EPI_BIAS_RESID = 3, EPI_BIAS_GELU = 4, EPI_SWIGLU = 5,
       EPI_QKV_ROPE = 6, EPI_LSE = 7,
       // fp32 execution (operands in the h3 split-fp16 layout, common.h; K is the concatenated 3K; fp16 MFMAs): fp32
       // outputs, fp32 bias / residual, h3-layout outputs for epilogues whose result feeds the next GEMM, or the LM
       // head's LSE partials
       EPI_F32 = 8, EPI_F32_BIAS = 9, EPI_F32_RESID = 10, EPI_F32_BIAS_RESID = 11, EPI_H3_BIAS_GELU = 12,
       EPI_H3_SWIGLU = 13, EPI_F32_QKV_ROPE = 14, EPI_F32_LSE = 15,
       // fp32 output = colscale[n] * product + fp32 residual: the relevance engine's input gradients through a
       // projection whose RMSNorm weight is applied on the output columns (the transposed weight then stays exact in
       // fp16: two products instead of three)
       EPI_F32_RESID_CS = 16,
       // the AttnLRP SwiGLU rule on the product (the MLP backward's dm GEMM): d = alpha (A . B^T) [M, N] with the saved
       // interleaved pre-activations gu [M, 2N] (residf / ldr) -> h3 planes [M, 2 (2N)] of the interleaved
       // (0.5 d u sig(g), 0.5 d g sig(g)) at unit scale (alpha carries the caller's bound-derived scale: no row max,
       // so no separate rule pass over an fp32 dm)
       EPI_H3_LRP_SWIGLU = 17,
       // fp32 output = product + fp32 residual, plus the next RMSNorm's producer side (the separate RMSNorm pass goes):
       // the h3 planes [M, 2N] of p_m (C_m * colscale) at a power-of-two row scale p_m from a bound on |C_m * colscale|,
       // prinv[m] = 1 / p_m and the row sum-of-squares partials ssq_out[m, N / 112] of C; the consumer GEMM takes
       // rscale[m] = rsqrt(sum ssq_out[m] / N + eps) * prinv[m] (np_scale)
       EPI_F32_RESID_NP = 18 };
constexpr bool epi_f32(int e) { return e >= EPI_F32; }
constexpr bool epi_plain(int e) {  // none / bias / residual epilogues (the 256x224 kernel's set)
  return e == EPI_NONE || e == EPI_BIAS || e == EPI_RESID || e == EPI_BIAS_RESID || e == EPI_F32 ||
         e == EPI_F32_BIAS || e == EPI_F32_RESID || e == EPI_F32_BIAS_RESID || e == EPI_F32_RESID_CS ||
         e == EPI_F32_RESID_NP;
}

struct GemmArgs {
  const bf16_t* A; const bf16_t* B; bf16_t* C;
  int M, N, K, lda, ldb, ldc;
  const bf16_t* bias; const bf16_t* resid; int ldr;
  // fp32 epilogues: fp32 output / bias / residual (C may alias resid), h3 outputs go to C (fp16 planes) with
  // ldc = 2 * width
  float* Cf; const float* biasf; const float* residf;
  float* qf; float* kf; float* vtf;
  float* vf;   // fp32 QKV, optional: V row-major [B, Hkv, S, 64] (the AttnLRP backward's operand) next to V^T / planes
  // EPI_F32_RESID_CS, optional: C also as the 2-plane h3 activation [M, 2N] (planes) of s_m C at the power-of-two row
  // scale s_m from the caller's bound 2^15 (bnd_a[m] + bnd_b[m] bnd_c) on |C row m|, and prinv[m] = 1 / s_m - the
  // next backward GEMM's input without a row-max pass (plane_scale)
  f16_t* planes; float* prinv; const float* bnd_a; const float* bnd_b; float bnd_c;
  // EPI_F32_RESID_NP: the bound on |C_m * colscale| is np_g (np_rn / bnd_b[m] + bnd_c) with bnd_b the residual input's
  // RMSNorm normalisers rsqrt(mean(x_m^2) + eps) (np_rn / bnd_b[m] = sqrt(K mean + K eps) >= ||x_m||_2 >= max |x_m|, np_rn =
  // sqrt(N)), bnd_c a bound on |product| and np_g = max |colscale|
  float np_g, np_rn;
  // QKV_ROPE
  bf16_t* qout; bf16_t* kout; bf16_t* vtout;
  const float* cosT; const float* sinT;
  int S, Hq, Hkv, s_pad; float q_scale;
  // fp32 QKV, optional: K / V^T also as scaled fp16 h3 planes for the attention kernel's LDS-DMA staging
  // (kp [B, Hkv, 2, S, 64], vp [B, Hkv, 2, 64, s_pad] in the kernel's key order; kv_plane_pos)
  f16_t* kp; f16_t* vp; float kv_sk, kv_sv;
  // LSE
  const int64_t* targets; float* part_max; float* part_sum; float* tgt_logit; int nparts;
  // fused RMSNorm: consumer side (row scale rscale[m] = rsqrt(mean(x_m^2) + eps), the norm weight is
  // pre-folded into B) and producer side (per-row sum of squares of the stored bf16 outputs, one
  // partial per 64-column slab: ssq_out[m, n/64])
  const float* rscale; float* ssq_out;
  const float* colscale;   // EPI_F32_RESID_CS: per-output-column factor of the product
  // consumer side without a row_rscale launch (QKV): rscale[m] computed at tile start from the producer's
  // partials, rsqrt(sum_p ssq_in[m, p] * norm_inv_k + norm_eps); takes precedence over rscale
  const float* ssq_in; int ssq_parts; float norm_inv_k, norm_eps;
  int walk;      // persistent four-wave kernel's tile walk: 0 = strided by the grid size, 1 = XCD-contiguous chunks
  int store_wait = 0;  // four-wave kernel: the wait after a full tile's epilogue leaves its last stores in flight
  int h3k;      // > 0: A is a 2-plane h3 activation [M, 2 h3k] (common.h h3_acol) of the K' = 3 h3k (or 2 h3k) GEMM
  int pairb;     // h3 two-product GEMM (K' = 2 h3k, B the single fp16 plane [N, h3k]): K-tiles interleave the planes,
                 // t -> A plane (t odd: hi, even: lo) column 64 (t >> 1), B column 64 (t >> 1) (b_kcol)
  float alpha = 1.f;      // h3: 1 / (s_a s_b), the product's scale (applied with the row scale)
  float out_scale = 1.f;  // h3 outputs (SwiGLU / GELU): the next GEMM's input scale s_a
  float* raw = nullptr;     // EPI_H3_SWIGLU, optional: the scaled pre-activations (gate|up interleaved) as fp32 [M, N]
                            // too, bit-identical to EPI_F32 (the AttnLRP forward saves them for the SwiGLU rule)
  bf16_t* rawb = nullptr;   // EPI_SWIGLU, optional: the same as bf16 [M, N], bit-identical to EPI_NONE
};

// element column of A holding GEMM column k (k a K-tile start)
__device__ __forceinline__ int a_kcol(const GemmArgs& a, int k) {
  if (a.pairb) return ((k >> 6) & 1 ? 0 : a.h3k) + ((k >> 7) << 6);
  return a.h3k ? h3_acol(k, a.h3k) : k;
}
// element column of B holding GEMM column k (k a K-tile start): the two K-tiles of a pair share one B tile
__device__ __forceinline__ int b_kcol(const GemmArgs& a, int k) { return a.pairb ? (k >> 7) << 6 : k; }

// 16x16x32 MFMA on bf16 (bf16 mode) or fp16 (h3 planes of the fp32 mode) operands held as raw 16-bit words
template <bool F16>
__device__ __forceinline__ f32x4_t mfma16x32(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

constexpr int BK = 64;
constexpr int GROUP_M = 8;

// Tile configurations: every wave owns a (MI*16) x 64 output slab (the 64-wide column slab is what
// the QKV/RoPE (one head) and SwiGLU (gate/up pairs) epilogues rely on).
template <int BM_, int BN_, int NWM_, int NWN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, NWM = NWM_, NWN = NWN_;
  static constexpr int NW = NWM * NWN, NT = 64 * NW;
  static constexpr int WTM = BM / NWM, MI = WTM / 16;
  static_assert(BN / NWN == 64, "wave column slab must be 64");
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  static constexpr int A_INSTR = BM / 8 / NW, B_INSTR = BN / 8 / NW;  // 1-KiB glds per wave per K-tile
  static constexpr int LDS = 2 * STAGE;
};
using C128 = Cfg<128, 128, 2, 2>;   // 4 waves, 64 KiB LDS, 2 blocks/CU

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }


__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float silu(float x) { return fast_silu(x); }

// Per-lane source pointers of this wave's staging instructions (hoisted out of the K loop): instruction
// i of wave w writes LDS rows [8*(i*NW+w), +8) of the tile, lane l -> row +l/8, physical 16-B chunk l%8,
// which holds logical chunk (l%8) ^ swz(row) (swizzle applied on the source side, LDS image lane-linear).
template <int NI, int NW>
__device__ __forceinline__ void stage_ptrs(const bf16_t* __restrict__ src, int ld, int row0, int row_max, int wave,
                                           int lane, const bf16_t* (&p)[NI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int blk = i * NW + wave;
    const int r = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz(r);
    int gr = row0 + r;
    gr = gr < row_max ? gr : row_max - 1;
    p[i] = src + (size_t)gr * ld + c * 8;
  }
}
template <int NI, int NW>
__device__ __forceinline__ void stage_issue(const bf16_t* const (&p)[NI], int k0, char* lds, int wave) {
#pragma unroll
  for (int i = 0; i < NI; ++i) glds16(p[i] + k0, lds + (i * NW + wave) * 1024);
}

__device__ __forceinline__ bf16x8_t read_frag(const char* lds, int r, int c) {
  return *(const bf16x8_t*)(lds + r * 128 + ((c ^ swz(r)) << 4));
}

// SwiGLU h3 epilogue of one 16-row group of a 64-column slab: gate/up interleaved in 16-column blocks (acc4[2p] gate,
// acc4[2p+1] up of output columns 16p + 4g + r) -> the 8 output columns pair_col(g) .. + 7 of the lane's row as the
// two h3 planes H, L (16 bytes each).  silu via v_exp_f32 / v_rcp_f32 (about 1 ulp each: fp32-level, as the h3
// products; the IEEE-exact expf and division were a third of this epilogue's VALU time).  The accumulators arrive
// unscaled (product scale f = row scale x alpha): the gate's f folds into the exp2 argument and f^2 s into one output
// multiply, on packed-f32 pairs: o = (g u) (1 / (1 + 2^(-f log2e g))) f^2 s.  The two 4-column groups of a plane are
// pair-swapped (permlane16: every lane must execute it, partners share the row) into 8 consecutive columns.
__device__ __forceinline__ void swiglu_h3_rowgroup(const GemmArgs& a, const f32x4_t (&acc4)[4], float f, u32x4_t& H,
                                                   u32x4_t& L) {
  const f32x2_t c1 = {-1.4426950408889634f * f, -1.4426950408889634f * f};
  const f32x2_t k2 = {f * f * a.out_scale, f * f * a.out_scale};
  u32x2_t hw[2], lw[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2_t gg = {acc4[2 * p][2 * h], acc4[2 * p][2 * h + 1]};
      const f32x2_t uu = {acc4[2 * p + 1][2 * h], acc4[2 * p + 1][2 * h + 1]};
      f32x2_t o = gg * uu;
      const f32x2_t t = gg * c1;
      f32x2_t e = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
      e = e + f32x2_t{1.f, 1.f};
      o = o * f32x2_t{__builtin_amdgcn_rcpf(e[0]), __builtin_amdgcn_rcpf(e[1])};
      o = o * k2;
      const u32x2_t hl = split2h_pk(o[0], o[1]);
      hw[p][h] = hl[0];
      lw[p][h] = hl[1];
    }
  }
  H = pair_swap16(hw[0], hw[1]);
  L = pair_swap16(lw[0], lw[1]);
}

// GemmArgs::raw: the 16-column groups acc4[0..3] of row m (columns n + 16 j + 4g .. + 3) times the product scale f,
// the values EPI_F32 stores.
__device__ __forceinline__ void swiglu_raw_store(const GemmArgs& a, const f32x4_t (&acc4)[4], float f, int m, int n,
                                                 int g) {
  if (m >= a.M) return;
  float* dst = a.raw + (size_t)m * a.N + n + 4 * g;
#pragma unroll
  for (int j = 0; j < 4; ++j) store_nt((f32x4_t*)(dst + 16 * j), acc4[j] * f);   // 1.27 GB, read in the backward
}

// Exchange of two 16-byte chunks between lanes r and r ^ 8 of each 16-lane row (DPP row_ror:8): lanes r < 8 keep X
// and get the X of lane r + 8 in B; lanes r >= 8 get the Y of lane r - 8 in A and keep Y in B.  For X / Y = the
// chunks of row r in the left / right 64-byte half of a 128-byte line, A then holds rows 0-7 and B rows 8-15 of the
// 16-row group as full lines (8 lanes per row).
__device__ __forceinline__ void line_exchange8(const u32x4_t& X, const u32x4_t& Y, bool lo8, u32x4_t& A, u32x4_t& B) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t t = lo8 ? Y[d] : X[d];
    const uint32_t u = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, 0x128, 0xF, 0xF, false);   // row_ror:8
    A[d] = lo8 ? X[d] : u;
    B[d] = lo8 ? u : Y[d];
  }
}

// SwiGLU h3 epilogue of the four-wave 256x256 kernel with full-line stores: the wave's 128 accumulator columns are 64
// output columns = one 128-byte line per plane and row, written 8 rows x 128 bytes per store instruction (the two
// 64-column slabs of a row group exchanged between lanes r and r ^ 8) instead of 16 rows x 64 bytes - half the
// store cost of the per-slab layout (ablation: 1 KiB-contiguous stores, profiles/history/r02k_gemm_epilogue_ablations.log).
template <int MI8>
__device__ __forceinline__ void swiglu_h3_lines_4w(const GemmArgs& a, f32x4_t (&acc)[MI8][8], const float (&rs)[MI8],
                                                   int m0, int n0, int lane, int wm, int wn) {
  const int r = lane & 15, g = lane >> 4;
  const bool lo8 = r < 8;
  const int col = n0 / 2 + wn * 64 + (lo8 ? 0 : 32) + pair_col(g);   // output column of the lane's chunk in A and B
  f16_t* const base = a.C + col;
#pragma unroll
  for (int i = 0; i < MI8; ++i) {
    f32x4_t c0[4], c1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c0[j] = acc[i][j];
      c1[j] = acc[i][4 + j];
      asm volatile("" : "+v"(c0[j]), "+v"(c1[j]));
    }
    const float f = rs[i] * a.alpha;
    if (a.raw) {   // (full-line stores here, as for the planes, measured equal: profiles/history/r05/raw_store_ab.log)
      const int m = m0 + wm * 128 + i * 16 + r;
      swiglu_raw_store(a, c0, f, m, n0 + wn * 128, g);
      swiglu_raw_store(a, c1, f, m, n0 + wn * 128 + 64, g);
    }
    u32x4_t H0, L0, H1, L1;
    swiglu_h3_rowgroup(a, c0, f, H0, L0);
    swiglu_h3_rowgroup(a, c1, f, H1, L1);
    u32x4_t HA, HB, LA, LB;
    line_exchange8(H0, H1, lo8, HA, HB);
    line_exchange8(L0, L1, lo8, LA, LB);
    const int ma = m0 + wm * 128 + i * 16 + (r & 7), mb = ma + 8;
    if (ma < a.M) {
      store_nt((u32x4_t*)(base + (size_t)ma * a.ldc), HA);
      store_nt((u32x4_t*)(base + (size_t)ma * a.ldc + a.N / 2), LA);
    }
    if (mb < a.M) {
      store_nt((u32x4_t*)(base + (size_t)mb * a.ldc), HB);
      store_nt((u32x4_t*)(base + (size_t)mb * a.ldc + a.N / 2), LB);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// AttnLRP SwiGLU rule epilogue of the four-wave 256x256 kernel (EPI_H3_LRP_SWIGLU): the wave's 128 rows x 128 dm
// columns are 8 interleave blocks per 16-row group, whose gate|up pre-activations (a 128-byte line per row and block)
// the rule reads.  Row group i + 1's loads are issued before group i computes and stores, so every wait finds its
// loads long in flight (the per-slab epilogue waited a full memory round trip per group and made the fused GEMM as
// slow as the GEMM plus the rule's own pass).
__device__ __forceinline__ void lrp_swiglu_4w(const GemmArgs& a, f32x4_t (&acc)[8][8], int m0, int n0, int lane,
                                              int wm, int wn) {
  if (n0 + wn * 128 >= a.N) return;   // empty half of a partial column tile (wave-uniform)
  const int r = lane & 15, g = lane >> 4;
  const int W = 2 * a.N;
  const int cb = (n0 + wn * 128) * 2 + g * 4;   // gu / plane column of the lane's gate chunk in block 0
  f32x4_t gb[2][8], ub[2][8];
  auto load = [&](int i, int b) {
    const int m = min(m0 + wm * 128 + i * 16 + r, a.M - 1);
    const float* gr = a.residf + (size_t)m * a.ldr + cb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gb[b][j] = *(const f32x4_t*)(gr + 32 * j);
      ub[b][j] = *(const f32x4_t*)(gr + 32 * j + 16);
    }
  };
  load(0, 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int b = i & 1;
    if (i + 1 < 8) load(i + 1, b ^ 1);
    f32x4_t c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      c[j] = acc[i][j];
      asm volatile("" : "+v"(c[j]));
    }
    const int m = m0 + wm * 128 + i * 16 + r;
    // the gate half (columns 4g..) and the up half (16 + 4g..) of block j exchanged between lanes l, l ^ 16 (same row:
    // every lane takes part) into 8 consecutive columns pair_col(g): one 16-byte store per plane instead of two 8-byte
    // ones - the fused GEMM 996-1005 against 1098-1104 us; plain stores (nontemporal: 1057-1061 us, the next GEMM reads
    // these planes; profiles/history/r05/lrp_epi17/)
    f16_t* dst = a.C + (size_t)min(m, a.M - 1) * a.ldc + (n0 + wn * 128) * 2 + pair_col(g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dg[4], du[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gv = gb[b][j][q];
        const float h = 0.5f * a.alpha * c[j][q] * fast_sigmoid(gv);
        dg[q] = h * ub[b][j][q];
        du[q] = h * gv;
      }
      const u32x2_t g0 = split2h_pk(dg[0], dg[1]), g1 = split2h_pk(dg[2], dg[3]);
      const u32x2_t u0 = split2h_pk(du[0], du[1]), u1 = split2h_pk(du[2], du[3]);
      const u32x4_t H = pair_swap16(u32x2_t{g0[0], g1[0]}, u32x2_t{u0[0], u1[0]});
      const u32x4_t L = pair_swap16(u32x2_t{g0[1], g1[1]}, u32x2_t{u0[1], u1[1]});
      if (m < a.M) {
        *(u32x4_t*)(dst + 32 * j) = H;
        *(u32x4_t*)(dst + 32 * j + W) = L;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---- K / V^T h3 planes from the fp32 QKV epilogues (GemmArgs::kp / vp).  split2h of s x: bit-identical to the split
// flash_attn_fwd_x6_kernel applies to the fp32 K / V^T it stages itself.  V^T keys are stored in the order the
// kernel's P^T operand holds them: within each 32-key block, lane group g's k-slots 8g..8g+7 are keys
// {4g..4g+3, 16+4g..16+4g+3}, so key 32 s + 16 hf + 4 a + r sits at element 8 (4 s + a) + 4 hf + r of its 64-key tile.
__device__ __forceinline__ int kv_plane_pos(int pos) {
  const int k = pos & 63;
  return (pos & ~63) | ((4 * (k >> 5) + ((k >> 2) & 3)) << 3) | (((k >> 4) & 1) << 2) | (k & 3);
}
__device__ __forceinline__ void store_k_planes4(const GemmArgs& a, int b, int hk, int pos, int d, const float (&v)[4]) {
  store_h3_4(a.kp + ((size_t)(b * a.Hkv + hk) * 2 * a.S + pos) * 64, a.S * 64, d, v, a.kv_sk);
}
__device__ __forceinline__ void store_vt_plane1(const GemmArgs& a, int b, int hv, int pos, int d, float v) {
  float hi, lo;
  split2h(v * a.kv_sv, hi, lo);
  const size_t o = ((size_t)(b * a.Hkv + hv) * 2 * 64 + d) * a.s_pad + kv_plane_pos(pos);
  a.vp[o] = __builtin_bit_cast(uint16_t, (_Float16)hi);
  a.vp[o + (size_t)64 * a.s_pad] = __builtin_bit_cast(uint16_t, (_Float16)lo);
}

// s_m of GemmArgs::planes: 2^(15 - E) for the bound 2^15 (bnd_a[m] + bnd_b[m] bnd_c) = f 2^E, f in [0.5, 1)
__device__ __forceinline__ float plane_scale(const GemmArgs& a, int m) {
  int e;
  (void)frexpf(32768.f * (a.bnd_a[m] + a.bnd_b[m] * a.bnd_c), &e);
  return ldexpf(1.f, 15 - e);
}

// p_m of EPI_F32_RESID_NP: 2^(14 - E) for the bound u = np_g (np_rn / bnd_b[m] + bnd_c) = f 2^E, f in [0.5, 1), so that
// p_m |C_m colscale| < 2^14 (fp16 max 65504: 2x headroom for the fp32 rounding of C)
__device__ __forceinline__ float np_scale(const GemmArgs& a, int m) {
  int e;
  (void)frexpf(a.np_g * (a.np_rn / a.bnd_b[m] + a.bnd_c), &e);
  return ldexpf(1.f, 14 - e);
}

// ---- fp32-execution epilogues (EPI >= EPI_F32).  Same ownership as gemm_epilogue below: lane owns rows
// m0 + wm*WTM + i*16 + (lane&15) and columns nw + j*16 + 4*(lane>>4) + r of the wave's 64-column slab, so every
// output is 4 consecutive fp32 values (one 16-byte store) or 4 consecutive values of each of the two h3 planes.
template <int EPI, int RH, class CF>
__device__ __forceinline__ void gemm_epilogue_f32(const GemmArgs& a, f32x4_t (&acc)[CF::MI][4], int m0, int nw,
                                                  int lane, int wm, const float (&rs)[CF::MI]) {
  constexpr int MI = CF::MI;
  const int g = lane >> 4;
  if constexpr (EPI == EPI_F32_QKV_ROPE) {
    const int head = nw / 64;  // global head slot in [q heads | k heads | v heads]
    const bool is_v = head >= a.Hq + a.Hkv;
    f32x4_t bw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bw[j] = *(const f32x4_t*)(a.biasf + nw + j * 16 + g * 4);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
      const int mm = m < a.M ? m : a.M - 1;
      const int b = mm / a.S, pos = mm - b * a.S;
      float v[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] = acc[i][j][r] + bw[j][r];
      if constexpr (RH >= 16) {
        constexpr int DJ = RH / 16;
        if (!is_v) {
          float o[4][4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (j * 16 >= 2 * RH) { o[j][r] = v[j][r]; continue; }
              const bool lo = j * 16 < RH;
              const int fi = (lo ? j : j - DJ) * 16 + g * 4 + r;
              const float c = a.cosT[pos * RH + fi], sv = a.sinT[pos * RH + fi];
              const float y = lo ? v[(j + DJ) & 3][r] : v[(j - DJ) & 3][r];
              o[j][r] = lo ? (v[j][r] * c - y * sv) : (v[j][r] * c + y * sv);
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] = o[j][r];
        }
      } else if constexpr (RH > 0) {
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = __shfl_xor(v[0][r], 4 * RH, 64);
        if (!is_v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int d = g * 4 + r;
            if (d < 2 * RH) {
              const bool lo = d < RH;
              const int fi = lo ? d : d - RH;
              const float c = a.cosT[pos * RH + fi], s = a.sinT[pos * RH + fi];
              v[0][r] = lo ? (v[0][r] * c - p[r] * s) : (v[0][r] * c + p[r] * s);
            }
          }
        }
      }
      if (m >= a.M) continue;
      if (!is_v) {
        const float sc = head < a.Hq ? a.q_scale : 1.f;
        float* dst = head < a.Hq ? a.qf + (((size_t)b * a.Hq + head) * a.S + pos) * 64
                                 : a.kf + (((size_t)b * a.Hkv + (head - a.Hq)) * a.S + pos) * 64;
        if (head < a.Hq || a.kf) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            *(f32x4_t*)(dst + j * 16 + g * 4) = f32x4_t{v[j][0] * sc, v[j][1] * sc, v[j][2] * sc, v[j][3] * sc};
        }
        if (head >= a.Hq && a.kp) {
#pragma unroll
          for (int j = 0; j < 4; ++j) store_k_planes4(a, b, head - a.Hq, pos, j * 16 + g * 4, v[j]);
        }
      } else {
        if (a.vf) {
          float* dst = a.vf + (((size_t)b * a.Hkv + (head - a.Hq - a.Hkv)) * a.S + pos) * 64;
#pragma unroll
          for (int j = 0; j < 4; ++j) *(f32x4_t*)(dst + j * 16 + g * 4) = f32x4_t{v[j][0], v[j][1], v[j][2], v[j][3]};
        }
        if (a.vtf) {
          float* dst = a.vtf + ((size_t)b * a.Hkv + (head - a.Hq - a.Hkv)) * 64 * (size_t)a.s_pad + pos;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(size_t)(j * 16 + g * 4 + r) * a.s_pad] = v[j][r];
        }
        if (a.vp) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) store_vt_plane1(a, b, head - a.Hq - a.Hkv, pos, j * 16 + g * 4 + r, v[j][r]);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
    if constexpr (EPI == EPI_H3_SWIGLU) {
      u32x4_t H, Lw;
      if (a.raw) swiglu_raw_store(a, acc[i], rs[i] * a.alpha, m, nw, g);
      swiglu_h3_rowgroup(a, acc[i], rs[i] * a.alpha, H, Lw);
      if (m < a.M) {
        f16_t* dst = a.C + (size_t)m * a.ldc + nw / 2 + pair_col(g);
        *(u32x4_t*)dst = H;
        *(u32x4_t*)(dst + a.N / 2) = Lw;
      }
      continue;
    }
    if constexpr (EPI == EPI_H3_BIAS_GELU) {   // same 16-byte plane stores for the column-group pairs (0,1) (2,3)
      u32x2_t hw[4], lw[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4_t bw = *(const f32x4_t*)(a.biasf + nw + j * 16 + g * 4);
        float hi[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) hi[r] = gelu_erf(acc[i][j][r] + bw[r]) * a.out_scale;
        const u32x2_t t0 = split2h_pk(hi[0], hi[1]), t1 = split2h_pk(hi[2], hi[3]);
        hw[j] = u32x2_t{t0[0], t1[0]};
        lw[j] = u32x2_t{t0[1], t1[1]};
      }
#pragma unroll
      for (int q2 = 0; q2 < 2; ++q2) {
        const u32x4_t H = pair_swap16(hw[2 * q2], hw[2 * q2 + 1]), Lw = pair_swap16(lw[2 * q2], lw[2 * q2 + 1]);
        if (m < a.M) {
          f16_t* dst = a.C + (size_t)m * a.ldc + nw + q2 * 32 + pair_col(g);
          *(u32x4_t*)dst = H;
          *(u32x4_t*)(dst + a.N) = Lw;
        }
      }
      continue;
    }
    if constexpr (EPI == EPI_H3_LRP_SWIGLU) {   // a 16-column j group is one interleave block: gate|up = 128 B of gu
      if (m >= a.M) continue;
      const float* gr = a.residf + (size_t)m * a.ldr;
      f16_t* dst = a.C + (size_t)m * a.ldc;
      const int W = 2 * a.N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nw + j * 16 + g * 4;
        const int col = (n >> 4) * 32 + (n & 15);
        const f32x4_t gv = *(const f32x4_t*)(gr + col), uv = *(const f32x4_t*)(gr + col + 16);
        float dg[4], du[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float sg = fast_sigmoid(gv[r]), h = 0.5f * acc[i][j][r] * sg;
          dg[r] = h * uv[r];
          du[r] = h * gv[r];
        }
        store_h3_4(dst, W, col, dg, 1.f);
        store_h3_4(dst, W, col + 16, du, 1.f);
      }
      continue;
    }
    if (m >= a.M) continue;
    {
      float ps = 0.f;
      if constexpr (EPI == EPI_F32_RESID_CS) {
        if (a.planes) {
          ps = plane_scale(a, m);
          if (nw == 0 && g == 0) a.prinv[m] = 1.f / ps;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = nw + j * 16 + g * 4;
        float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (EPI == EPI_F32_RESID_CS) {
          const f32x4_t cw = *(const f32x4_t*)(a.colscale + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] *= cw[r];
        }
        if constexpr (EPI == EPI_F32_BIAS || EPI == EPI_F32_BIAS_RESID) {
          const f32x4_t bw = *(const f32x4_t*)(a.biasf + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] += bw[r];
        }
        if constexpr (EPI == EPI_F32_RESID || EPI == EPI_F32_BIAS_RESID || EPI == EPI_F32_RESID_CS) {
          const f32x4_t rw = *(const f32x4_t*)(a.residf + (size_t)m * a.ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] += rw[r];
        }
        *(f32x4_t*)(a.Cf + (size_t)m * a.ldc + n) = f32x4_t{o[0], o[1], o[2], o[3]};
        if constexpr (EPI == EPI_F32_RESID_CS) {
          if (a.planes) store_h3_4(a.planes + (size_t)m * (2 * a.N), a.N, n, o, ps);
        }
      }
    }
  }
}

// ---- epilogue: lane owns rows m0 + wm*WTM + i*16 + (lane&15), columns n0 + wn*64 + j*16 + 4*(lane>>4) + r
template <int EPI, int RH, class CF>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& a, f32x4_t (&acc)[CF::MI][4], int m0, int n0,
                                              int lane, int wm, int wn, const float (&rs)[CF::MI],
                                              char* lds = nullptr) {
  constexpr int MI = CF::MI;
  const int g = lane >> 4;
  const int nw = n0 + wn * 64;  // first column of this wave's 64-wide slab
  if (nw >= a.N) return;        // slab beyond N in a partial last column tile (wave-uniform)

  if constexpr (epi_f32(EPI)) {  // h3 operands: the product's scale alpha with the optional row scale
    if constexpr (EPI != EPI_H3_SWIGLU) {   // (the SwiGLU epilogue folds it into its constants)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const float f = rs[i] * a.alpha;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] *= f;
      }
    }
    if constexpr (EPI != EPI_F32_LSE) return gemm_epilogue_f32<EPI, RH, CF>(a, acc, m0, nw, lane, wm, rs);
  } else if (a.rscale || a.ssq_in) {  // fused RMSNorm of the A operand: per-row scale (prefetched at tile start)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] *= rs[i];
  }

  if constexpr (EPI == EPI_LSE || EPI == EPI_F32_LSE) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, acc[i][j][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) se += __expf(acc[i][j][r] - mx);
      se += __shfl_xor(se, 16, 64);
      se += __shfl_xor(se, 32, 64);
      if (m < a.M) {
        if (g == 0) {
          a.part_max[(size_t)m * a.nparts + nw / 64] = mx;
          a.part_sum[(size_t)m * a.nparts + nw / 64] = se;
        }
        const int64_t tg = a.targets[m];
        const int64_t off = tg - nw;
        if (off >= 0 && off < 64) {
          const int j = (int)(off >> 4), rr = (int)(off & 3), gg = (int)((off >> 2) & 3);
          if (gg == g) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (jj == j && r == rr) a.tgt_logit[m] = acc[i][jj][r];
          }
        }
      }
    }
    return;
  }

  if constexpr (EPI == EPI_QKV_ROPE) {
    const int head = nw / 64;  // global head slot in [q heads | k heads | v heads]
    const bool is_v = head >= a.Hq + a.Hkv;
    // Every global load of the epilogue (bias, RoPE tables of all row groups) is issued before the first store:
    // vmcnt counts stores too, so a load waited between the stores of two row groups would drain them.
    u32x2_t bw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bw[j] = *(const u32x2_t*)(a.bias + nw + j * 16 + g * 4);
    constexpr int NJ = RH >= 16 ? RH / 16 : 1;  // register groups in the rotated low half
    f32x4_t cs[MI][NJ], sn[MI][NJ];
    int bi[MI], pi[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
      const int mm = m < a.M ? m : a.M - 1;
      bi[i] = mm / a.S;
      pi[i] = mm - bi[i] * a.S;
      if constexpr (RH >= 16) {
        if (!is_v) {
          // cos/sin of the 4 consecutive frequencies this lane needs per 16-column group: one float4 each
          // (the frequency index of column d is d mod RH, shared by the pair (d, d+RH))
#pragma unroll
          for (int jf = 0; jf < NJ; ++jf) {
            cs[i][jf] = *(const f32x4_t*)(a.cosT + pi[i] * RH + jf * 16 + g * 4);
            sn[i][jf] = *(const f32x4_t*)(a.sinT + pi[i] * RH + jf * 16 + g * 4);
          }
        }
      }
    }
    // V heads: transpose the wave's 64-row x 64-d slab through LDS ([d][row], row stride 72 elements) and store
    // V^T rows as 16-byte chunks of 8 positions, instead of 16 scattered 2-byte stores per lane and row group.
    // Needs the slab's 64 rows inside one window and < M (S % 64 == 0), and the LDS (free after the K loop).
    const int row0 = m0 + wm * CF::WTM;
    const bool v_lds = is_v && lds && CF::WTM == 64 && a.S % 64 == 0 && row0 + 63 < a.M;
    bf16_t* tl = v_lds ? (bf16_t*)(lds + (wm * CF::NWN + wn) * (64 * 72 * 2)) : nullptr;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
      const int b = bi[i], pos = pi[i];
      float v[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j][0] = acc[i][j][0] + bf_lo(bw[j][0]);
        v[j][1] = acc[i][j][1] + bf_hi(bw[j][0]);
        v[j][2] = acc[i][j][2] + bf_lo(bw[j][1]);
        v[j][3] = acc[i][j][3] + bf_hi(bw[j][1]);
      }
      if constexpr (RH >= 16) {
        // rotate_half partner of column d is d +- RH: register j +- RH/16, same lane.
        constexpr int DJ = RH / 16;
        if (!is_v) {
          float o[4][4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (j * 16 >= 2 * RH) { o[j][r] = v[j][r]; continue; }
              const bool lo = j * 16 < RH;
              const int jf = lo ? j : j - DJ;
              const float c = cs[i][jf][r], sv = sn[i][jf][r];
              const float y = lo ? v[(j + DJ) & 3][r] : v[(j - DJ) & 3][r];
              o[j][r] = lo ? (v[j][r] * c - y * sv) : (v[j][r] * c + y * sv);
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] = o[j][r];
        }
      } else if constexpr (RH > 0) {
        // rotated dims live in register group j == 0; partner lane = lane ^ (4*RH)
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = __shfl_xor(v[0][r], 4 * RH, 64);
        if (!is_v) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int d = g * 4 + r;
            if (d < 2 * RH) {
              const bool lo = d < RH;
              const int fi = lo ? d : d - RH;
              const float c = a.cosT[pos * RH + fi], s = a.sinT[pos * RH + fi];
              v[0][r] = lo ? (v[0][r] * c - p[r] * s) : (v[0][r] * c + p[r] * s);
            }
          }
        }
      }
      if (!is_v) {  // q / k rows: 16-byte stores after the pair swap (head is wave-uniform, m per row)
        const float sc = head < a.Hq ? a.q_scale : 1.f;
        bf16_t* dst = head < a.Hq ? a.qout + (((size_t)b * a.Hq + head) * a.S + pos) * 64
                                  : a.kout + (((size_t)b * a.Hkv + (head - a.Hq)) * a.S + pos) * 64;
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
          u32x2_t w0, w1;
          w0[0] = pack_bf2(v[2 * q2][0] * sc, v[2 * q2][1] * sc);
          w0[1] = pack_bf2(v[2 * q2][2] * sc, v[2 * q2][3] * sc);
          w1[0] = pack_bf2(v[2 * q2 + 1][0] * sc, v[2 * q2 + 1][1] * sc);
          w1[1] = pack_bf2(v[2 * q2 + 1][2] * sc, v[2 * q2 + 1][3] * sc);
          const u32x4_t w = pair_swap16(w0, w1);
          if (m < a.M) *(u32x4_t*)(dst + q2 * 32 + pair_col(g)) = w;
        }
      } else if (v_lds) {
        const int rl = i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) tl[(j * 16 + g * 4 + r) * 72 + rl] = f2bf(v[j][r]);
      } else {
        if (m >= a.M) continue;
        bf16_t* dst = a.vtout + ((size_t)b * a.Hkv + (head - a.Hq - a.Hkv)) * 64 * (size_t)a.s_pad + pos;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) dst[(size_t)(j * 16 + g * 4 + r) * a.s_pad] = f2bf(v[j][r]);
      }
    }
    if (v_lds) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done before it reads them back
      const int b = bi[0], pos0 = pi[0] - (lane & 15);  // slab's first row (64-aligned, one window)
      bf16_t* vbase = a.vtout + ((size_t)b * a.Hkv + (head - a.Hq - a.Hkv)) * 64 * (size_t)a.s_pad + pos0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = k * 64 + lane, d = c >> 3, pc = c & 7;
        const u32x4_t w = *(const u32x4_t*)(tl + d * 72 + pc * 8);
        *(u32x4_t*)(vbase + (size_t)d * a.s_pad + pc * 8) = w;
      }
    }
    return;
  }

#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = m0 + wm * CF::WTM + i * 16 + (lane & 15);
    const bool ok = m < a.M;
    if constexpr (EPI == EPI_SWIGLU) {
      if (a.rawb && ok) {   // the pre-activations as EPI_NONE would store them (columns nw + 16 j + 4 g .. + 3)
        bf16_t* rp = a.rawb + (size_t)m * a.N + nw + g * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *(u32x2_t*)(rp + j * 16) = u32x2_t{pack_bf2(acc[i][j][0], acc[i][j][1]), pack_bf2(acc[i][j][2], acc[i][j][3])};
      }
      u32x2_t w[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        // silu(g) * u on float pairs: the multiplies and the add issue as v_pk_* (two lanes' worth per VALU
        // slot), leaving the two transcendentals per output (v_exp_f32, v_rcp_f32) as the epilogue's cost
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2_t gg = {acc[i][2 * p][2 * h], acc[i][2 * p][2 * h + 1]};
          const f32x2_t uu = {acc[i][2 * p + 1][2 * h], acc[i][2 * p + 1][2 * h + 1]};
          const f32x2_t t = gg * f32x2_t{-1.4426950408889634f, -1.4426950408889634f};
          f32x2_t e = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
          e = e + f32x2_t{1.f, 1.f};
          const f32x2_t r = {__builtin_amdgcn_rcpf(e[0]), __builtin_amdgcn_rcpf(e[1])};
          const f32x2_t o = (gg * uu) * r;
          w[p][h] = pack_bf2(o[0], o[1]);
        }
      }
      const u32x4_t wv = pair_swap16(w[0], w[1]);   // every lane swaps (partners share m)
      if (ok) *(u32x4_t*)(a.C + (size_t)m * a.ldc + nw / 2 + pair_col(g)) = wv;
    } else {
      float ss = 0.f;
      const int mr = ok ? m : a.M - 1;   // clamped row for loads; every lane takes part in the swaps
#pragma unroll
      for (int q2 = 0; q2 < 2; ++q2) {
        u32x2_t w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int j = 2 * q2 + h;
          const int n = nw + j * 16 + g * 4;
          float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU) {
            const u32x2_t bw = *(const u32x2_t*)(a.bias + n);
            o[0] += bf_lo(bw[0]); o[1] += bf_hi(bw[0]); o[2] += bf_lo(bw[1]); o[3] += bf_hi(bw[1]);
          }
          if constexpr (EPI == EPI_BIAS_GELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = gelu_erf(o[r]);
          }
          if constexpr (EPI == EPI_RESID || EPI == EPI_BIAS_RESID) {
            const u32x2_t rw = *(const u32x2_t*)(a.resid + (size_t)mr * a.ldr + n);
            o[0] += bf_lo(rw[0]); o[1] += bf_hi(rw[0]); o[2] += bf_lo(rw[1]); o[3] += bf_hi(rw[1]);
          }
          w[h][0] = pack_bf2(o[0], o[1]);
          w[h][1] = pack_bf2(o[2], o[3]);
          const float v0 = bf_lo(w[h][0]), v1 = bf_hi(w[h][0]), v2 = bf_lo(w[h][1]), v3 = bf_hi(w[h][1]);
          ss += v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;  // of the stored (rounded) values
        }
        const u32x4_t wv = pair_swap16(w[0], w[1]);
        if (ok) *(u32x4_t*)(a.C + (size_t)m * a.ldc + nw + q2 * 32 + pair_col(g)) = wv;
      }
      if (a.ssq_out) {  // uniform branch: every lane takes part in the shuffles
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        if (ok && g == 0) a.ssq_out[(size_t)m * (a.N / 64) + nw / 64] = ss;
      }
    }
  }
}

// Row sums of NP sum-of-squares partials with every load issued before the first add (one round trip)
template <int MI, int WTM, int NP>
__device__ __forceinline__ void rscale_from_partials(const GemmArgs& a, int m0, int wm, int lane, float (&rs)[MI]) {
  float v[MI][NP];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    int m = m0 + wm * WTM + i * 16 + (lane & 15);
    m = m < a.M ? m : a.M - 1;
    const float* p = a.ssq_in + (size_t)m * NP;
    if constexpr (NP % 4 == 0) {
#pragma unroll
      for (int j = 0; j < NP; j += 4) *(f32x4_t*)&v[i][j] = *(const f32x4_t*)(p + j);
    } else {
#pragma unroll
      for (int j = 0; j < NP; j += 2) {
        const u32x2_t w = *(const u32x2_t*)(p + j);
        v[i][j] = __uint_as_float(w[0]);
        v[i][j + 1] = __uint_as_float(w[1]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < NP; ++j) ss += v[i][j];
    rs[i] = rsqrtf(ss * a.norm_inv_k + a.norm_eps);
  }
}

template <int MI, int WTM>
__device__ __forceinline__ void load_rscale(const GemmArgs& a, int m0, int wm, int lane, float (&rs)[MI]) {
  // partial counts of the producers: 8 (256x224 GEMMs' 112-column slabs), 14 (64-column slabs of H=896).  Only
  // compiled into the 128x128 tiles (the QKV GEMM): the 256-VGPR 256x256 loops spill with the extra registers.
  if constexpr (MI <= 4) {
    if (a.ssq_in) {
      if (a.ssq_parts == 8) return rscale_from_partials<MI, WTM, 8>(a, m0, wm, lane, rs);
      return rscale_from_partials<MI, WTM, 14>(a, m0, wm, lane, rs);
    }
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    int m = m0 + wm * WTM + i * 16 + (lane & 15);
    m = m < a.M ? m : a.M - 1;
    rs[i] = a.rscale ? a.rscale[m] : 1.f;
  }
}

template <int MI>
__device__ __forceinline__ void zero_acc(f32x4_t (&acc)[MI][4]) {
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
}

// 32-bit LDS address of a pointer into dynamic shared memory
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// ds_read_b128 hidden from the compiler's waitcnt insertion: the caller owns the lgkmcnt accounting.
#define DS_READ_B128(dst, vaddr, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(vaddr), "i"(off))
// MFMA with the accumulator pinned to AGPRs: a one-wave-per-SIMD kernel holding 256 accumulator registers needs
// them in the AGPR half of the unified file (the builtin's VGPR form spills).  The hazard recognizer does not see
// into the asm: readers of the accumulators wait MFMA_DRAIN first, and zeroed accumulators are separated from
// their first MFMA by ACC_SETTLE.
#define MFMA_AGPR(acc, a, b) asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b))
#define MFMA_DRAIN() asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory")
#define ACC_SETTLE() asm volatile("s_nop 4" ::: "memory")
#define MFMA_AGPR_FIRST(acc, a, b) asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b))
// fp16 operands (the h3 planes of the fp32 mode)
#define MFMA_AGPR_H(acc, a, b) asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b))
#define MFMA_AGPR_FIRST_H(acc, a, b) asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b))

// Persistent tile walk of workgroup bid out of G.  Workgroups are dispatched round-robin over the 8 XCDs
// (bid & 7), and xcd_remap numbers the workgroups of one XCD consecutively (base .. base+cx-1).
//   chunked (default): XCD x owns the contiguous range [T*base/G, T*(base+cx)/G) of the grouped-M tile order
//     and its cx workgroups take tiles lo+l, lo+l+cx, ...  Consecutive rounds of an XCD stay inside one
//     GROUP_M band, so its 8 A panels stay in the XCD's L2 and only the next B panels are fetched (for the
//     gate/up shape: 4 new panels per round of 32 tiles instead of 12).
//   strided: tiles v, v+G, v+2G, ... with v = xcd_remap(bid): every round jumps to a new region of the order.
struct TileWalk { int first, stride, end; };
__device__ __forceinline__ TileWalk tile_walk(int bid, int G, int ntiles, int chunked) {
  if (!chunked) return {xcd_remap(bid, G), G, ntiles};
  const int x = bid & 7, l = bid >> 3, q = G >> 3, r = G & 7;
  const int cx = q + (x < r ? 1 : 0);
  const int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int lo = (int)((long long)ntiles * base / G), hi = (int)((long long)ntiles * (base + cx) / G);
  return {lo + l, cx, hi};
}

__device__ __forceinline__ void tile_origin(int id, int M, int N, int BM, int BN, int& m0, int& n0) {
  // grouped-M order: GROUP_M consecutive m-panels sweep the n-panels together (A panels stay in L2)
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const int group = id / (GROUP_M * tn);
  const int first_m = group * GROUP_M;
  const int gsz = min(tm - first_m, GROUP_M);
  const int in_g = id - group * GROUP_M * tn;
  m0 = (first_m + in_g % gsz) * BM;
  n0 = (in_g / gsz) * BN;
}

template <int EPI, int RH, class CF>
__global__ __launch_bounds__(CF::NT, 2) void gemm_bf16_kernel(GemmArgs a) {
  // One tile per workgroup (2 workgroups per CU hide each other's prologue/epilogue); fragments are read right before
  // use.  The small-M / odd-N shapes the persistent four-wave kernel does not fill the chip with.
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = CF::BM, BN = CF::BN, MI = CF::MI, NW = CF::NW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / CF::NWN, wn = wave % CF::NWN;
  const int tm = (a.M + BM - 1) / BM, tn = (a.N + BN - 1) / BN;  // last column tile may be partial
  const int ntiles = tm * tn;

  f32x4_t acc[MI][4];
  zero_acc<MI>(acc);
  const bf16_t* pa[CF::A_INSTR];
  const bf16_t* pb[CF::B_INSTR];
  // Fragment addresses in the swizzled LDS image.  The swizzle of row r is (r>>1)&7 and every fragment
  // row is lane&15 plus a multiple of 16, so it depends on the lane only: one base per k-half, the
  // m/n tile offsets are immediates (2 KiB per 16 rows).
  const int sw = ((lane & 15) >> 1) & 7;
  int abase[2], bbase[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int c = ks * 4 + (lane >> 4);
    abase[ks] = (wm * CF::WTM + (lane & 15)) * 128 + ((c ^ sw) << 4);
    bbase[ks] = CF::A_BYTES + (wn * 64 + (lane & 15)) * 128 + ((c ^ sw) << 4);
  }
  constexpr int MG = MI / 4;
  bf16x8_t XA[4], XB[4];
  auto ld = [&](bf16x8_t(&FA)[4], bf16x8_t(&FB)[4], const char* buf, int ks, int mg) {
#pragma unroll
    for (int i = 0; i < 4; ++i) FA[i] = *(const bf16x8_t*)(buf + abase[ks] + (mg * 4 + i) * 2048);
#pragma unroll
    for (int j = 0; j < 4; ++j) FB[j] = *(const bf16x8_t*)(buf + bbase[ks] + j * 2048);
  };
  auto mma = [&](const bf16x8_t(&FA)[4], const bf16x8_t(&FB)[4], int mg) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[mg * 4 + i][j] = mfma16x32<epi_f32(EPI)>(FB[j], FA[i], acc[mg * 4 + i][j]);
  };
  auto stage = [&](int k0, char* buf) {
    stage_issue<CF::A_INSTR, NW>(pa, a_kcol(a, k0), buf, wave);
    stage_issue<CF::B_INSTR, NW>(pb, b_kcol(a, k0), buf + CF::A_BYTES, wave);
  };
  const int nk = a.K / BK;
  int m0, n0;
  tile_origin(xcd_remap(blockIdx.x, ntiles), a.M, a.N, BM, BN, m0, n0);
  float rs[MI];
  load_rscale<MI, CF::WTM>(a, m0, wm, lane, rs);
  stage_ptrs<CF::A_INSTR, NW>(a.A, a.lda, m0, a.M, wave, lane, pa);
  stage_ptrs<CF::B_INSTR, NW>(a.B, a.ldb, n0, a.N, wave, lane, pb);
  stage(0, smem);
  wait_vmcnt0();
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t & 1) * CF::STAGE;
    if (t + 1 < nk) stage((t + 1) * BK, smem + ((t + 1) & 1) * CF::STAGE);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int mg = 0; mg < MG; ++mg) {
        ld(XA, XB, cur, ks, mg);
        mma(XA, XB, mg);
      }
    }
    wait_vmcnt0();
    __syncthreads();
  }
  gemm_epilogue<EPI, RH, CF>(a, acc, m0, n0, lane, wm, wn, rs, smem);  // LDS free: K loop done
}

// ---- 256x224 tiles for N = 896 (Qwen2 hidden size: O-proj and MLP down, both residual epilogues) ------------------
// 896 = 3.5 x 256: the 256x256 tile computes a half-empty last column tile (1/8 of all MFMAs wasted), and no
// power-of-two tile both avoids that and gives a tile count that divides the 256 CUs.  896 = 4 x 224 does:
// 128 x 4 = 512 tiles for M = 32768 (exactly 2 per CU), run by the four-wave kernel as 128 x 112 wave tiles whose
// epilogue works on 64 x 112 halves (w7_epilogue).  Row sum-of-squares partials (fused RMSNorm producer) are per
// 112-column wave slab: ssq_out[m, N / 112].
namespace w7 {
constexpr int MI = 4, NJ = 7;   // a 64 x 112 epilogue half: 4 x 7 accumulators of 16 x 16
}  // namespace w7

template <int EPI>
__device__ __forceinline__ void w7_epilogue(const GemmArgs& a, f32x4_t (&acc)[w7::MI][w7::NJ], int m0, int n0,
                                            int lane, int wm, int wn) {
  const int g = lane >> 4;
  const int nw = n0 + wn * 112;
  const int P = a.N / 112;
  static_assert(!epi_f32(EPI), "fp32 epilogues of the 224-wide tiles: w4_f32_epilogue_224");
  constexpr bool RES = EPI == EPI_RESID || EPI == EPI_BIAS_RESID;
  // every residual load of the slab is issued up front (4 x 7 x 8 B per lane): one global round trip instead of
  // one per 16-row group (the per-group load -> wait -> use chain cost ~30 % of the O-proj GEMM's time)
  // (vmcnt also counts stores on gfx9: a load waited between the stores of two groups drains those stores too,
  // so the row scales are fetched up front as well)
  u32x2_t rv[w7::MI][w7::NJ];
  float rsv[w7::MI];
#pragma unroll
  for (int i = 0; i < w7::MI; ++i) {
    int mr = m0 + wm * 64 + i * 16 + (lane & 15);
    mr = mr < a.M ? mr : a.M - 1;
    rsv[i] = a.rscale ? a.rscale[mr] : 1.f;
    if constexpr (RES) {
      const bf16_t* rrow = a.resid + (size_t)mr * a.ldr + nw + g * 4;
#pragma unroll
      for (int j = 0; j < w7::NJ; ++j) rv[i][j] = *(const u32x2_t*)(rrow + j * 16);
    }
  }
#pragma unroll
  for (int i = 0; i < w7::MI; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    const bool ok = m < a.M;
    const float rs = rsv[i];
    float ss = 0.f;
    u32x2_t w[w7::NJ];
#pragma unroll
    for (int j = 0; j < w7::NJ; ++j) {
      const int n = nw + j * 16 + g * 4;
      float o[4] = {acc[i][j][0] * rs, acc[i][j][1] * rs, acc[i][j][2] * rs, acc[i][j][3] * rs};
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID) {
        const u32x2_t bw = *(const u32x2_t*)(a.bias + n);
        o[0] += bf_lo(bw[0]); o[1] += bf_hi(bw[0]); o[2] += bf_lo(bw[1]); o[3] += bf_hi(bw[1]);
      }
      if constexpr (RES) {
        const u32x2_t rw = rv[i][j];
        o[0] += bf_lo(rw[0]); o[1] += bf_hi(rw[0]); o[2] += bf_lo(rw[1]); o[3] += bf_hi(rw[1]);
      }
      w[j][0] = pack_bf2(o[0], o[1]);
      w[j][1] = pack_bf2(o[2], o[3]);
      const float v0 = bf_lo(w[j][0]), v1 = bf_hi(w[j][0]), v2 = bf_lo(w[j][1]), v3 = bf_hi(w[j][1]);
      ss += v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;  // of the stored (rounded) values
    }
    bf16_t* row = a.C + (size_t)(ok ? m : a.M - 1) * a.ldc + nw;
#pragma unroll
    for (int q2 = 0; q2 < 3; ++q2) {  // column groups (0,1) (2,3) (4,5): 16-byte stores after the pair swap
      const u32x4_t wv = pair_swap16(w[2 * q2], w[2 * q2 + 1]);
      if (ok) *(u32x4_t*)(row + q2 * 32 + pair_col(g)) = wv;
    }
    if (ok) *(u32x2_t*)(row + 96 + g * 4) = w[6];  // group 6: 8-byte store
    if (a.ssq_out) {  // uniform branch: every lane takes part in the shuffles
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (ok && g == 0) a.ssq_out[(size_t)m * P + nw / 112] = ss;
    }
  }
}

// ---- four-wave persistent GEMM: 128 x (BN/2) wave tiles, one wave per SIMD ------------------------------------
// Four waves (2 x 2) per 256 x BN tile (BN = 256, or 224 for the N = 896 residual GEMMs), each owning a 128 x BN/2
// block = 8 x NJ v_mfma_f32_16x16x32_bf16 accumulators (NJ = BN/32: 256 / 224 AGPRs, the accumulator half of the
// 512-entry unified register file of a one-wave-per-SIMD kernel; see MFMA_AGPR).  Per 32-wide K-half a wave reads
// 8 A + NJ B fragments for 8 NJ MFMAs - about half the LDS reads per MFMA of the eight-wave 128x64 / 64x112 wave
// tiles - and no partner wave shares its SIMD's matrix pipe.  K-tiles of BK = 64 (full 128-byte LDS rows, the
// swizzled 128-byte-row image), double-buffered (2 x (32 + BN/8) KiB); fragments double-buffered in registers (X = K-half
// 0, Y = K-half 1).  Per K-tile t (buffer t & 1):
//   M(t,0): 8 NJ MFMAs on X, interleaved with the ds_reads of K-half 1 into Y
//   lgkmcnt(0) (Y landed), vmcnt(0) (K-tile t+1's DMA, issued during M(t-1,1), landed), ONE barrier
//   M(t,1): 8 NJ MFMAs on Y, interleaved with the 8 + NJ glds of K-tile t+2 into buffer t & 1 (every wave's reads
//           of it retired before the barrier) and the ds_reads of K-tile t+1's K-half 0 into X
// so each DMA has two K-halves to land.  The K-tile stream runs through all of the workgroup's tiles (persistent,
// grid-strided walk); a tile's epilogue runs after its last M(t,1), one 64-row quarter / half at a time with the
// shared epilogues (gemm_epilogue for BN = 256 as a 4 x 4 layout of 64 x 64 slabs, w7_epilogue for BN = 224 as
// 4 x 2 slabs of 64 x 112).
namespace w4 {
template <int BN> struct Geo {
  static constexpr int NJ = BN / 32;                    // wave column groups of 16
  static constexpr int NB = BN / 32;                    // B glds blocks per wave per K-tile (BN/8 blocks of 1 KiB)
  static constexpr int BOFF = 32768, TB = 32768 + BN * 128;   // B tile offset, K-tile buffer bytes
  static constexpr int NR = 8 + NJ;                     // fragment reads (and glds) per wave per K-half (K-tile)
  static constexpr int MF = 8 * NJ;                     // MFMAs per wave per K-half
  static constexpr int LDS = 2 * TB;
  // R3 (paired-B h3 GEMMs): three A slots of 32 KiB in a ring, then the two pair B regions - a K-tile's DMA spread
  // over both K-halves (96 KiB + 2 x BN/8 KiB <= 160 KiB for BN <= 256)
  static constexpr int LDS_R3 = 3 * 32768 + 2 * BN * 128;
};
// position (MFMA index) after which work item r of NR is issued: evenly spread over the MF MFMAs
template <int MF, int NR>
__device__ constexpr int slot_pos(int r) { return (r + 1) * MF / NR - 1; }
}  // namespace w4

// ---- 256 x 192 QKV tiles (fp32 mode, N = 1152 = 6 x 192: 768 tiles = exactly 3 rounds of the 256 CUs, where 256-wide
// tiles give 4.5 column tiles, a half-empty fifth and 2.5 rounds).  A wave's 96-column slab is 1.5 heads, so the
// tile's weight rows are loaded permuted: 16-row blocks 1 and 2 of every head swapped (q192_feat), which puts each
// RoPE pair of blocks - dims [0,16) with [32,48), [16,32) with [48,64) - into adjacent MFMA column groups (2p, 2p+1):
// the rotation partner of a lane's value is in the same lane, and no pair straddles the two waves.
__device__ __forceinline__ int q192_feat(int col) {   // tile column (permuted order) -> weight output feature
  const int q = (col >> 4) & 3;
  return (col & ~63) | ((q == 1 ? 2 : q == 2 ? 1 : q) << 4) | (col & 15);
}

// c: the virtual wave vw's 64 x 96 slab (rows m0 + vw 64 + i 16 + (lane & 15), columns nw + j 16 + 4 g + r); RH = 32
// (full 64-dim rotary: pair offset 32) or 0 (no rotary)
// bias of the wave's 96 columns (permuted order), loaded once per tile for both 64-row halves: the second half's
// reload came after the first half's stores, and waiting for it drained them (bench-shape probe 158.5-161.9 us against
// 162.5-165.8, same box; docs/RESULTS.md section 6)
__device__ __forceinline__ void qkv192_bias(const GemmArgs& a, int n0, int lane, int wn, f32x4_t (&bw)[6]) {
  const int nw = n0 + wn * 96;
#pragma unroll
  for (int j = 0; j < 6; ++j) bw[j] = *(const f32x4_t*)(a.biasf + q192_feat(nw + j * 16) + (lane >> 4) * 4);
}

template <int RH>
__device__ __forceinline__ void qkv192_epilogue(const GemmArgs& a, f32x4_t (&c)[4][6], const f32x4_t (&bw)[6], int m0,
                                                int n0, int lane, int vw, int wn) {
  static_assert(RH == 0 || RH == 32, "192-wide QKV tiles: full rotary or none");
  const int g = lane >> 4;
  const int nw = n0 + wn * 96;
  // every global load of the epilogue (bias - by the caller, before the first half - and the RoPE tables of all four
  // row groups for both low-half dim groups 4g and 16 + 4g) is issued before the first store: vmcnt counts stores
  // too, so a load waited between two groups' stores would drain them
  int bi[4], pi[4];
  f32x4_t cs[4][2], sn[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = min(m0 + vw * 64 + i * 16 + (lane & 15), a.M - 1);
    bi[i] = m / a.S;
    pi[i] = m - bi[i] * a.S;
    if constexpr (RH == 32) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        cs[i][hf] = *(const f32x4_t*)(a.cosT + pi[i] * 32 + hf * 16 + g * 4);
        sn[i][hf] = *(const f32x4_t*)(a.sinT + pi[i] * 32 + hf * 16 + g * 4);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + vw * 64 + i * 16 + (lane & 15);
    if (m >= a.M) continue;
    const int b = bi[i], pos = pi[i];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int col = nw + 32 * p;                       // block 2p: q = 0 or 2 of its head
      const int head = col >> 6;                         // wave-uniform
      const int hf = ((col >> 4) & 3) ? 1 : 0;           // low-half dims d .. d+3 (d = 16 hf + 4g), partners d+32
      const int d = hf * 16 + g * 4;
      f32x4_t lo = c[i][2 * p] * a.alpha + bw[2 * p];
      f32x4_t hi = c[i][2 * p + 1] * a.alpha + bw[2 * p + 1];
      const bool is_v = head >= a.Hq + a.Hkv;
      if (!is_v) {
        if constexpr (RH == 32) {
          const f32x4_t cv = hf ? cs[i][1] : cs[i][0], sv = hf ? sn[i][1] : sn[i][0];
          const f32x4_t l2 = lo * cv - hi * sv;
          hi = hi * cv + lo * sv;
          lo = l2;
        }
        const float sc = head < a.Hq ? a.q_scale : 1.f;
        float* dst = head < a.Hq ? a.qf + (((size_t)b * a.Hq + head) * a.S + pos) * 64
                                 : a.kf + (((size_t)b * a.Hkv + (head - a.Hq)) * a.S + pos) * 64;
        if (head < a.Hq || a.kf) {   // (fp32 K skipped when only its planes are wanted: head is wave-uniform)
          *(f32x4_t*)(dst + d) = lo * sc;
          *(f32x4_t*)(dst + d + 32) = hi * sc;
        }
        if (head >= a.Hq && a.kp) {
          const float l4[4] = {lo[0], lo[1], lo[2], lo[3]}, h4[4] = {hi[0], hi[1], hi[2], hi[3]};
          store_k_planes4(a, b, head - a.Hq, pos, d, l4);
          store_k_planes4(a, b, head - a.Hq, pos, d + 32, h4);
        }
      } else {
        if (a.vf) {
          float* dst = a.vf + (((size_t)b * a.Hkv + (head - a.Hq - a.Hkv)) * a.S + pos) * 64;
          *(f32x4_t*)(dst + d) = lo;
          *(f32x4_t*)(dst + d + 32) = hi;
        }
        if (a.vtf) {
          float* dst = a.vtf + ((size_t)b * a.Hkv + (head - a.Hq - a.Hkv)) * 64 * (size_t)a.s_pad + pos;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dst[(size_t)(d + r) * a.s_pad] = lo[r];
            dst[(size_t)(d + 32 + r) * a.s_pad] = hi[r];
          }
        }
        if (a.vp) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            store_vt_plane1(a, b, head - a.Hq - a.Hkv, pos, d + r, lo[r]);
            store_vt_plane1(a, b, head - a.Hq - a.Hkv, pos, d + 32 + r, hi[r]);
          }
        }
      }
    }
  }
}

// bf16 QKV on the 256 x 192 tiles: the same permuted column order and RoPE pairing as qkv192_epilogue, with the fused
// RMSNorm's row scale rq (from the producer's sum-of-squares partials), the bf16 bias, and the bf16 outputs of the
// 128 x 128 EPI_QKV_ROPE epilogue: q (scaled) / k [B, H, S, 64], V^T [B, Hkv, 64, s_pad] (2-byte stores: the LDS
// holds the next tile's staging here).
template <int RH>
__device__ __forceinline__ void qkv192_bf16_epilogue(const GemmArgs& a, f32x4_t (&c)[4][6], const float (&rq)[4],
                                                     int m0, int n0, int lane, int vw, int wn) {
  static_assert(RH == 0 || RH == 32, "192-wide QKV tiles: full rotary or none");
  const int g = lane >> 4;
  const int nw = n0 + wn * 96;
  u32x2_t bw[6];   // all the epilogue's loads before the first store (vmcnt counts stores too)
#pragma unroll
  for (int j = 0; j < 6; ++j) bw[j] = *(const u32x2_t*)(a.bias + q192_feat(nw + j * 16) + g * 4);
  int bi[4], pi[4];
  f32x4_t cs[4][2], sn[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = min(m0 + vw * 64 + i * 16 + (lane & 15), a.M - 1);
    bi[i] = m / a.S;
    pi[i] = m - bi[i] * a.S;
    if constexpr (RH == 32) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        cs[i][hf] = *(const f32x4_t*)(a.cosT + pi[i] * 32 + hf * 16 + g * 4);
        sn[i][hf] = *(const f32x4_t*)(a.sinT + pi[i] * 32 + hf * 16 + g * 4);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + vw * 64 + i * 16 + (lane & 15);
    if (m >= a.M) continue;
    const int b = bi[i], pos = pi[i];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int col = nw + 32 * p;                       // block 2p: q = 0 or 2 of its head
      const int head = col >> 6;                         // wave-uniform
      const int hf = ((col >> 4) & 3) ? 1 : 0;           // low-half dims d .. d+3 (d = 16 hf + 4g), partners d+32
      const int d = hf * 16 + g * 4;
      const u32x2_t bl = bw[2 * p], bh = bw[2 * p + 1];
      f32x4_t lo = c[i][2 * p] * rq[i] + f32x4_t{bf_lo(bl[0]), bf_hi(bl[0]), bf_lo(bl[1]), bf_hi(bl[1])};
      f32x4_t hi = c[i][2 * p + 1] * rq[i] + f32x4_t{bf_lo(bh[0]), bf_hi(bh[0]), bf_lo(bh[1]), bf_hi(bh[1])};
      if (head < a.Hq + a.Hkv) {
        if constexpr (RH == 32) {
          const f32x4_t cv = hf ? cs[i][1] : cs[i][0], sv = hf ? sn[i][1] : sn[i][0];
          const f32x4_t l2 = lo * cv - hi * sv;
          hi = hi * cv + lo * sv;
          lo = l2;
        }
        const float sc = head < a.Hq ? a.q_scale : 1.f;
        bf16_t* dst = head < a.Hq ? a.qout + (((size_t)b * a.Hq + head) * a.S + pos) * 64
                                  : a.kout + (((size_t)b * a.Hkv + (head - a.Hq)) * a.S + pos) * 64;
        *(u32x2_t*)(dst + d) = u32x2_t{pack_bf2(lo[0] * sc, lo[1] * sc), pack_bf2(lo[2] * sc, lo[3] * sc)};
        *(u32x2_t*)(dst + d + 32) = u32x2_t{pack_bf2(hi[0] * sc, hi[1] * sc), pack_bf2(hi[2] * sc, hi[3] * sc)};
      } else {
        bf16_t* dst = a.vtout + ((size_t)b * a.Hkv + (head - a.Hq - a.Hkv)) * 64 * (size_t)a.s_pad + pos;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dst[(size_t)(d + r) * a.s_pad] = f2bf(lo[r]);
          dst[(size_t)(d + 32 + r) * a.s_pad] = f2bf(hi[r]);
        }
      }
    }
  }
}

// fp32-output epilogue of the four-wave 256x224 kernel (O-projection / down + fp32 residual): the wave's 128 x 112
// block in four pairs of 16-row groups, the residual (and row-scale) loads running two pairs ahead of the stores.
// (vmcnt counts stores too: with each pair's loads issued after the previous pair's stores, every wait drained those
// stores and the epilogue was four serial memory round trips per tile - 37 % of the O-projection's time.)
// Reads the accumulators in place (C may alias the residual: a pair's loads are rows no earlier store wrote).
template <int EPI>
__device__ __forceinline__ void w4_f32_epilogue_224(const GemmArgs& a, f32x4_t (&acc)[8][7], int m0, int n0,
                                                    int lane, int wm, int wn) {
  constexpr bool NP = EPI == EPI_F32_RESID_NP;
  constexpr bool RESF = EPI == EPI_F32_RESID || EPI == EPI_F32_BIAS_RESID || EPI == EPI_F32_RESID_CS || NP;
  constexpr bool BIAS = EPI == EPI_F32_BIAS || EPI == EPI_F32_BIAS_RESID;
  constexpr bool CS = EPI == EPI_F32_RESID_CS;
  const int g = lane >> 4;
  const int nw = n0 + wn * 112;
  const int rbase = m0 + wm * 128 + (lane & 15);
  f32x4_t bw[BIAS || CS || NP ? 7 : 1];   // bias, or the column scales / the next norm's weight (never both)
  if constexpr (BIAS) {
#pragma unroll
    for (int j = 0; j < 7; ++j) bw[j] = *(const f32x4_t*)(a.biasf + nw + j * 16 + g * 4);
  }
  if constexpr (CS || NP) {
#pragma unroll
    for (int j = 0; j < 7; ++j) bw[j] = *(const f32x4_t*)(a.colscale + nw + j * 16 + g * 4);
  }
  f32x4_t rv[2][2][RESF ? 7 : 1];
  float rsv[2][2], psv[2][2];
  auto load = [&](int pr, int buf) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
      const int mr = min(rbase + (2 * pr + i2) * 16, a.M - 1);
      rsv[buf][i2] = (a.rscale ? a.rscale[mr] : 1.f) * a.alpha;
      if constexpr (CS) psv[buf][i2] = a.planes ? plane_scale(a, mr) : 0.f;
      if constexpr (NP) psv[buf][i2] = np_scale(a, mr);
      if constexpr (RESF) {
        const float* rrow = a.residf + (size_t)mr * a.ldr + nw + g * 4;
#pragma unroll
        for (int j = 0; j < 7; ++j) rv[buf][i2][j] = *(const f32x4_t*)(rrow + j * 16);
      }
    }
  };
  load(0, 0);
  load(1, 1);
#pragma unroll
  for (int pr = 0; pr < 4; ++pr) {
    const int buf = pr & 1;
    f32x4_t c[2][7];
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        c[i2][j] = acc[2 * pr + i2][j];
        asm volatile("" : "+v"(c[i2][j]));
      }
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
      const int m = rbase + (2 * pr + i2) * 16;
      float ss = 0.f;
      if (m < a.M) {
        float* row = a.Cf + (size_t)m * a.ldc + nw + g * 4;
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          f32x4_t o = c[i2][j] * rsv[buf][i2];
          if constexpr (CS) o *= bw[j];
          if constexpr (BIAS) o += bw[j];
          if constexpr (RESF) o += rv[buf][i2][j];
          *(f32x4_t*)(row + j * 16) = o;
          if constexpr (CS) {
            if (a.planes) {
              const float v4[4] = {o[0], o[1], o[2], o[3]};
              store_h3_4(a.planes + (size_t)m * (2 * a.N), a.N, nw + j * 16 + g * 4, v4, psv[buf][i2]);
            }
          }
          if constexpr (NP) {
            const f32x4_t n4 = o * bw[j];
            const float v4[4] = {n4[0], n4[1], n4[2], n4[3]};
            store_h3_4(a.planes + (size_t)m * (2 * a.N), a.N, nw + j * 16 + g * 4, v4, psv[buf][i2]);
            ss += o[0] * o[0] + o[1] * o[1] + o[2] * o[2] + o[3] * o[3];
          }
        }
        if constexpr (CS) {
          if (a.planes && nw == 0 && g == 0) a.prinv[m] = 1.f / psv[buf][i2];
        }
      }
      if constexpr (NP) {   // uniform: every lane takes part in the shuffles (the 4 lanes of a row: g = 0..3)
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        if (m < a.M && g == 0) {
          a.ssq_out[(size_t)m * (a.N / 112) + nw / 112] = ss;
          if (nw == 0) a.prinv[m] = 1.f / psv[buf][i2];
        }
      }
    }
    if (pr + 2 < 4) load(pr + 2, buf);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// PB (h3 two-product GEMMs, GemmArgs::pairb): the B tile of K-tile pair p (K-tiles 2p, 2p+1 = the two A planes
// against the same weight columns) lives in the B region of buffer p & 1 and is staged with the pair's even K-tile
// only - a quarter less L2 -> LDS traffic.  The K loop is unrolled by two so that every DMA / read switch stays
// compile-time (nk is even: pairs never straddle tiles).
//
// R3 (with PB): the A tiles live in a ring of three LDS slots (K-tile q in slot q mod 3) and the pair B tiles in two
// regions after them, which frees a slot one K-half earlier and lets the DMA be SPREAD over both K-halves instead of
// issued in one: M(u,0) stages K-tile u+2's 8 A pieces into slot (u+2) mod 3 (K-tile u-1's, whose last reads - K-half 1
// in M(u-1,0) - retired before ktile(u-1)'s barrier), M(u,1) its NB B pieces when u+2 is even (into the B region of
// pair (u+2)/2 = pair u/2 - 1's, last read in M(u-1,0) too) and advances the stream.  Per K-half at most 8 or NB pieces
// instead of 0 and 8+NB: an LDS-DMA piece costs its wave ~60 issue cycles among bare MFMAs and 100-185 in a K-half
// already carrying 8 pieces and 16 fragment reads (MI355X_MICROARCH constants).  Every wait before M(u,1) is vmcnt(8):
// K-tile u+1's last piece was issued before M(u,0)'s 8.  The prologue is PB's (K-tile 0, K-tile 1's A, vmcnt(8)).
// RING: 0 the two buffers, 1 R3, 2 the two buffers with the B pieces spread (PB): the B region of pair t/2 + 1 (t
// even) is pair t/2 - 1's, last read in M(t-1,0), so M(t,0) stages K-tile t+2's NB B pieces and M(t,1) its 8 A pieces
// (per K-half NB, 8, 0, 8 instead of 0, 8+NB, 0, 8; no extra LDS); the wait before M(t,1) is vmcnt(NB), before
// M(t+1,1) vmcnt(0).
//
// Stores after an epilogue (GemmArgs::store_wait): vmcnt counts stores, and retires in issue order, so the first wait
// of the next tile - for the K-tile whose DMA M(t,1) issued just before the epilogue - also drained the whole
// epilogue's stores.  epi_tail_stores<EPI, BN>() is a lower bound on the vector-memory ops every wave issues after the
// last of its epilogue's own waits, when the tile is full (no guarded row skips a store): vmcnt(that + the DMA
// issued after K-tile t+1) still retires K-tile t+1's DMA and leaves those stores in flight.
//   SwiGLU 256x256 (swiglu_h3_lines_4w): no loads; 8 row groups x 4 line stores = 32.
//   fp32 256x224 (w4_f32_epilogue_224): row pair 3's residual loads are issued after pair 1's stores and waited for
//   before pair 3 computes; pairs 2 and 3 store 2 x 2 x 7 = 28 after that wait.
template <int EPI, int BN>
__device__ constexpr int epi_tail_stores() {
  if constexpr (BN == 256 && EPI == EPI_H3_SWIGLU) return 32;
  else if constexpr (BN == 224 && epi_f32(EPI)) return 28;
  else return 0;
}
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

template <int EPI, int RH, int BN, bool PB = false, int RING = 0>
__global__ __launch_bounds__(256, 1) void gemm_4w_kernel(GemmArgs a) {
  static_assert(!PB || epi_f32(EPI), "paired B: h3 GEMMs");
  static_assert(RING == 0 || PB, "spread DMA schedules: paired-B GEMMs");
  constexpr bool R3 = RING == 1, SP2 = RING == 2;
  static_assert(BN != 192 || ((EPI == EPI_F32_QKV_ROPE || EPI == EPI_QKV_ROPE) && (RH == 0 || RH == 32)),
                "192-wide tiles: QKV only");
  static_assert(BN == 192 || BN == 224 || BN == 256, "tile width");
  using Gm = w4::Geo<BN>;
  constexpr int NJ = Gm::NJ, NB = Gm::NB, BOFF = Gm::BOFF, TB = Gm::TB, NR = Gm::NR, MF = Gm::MF;
  // LDS geometry: A tile of K-tile q at aslot(q); B tiles at BREG + region * BSTRIDE (PB: region = pair parity)
  constexpr int BREG = R3 ? 3 * 32768 : BOFF, BSTRIDE = R3 ? BN * 128 : TB;
  auto aslot = [](int q) -> uint32_t { return R3 ? (uint32_t)(q % 3) * 32768u : (uint32_t)(q & 1) * TB; };
  using CQ = Cfg<256, 256, 4, 4>;   // BN = 256 epilogue view: 64x64 slabs
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tm = (a.M + 255) / 256, tn = (a.N + BN - 1) / BN, ntiles = tm * tn;
  // strided walk (a.walk 0): at any time the whole chip works on ~256 consecutive grouped-M tiles, so every XCD
  // shares the same 8 A panels through the Infinity Cache (the per-XCD chunked walk was 3-8 % slower on the
  // M = 32768 shapes); the QKV GEMMs walk XCD-chunked (a.walk 1)
  const TileWalk walk = tile_walk(blockIdx.x, gridDim.x, ntiles, a.walk);

  const int tile0 = walk.first, G = walk.stride;
  if (tile0 >= walk.end) return;
  const int nk = a.K / 64;
  const int ntw = (walk.end - 1 - tile0) / G + 1;   // tiles of this workgroup
  const int total = ntw * nk;                       // K-tiles of this workgroup

  // ---- DMA: wave w stages 1-KiB blocks w, w+4, ... of each operand tile (8 rows of 128 B each)
  const char* sa = nullptr;
  const char* sb = nullptr;
  uint32_t oa[8], ob[NB];
  auto set_stage_tile = [&](int t) {
    int m0, n0;
    tile_origin(t, a.M, a.N, 256, BN, m0, n0);
    sa = (const char*)(a.A + (size_t)m0 * a.lda);
    sb = (const char*)(a.B + (size_t)n0 * a.ldb);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = (i * 4 + wave) * 8 + (lane >> 3);
      oa[i] = (uint32_t)(min(r, a.M - 1 - m0) * a.lda + ((lane & 7) ^ swz(r)) * 8) * 2u;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int r = (i * 4 + wave) * 8 + (lane >> 3);
      // 192-wide QKV tiles (head-aligned n0): LDS row r holds weight row q192_feat(n0 + r)
      const int rb = BN == 192 ? q192_feat(n0 + r) - n0 : r;
      ob[i] = (uint32_t)(min(rb, a.N - 1 - n0) * a.ldb + ((lane & 7) ^ swz(r)) * 8) * 2u;
    }
  };
  int st_q = 0, st_kt = 0, st_tile = tile0;
  set_stage_tile(st_tile);
  // item r < 8: A block, else B block r - 8 (with PB into the K-tile pair's slot; its callers skip the B items of
  // odd K-tiles at compile time)
  auto dma_item = [&](int r, char* buf, int kba, int kb) {
    if (r < 8) {
      glds16(sa + kba + oa[r], buf + (r * 4 + wave) * 1024);
    } else {
      char* bbuf = PB ? smem + BREG + ((st_q >> 1) & 1) * BSTRIDE : buf + BOFF;
      glds16(sb + kb + ob[r - 8], bbuf + ((r - 8) * 4 + wave) * 1024);
    }
  };
  // byte offsets of the stream K-tile's A and B columns (h3 operands: the plane remap / pair mapping, computed once per
  // K-tile where the wave waits anyway, not on the MFMA issue path)
  int st_kba = a_kcol(a, 0) * 2, st_kb = 0;
  auto advance_stage = [&]() {   // the DMA stream stops (repeats its last K-tile) at the end
    ++st_q;
    if (st_q >= total) {
      st_kt = nk - 1;
    } else if (++st_kt == nk) {
      st_kt = 0;
      st_tile += G;
      set_stage_tile(st_tile);
    }
    st_kba = a_kcol(a, st_kt * 64) * 2;
    st_kb = b_kcol(a, st_kt * 64) * 2;
  };
  auto stage_all = [&](auto with_b) {
    char* buf = smem + aslot(st_q);
    const int kb = st_kb, kba = st_kba;
#pragma unroll
    for (int r = 0; r < (decltype(with_b)::value ? NR : 8); ++r) dma_item(r, buf, kba, kb);
    advance_stage();
  };

  // ---- fragments
  const int sw = ((lane & 15) >> 1) & 7;
  uint32_t abase[2], bbase[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int c = ks * 4 + (lane >> 4);
    abase[ks] = lds_addr(smem) + (wm * 128 + (lane & 15)) * 128 + ((c ^ sw) << 4);
    bbase[ks] = lds_addr(smem) + BREG + (wn * (BN / 2) + (lane & 15)) * 128 + ((c ^ sw) << 4);
  }
  bf16x8_t XA[8], XB[NJ], YA[8], YB[NJ];
  f32x4_t acc[8][NJ];

  // 8 NJ MFMAs on (FA, FB) with the NR fragment reads of K-half ks of buffer bo into (GA, GB) and, with DMA, the NR
  // glds of the stream's next K-tile spread evenly between them.  The switches are compile-time (runtime-predicated
  // asm register writes make the allocator spill the fragments); first_c: the tile's first MFMAs start from zero.
  // dm_c: 0 no DMA; 1 the stream K-tile's A pieces and, with dmab, its B pieces, then advance; 2 (R3) its A pieces
  // only, spread over the NR work items; 3 (R3) its B pieces (with dmab) spread, then advance; 4 (SP2) its B pieces
  // (with dmab) spread; 5 (SP2) its A pieces spread, then advance
  auto mma = [&](const bf16x8_t(&FA)[8], const bf16x8_t(&FB)[NJ], bf16x8_t(&GA)[8], bf16x8_t(&GB)[NJ], uint32_t bo,
                 uint32_t boB, int ks, auto first_c, auto dm_c, auto read_c, auto dmab_c) {
    constexpr bool first = decltype(first_c)::value;
    constexpr int dm = decltype(dm_c)::value;
    constexpr bool read_on = decltype(read_c)::value, dma_b = decltype(dmab_c)::value;
    const uint32_t va = abase[ks] + bo, vb = bbase[ks] + boB;
    char* dbuf = smem + aslot(st_q);
    const int kb = st_kb, kba = st_kba;
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      // MFMAs slot_pos(rr-1)+1 .. slot_pos(rr), then work item rr
#pragma unroll
      for (int n = (rr == 0 ? 0 : w4::slot_pos<MF, NR>(rr - 1) + 1); n <= w4::slot_pos<MF, NR>(rr); ++n) {
        const int i = n / NJ, j = n % NJ;
        if constexpr (epi_f32(EPI)) {
          if constexpr (first) MFMA_AGPR_FIRST_H(acc[i][j], FB[j], FA[i]);
          else MFMA_AGPR_H(acc[i][j], FB[j], FA[i]);
        } else {
          if constexpr (first) MFMA_AGPR_FIRST(acc[i][j], FB[j], FA[i]);
          else MFMA_AGPR(acc[i][j], FB[j], FA[i]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (read_on) {
        if (rr < 8) DS_READ_B128(GA[rr], va, rr * 2048);
        else DS_READ_B128(GB[rr - 8], vb, (rr - 8) * 2048);
      }
      // rr is a compile-time index of the unrolled loop; spread pieces: piece floor(rr n / NR) at the rr where it steps
      if constexpr (dm == 1) {
        if (rr < 8 || dma_b) dma_item(rr, dbuf, kba, kb);
      } else if constexpr (dm == 2 || dm == 5) {
        if ((rr * 8) % NR < 8) dma_item(rr * 8 / NR, dbuf, kba, kb);
      } else if constexpr (dm == 3 || dm == 4) {
        if (dma_b && (rr * NB) % NR < NB) dma_item(8 + rr * NB / NR, dbuf, kba, kb);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (dm == 1 || dm == 3 || dm == 5) advance_stage();
  };

  // prologue: K-tiles 0 and 1 in flight, K-tile 0 landed and visible, its K-half 0 fragments in X
  stage_all(std::true_type{});
  if (total > 1) {
    stage_all(std::integral_constant<bool, !PB>{});
    if constexpr (PB) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // K-tile 1 staged its 8 A blocks only
    else if constexpr (NR == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (NR == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) DS_READ_B128(XA[i], abase[0], i * 2048);
#pragma unroll
  for (int j = 0; j < NJ; ++j) DS_READ_B128(XB[j], bbase[0], j * 2048);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  int tile = tile0, kt = 0, m0, n0;
  bool epi_full = false;   // the previous tile's epilogue issued its epi_tail_stores (store_wait on, full tile)
  tile_origin(tile, a.M, a.N, 256, BN, m0, n0);
  float rs[8];
  auto load_rs = [&](int mt) {
    if constexpr (BN == 256 || BN == 192) {
      if constexpr (EPI == EPI_QKV_ROPE) {
        if (a.ssq_in) {   // fused RMSNorm from the producer's sum-of-squares partials (the bf16 QKV GEMM)
          if (a.ssq_parts == 8) rscale_from_partials<8, 128, 8>(a, mt, wm, lane, rs);
          else rscale_from_partials<8, 128, 14>(a, mt, wm, lane, rs);
          return;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = min(mt + wm * 128 + i * 16 + (lane & 15), a.M - 1);
        rs[i] = a.rscale ? a.rscale[m] : 1.f;
      }
    }
  };
  load_rs(m0);
  // K-tile t of the stream; dmab_c: the DMA issued in M(t,1) (K-tile t + 2) includes the B tile; end_c: K-tile t
  // may be its tile's last (with PB only odd K-tiles can be)
  auto ktile = [&](int t, auto dmab_c, auto end_c) {
    const uint32_t bo = aslot(t), bn = aslot(t + 1);
    const uint32_t boB = PB ? ((t >> 1) & 1) * BSTRIDE : bo, bnB = PB ? (((t + 1) >> 1) & 1) * BSTRIDE : bn;
    // M(t,0) on X, K-half 1 of K-tile t -> Y
    __builtin_amdgcn_sched_barrier(0);
    // R3: K-tile t+2's A pieces; SP2: its B pieces (t even)
    using DM0 = std::integral_constant<int, R3 ? 2 : (SP2 && decltype(dmab_c)::value) ? 4 : 0>;
    if (kt == 0) mma(XA, XB, YA, YB, bo, boB, 1, std::true_type{}, DM0{}, std::true_type{}, dmab_c);
    else mma(XA, XB, YA, YB, bo, boB, 1, std::false_type{}, DM0{}, std::true_type{}, dmab_c);
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < total) {
      // K-tile t+1 landed (R3: K-tile t+2's 8 A pieces, issued in M(t,0), may stay in flight).  After a full tile's
      // epilogue its last TS stores may too (issued after M(t-1,1)'s DMA; with R3 they precede M(t,0)'s, so R3 waits
      // for them)
      constexpr int N0 = R3 ? 8 : (SP2 && decltype(dmab_c)::value) ? NB : 0;   // SP2: M(t,0)'s B pieces
      constexpr int TS = epi_tail_stores<EPI, BN>();
      if constexpr (TS > 0 && RING == 0) {
        if (kt == 0 && epi_full) wait_vm_lgkm0<N0 + TS>();
        else wait_vm_lgkm0<N0>();
      } else {
        wait_vm_lgkm0<N0>();
      }
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if constexpr ((BN == 256 || BN == 192) && (RING == 0 || (SP2 && !decltype(dmab_c)::value))) {
      // The row scales load_rs issued at the tile's start are older than the DMA the wait above leaves in flight, so
      // they have landed: hand them to the compiler as fresh values on every path here.  Otherwise its own wait for
      // them sits at their first use in the epilogue, as vmcnt(0), and also drains the DMA issued just before it.
      // (The compiler puts its own vmcnt(0) before these asm statements on the first K-tile after load_rs: only where
      // the wait above is vmcnt(0) anyway - two buffers, SP2's odd K-tiles; with store_wait it voids vmcnt(TS).)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(rs[i]));
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // M(t,1) on Y, K-tile t+2 -> buffer t & 1 (R3: its B pieces), K-half 0 of K-tile t+1 -> X.  Unconditional: past
    // the end of the stream the DMA re-reads the last K-tile into a buffer nobody reads again and X gets values nobody
    // consumes.
    // (A runtime switch between read / no-read copies of this loop makes the allocator spill the fragments.)
    mma(YA, YB, XA, XB, bn, bnB, 0, std::false_type{}, std::integral_constant<int, R3 ? 3 : SP2 ? 5 : 1>{},
        std::true_type{}, dmab_c);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ++kt;
    if (decltype(end_c)::value && kt == nk) {
      // all MFMAs of the tile were issued; the epilogue reads the accumulators after they drain
      MFMA_DRAIN();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (BN == 256 && EPI == EPI_H3_SWIGLU) {
        swiglu_h3_lines_4w<8>(a, acc, rs, m0, n0, lane, wm, wn);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (BN == 256 && EPI == EPI_H3_LRP_SWIGLU) {
        lrp_swiglu_4w(a, acc, m0, n0, lane, wm, wn);
        __builtin_amdgcn_sched_barrier(0);
      } else if constexpr (BN == 256) {
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          // one 64x64 slab at a time (row half ih, column half h), as virtual wave (2 wm + ih, 2 wn + h) of a 4x4
          // layout: its accumulators are copied to VGPRs here (the scheduler would otherwise hoist all the reads)
          const int ih = qd >> 1, h = qd & 1;
          f32x4_t c[4][4];
          float rq[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            rq[i] = rs[ih * 4 + i];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              c[i][j] = acc[ih * 4 + i][h * 4 + j];
              asm volatile("" : "+v"(c[i][j]));
            }
          }
          if (n0 + wn * 128 + h * 64 < a.N) gemm_epilogue<EPI, RH, CQ>(a, c, m0, n0, lane, wm * 2 + ih, wn * 2 + h, rq);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else if constexpr (BN == 192) {
        f32x4_t bw[6];
        if constexpr (EPI != EPI_QKV_ROPE) qkv192_bias(a, n0, lane, wn, bw);
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {   // 64 x 96 halves
          f32x4_t c[4][6];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
              c[i][j] = acc[ih * 4 + i][j];
              asm volatile("" : "+v"(c[i][j]));
            }
          if constexpr (EPI == EPI_QKV_ROPE) {
            const float rq[4] = {rs[ih * 4], rs[ih * 4 + 1], rs[ih * 4 + 2], rs[ih * 4 + 3]};
            qkv192_bf16_epilogue<RH>(a, c, rq, m0, n0, lane, wm * 2 + ih, wn);
          } else {
            qkv192_epilogue<RH>(a, c, bw, m0, n0, lane, wm * 2 + ih, wn);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      } else if constexpr (epi_f32(EPI)) {
        w4_f32_epilogue_224<EPI>(a, acc, m0, n0, lane, wm, wn);
        __builtin_amdgcn_sched_barrier(0);
      } else {
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {   // 64 x 112 halves as virtual waves (2 wm + ih, wn) of the W7 layout
          f32x4_t c[4][NJ];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              c[i][j] = acc[ih * 4 + i][j];
              asm volatile("" : "+v"(c[i][j]));
            }
          w7_epilogue<EPI>(a, c, m0, n0, lane, wm * 2 + ih, wn);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      epi_full = a.store_wait && m0 + 256 <= a.M && n0 + BN <= a.N;
      tile += G;
      kt = 0;
      if (tile < walk.end) {
        tile_origin(tile, a.M, a.N, 256, BN, m0, n0);
        load_rs(m0);
      }
      // the next tile's first K-half fragments again (K-tile t+1 landed in buffer bn before this K-tile's barrier):
      // re-reading them here leaves the copies read during M(t,1) dead across the epilogue, which gets their VGPRs
#pragma unroll
      for (int i = 0; i < 8; ++i) DS_READ_B128(XA[i], abase[0] + bn, i * 2048);
#pragma unroll
      for (int j = 0; j < NJ; ++j) DS_READ_B128(XB[j], bbase[0] + bnB, j * 2048);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  };
#pragma unroll 1
  for (int t = 0; t < total; t += PB ? 2 : 1) {
    if constexpr (PB) {   // (R3: M(t,0) / M(t,1) stage K-tile t+2's A / B, M(t+1,0) K-tile t+3's A)
      ktile(t, std::true_type{}, std::false_type{});       // M(t,1) stages K-tile t+2 (even): A and the pair's B
      ktile(t + 1, std::false_type{}, std::true_type{});   // M(t+1,1) stages K-tile t+3 (odd): A only
    } else {
      ktile(t, std::true_type{}, std::true_type{});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

static int g_tile_override = 0;  // 0 automatic; 128, 192, 224 or 256 force a tile at any M (tests only)

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <int EPI, int RH, class CF>
static int launch_cfg(const GemmArgs& a, hipStream_t st) {
  const int grid = ((a.M + CF::BM - 1) / CF::BM) * ((a.N + CF::BN - 1) / CF::BN);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, RH, CF>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              CF::LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_bf16_kernel<EPI, RH, CF>), dim3(grid), dim3(CF::NT), CF::LDS, st, a);
  return (int)hipGetLastError();
}

// four-wave tile walk forced for every GEMM (A/B measurements): EDGE_GEMM_WALK=0 / 1, unset or -1 = by GEMM
static int g_walk_override = [] {
  const char* e = getenv("EDGE_GEMM_WALK");
  return (e && (e[0] == '0' || e[0] == '1')) ? e[0] - '0' : -1;
}();

// GemmArgs::store_wait for the four-wave kernels: EDGE_GEMM_STORE_WAIT (1 / 0) or edge_gemm_set_store_wait
static int g_store_wait = -1;
static int store_wait() {
  if (g_store_wait < 0) {
    const char* e = getenv("EDGE_GEMM_STORE_WAIT");
    g_store_wait = (e && e[0] && e[0] != '0') ? 1 : 0;
  }
  return g_store_wait;
}

// the persistent four-wave kernel: one workgroup per CU walks its tiles (walk 0 strided, 1 XCD-chunked)
template <int EPI, int RH, int BN, bool PB, int RING = 0>
static int launch_4w_pb(const GemmArgs& args, hipStream_t st, int walk) {
  GemmArgs a = args;
  a.walk = g_walk_override >= 0 ? g_walk_override : walk;
  a.store_wait = store_wait();
  const int tiles = ((a.M + 255) / 256) * ((a.N + BN - 1) / BN);
  const int grid = std::min(tiles, num_cus());
  constexpr int lds = RING == 1 ? w4::Geo<BN>::LDS_R3 : w4::Geo<BN>::LDS;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_4w_kernel<EPI, RH, BN, PB, RING>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_4w_kernel<EPI, RH, BN, PB, RING>), dim3(grid), dim3(256), lds, st, a);
  return (int)hipGetLastError();
}

// DMA schedule of the paired-B four-wave kernels per tile width (gemm_4w_kernel RING): three decimal digits for the
// 192- (QKV), 224- (O-projection / down) and 256-wide (gate/up, LM head) tiles, each 0 two buffers, 1 the three-slot
// ring (R3), 2 the two buffers with B spread (SP2).  EDGE_GEMM_RING or edge_gemm_set_ring; default 022 (SP2 on the
// O-projection / down and gate/up GEMMs: +1.0-1.2 % on the fp32 bench against 010, same box, 3 of 3 rounds; 010 was
// +0.5-0.7 % against 000; the QKV stays on two plain buffers - docs/RESULTS.md section 6)
static int g_ring = -1;
static int ring_mode(int bn) {
  if (g_ring < 0) {
    const char* e = getenv("EDGE_GEMM_RING");
    g_ring = 22;
    if (e && strlen(e) == 3 && strspn(e, "012") == 3) g_ring = atoi(e);
  }
  return (bn == 192 ? g_ring / 100 : bn == 224 ? g_ring / 10 : g_ring) % 10;
}

template <int EPI, int RH, int BN = 256>
static int launch_4w(const GemmArgs& a, hipStream_t st, int walk = 0) {
  if constexpr (epi_f32(EPI)) {
    if (a.pairb) {
      const int r = ring_mode(BN);
      if (r == 1) return launch_4w_pb<EPI, RH, BN, true, 1>(a, st, walk);
      if (r == 2) return launch_4w_pb<EPI, RH, BN, true, 2>(a, st, walk);
      return launch_4w_pb<EPI, RH, BN, true>(a, st, walk);
    }
  }
  return launch_4w_pb<EPI, RH, BN, false>(a, st, walk);
}

// The 256x224 tiles take the plain / bias / residual epilogues of N % 224 == 0 shapes that 256 does not divide (the
// Qwen2 hidden size 896 = 3.5 x 256 = 4 x 224: no half-empty column tile), when 256-row tiles fill the chip; tests
// force them at small M with tile override 224.
static bool use_224(int M, int N, int K, int epi) {
  if (!epi_plain(epi)) return false;
  if (N % 224 || N % 256 == 0 || K < 2 * BK) return false;
  if (g_tile_override) return g_tile_override == 224;
  return (long long)((M + 255) / 256) * (N / 224) >= 256;
}

// Kernel choice by shape: the persistent four-wave kernel (256 x 256 / 224 / 192 tiles) when its tiles fill the chip,
// the 128x128 kernel otherwise (small M, N not a multiple of the tile).
template <int EPI, int RH = 0>
static int launch(const GemmArgs& a, hipStream_t st) {
  if constexpr (epi_plain(EPI)) {
    if (use_224(a.M, a.N, a.K, EPI)) return launch_4w<EPI, 0, 224>(a, st);
  }
  if constexpr (EPI == EPI_QKV_ROPE || EPI == EPI_F32_QKV_ROPE) {
    // fp32-mode (h3) QKV: 256x192 tiles when 192 divides N and 256 does not (N = 1152: 768 tiles, three full rounds
    // of the chip), else 256x256 when they fill it; the XCD-chunked walk keeps an XCD's rounds inside one GROUP_M
    // band, re-using its A panels from L2 (h3 QKV at M = 32768: 144 vs 159 us strided, profiles/history/r02h_gemm_explore.log).
    // The bf16 QKV (K = 896, fused RMSNorm row scale) stays on 128x128 tiles unless a test forces a tile.
    const long long tiles = (long long)((a.M + 255) / 256) * ((a.N + 255) / 256);
    if constexpr (RH == 0 || RH == 32) {
      const long long t192 = (long long)((a.M + 255) / 256) * (a.N / 192);
      if (a.N % 192 == 0 && a.N % 256 &&
          (g_tile_override == 192 || (EPI == EPI_F32_QKV_ROPE && t192 >= 256 && !g_tile_override)))
        return launch_4w<EPI, RH, 192>(a, st, 1);
    }
    if (g_tile_override == 256 || (EPI == EPI_F32_QKV_ROPE && tiles >= 256 && !g_tile_override))
      return launch_4w<EPI, RH>(a, st, 1);
    return launch_cfg<EPI, RH, C128>(a, st);
  } else if constexpr (EPI == EPI_LSE || EPI == EPI_F32_LSE) {
    // LM head on the scored rows (M = 2048 at the bench batch, N = vocab): 256x256 persistent tiles when they fill
    // the chip (per-64-column LSE partials per quarter), else 128x128
    const bool big = a.N % 128 == 0 && (long long)((a.M + 255) / 256) * ((a.N + 255) / 256) >= 256;
    if (big && g_tile_override != 128) return launch_4w<EPI, RH>(a, st);
    return launch_cfg<EPI, RH, C128>(a, st);
  } else {
    // a partial last column tile (N % 256 == 128) wastes at most 1/(2*tn) of the MFMA work
    const int tn = (a.N + 255) / 256;
    const bool fits = a.N % 256 == 0 || (a.N % 128 == 0 && tn >= 4 && EPI != EPI_SWIGLU && EPI != EPI_H3_SWIGLU);
    const bool big = fits && ((long long)((a.M + 255) / 256) * tn >= 256);
    const bool use256 = g_tile_override ? g_tile_override == 256 && fits : big;
    if (!use256) return launch_cfg<EPI, RH, C128>(a, st);
    return launch_4w<EPI, RH>(a, st);
  }
}

EDGE_API int edge_gemm_set_tile(int t) {
  g_tile_override = t;
  return 0;
}

// the paired-B GEMMs' DMA schedules (ring_mode): code = 100 x (192 tiles) + 10 x (224) + (256), digits 0 / 1 / 2;
// -1: from EDGE_GEMM_RING
EDGE_API int edge_gemm_set_ring(int code) {
  const bool ok = code >= 0 && code / 100 <= 2 && code / 10 % 10 <= 2 && code % 10 <= 2;
  g_ring = ok ? code : -1;
  return 0;
}

// 1: the four-wave kernels leave a full tile's last epilogue stores in flight across the next tile's first wait
// (GemmArgs::store_wait), 0: that wait drains them; -1: from EDGE_GEMM_STORE_WAIT
EDGE_API int edge_gemm_set_store_wait(int on) {
  g_store_wait = on;
  return 0;
}

// Number of row sum-of-squares partials edge_gemm writes for this shape (ssq_out is [M, parts]): one per
// 64-column slab, or one per 112-column wave slab on the 256x224 kernel.  act/bias/resid as edge_gemm.
EDGE_API int edge_gemm_ssq_parts(int M, int N, int K, int act, int has_bias, int has_resid) {
  if (act) return N / 64;
  const int epi = has_bias ? (has_resid ? EPI_BIAS_RESID : EPI_BIAS) : (has_resid ? EPI_RESID : EPI_NONE);
  return use_224(M, N, K, epi) ? N / 112 : N / 64;
}

static int check_shapes(const GemmArgs& a) {
  if (a.M <= 0) return -1;
  if (a.N % 128 || a.K % BK || a.N <= 0 || a.K <= 0) return (int)hipErrorInvalidValue;
  if (a.lda % 8 || a.ldb % 8) return (int)hipErrorInvalidValue;
  return 0;
}

EDGE_API int edge_gemm(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       const void* bias, const void* resid, int ldr, int act, const float* rscale, float* ssq_out,
                       hipStream_t st) {
  GemmArgs a{};
  a.rscale = rscale; a.ssq_out = ssq_out;
  if (ssq_out && (N % 64 || act == 2)) return (int)hipErrorInvalidValue;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = (bf16_t*)C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.bias = (const bf16_t*)bias; a.resid = (const bf16_t*)resid; a.ldr = ldr;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  // the epilogues store 16-byte vectors (pair-swapped columns): 16-B aligned output rows
  if (ldc % 8 || ((uintptr_t)C & 15) || (resid && ldr % 4)) return (int)hipErrorInvalidValue;
  // act: 0 none, 1 gelu, 2 swiglu-interleaved
  if (act == 2) return bias || resid ? (int)hipErrorInvalidValue : launch<EPI_SWIGLU>(a, st);
  if (act == 1) return resid || !bias ? (int)hipErrorInvalidValue : launch<EPI_BIAS_GELU>(a, st);
  if (bias && resid) return launch<EPI_BIAS_RESID>(a, st);
  if (bias) return launch<EPI_BIAS>(a, st);
  if (resid) return launch<EPI_RESID>(a, st);
  return launch<EPI_NONE>(a, st);
}

// EPI_SWIGLU that also stores the (row-scaled) pre-activations raw [M, N] bf16, bit-identical to edge_gemm act 0
// (the bf16 AttnLRP forward saves them for the SwiGLU rule; one GEMM instead of a GEMM and a SwiGLU pass).
EDGE_API int edge_gemm_swiglu_raw(const void* A, const void* B, void* C, void* raw, int M, int N, int K, int lda,
                                  int ldb, int ldc, const float* rscale, hipStream_t st) {
  GemmArgs a{};
  a.rscale = rscale;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = (bf16_t*)C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.rawb = (bf16_t*)raw;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  if (!raw || ((uintptr_t)raw & 15) || ldc % 8 || ((uintptr_t)C & 15)) return (int)hipErrorInvalidValue;
  return launch<EPI_SWIGLU>(a, st);
}

EDGE_API int edge_gemm_qkv_rope(const void* X, const void* W, const void* bias, void* q, void* k, void* vt,
                                const float* cosT, const float* sinT, int M, int K, int S, int Hq, int Hkv,
                                int rot_dim, int s_pad, float q_scale, const float* rscale, const float* ssq_in,
                                int ssq_parts, float norm_eps, hipStream_t st) {
  GemmArgs a{};
  a.rscale = rscale;
  a.ssq_in = ssq_in; a.ssq_parts = ssq_parts; a.norm_inv_k = 1.f / (float)K; a.norm_eps = norm_eps;
  if (ssq_in && ssq_parts != 8 && ssq_parts != 14) return (int)hipErrorInvalidValue;
  if (ssq_in && ((uintptr_t)ssq_in & 15)) return (int)hipErrorInvalidValue;
  a.A = (const bf16_t*)X; a.B = (const bf16_t*)W;
  a.M = M; a.N = (Hq + 2 * Hkv) * 64; a.K = K; a.lda = K; a.ldb = K;
  a.bias = (const bf16_t*)bias;
  a.qout = (bf16_t*)q; a.kout = (bf16_t*)k; a.vtout = (bf16_t*)vt;
  a.cosT = cosT; a.sinT = sinT; a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.s_pad = s_pad;
  a.q_scale = q_scale;
  if (!bias || M % S) return (int)hipErrorInvalidValue;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  switch (rot_dim) {
    case 0: return launch<EPI_QKV_ROPE, 0>(a, st);
    case 8: return launch<EPI_QKV_ROPE, 4>(a, st);
    case 16: return launch<EPI_QKV_ROPE, 8>(a, st);
    case 32: return launch<EPI_QKV_ROPE, 16>(a, st);
    case 64: return launch<EPI_QKV_ROPE, 32>(a, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// h3 operand geometry: K' = Kx = terms x kplane, terms 3 (B' = [b_hi | b_lo | b_hi] [N, 3K]) or 2 (a weight exact in
// fp16, b_lo = 0 - e.g. a bf16 or fp16 checkpoint: B = b_hi [N, K] once, the K-tiles interleave A' = a_lo / a_hi
// against the same B tile, GemmArgs::pairb)
static bool h3_geometry_ok(int Kx, int kplane) {
  return kplane > 0 && kplane % BK == 0 && (Kx == 2 * kplane || Kx == 3 * kplane);
}

// fp32 execution (h3 operands, common.h): A a 2-plane h3 activation [M, 2K] (K = kplane, lda >= 2K), B the h3
// weight [N, Kx] with Kx = 3K (or 2K, h3_geometry_ok); alpha = 1 / (s_a s_b).  act 0 none -> fp32 C [M, ldc] (+ fp32 bias, + fp32
// residual, which may alias C); act 1 bias + GELU -> h3 output [M, 2N] in C (fp16 planes, ldc = 2N) at scale
// out_scale; act 2 interleaved SwiGLU -> h3 output [M, 2 (N/2)] (ldc = N).
EDGE_API int edge_gemm_f32(const void* A, const void* B, void* C, int M, int N, int Kx, int kplane, int lda, int ldb,
                           int ldc, const float* bias, const float* resid, int ldr, int act, const float* rscale,
                           float alpha, float out_scale, hipStream_t st) {
  GemmArgs a{};
  a.rscale = rscale;  // optional per-row scale of the product (before bias / activation / residual)
  a.alpha = alpha; a.out_scale = out_scale;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B;
  a.M = M; a.N = N; a.K = Kx; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.biasf = bias; a.residf = resid; a.ldr = ldr;
  a.h3k = kplane;   // A: 2-plane activation rows (lda >= 2 kplane)
  a.pairb = Kx == 2 * kplane;
  if (!h3_geometry_ok(Kx, kplane) || lda < 2 * kplane || ldb < (a.pairb ? kplane : Kx) || !(alpha > 0.f) ||
      !(out_scale > 0.f))
    return (int)hipErrorInvalidValue;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  if (((uintptr_t)C & 15) || ldc % 4 || (resid && (ldr % 4 || ((uintptr_t)resid & 15))) ||
      (bias && ((uintptr_t)bias & 15)))
    return (int)hipErrorInvalidValue;
  if (act == 2) {
    if (bias || resid || ldc != 2 * (N / 2)) return (int)hipErrorInvalidValue;
    a.C = (bf16_t*)C;
    return launch<EPI_H3_SWIGLU>(a, st);
  }
  if (act == 1) {
    if (resid || !bias || ldc != 2 * N) return (int)hipErrorInvalidValue;
    a.C = (bf16_t*)C;
    return launch<EPI_H3_BIAS_GELU>(a, st);
  }
  a.Cf = (float*)C;
  if (bias && resid) return launch<EPI_F32_BIAS_RESID>(a, st);
  if (bias) return launch<EPI_F32_BIAS>(a, st);
  if (resid) return launch<EPI_F32_RESID>(a, st);
  return launch<EPI_F32>(a, st);
}

// EPI_H3_SWIGLU that also stores the scaled pre-activations: raw = rscale[m] * alpha * (A . B^T) as fp32 [M, N]
// (what edge_gemm_f32 with act 0 returns, bit for bit) next to the SwiGLU h3 planes in C (as edge_gemm_f32 act 2).
EDGE_API int edge_gemm_f32_swiglu_raw(const void* A, const void* B, void* C, float* raw, int M, int N, int Kx,
                                      int kplane, int lda, int ldb, int ldc, const float* rscale, float alpha,
                                      float out_scale, hipStream_t st) {
  if (!raw || ((uintptr_t)raw & 15) || N % 16) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.rscale = rscale;
  a.alpha = alpha; a.out_scale = out_scale;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B;
  a.M = M; a.N = N; a.K = Kx; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.h3k = kplane;
  a.pairb = Kx == 2 * kplane;
  if (!h3_geometry_ok(Kx, kplane) || lda < 2 * kplane || ldb < (a.pairb ? kplane : Kx) || !(alpha > 0.f) ||
      !(out_scale > 0.f) || ldc != 2 * (N / 2) || ((uintptr_t)C & 15))
    return (int)hipErrorInvalidValue;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  a.C = (bf16_t*)C;
  a.raw = raw;
  return launch<EPI_H3_SWIGLU>(a, st);
}

// EPI_F32_RESID_CS: C = colscale[n] * rscale[m] * alpha * (A . B^T) + resid (h3 operands as edge_gemm_f32; C may
// alias resid).
// planes / prinv / bnd_a / bnd_b / bnd_c (all or none): C also as the h3 activation [M, 2N] at the bound-derived
// row scales (GemmArgs::planes).
EDGE_API int edge_gemm_f32_cs(const void* A, const void* B, float* C, int M, int N, int Kx, int kplane, int lda, int ldb,
                              int ldc, const float* colscale, const float* resid, int ldr, const float* rscale,
                              float alpha, void* planes, float* prinv, const float* bnd_a, const float* bnd_b,
                              float bnd_c, hipStream_t st) {
  GemmArgs a{};
  a.rscale = rscale;
  a.colscale = colscale;
  a.alpha = alpha;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B;
  a.M = M; a.N = N; a.K = Kx; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.residf = resid; a.ldr = ldr; a.Cf = C;
  a.h3k = kplane;
  a.pairb = Kx == 2 * kplane;
  a.planes = (f16_t*)planes; a.prinv = prinv; a.bnd_a = bnd_a; a.bnd_b = bnd_b; a.bnd_c = bnd_c;
  if (!colscale || !resid || !h3_geometry_ok(Kx, kplane) || lda < 2 * kplane || ldb < (a.pairb ? kplane : Kx) ||
      !(alpha > 0.f))
    return (int)hipErrorInvalidValue;
  if (planes && (!prinv || !bnd_a || !bnd_b || !(bnd_c >= 0.f) || ((uintptr_t)planes & 7)))
    return (int)hipErrorInvalidValue;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  if (((uintptr_t)C & 15) || ldc % 4 || ldr % 4 || ((uintptr_t)resid & 15) || ((uintptr_t)colscale & 15))
    return (int)hipErrorInvalidValue;
  return launch<EPI_F32_RESID_CS>(a, st);
}

// EPI_F32_RESID_NP (the O-projection / down GEMM with the next RMSNorm's producer side): C = alpha (A . B^T) + resid
// (fp32, C may alias resid), planes [M, 2N] = h3 of p_m (C_m * g) with p_m from the bound g_max (sqrt(N) / rstd_in[m] +
// prod_bound) on |C_m * g| (np_scale), prinv[m] = 1 / p_m, ssq_out [M, N / 112] the row sum-of-squares partials of C.
// 256x224 tiles only (edge_gemm_f32_np_ok); A / B as edge_gemm_f32.
EDGE_API int edge_gemm_f32_np_ok(int M, int N, int Kx) { return use_224(M, N, Kx, EPI_F32_RESID_NP) ? 1 : 0; }

EDGE_API int edge_gemm_f32_np(const void* A, const void* B, float* C, int M, int N, int Kx, int kplane, int lda, int ldb,
                              int ldc, const float* resid, int ldr, float alpha, const float* g, const float* rstd_in,
                              float g_max, float prod_bound, void* planes, float* prinv, float* ssq_out, hipStream_t st) {
  GemmArgs a{};
  a.alpha = alpha;
  a.colscale = g;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B;
  a.M = M; a.N = N; a.K = Kx; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.residf = resid; a.ldr = ldr; a.Cf = C;
  a.h3k = kplane;
  a.pairb = Kx == 2 * kplane;
  a.planes = (f16_t*)planes; a.prinv = prinv; a.bnd_b = rstd_in; a.bnd_c = prod_bound; a.ssq_out = ssq_out;
  a.np_g = g_max; a.np_rn = sqrtf((float)N);
  if (!g || !resid || !rstd_in || !planes || !prinv || !ssq_out || !h3_geometry_ok(Kx, kplane) || lda < 2 * kplane ||
      ldb < (a.pairb ? kplane : Kx) || !(alpha > 0.f) || !(g_max > 0.f) || !(prod_bound >= 0.f))
    return (int)hipErrorInvalidValue;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  if (((uintptr_t)C & 15) || ldc % 4 || ldr % 4 || ((uintptr_t)resid & 15) || ((uintptr_t)g & 15) ||
      ((uintptr_t)planes & 7) || !use_224(M, N, Kx, EPI_F32_RESID_NP))
    return (int)hipErrorInvalidValue;
  return launch_4w<EPI_F32_RESID_NP, 0, 224>(a, st);
}

// EPI_H3_LRP_SWIGLU: C = h3 planes [M, 4N] (fp16, row stride 4N) of the SwiGLU LRP rule on d = alpha (A . B^T)
// [M, N] and the interleaved pre-activations gu [M, 2N] (row stride ldr); A / B as edge_gemm_f32.
EDGE_API int edge_gemm_f32_lrp_swiglu(const void* A, const void* B, void* C, const float* gu, int M, int N, int Kx,
                                      int kplane, int lda, int ldb, int ldr, float alpha, hipStream_t st) {
  GemmArgs a{};
  a.alpha = alpha;
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = (bf16_t*)C;
  a.M = M; a.N = N; a.K = Kx; a.lda = lda; a.ldb = ldb; a.ldc = 4 * N;
  a.residf = gu; a.ldr = ldr;
  a.h3k = kplane;
  a.pairb = Kx == 2 * kplane;
  if (!gu || !h3_geometry_ok(Kx, kplane) || lda < 2 * kplane || ldb < (a.pairb ? kplane : Kx) || !(alpha > 0.f) ||
      ldr < 2 * N || ldr % 4 || ((uintptr_t)gu & 15) || ((uintptr_t)C & 7))
    return (int)hipErrorInvalidValue;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  return launch<EPI_H3_LRP_SWIGLU>(a, st);
}

// fp32 QKV projection + bias + RoPE + head-major scatter: X [M, 2K] (h3 activation), W [(Hq+2Hkv)*64, 3K] (h3
// weight), alpha = 1 / (s_x s_w), fp32 bias, fp32 outputs q [B,Hq,S,64] (x q_scale), k [B,Hkv,S,64],
// vt [B,Hkv,64,s_pad].
// kp / vp (optional, both or neither): K and V^T also as scaled fp16 h3 planes at scales kv_sk / kv_sv (GemmArgs);
// with them vt may be null (the plane-staged attention reads no fp32 V^T).  vf (optional): V row-major fp32
// [B,Hkv,S,64] too (the AttnLRP backward's V).
EDGE_API int edge_gemm_qkv_rope_f32(const void* X, const void* W, const float* bias, float* q, float* k, float* vt,
                                    const float* cosT, const float* sinT, int M, int Kx, int kplane, int S, int Hq,
                                    int Hkv, int rot_dim, int s_pad, float q_scale, float alpha, void* kp, void* vp,
                                    float kv_sk, float kv_sv, float* vf, hipStream_t st) {
  GemmArgs a{};
  a.A = (const bf16_t*)X; a.B = (const bf16_t*)W;
  a.pairb = Kx == 2 * kplane;
  a.M = M; a.N = (Hq + 2 * Hkv) * 64; a.K = Kx; a.lda = 2 * kplane; a.ldb = a.pairb ? kplane : Kx;
  a.h3k = kplane;   // X: 2-plane activation rows [M, 2 kplane]
  a.alpha = alpha;
  a.biasf = bias; a.qf = q; a.kf = k; a.vtf = vt;
  a.cosT = cosT; a.sinT = sinT; a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.s_pad = s_pad;
  a.q_scale = q_scale;
  a.kp = (f16_t*)kp; a.vp = (f16_t*)vp; a.kv_sk = kv_sk; a.kv_sv = kv_sv;
  a.vf = vf;
  if (vf && ((uintptr_t)vf & 15)) return (int)hipErrorInvalidValue;
  if (!bias || M % S || !h3_geometry_ok(Kx, kplane) || ((uintptr_t)bias & 15) || !(alpha > 0.f))
    return (int)hipErrorInvalidValue;
  if ((kp == nullptr) != (vp == nullptr) || (kp && (!(kv_sk > 0.f) || !(kv_sv > 0.f) || ((uintptr_t)kp & 7))))
    return (int)hipErrorInvalidValue;
  // fp32 K / V^T may be skipped when their planes are written
  if (!q || (!k && !kp) || (!vt && !vp)) return (int)hipErrorInvalidValue;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  switch (rot_dim) {
    case 0: return launch<EPI_F32_QKV_ROPE, 0>(a, st);
    case 8: return launch<EPI_F32_QKV_ROPE, 4>(a, st);
    case 16: return launch<EPI_F32_QKV_ROPE, 8>(a, st);
    case 32: return launch<EPI_F32_QKV_ROPE, 16>(a, st);
    case 64: return launch<EPI_F32_QKV_ROPE, 32>(a, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// LM head + LSE partials.  alpha == 0: bf16 X [M, K], W [N, K].  alpha > 0: fp32 execution, X a 2-plane h3
// activation [M, 2 kplane] and W the h3 weight [N, K] (h3_geometry_ok), product scale alpha.
EDGE_API int edge_gemm_lse(const void* X, const void* W, const int64_t* targets, float* part_max, float* part_sum,
                           float* tgt_logit, int M, int N, int K, int kplane, float alpha, hipStream_t st) {
  GemmArgs a{};
  const bool h3 = alpha > 0.f;
  a.A = (const bf16_t*)X; a.B = (const bf16_t*)W;
  a.pairb = h3 && K == 2 * kplane;
  a.M = M; a.N = N; a.K = K; a.lda = h3 ? 2 * kplane : K; a.ldb = a.pairb ? kplane : K;
  if (h3 && !h3_geometry_ok(K, kplane)) return (int)hipErrorInvalidValue;
  a.h3k = h3 ? kplane : 0;
  a.alpha = h3 ? alpha : 1.f;
  a.targets = targets; a.part_max = part_max; a.part_sum = part_sum; a.tgt_logit = tgt_logit; a.nparts = N / 64;
  const int chk = check_shapes(a);
  if (chk) return chk < 0 ? 0 : chk;
  return h3 ? launch<EPI_F32_LSE>(a, st) : launch<EPI_LSE>(a, st);
}

// Combine the LSE partials: nll[m] = logsumexp_m - logit[target_m].
__global__ __launch_bounds__(256) void lse_reduce_kernel(const float* __restrict__ pmax, const float* __restrict__ psum,
                                                         const float* __restrict__ tgt, float* __restrict__ nll,
                                                         int nparts) {
  __shared__ float red[4];
  const int m = blockIdx.x;
  const float* pm = pmax + (size_t)m * nparts;
  const float* ps = psum + (size_t)m * nparts;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < nparts; i += 256) mx = fmaxf(mx, pm[i]);
  mx = block_max<256>(mx, red);
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += ps[i] * __expf(pm[i] - mx);
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) nll[m] = mx + logf(s) - tgt[m];
}

EDGE_API int edge_lse_reduce(const float* pmax, const float* psum, const float* tgt, float* nll, int M, int nparts,
                             hipStream_t st) {
  if (M <= 0) return 0;
  lse_reduce_kernel<<<M, 256, 0, st>>>(pmax, psum, tgt, nll, nparts);
  return (int)hipGetLastError();
}
