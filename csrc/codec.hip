// Boundary codec kernels: importance-ranked token selection and the
// quantize/pack / unpack/dequantize of the hidden state that crosses a pipeline-stage boundary.
//
// Wire message (offsets computed on the host, codec/wire.py, every section 16-byte aligned):
//   fixed k     : [header 32 B][class bitmask B x MW u32][scales][hi-class rows][lo-class rows]
//   variable k  : [header 32 B][class bitmask][k per window, B x i32][scales][lo-class rows][hi-class rows]
// (variable k = top-rho selection: each window quantizes the tokens outside its smallest importance mass
// reaching a threshold; window b's rows follow the sum of the k (or S - k) of the windows before it, and the hi
// section starts right after the Sum k lo rows, so the message is compact; the buffer has capacity for any k).
// A token whose bit is set belongs to the low-precision ("lo") class.  Rows of each class are stored in
// token order; a row's slot is the popcount of the mask bits before it, so the receiver needs nothing
// but the mask.  Row formats: 0 bf16, 1 int8, 2 int4 (two's-complement nibbles, even element in the low
// nibble), 3 int2 (ternary, 4 per byte).  Scale modes: 0 per token (fp32 [B*S]), 1 per window for the
// lo class (fp32 [B], reference Q1 "one global max-abs" int4), 2 per channel (fp32 [B*H]; reference
// channel_8/4/1_max store max|x_c|, channel_1_mean stores mean_c + 1e-8), 3 none (pass-through).
// Activations are bf16 or fp32 (the fp32 execution mode); row format 4 keeps a row in fp32 (the reference leaves
// its un-selected tokens in fp32, Experiments/Qwen2-0.5B/qwen_layer_wise.py:54-70).
#include "common.h"

enum { FMT_BF16 = 0, FMT_INT8 = 1, FMT_INT4 = 2, FMT_INT2 = 3, FMT_F32 = 4, FMT_MXFP4 = 5, FMT_MXFP8 = 6, FMT_GRP = 7 };
// Head-group rows (FMT_GRP): every 64-channel group g (one head's width) has its own bit width b_g in {2, 3, 4, 5, 6, 8}
// (the plan: one byte per group in the message at off_plan, chosen from the boundary's channel-group sensitivity) and
// its own max-abs scale s = max|x| / qmax_b (qmax = 2^(b-1) - 1: 1 / 3 / 7 / 15 / 31 / 127): row = [group 0 codes
// (8 b_0 bytes)] ... [group G-1 codes][G fp32 scales]; the group's 64 two's-complement b-bit codes form one
// little-endian bit stream (code c at bits [b c, b c + b)), so 8 consecutive codes are b whole bytes.
// OCP microscaling rows (FMT_MXFP4: E2M1 codes, FMT_MXFP8: E4M3 codes): blocks of 32 consecutive channels share one
// E8M0 scale 2^(floor(log2 max|x|) - emax) (emax 2 / 8), stored after the row's codes: [codes][H/32 scale bytes].
// Quantize / dequantize with gfx950's scaled converts (v_cvt_scalef32_pk_fp4_f32 / _fp8_f32 and the inverses:
// round-to-nearest-even of x / scale, saturating).
enum { SC_TOKEN = 0, SC_WINDOW = 1, SC_CHANNEL = 2, SC_NONE = 3 };
enum { CH_MAXABS = 0, CH_MEAN = 1 };

struct CodecArgs {
  void* x; uint8_t* msg;
  long long off_mask, off_scale, off_hi, off_lo;
  long long off_kvec;           // >= 0: variable-k layout (k per window at msg + off_kvec), else fixed k
  long long off_plan;           // >= 0: FMT_GRP bit plan (one byte per 64-channel group)
  int B, S, H, k, mw;           // mw: mask words per window
  int hi_fmt, lo_fmt, scale_mode, qmax_hi, qmax_lo, ch_kind;
  int grp_code_bytes;           // FMT_GRP: sum over groups of 8 b_g (row = codes + 4 G scale bytes)
};

__device__ __forceinline__ int fmt_row_bytes(int fmt, int H) {
  return fmt == FMT_F32 ? 4 * H : fmt == FMT_BF16 ? 2 * H : fmt == FMT_INT8 ? H : fmt == FMT_INT4 ? H / 2 :
         fmt == FMT_MXFP4 ? H / 2 + H / 32 : fmt == FMT_MXFP8 ? H + H / 32 : H / 4;
}
__device__ __forceinline__ int row_bytes(const CodecArgs& a, int fmt) {
  return fmt == FMT_GRP ? a.grp_code_bytes + 4 * (a.H / 64) : fmt_row_bytes(fmt, a.H);
}

__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// number of lo-class tokens before token j in window b, and the class of j
__device__ __forceinline__ int lo_prefix(const uint32_t* __restrict__ mask, int mw, int j, bool& is_lo) {
  const int lane = threadIdx.x & 63;
  const int wj = j >> 5;
  int cnt = 0;
  for (int w = lane; w < wj; w += 64) cnt += __popc(mask[w]);
  cnt = wave_isum(cnt);
  const uint32_t word = mask[wj];
  is_lo = (word >> (j & 31)) & 1u;
  return cnt + __popc(word & ((1u << (j & 31)) - 1u));
}

// ---------------------------------------------------------------------------------------------
// Token selection: one workgroup per window sorts the window's (importance, position) pairs
// ascending with an LDS bitonic sort of 64-bit keys (order-preserving float bits << 32 | position: ties by
// position, NaN ranked above +inf, -0 == +0 - the order of a stable torch.sort) and marks the first k positions
// as the lo class.
//   mode 0 (ratio)  : k given (reference int(ratio * S), qwen_layer_wise.py:57).
//   mode 1 (top-rho): in descending order, keep the shortest prefix whose mass reaches thr = 1 - 0.1 ratio and
//                     quantize the rest: keep = first i with sum_{j<i} desc_j >= thr (thr <= 0 -> 0, none -> S),
//                     k = S - keep (the intended semantics of pythia_model.py:92-112, its token-id indexing bug
//                     B21 fixed); the exclusive prefix sums are an LDS block scan.  k is written to kvec[b].
__device__ __forceinline__ uint32_t ord_key(float f) {
  if (f != f) return 0xFFFFFFFFu;                  // NaN last
  uint32_t u = __float_as_uint(f == 0.f ? 0.f : f);  // -0 -> +0
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_val(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

constexpr int SEL_T = 512;
__global__ __launch_bounds__(SEL_T) void select_sort_kernel(const float* __restrict__ imp, int S, int P, int mode,
                                                            int k_fixed, float thr, uint32_t* __restrict__ mask_out,
                                                            int mw, int* __restrict__ kvec) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];  // P keys, then mw mask words
  uint32_t* mwords = (uint32_t*)(keys + P);
  __shared__ float part[SEL_T];
  __shared__ int cut;
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* ib = imp + (size_t)b * S;
  for (int i = tid; i < P; i += SEL_T)
    keys[i] = i < S ? (((unsigned long long)ord_key(ib[i]) << 32) | (unsigned)i) : ~0ull;
  for (int w = tid; w < mw; w += SEL_T) mwords[w] = 0u;
  if (tid == 0) cut = S;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += SEL_T) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = keys[i], c = keys[ixj];
          if (((i & k) == 0) == (a > c)) { keys[i] = c; keys[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  int kk = k_fixed;
  if (mode == 1) {
    // descending value i = keys[S-1-i]; thread t owns the contiguous run [t*C, t*C + C) of descending positions
    const int C = (S + SEL_T - 1) / SEL_T;
    const int i0 = tid * C;
    float run = 0.f;
    for (int e = 0; e < C && i0 + e < S; ++e) run += key_val((uint32_t)(keys[S - 1 - (i0 + e)] >> 32));
    part[tid] = run;
    __syncthreads();
    for (int off = 1; off < SEL_T; off <<= 1) {  // Hillis-Steele inclusive scan of the run sums
      const float v = tid >= off ? part[tid - off] : 0.f;
      __syncthreads();
      part[tid] += v;
      __syncthreads();
    }
    float excl = tid ? part[tid - 1] : 0.f;
    for (int e = 0; e < C && i0 + e < S; ++e) {
      if (excl >= thr) { atomicMin(&cut, i0 + e); break; }
      excl += key_val((uint32_t)(keys[S - 1 - (i0 + e)] >> 32));
    }
    __syncthreads();
    kk = S - cut;
  }
  for (int p = tid; p < kk; p += SEL_T) {
    const int idx = (int)(keys[p] & 0xFFFFFFFFu);
    atomicOr(&mwords[idx >> 5], 1u << (idx & 31));
  }
  __syncthreads();
  uint32_t* mb = mask_out + (size_t)b * mw;
  for (int w = tid; w < mw; w += SEL_T) mb[w] = mwords[w];
  if (kvec && tid == 0) kvec[b] = kk;
}

// Variable-k layout: lo rows of the windows before b (Kb) and in total (Kt), by one wave.
__device__ __forceinline__ void kvar_prefix(const CodecArgs& a, int b, int& Kb, int& Kt) {
  const int lane = threadIdx.x & 63;
  const int* kv = (const int*)(a.msg + a.off_kvec);
  int before = 0, all = 0;
  for (int w = lane; w < a.B; w += 64) {
    const int v = kv[w];
    all += v;
    before += w < b ? v : 0;
  }
  Kb = wave_isum(before);
  Kt = wave_isum(all);
}

// Per-(window, channel) statistics over the window's rows (optionally only lo-class rows).
// mode 0: max|x|, mode 1: mean(x) + 1e-8.   grid (B, ceil(H/64)), 256 threads = 4 row groups x 64 ch.
__device__ __forceinline__ float ldx(const bf16_t* p, size_t i) { return bf2f(p[i]); }
__device__ __forceinline__ float ldx(const float* p, size_t i) { return p[i]; }

template <class T>
__global__ __launch_bounds__(256) void channel_stats_kernel(const T* __restrict__ x,
                                                            const uint32_t* __restrict__ mask, int mask_stride,
                                                            float* __restrict__ out, int S, int H, int mode,
                                                            int only_lo) {
  __shared__ float red[4][64];
  const int b = blockIdx.x, c = blockIdx.y * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  const uint32_t* mb = mask + (size_t)b * mask_stride;
  float acc = 0.f;
  if (c < H) {
    for (int j = rg; j < S; j += 4) {
      if (only_lo && !((mb[j >> 5] >> (j & 31)) & 1u)) continue;
      const float xv = ldx(x, ((size_t)b * S + j) * H + c);
      acc = mode == 0 ? fmaxf(acc, fabsf(xv)) : acc + xv;
    }
  }
  red[rg][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rg == 0 && c < H) {
    const int l = threadIdx.x;
    float r = mode == 0 ? fmaxf(fmaxf(red[0][l], red[1][l]), fmaxf(red[2][l], red[3][l]))
                        : (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    out[(size_t)b * H + c] = mode == 0 ? r : r / (float)S + 1e-8f;
  }
}

__global__ __launch_bounds__(256) void rowmax_kernel(const float* __restrict__ in, float* __restrict__ out, int H) {
  __shared__ float red[4];
  const float* r = in + (size_t)blockIdx.x * H;
  float m = 0.f;
  for (int c = threadIdx.x; c < H; c += 256) m = fmaxf(m, r[c]);
  m = block_max<256>(m, red);
  if (threadIdx.x == 0) out[blockIdx.x] = m;
}

// ---------------------------------------------------------------------------------------------
template <int NCH>
__device__ __forceinline__ void load_row8(const float* __restrict__ src, int H, float (&v)[NCH][8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < H) {
      const f32x4_t a = *(const f32x4_t*)(src + col), b = *(const f32x4_t*)(src + col + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[c][e] = a[e]; v[c][4 + e] = b[e]; }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] = 0.f;
    }
  }
}
template <int NCH>
__device__ __forceinline__ void load_row8(const bf16_t* __restrict__ src, int H, float (&v)[NCH][8]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < H) {
      const u32x4_t w = *(const u32x4_t*)(src + col);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[c][2 * e] = bf_lo(w[e]); v[c][2 * e + 1] = bf_hi(w[e]); }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[c][e] = 0.f;
    }
  }
}

__device__ __forceinline__ float qround(float t, float qmax, float qmin) { return fminf(fmaxf(rintf(t), qmin), qmax); }

typedef __attribute__((ext_vector_type(2))) short s16x2_t;

// E8M0 scale byte and value of a 32-channel block (4 lanes x 8 values): 2^(floor(log2 amax) - emax)
__device__ __forceinline__ int mx_scale_byte(float am, int emax) {
  const int e = am > 0.f ? (int)((__float_as_uint(am) >> 23) & 0xff) - 127 : -127;   // denormal amax -> -127
  const int sb = e - emax + 127;
  return sb < 0 ? 0 : (sb > 254 ? 254 : sb);
}
__device__ __forceinline__ float e8m0_value(int sb) { return sb ? __uint_as_float((uint32_t)sb << 23) : __uint_as_float(0x00400000u); }

__device__ __forceinline__ void mx_pack8(uint8_t* __restrict__ row, int H, int col, int fmt, const float (&v)[8]) {
  const int lane = threadIdx.x & 63;
  float am = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[e]));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  const int sb = mx_scale_byte(am, fmt == FMT_MXFP4 ? 2 : 8);
  const float X = e8m0_value(sb);
  if (fmt == FMT_MXFP4) {
    uint32_t w = 0;
    w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, v[0], v[1], X, 0);
    w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, v[2], v[3], X, 1);
    w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, v[4], v[5], X, 2);
    w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, v[6], v[7], X, 3);
    *(uint32_t*)(row + col / 2) = w;
    if ((lane & 3) == 0) row[H / 2 + col / 32] = (uint8_t)sb;
  } else {
    // x / X can reach 2^9 > 448 (E4M3 max): clamp first - the fp8 convert does not saturate (NaN code)
    const float lim = 448.f * X;
    float c[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) c[e] = fminf(fmaxf(v[e], -lim), lim);
    s16x2_t a = {0, 0}, b = {0, 0};
    a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(a, c[0], c[1], X, false);
    a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(a, c[2], c[3], X, true);
    b = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(b, c[4], c[5], X, false);
    b = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(b, c[6], c[7], X, true);
    u32x2_t w;
    w[0] = (uint32_t)(uint16_t)a[0] | ((uint32_t)(uint16_t)a[1] << 16);
    w[1] = (uint32_t)(uint16_t)b[0] | ((uint32_t)(uint16_t)b[1] << 16);
    *(u32x2_t*)(row + col) = w;
    if ((lane & 3) == 0) row[H + col / 32] = (uint8_t)sb;
  }
}

__device__ __forceinline__ void mx_unpack8(const uint8_t* __restrict__ row, int H, int col, int fmt, float (&o)[8]) {
  if (fmt == FMT_MXFP4) {
    const float X = e8m0_value(row[H / 2 + col / 32]);
    const uint32_t w = *(const uint32_t*)(row + col / 2);
    f32x2_t p0 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(w, X, 0), p1 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(w, X, 1);
    f32x2_t p2 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(w, X, 2), p3 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(w, X, 3);
    o[0] = p0[0]; o[1] = p0[1]; o[2] = p1[0]; o[3] = p1[1]; o[4] = p2[0]; o[5] = p2[1]; o[6] = p3[0]; o[7] = p3[1];
  } else {
    const float X = e8m0_value(row[H + col / 32]);
    const u32x2_t w = *(const u32x2_t*)(row + col);
    f32x2_t p0 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(w[0], X, false), p1 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(w[0], X, true);
    f32x2_t p2 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(w[1], X, false), p3 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(w[1], X, true);
    o[0] = p0[0]; o[1] = p0[1]; o[2] = p1[0]; o[3] = p1[1]; o[4] = p2[0]; o[5] = p2[1]; o[6] = p3[0]; o[7] = p3[1];
  }
}

// FMT_GRP: the 8 lanes holding channels [64 g, 64 g + 64) of a row (8 values each) quantize their group.
// Byte offset of group g's codes = sum_{g' < g} 8 b_g'.
__device__ __forceinline__ int grp_offset(const uint8_t* __restrict__ plan, int g) {
  int o = 0;
  for (int i = 0; i < g; ++i) o += 8 * plan[i];
  return o;
}
// The 8 codes of a lane are bytes [sub b, sub b + b) of the group's stream (sub = lane & 7), b-byte aligned: whole
// 8 / 4 / 2-byte stores for b = 8 / 4 / 2, 2-byte pieces for b = 6, single bytes for b = 3 / 5.
__device__ __forceinline__ void grp_store(uint8_t* __restrict__ dst, uint64_t w, int bits) {
  if (bits == 8) {
    *(u32x2_t*)dst = u32x2_t{(uint32_t)w, (uint32_t)(w >> 32)};
  } else if (bits == 4) {
    *(uint32_t*)dst = (uint32_t)w;
  } else if (bits == 2) {
    *(uint16_t*)dst = (uint16_t)w;
  } else if (bits == 6) {
#pragma unroll
    for (int i = 0; i < 3; ++i) ((uint16_t*)dst)[i] = (uint16_t)(w >> (16 * i));
  } else {
    for (int i = 0; i < bits; ++i) dst[i] = (uint8_t)(w >> (8 * i));
  }
}
__device__ __forceinline__ uint64_t grp_load(const uint8_t* __restrict__ src, int bits) {
  if (bits == 8) {
    const u32x2_t v = *(const u32x2_t*)src;
    return (uint64_t)v[0] | ((uint64_t)v[1] << 32);
  }
  if (bits == 4) return *(const uint32_t*)src;
  if (bits == 2) return *(const uint16_t*)src;
  uint64_t w = 0;
  if (bits == 6) {
#pragma unroll
    for (int i = 0; i < 3; ++i) w |= (uint64_t)((const uint16_t*)src)[i] << (16 * i);
  } else {
    for (int i = 0; i < bits; ++i) w |= (uint64_t)src[i] << (8 * i);
  }
  return w;
}
__device__ __forceinline__ void grp_pack8(uint8_t* __restrict__ row, const CodecArgs& a, int col,
                                          const float (&v)[8]) {
  const int lane = threadIdx.x & 63;
  const uint8_t* plan = a.msg + a.off_plan;
  const int g = col >> 6, bits = plan[g];
  const int qmax = (1 << (bits - 1)) - 1;
  float am = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[e]));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  am = fmaxf(am, __shfl_xor(am, 4, 64));
  const float s = am / (float)qmax;
  const float inv = am > 0.f ? 1.f / s : 0.f;
  const float qf = (float)qmax;
  const uint64_t mask = (1ull << bits) - 1;
  uint64_t w = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) w |= ((uint64_t)(int64_t)(int)qround(v[e] * inv, qf, -qf) & mask) << (bits * e);
  const int sub = lane & 7;
  grp_store(row + grp_offset(plan, g) + sub * bits, w, bits);
  if (sub == 0) *(float*)(row + a.grp_code_bytes + 4 * g) = s;
}
__device__ __forceinline__ bool grp_bits_ok(int b) { return b == 2 || b == 3 || b == 4 || b == 5 || b == 6 || b == 8; }
__device__ __forceinline__ void grp_unpack8(const uint8_t* __restrict__ row, const CodecArgs& a, int col,
                                            float (&o)[8]) {
  const int lane = threadIdx.x & 63;
  const uint8_t* plan = a.msg + a.off_plan;
  const int g = col >> 6;
  const int sub = lane & 7;
  // the plan bytes come from the message: a width outside GROUP_BITS (a corrupt or version-mismatched message) or a
  // group stream reaching past the row's code bytes decodes to NaN - loud - instead of a shift by 32 or a read past
  // the row (invalid widths count 0 bytes in the offset)
  int off = 0;
  bool bad = false;
  for (int i = 0; i < g; ++i) {
    const int b = plan[i];
    bad |= !grp_bits_ok(b);
    off += grp_bits_ok(b) ? 8 * b : 0;
  }
  const int bits = plan[g];
  bad |= !grp_bits_ok(bits) || off + 8 * bits > a.grp_code_bytes;
  if (bad) {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = __builtin_nanf("");
    return;
  }
  const uint64_t w = grp_load(row + off + sub * bits, bits);
  const float s = *(const float*)(row + a.grp_code_bytes + 4 * g);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int q = ((int)((uint32_t)(w >> (bits * e)) << (32 - bits))) >> (32 - bits);   // sign-extend b bits
    o[e] = (float)q * s;
  }
}

template <int NCH, class T>
__global__ __launch_bounds__(256) void pack_kernel(CodecArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.B * a.S) return;
  const int lane = threadIdx.x & 63;
  const int b = row / a.S, j = row - b * a.S;
  const uint32_t* mask = (const uint32_t*)(a.msg + a.off_mask) + (size_t)b * a.mw;
  bool is_lo;
  const int slot_lo = lo_prefix(mask, a.mw, j, is_lo);
  const int fmt = is_lo ? a.lo_fmt : a.hi_fmt;
  const int qmax = is_lo ? a.qmax_lo : a.qmax_hi;
  const int rb = row_bytes(a, fmt);
  uint8_t* dst;
  if (a.off_kvec >= 0) {
    int Kb, Kt;
    kvar_prefix(a, b, Kb, Kt);
    const long long off_hi = a.off_lo + (((long long)Kt * row_bytes(a, a.lo_fmt) + 15) & ~15ll);
    dst = is_lo ? a.msg + a.off_lo + ((size_t)Kb + slot_lo) * rb
                : a.msg + off_hi + ((size_t)b * a.S - Kb + (j - slot_lo)) * rb;
  } else {
    dst = is_lo ? a.msg + a.off_lo + ((size_t)b * a.k + slot_lo) * rb
                : a.msg + a.off_hi + ((size_t)b * (a.S - a.k) + (j - slot_lo)) * rb;
  }
  float v[NCH][8];
  load_row8<NCH>((const T*)a.x + (size_t)row * a.H, a.H, v);
  float* scales = (float*)(a.msg + a.off_scale);

  // scale / quantiser for this row
  float inv = 0.f, mul = 0.f;  // code = round(x * inv) for token & channel; window mode uses ref formula
  const bool raw = fmt == FMT_BF16 || fmt == FMT_F32 || fmt == FMT_MXFP4 || fmt == FMT_MXFP8 || fmt == FMT_GRP;
  if (raw && a.scale_mode == SC_TOKEN && lane == 0) scales[row] = 0.f;
  if (!raw) {
    if (a.scale_mode == SC_TOKEN) {
      float am = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(v[c][e]));
      am = wave_max(am);
      const float s = am / (float)qmax;
      if (lane == 0) scales[row] = s;
      inv = am > 0.f ? 1.f / s : 0.f;
    } else if (a.scale_mode == SC_WINDOW) {
      mul = scales[b];  // max|x| over the window's lo rows
    }
  }
  const float qmaxf = (float)qmax;
  const float qminf = a.scale_mode == SC_WINDOW ? -(float)(qmax + 1) : -(float)qmax;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col >= a.H) continue;
    int q[8];
    if (fmt == FMT_F32) {
      *(f32x4_t*)(dst + col * 4) = f32x4_t{v[c][0], v[c][1], v[c][2], v[c][3]};
      *(f32x4_t*)(dst + col * 4 + 16) = f32x4_t{v[c][4], v[c][5], v[c][6], v[c][7]};
      continue;
    }
    if (fmt == FMT_MXFP4 || fmt == FMT_MXFP8) {
      mx_pack8(dst, a.H, col, fmt, v[c]);
      continue;
    }
    if (fmt == FMT_GRP) {
      grp_pack8(dst, a, col, v[c]);
      continue;
    }
    if (fmt == FMT_BF16) {
      u32x4_t w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = pack_bf2(v[c][2 * e], v[c][2 * e + 1]);
      *(u32x4_t*)(dst + col * 2) = w;
      continue;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xv = v[c][e];
      float t;
      if (a.scale_mode == SC_TOKEN) {
        t = qround(xv * inv, qmaxf, qminf);
      } else if (a.scale_mode == SC_WINDOW) {
        // reference Q1: round(clamp(x / m * 7, -8, 7))
        t = mul > 0.f ? rintf(fminf(fmaxf(xv / mul * qmaxf, qminf), qmaxf)) : 0.f;
      } else {
        const float sc = scales[(size_t)b * a.H + col + e];
        if (a.ch_kind == CH_MEAN || qmax == 1) {
          t = sc != 0.f ? fminf(fmaxf(rintf(xv / sc), -1.f), 1.f) : 0.f;       // ternary (reference clamps)
        } else {
          t = sc > 0.f ? rintf(xv / sc * qmaxf) : 0.f;                         // reference: no clamp
        }
      }
      q[e] = (int)t;
    }
    if (fmt == FMT_INT8) {
      u32x2_t w;
      w[0] = (q[0] & 255) | ((q[1] & 255) << 8) | ((q[2] & 255) << 16) | ((uint32_t)(q[3] & 255) << 24);
      w[1] = (q[4] & 255) | ((q[5] & 255) << 8) | ((q[6] & 255) << 16) | ((uint32_t)(q[7] & 255) << 24);
      *(u32x2_t*)(dst + col) = w;
    } else if (fmt == FMT_INT4) {
      uint32_t w = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) w |= (uint32_t)(q[e] & 15) << (4 * e);
      *(uint32_t*)(dst + col / 2) = w;
    } else {
      uint32_t w = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) w |= (uint32_t)(q[e] & 3) << (2 * e);
      *(uint16_t*)(dst + col / 4) = (uint16_t)w;
    }
  }
}

__device__ __forceinline__ void store8(bf16_t* dst, const float (&o)[8]) {
  u32x4_t w;
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = pack_bf2(o[2 * e], o[2 * e + 1]);
  *(u32x4_t*)dst = w;
}
__device__ __forceinline__ void store8(float* dst, const float (&o)[8]) {
  *(f32x4_t*)dst = f32x4_t{o[0], o[1], o[2], o[3]};
  *(f32x4_t*)(dst + 4) = f32x4_t{o[4], o[5], o[6], o[7]};
}

template <int NCH, class T>
__global__ __launch_bounds__(256) void unpack_kernel(CodecArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.B * a.S) return;
  const int lane = threadIdx.x & 63;
  const int b = row / a.S, j = row - b * a.S;
  const uint32_t* mask = (const uint32_t*)(a.msg + a.off_mask) + (size_t)b * a.mw;
  bool is_lo;
  const int slot_lo = lo_prefix(mask, a.mw, j, is_lo);
  const int fmt = is_lo ? a.lo_fmt : a.hi_fmt;
  const int qmax = is_lo ? a.qmax_lo : a.qmax_hi;
  const int rb = row_bytes(a, fmt);
  const uint8_t* src;
  if (a.off_kvec >= 0) {
    int Kb, Kt;
    kvar_prefix(a, b, Kb, Kt);
    const long long off_hi = a.off_lo + (((long long)Kt * row_bytes(a, a.lo_fmt) + 15) & ~15ll);
    src = is_lo ? a.msg + a.off_lo + ((size_t)Kb + slot_lo) * rb
                : a.msg + off_hi + ((size_t)b * a.S - Kb + (j - slot_lo)) * rb;
  } else {
    src = is_lo ? a.msg + a.off_lo + ((size_t)b * a.k + slot_lo) * rb
                : a.msg + a.off_hi + ((size_t)b * (a.S - a.k) + (j - slot_lo)) * rb;
  }
  const float* scales = (const float*)(a.msg + a.off_scale);
  float s = 0.f;
  if (fmt != FMT_BF16 && fmt != FMT_F32 && fmt != FMT_MXFP4 && fmt != FMT_MXFP8 && fmt != FMT_GRP) {
    if (a.scale_mode == SC_TOKEN) s = scales[row];
    else if (a.scale_mode == SC_WINDOW) s = scales[b];
  }
  T* out = (T*)a.x + (size_t)row * a.H;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col >= a.H) continue;
    if (fmt == FMT_BF16 || fmt == FMT_F32) {
      float o[8];
      if (fmt == FMT_F32) {
        const f32x4_t x0 = *(const f32x4_t*)(src + col * 4), x1 = *(const f32x4_t*)(src + col * 4 + 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) { o[e] = x0[e]; o[4 + e] = x1[e]; }
      } else {
        const u32x4_t w = *(const u32x4_t*)(src + col * 2);
#pragma unroll
        for (int e = 0; e < 4; ++e) { o[2 * e] = bf_lo(w[e]); o[2 * e + 1] = bf_hi(w[e]); }
      }
      store8(out + col, o);
      continue;
    }
    if (fmt == FMT_MXFP4 || fmt == FMT_MXFP8) {
      float o[8];
      mx_unpack8(src, a.H, col, fmt, o);
      store8(out + col, o);
      continue;
    }
    if (fmt == FMT_GRP) {
      float o[8];
      grp_unpack8(src, a, col, o);
      store8(out + col, o);
      continue;
    }
    int q[8];
    if (fmt == FMT_INT8) {
      const u32x2_t w = *(const u32x2_t*)(src + col);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        q[e] = (int)(int8_t)((w[0] >> (8 * e)) & 255);
        q[4 + e] = (int)(int8_t)((w[1] >> (8 * e)) & 255);
      }
    } else if (fmt == FMT_INT4) {
      const uint32_t w = *(const uint32_t*)(src + col / 2);
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = ((int)(w << (28 - 4 * e))) >> 28;
    } else {
      const uint32_t w = *(const uint16_t*)(src + col / 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = ((int)(w << (30 - 2 * e))) >> 30;
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float qf = (float)q[e];
      if (a.scale_mode == SC_TOKEN) o[e] = qf * s;
      else if (a.scale_mode == SC_WINDOW) o[e] = qf / (float)qmax * s;            // reference: q / 7 * m
      else {
        const float sc = scales[(size_t)b * a.H + col + e];
        o[e] = (a.ch_kind == CH_MEAN || qmax == 1) ? qf * sc : qf * sc / (float)qmax;
      }
    }
    store8(out + col, o);
  }
}

#define DISPATCH_NCH(H, ...)                                          \
  do {                                                                \
    const int _nch = ((H) / 8 + 63) / 64;                             \
    if (_nch <= 1) { constexpr int NCH = 1; __VA_ARGS__; }            \
    else if (_nch <= 2) { constexpr int NCH = 2; __VA_ARGS__; }       \
    else if (_nch <= 4) { constexpr int NCH = 4; __VA_ARGS__; }       \
    else if (_nch <= 8) { constexpr int NCH = 8; __VA_ARGS__; }       \
    else return (int)hipErrorInvalidValue;                            \
  } while (0)

static CodecArgs make_args(void* x, void* msg, long long om, long long os, long long oh, long long ol, long long okv,
                           long long opl, int B, int S, int H, int k, int hi_fmt, int lo_fmt, int scale_mode,
                           int qmax_hi, int qmax_lo, int ch_kind, int grp_code_bytes) {
  CodecArgs a;
  a.x = x; a.msg = (uint8_t*)msg;
  a.off_mask = om; a.off_scale = os; a.off_hi = oh; a.off_lo = ol; a.off_kvec = okv; a.off_plan = opl;
  a.grp_code_bytes = grp_code_bytes;
  a.B = B; a.S = S; a.H = H; a.k = k; a.mw = ((S + 63) / 64) * 2;
  a.hi_fmt = hi_fmt; a.lo_fmt = lo_fmt; a.scale_mode = scale_mode; a.qmax_hi = qmax_hi; a.qmax_lo = qmax_lo;
  a.ch_kind = ch_kind;
  return a;
}

// mode 0: k least important per window; mode 1: top-rho cut at mass thr, k per window -> msg + off_kvec (int32).
EDGE_API int edge_select(const float* imp, int B, int S, int k, void* msg, long long off_mask, int mode, float thr,
                         long long off_kvec, hipStream_t st) {
  if (B <= 0) return 0;
  if (S <= 0 || S > 8192 || (mode == 1 && off_kvec < 0)) return (int)hipErrorInvalidValue;
  int P = 1;
  while (P < S) P <<= 1;
  const int mw = ((S + 63) / 64) * 2;
  const size_t lds = (size_t)P * 8 + (size_t)mw * 4;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)select_sort_kernel,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(select_sort_kernel, dim3(B), dim3(SEL_T), lds, st, imp, S, P, mode, k, thr,
                     (uint32_t*)((uint8_t*)msg + off_mask), mw, off_kvec >= 0 ? (int*)((uint8_t*)msg + off_kvec) : nullptr);
  return (int)hipGetLastError();
}

// Constant lo-class mask (k = 0 or k = S): a kernel, not hipMemsetAsync - inside a captured HIP graph the memset node
// was measured to lose its order against the message's zero fill (replays produced an all-zero mask for k = S).
__global__ __launch_bounds__(256) void set_mask_kernel(uint32_t* __restrict__ mask, size_t nwords, uint32_t v) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < nwords) mask[i] = v;
}

EDGE_API int edge_set_mask(void* msg, long long off_mask, int B, int S, int all_lo, hipStream_t st) {
  const int mw = ((S + 63) / 64) * 2;
  const size_t n = (size_t)B * mw;
  if (!n) return 0;
  if (off_mask % 4) return (int)hipErrorInvalidValue;
  set_mask_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>((uint32_t*)((uint8_t*)msg + off_mask), n,
                                                                all_lo ? 0xffffffffu : 0u);
  return (int)hipGetLastError();
}

// channel_stats: mode 0 max|x|, 1 mean+1e-8; only_lo restricts to lo-class rows.  out: [B, H] fp32
EDGE_API int edge_channel_stats(const void* x, const void* msg, long long off_mask, float* out, int B, int S, int H,
                                int mode, int only_lo, int x_f32, hipStream_t st) {
  if (B <= 0) return 0;
  const int mw = ((S + 63) / 64) * 2;
  const uint32_t* mask = (const uint32_t*)((const uint8_t*)msg + off_mask);
  if (x_f32)
    hipLaunchKernelGGL(channel_stats_kernel<float>, dim3(B, (H + 63) / 64), dim3(256), 0, st, (const float*)x, mask,
                       mw, out, S, H, mode, only_lo);
  else
    hipLaunchKernelGGL(channel_stats_kernel<bf16_t>, dim3(B, (H + 63) / 64), dim3(256), 0, st, (const bf16_t*)x, mask,
                       mw, out, S, H, mode, only_lo);
  return (int)hipGetLastError();
}

EDGE_API int edge_rowmax(const float* in, float* out, int R, int H, hipStream_t st) {
  if (R <= 0) return 0;
  rowmax_kernel<<<R, 256, 0, st>>>(in, out, H);
  return (int)hipGetLastError();
}

// grp_code_bytes: FMT_GRP rows' code bytes (sum 8 b_g over the plan at msg + opl; 0 without FMT_GRP)
EDGE_API int edge_pack(const void* x, void* msg, long long om, long long os, long long oh, long long ol, long long okv,
                       long long opl, int B, int S, int H, int k, int hi_fmt, int lo_fmt, int scale_mode, int qmax_hi,
                       int qmax_lo, int ch_kind, int grp_code_bytes, int x_f32, hipStream_t st) {
  if (H % 32) return (int)hipErrorInvalidValue;
  if ((hi_fmt == FMT_GRP || lo_fmt == FMT_GRP) && (H % 64 || opl < 0 || grp_code_bytes <= 0))
    return (int)hipErrorInvalidValue;
  CodecArgs a = make_args((void*)x, msg, om, os, oh, ol, okv, opl, B, S, H, k, hi_fmt, lo_fmt, scale_mode, qmax_hi,
                          qmax_lo, ch_kind, grp_code_bytes);
  const int rows = B * S;
  if (rows <= 0) return 0;
  if (x_f32) DISPATCH_NCH(H, hipLaunchKernelGGL((pack_kernel<NCH, float>), dim3((rows + 3) / 4), dim3(256), 0, st, a));
  else DISPATCH_NCH(H, hipLaunchKernelGGL((pack_kernel<NCH, bf16_t>), dim3((rows + 3) / 4), dim3(256), 0, st, a));
  return (int)hipGetLastError();
}

EDGE_API int edge_unpack(void* x, const void* msg, long long om, long long os, long long oh, long long ol,
                         long long okv, long long opl, int B, int S, int H, int k, int hi_fmt, int lo_fmt,
                         int scale_mode, int qmax_hi, int qmax_lo, int ch_kind, int grp_code_bytes, int x_f32,
                         hipStream_t st) {
  if (H % 32) return (int)hipErrorInvalidValue;
  if ((hi_fmt == FMT_GRP || lo_fmt == FMT_GRP) && (H % 64 || opl < 0 || grp_code_bytes <= 0))
    return (int)hipErrorInvalidValue;
  CodecArgs a = make_args(x, (void*)msg, om, os, oh, ol, okv, opl, B, S, H, k, hi_fmt, lo_fmt, scale_mode, qmax_hi,
                          qmax_lo, ch_kind, grp_code_bytes);
  const int rows = B * S;
  if (rows <= 0) return 0;
  if (x_f32) DISPATCH_NCH(H, hipLaunchKernelGGL((unpack_kernel<NCH, float>), dim3((rows + 3) / 4), dim3(256), 0, st, a));
  else DISPATCH_NCH(H, hipLaunchKernelGGL((unpack_kernel<NCH, bf16_t>), dim3((rows + 3) / 4), dim3(256), 0, st, a));
  return (int)hipGetLastError();
}
