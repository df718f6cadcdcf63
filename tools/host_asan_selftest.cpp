// Host-side AddressSanitizer sweep of the native libraries.
//
// Built by tools/build_host_asan.sh: every csrc/*.hip and csrc/comm/rccl_comm.cpp compiled with
// `-Xarch_host -fsanitize=address` (host code instrumented, the gfx950 code objects unchanged - GPU ASan / XNACK
// are not available on this pool) and linked with this driver into one executable, so the ASan runtime is linked
// in (no preload).  It drives the C ABI entry points the Python layer uses - GEMMs with every epilogue family,
// fp32 (h3) GEMM, norms, attention, codec select/pack/unpack, argument validation paths, and an RCCL world-1
// loopback - on small shapes, and checks the return codes.  Any heap / stack misuse in the host code (argument
// structs, dispatch tables, layout arithmetic, communicator lifetime) aborts with an ASan report.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
int edge_gemm(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, const void* bias,
              const void* resid, int ldr, int act, const float* rscale, float* ssq_out, hipStream_t st);
int edge_gemm_f32(const void* A, const void* B, void* C, int M, int N, int Kx, int kplane, int lda, int ldb, int ldc,
                  const float* bias, const float* resid, int ldr, int act, const float* rscale, float alpha,
                  float out_scale, hipStream_t st);
int edge_rmsnorm_f32(const float* x, const float* w, void* y, const int* rows, int R, int H, float eps,
                     float h3_scale, hipStream_t st);
int edge_flash_attn_fwd_f32(const float* q, const float* k, const float* vt, void* o, float* lse,
                            const float* n_rows, int B, int Hq, int Hkv, int S, int s_pad, float out_h3_scale,
                            float sq, float sk, float sv, hipStream_t st);
int edge_select(const float* imp, int B, int S, int k, void* msg, long long off_mask, int mode, float thr,
                long long off_kvec, hipStream_t st);
int edge_pack(const void* x, void* msg, long long om, long long os, long long oh, long long ol, long long okv,
              long long opl, int B, int S, int H, int k, int hi_fmt, int lo_fmt, int scale_mode, int qmax_hi,
              int qmax_lo, int ch_kind, int grp_code_bytes, int x_f32, hipStream_t st);
int edge_unpack(void* x, const void* msg, long long om, long long os, long long oh, long long ol, long long okv,
                long long opl, int B, int S, int H, int k, int hi_fmt, int lo_fmt, int scale_mode, int qmax_hi,
                int qmax_lo, int ch_kind, int grp_code_bytes, int x_f32, hipStream_t st);
int edge_rccl_id_bytes();
int edge_rccl_unique_id(char* out);
int edge_rccl_init(void** handle, int nranks, const char* id_bytes, int rank, int device);
int edge_rccl_destroy(void* handle);
int edge_rccl_group_start();
int edge_rccl_group_end();
int edge_rccl_send(void* handle, const void* buf, long long bytes, int peer);
int edge_rccl_recv(void* handle, void* buf, long long bytes, int peer);
int edge_rccl_stream_sync(void* handle);
}

static int g_fail = 0;
#define EXPECT(expr, want)                                                                    \
  do {                                                                                        \
    const int _rc = (expr);                                                                   \
    if (_rc != (want)) {                                                                      \
      std::fprintf(stderr, "FAIL %s:%d %s -> %d (want %d)\n", __FILE__, __LINE__, #expr, _rc, \
                   (int)(want));                                                              \
      ++g_fail;                                                                               \
    }                                                                                         \
  } while (0)

static void* dalloc(size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMemset(p, 0, bytes) != hipSuccess) {
    std::fprintf(stderr, "hipMalloc(%zu) failed\n", bytes);
    std::exit(2);
  }
  return p;
}

int main() {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    std::printf("no GPU: host-only checks skipped\n");
    return 0;
  }
  std::vector<void*> bufs;
  auto A = [&](size_t n) { bufs.push_back(dalloc(n)); return bufs.back(); };
  hipStream_t st = nullptr;

  // bf16 GEMMs: plain, bias, residual, SwiGLU, GELU; 128x128 and persistent paths (M large enough for 256 tiles)
  for (int M : {300, 8192}) {
    const int N = 512, K = 256;
    void *a = A((size_t)M * K * 2), *b = A((size_t)N * K * 2), *c = A((size_t)M * N * 2), *bias = A(N * 2),
         *res = A((size_t)M * N * 2);
    EXPECT(edge_gemm(a, b, c, M, N, K, K, K, N, nullptr, nullptr, 0, 0, nullptr, nullptr, st), 0);
    EXPECT(edge_gemm(a, b, c, M, N, K, K, K, N, bias, res, N, 0, nullptr, nullptr, st), 0);
    EXPECT(edge_gemm(a, b, c, M, N, K, K, K, N / 2, nullptr, nullptr, 0, 2, nullptr, nullptr, st), 0);
    EXPECT(edge_gemm(a, b, c, M, N, K, K, K, N, bias, nullptr, 0, 1, nullptr, nullptr, st), 0);
    float* ssq = (float*)A((size_t)M * (N / 64) * 4);
    EXPECT(edge_gemm(a, b, c, M, N, K, K, K, N, nullptr, res, N, 0, nullptr, ssq, st), 0);
  }
  // N = 896 residual GEMM (the 256x224 kernels)
  {
    const int M = 32768, N = 896, K = 128;
    void *a = A((size_t)M * K * 2), *b = A((size_t)N * K * 2), *c = A((size_t)M * N * 2);
    EXPECT(edge_gemm(a, b, c, M, N, K, K, K, N, nullptr, c, N, 0, nullptr, nullptr, st), 0);
  }
  // argument validation: N not a multiple of 128, empty M
  EXPECT(edge_gemm(bufs[0], bufs[1], bufs[2], 300, 100, 256, 256, 256, 100, nullptr, nullptr, 0, 0, nullptr, nullptr,
                   st), (int)hipErrorInvalidValue);
  EXPECT(edge_gemm(bufs[0], bufs[1], bufs[2], 0, 512, 256, 256, 256, 512, nullptr, nullptr, 0, 0, nullptr, nullptr,
                   st), 0);

  // fp32 mode: h3 GEMM (2-plane activation [M, 2K], weight [N, 3K]), fp32 out + SwiGLU h3 out, RMSNorm -> h3
  {
    const int M = 4096, N = 512, K = 128, Kx = 3 * K;
    void *a = A((size_t)M * 2 * K * 2), *b = A((size_t)N * Kx * 2), *c = A((size_t)M * N * 4),
         *c3 = A((size_t)M * 2 * (N / 2) * 2);
    EXPECT(edge_gemm_f32(a, b, c, M, N, Kx, K, 2 * K, Kx, N, nullptr, nullptr, 0, 0, nullptr, 1.f, 1.f, st), 0);
    EXPECT(edge_gemm_f32(a, b, c, M, N, 2 * K, K, 2 * K, 2 * K, N, nullptr, nullptr, 0, 0, nullptr, 1.f, 1.f, st), 0);
    EXPECT(edge_gemm_f32(a, b, c3, M, N, Kx, K, 2 * K, Kx, 2 * (N / 2), nullptr, nullptr, 0, 2, nullptr, 1.f, 1.f, st),
           0);
    EXPECT(edge_gemm_f32(a, b, c, M, N, Kx, K, K, Kx, N, nullptr, nullptr, 0, 0, nullptr, 1.f, 1.f, st),
           (int)hipErrorInvalidValue);   // lda smaller than the 2-plane row
    EXPECT(edge_gemm_f32(a, b, c, M, N, Kx, K, 2 * K, Kx, N, nullptr, nullptr, 0, 0, nullptr, 0.f, 1.f, st),
           (int)hipErrorInvalidValue);   // no product scale
    float *x = (float*)A((size_t)M * K * 4), *w = (float*)A(K * 4);
    EXPECT(edge_rmsnorm_f32(x, w, c3, nullptr, M, K, 1e-6f, 1.f, st), 0);
  }
  // fp32 attention + LSE
  {
    const int B = 2, Hq = 4, Hkv = 2, S = 100, sp = 128;
    float *q = (float*)A((size_t)B * Hq * S * 64 * 4), *k = (float*)A((size_t)B * Hkv * S * 64 * 4),
          *vt = (float*)A((size_t)B * Hkv * 64 * sp * 4), *o = (float*)A((size_t)B * S * Hq * 64 * 4),
          *lse = (float*)A((size_t)B * Hq * S * 4);
    EXPECT(edge_flash_attn_fwd_f32(q, k, vt, o, lse, nullptr, B, Hq, Hkv, S, sp, 0.f, 0.f, 0.f, 0.f, st), 0);
    EXPECT(edge_flash_attn_fwd_f32(q, k, vt, o, lse, nullptr, B, Hq, Hkv, S, sp, 0.f, 1.f, 1.f, 1.f, st), 0);
    EXPECT(edge_flash_attn_fwd_f32(q, k, vt, o, lse, nullptr, B, Hq, Hkv, S, 100, 0.f, 0.f, 0.f, 0.f, st),
           (int)hipErrorInvalidValue);
  }
  // codec: mixed int4 / int8 per-token message, fixed k (layout of codec/wire.py for B 2, S 64, H 256, k 32)
  {
    const int B = 2, S = 64, H = 256, k = 32;
    const long long om = 32, os = 48, oh = os + B * S * 4, ol = oh + (long long)B * (S - k) * H,
                    total = ol + (long long)B * k * H / 2;
    float *x = (float*)A((size_t)B * S * H * 4), *imp = (float*)A((size_t)B * S * 4);
    void* msg = A(total);
    EXPECT(edge_select(imp, B, S, k, msg, om, 0, 0.f, -1, st), 0);
    EXPECT(edge_pack(x, msg, om, os, oh, ol, -1, -1, B, S, H, k, 1, 2, 0, 127, 7, 0, 0, 1, st), 0);
    EXPECT(edge_unpack(x, msg, om, os, oh, ol, -1, -1, B, S, H, k, 1, 2, 0, 127, 7, 0, 0, 1, st), 0);
    EXPECT(edge_pack(x, msg, om, os, oh, ol, -1, -1, B, S, 100, k, 1, 2, 0, 127, 7, 0, 0, 1, st),
           (int)hipErrorInvalidValue);   // H not a multiple of 32
    EXPECT(edge_select(imp, B, 9000, k, msg, om, 0, 0.f, -1, st), (int)hipErrorInvalidValue);
  }
  EXPECT((int)hipDeviceSynchronize(), 0);

  // RCCL world-1 loopback through the native communicator
  {
    std::vector<char> id(edge_rccl_id_bytes());
    EXPECT(edge_rccl_unique_id(id.data()), 0);
    void* comm = nullptr;
    EXPECT(edge_rccl_init(&comm, 1, id.data(), 0, 0), 0);
    void *s = A(1 << 20), *r = A(1 << 20);
    EXPECT(edge_rccl_group_start(), 0);
    EXPECT(edge_rccl_send(comm, s, 1 << 20, 0), 0);
    EXPECT(edge_rccl_recv(comm, r, 1 << 20, 0), 0);
    EXPECT(edge_rccl_group_end(), 0);
    EXPECT(edge_rccl_stream_sync(comm), 0);
    EXPECT(edge_rccl_destroy(comm), 0);
  }
  for (void* p : bufs) (void)hipFree(p);
  std::printf("%s: %d failures\n", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
