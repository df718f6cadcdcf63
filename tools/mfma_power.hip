// Sustained MFMA throughput of the two fp16 matrix-core shapes under the chip's power limit: every wave of a grid that
// fills all CUs issues back-to-back independent MFMAs on register operands (rotated every step so the operand bits
// toggle as in a GEMM) for ~50 ms per launch, 40 launches in a row; per launch the achieved TFLOP/s.  At a full MFMA
// pipe the rate is clock x peak, so the sustained rate of each shape is its clock under the same power cap: a shape
// that sustains more TFLOP/s costs less energy per FLOP (tools/mfma_power.hip; docs/RESULTS.md round 5).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_power tools/mfma_power.hip
// Run:   tools/bin/mfma_power [launches] [iters per launch]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// SHAPE 0: v_mfma_f32_16x16x32_f16 (16384 FLOP), 8 accumulators; SHAPE 1: v_mfma_f32_32x32x16_f16 (32768 FLOP),
// 4 accumulators: the same FLOPs per step and the same operand registers read per FLOP.
template <int SHAPE>
__global__ __launch_bounds__(256) void mfma_burn(const _Float16* __restrict__ src, float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  f16x8_t a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[i][e] = src[(lane * 8 + e + 97 * i) & 4095];
      b[i][e] = src[(lane * 8 + e + 389 * i + 2048) & 4095];
    }
  float s = 0.f;
  if constexpr (SHAPE == 0) {
    f32x4_t acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; it += 4) {   // operand rotation unrolled: compile-time register indices
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(j + u) & 3], b[((j >> 1) + u) & 3], acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
  } else if constexpr (SHAPE == 2) {
    // 16x16x32 with the four-wave GEMM's LDS traffic: per 8 MFMAs two 16-byte fragment reads (8 A + 8 B reads per
    // 64 MFMAs of a 128x128 wave tile), each feeding the MFMAs of the next step
    __shared__ __attribute__((aligned(16))) _Float16 lds[256 * 8 * 8];
    for (int i = threadIdx.x; i < 256 * 8 * 8; i += 256) lds[i] = src[i & 4095];
    __syncthreads();
    f32x4_t acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const f16x8_t* L = (const f16x8_t*)lds;
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[(j + u) & 3], b[((j >> 1) + u) & 3], acc[j], 0, 0, 0);
        const int o = ((it + u) * 64 + threadIdx.x) & 2047;
        a[(u + 2) & 3] = L[o];
        b[(u + 2) & 3] = L[(o + 1024) & 2047];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
  } else {
    f32x16_t acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(j + u) & 3], b[(j + 1 + u) & 3], acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][15];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int SHAPE>
static void run(const _Float16* src, float* out, int grid, int launches, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double flop_per_launch = (double)grid * 4 /*waves*/ * iters * 131072.0;   // 8 x 16384 = 4 x 32768 per step
  double sum = 0.0;
  std::vector<double> tf;
  for (int l = 0; l < launches; ++l) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(mfma_burn<SHAPE>, dim3(grid), dim3(256), 0, 0, src, out, iters);
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double t = flop_per_launch / (ms * 1e-3) / 1e12;
    tf.push_back(t);
    sum += ms;
  }
  printf("{\"shape\": \"%s\", \"launches\": %d, \"ms_total\": %.1f, \"tflops_first\": %.1f, \"tflops_last\": %.1f, "
         "\"tflops_per_launch\": [",
         SHAPE == 0 ? "16x16x32_f16" : SHAPE == 2 ? "16x16x32_f16+lds_reads" : "32x32x16_f16", launches, sum,
         tf.front(), tf.back());
  for (size_t i = 0; i < tf.size(); ++i) printf("%s%.1f", i ? ", " : "", tf[i]);
  printf("]}\n");
  fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 40;
  const int iters = argc > 2 ? atoi(argv[2]) : 200000;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = cus * 2;   // two 4-wave workgroups per CU: two waves per SIMD keep the MFMA pipe full
  std::vector<_Float16> h(4096);
  unsigned x = 12345u;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (_Float16)(((int)(x >> 9) % 2001 - 1000) / 1000.0f);
  }
  _Float16* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * sizeof(_Float16)));
  CHECK(hipMalloc(&out, (size_t)grid * 256 * sizeof(float)));
  CHECK(hipMemcpy(src, h.data(), h.size() * sizeof(_Float16), hipMemcpyHostToDevice));
  // alternate the shapes twice, so that neither always runs on the cooler chip
  run<0>(src, out, grid, launches, iters);
  run<1>(src, out, grid, launches, iters);
  run<2>(src, out, grid, launches, iters);
  run<0>(src, out, grid, launches, iters);
  run<1>(src, out, grid, launches, iters);
  run<2>(src, out, grid, launches, iters);
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
