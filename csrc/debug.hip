// Debug-only kernels (never launched unless EDGE_POISON=2, see utils/poison.py).
//
// lds_poison_kernel: fills the whole LDS of every CU and the whole register file of every SIMD (256 VGPRs + 256
// AGPRs per lane) with all-ones bits - NaN as fp32, fp16 and bf16 - and exits.  Launched on the current stream right
// before every framework kernel, it makes a kernel that reads LDS or a register it never wrote for this workgroup see
// NaN deterministically, instead of whatever an earlier workgroup (of this process, or of another process sharing the
// GPU) happened to leave there.  Neither LDS nor registers are cleared between workgroups by the hardware.
#include "common.h"

constexpr int POISON_T = 256;

#define A8(n) "a" #n "0", "a" #n "1", "a" #n "2", "a" #n "3", "a" #n "4", "a" #n "5", "a" #n "6", "a" #n "7"

__global__ __launch_bounds__(POISON_T) void lds_poison_kernel(int lds_words) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < lds_words; i += POISON_T) lds[i] = 0xFFFFFFFFu;
  // every AGPR: v_accvgpr_write of all-ones; the clobber list makes the allocator give this wave all 256
  uint32_t ones = 0xFFFFFFFFu;
  asm volatile(
      ".irp n, 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31\n\t"
      "v_accvgpr_write_b32 a\\n, %0\n\t"
      "v_accvgpr_write_b32 a[\\n+32], %0\n\t"
      "v_accvgpr_write_b32 a[\\n+64], %0\n\t"
      "v_accvgpr_write_b32 a[\\n+96], %0\n\t"
      "v_accvgpr_write_b32 a[\\n+128], %0\n\t"
      "v_accvgpr_write_b32 a[\\n+160], %0\n\t"
      "v_accvgpr_write_b32 a[\\n+192], %0\n\t"
      "v_accvgpr_write_b32 a[\\n+224], %0\n\t"
      ".endr"
      :
      : "v"(ones)
      : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a255", "memory");
  // every VGPR above the few this kernel needs: v_mov of all-ones
  asm volatile(
      ".irp n, 8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31\n\t"
      "v_mov_b32 v\\n, -1\n\t"
      "v_mov_b32 v[\\n+24], -1\n\t"
      "v_mov_b32 v[\\n+48], -1\n\t"
      "v_mov_b32 v[\\n+72], -1\n\t"
      "v_mov_b32 v[\\n+96], -1\n\t"
      "v_mov_b32 v[\\n+120], -1\n\t"
      "v_mov_b32 v[\\n+144], -1\n\t"
      "v_mov_b32 v[\\n+168], -1\n\t"
      "v_mov_b32 v[\\n+192], -1\n\t"
      "v_mov_b32 v[\\n+216], -1\n\t"
      ".endr\n\t"
      "v_mov_b32 v240, -1\n\tv_mov_b32 v241, -1\n\tv_mov_b32 v242, -1\n\tv_mov_b32 v243, -1\n\t"
      "v_mov_b32 v244, -1\n\tv_mov_b32 v245, -1\n\tv_mov_b32 v246, -1\n\tv_mov_b32 v247, -1\n\t"
      "v_mov_b32 v248, -1\n\tv_mov_b32 v249, -1\n\tv_mov_b32 v250, -1\n\tv_mov_b32 v251, -1\n\t"
      "v_mov_b32 v252, -1\n\tv_mov_b32 v253, -1\n\tv_mov_b32 v254, -1\n\tv_mov_b32 v255, -1"
      :
      :
      : "v8", "v255", "memory");
}

static int g_poison_bytes = -1;

EDGE_API int edge_poison_lds(hipStream_t st) {
  if (g_poison_bytes < 0) {
    int dev = 0, lds = 65536;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
    if (lds <= 0) lds = 65536;
    if (hipFuncSetAttribute((const void*)lds_poison_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      lds = 65536;
    g_poison_bytes = lds;
  }
  // 8 workgroups per CU of 256 CUs, each filling the largest LDS allocation a workgroup can have
  hipLaunchKernelGGL(lds_poison_kernel, dim3(2048), dim3(POISON_T), g_poison_bytes, st, g_poison_bytes / 4);
  return (int)hipGetLastError();
}

EDGE_API int edge_poison_lds_bytes() { return g_poison_bytes; }
