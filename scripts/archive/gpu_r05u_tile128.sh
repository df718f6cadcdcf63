# Round 5: two workgroups per CU (two waves per SIMD, the 128x128 kernel: one wave's epilogue can overlap the other's
# MFMAs) against the one-wave-per-SIMD 256x256 persistent kernel on the bench's gate/up + SwiGLU and down + residual.
set -o pipefail
O=gpurun_out/${OUT:-r05u}
mkdir -p $O
for r in 1 2; do
  for op in gateup down; do
    for t in 0 128; do
      timeout -k 10 120 python tools/kernel_probe.py --op $op --tile $t --iters 12 2>/dev/null >> $O/probe.log || exit 1
    done
  done
done
cat $O/probe.log
exit 0
