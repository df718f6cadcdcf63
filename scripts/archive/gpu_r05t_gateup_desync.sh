# Round 5: can the gate/up GEMM's epilogue (14 % of it under sustained load, scripts/gpu_r05s_gemm_epi.sh) be hidden?
# Probe builds from scratch copies of gemm.hip (macros not in the committed tree): RELAX - the first K-tile wait after
# the SwiGLU epilogue is vmcnt(32) (the DMA only) instead of vmcnt(0) (the epilogue's 32 stores too); DESYNC7 - odd
# workgroups start ~7 x 8128 cycles late, so the CUs' epilogues stop coinciding; both; and the no-epilogue bound.
set -o pipefail
O=gpurun_out/${OUT:-r05t}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/prod  /" >> $O/probe.log || exit 1
  for v in RELAX DESYNC7 RELAXDESYNC7 noepi_all; do
    timeout -k 10 120 env EDGE_KERNEL_LIB=$PWD/build/probe/libedge_kernels_$v.so python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/$v /" >> $O/probe.log || exit 1
  done
done
cat $O/probe.log
exit 0
