# Round 5: the SwiGLU epilogue without its stores (NOSTORE: every value computed, the stores predicated off by a
# condition no lane meets; scratch copy of gemm.hip, macro not committed) against production, gate/up sustained,
# interleaved; plus rocprofv3 PMC of both (MFMA busy, clock) in their own runs.
set -o pipefail
O=gpurun_out/${OUT:-r05y}
mkdir -p $O
NS=$PWD/build/probe/libedge_kernels_NOSTORE.so
for r in 1 2 3; do
  timeout -k 10 120 python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/prod    /" >> $O/probe.log || exit 1
  timeout -k 10 120 env EDGE_KERNEL_LIB=$NS python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/NOSTORE /" >> $O/probe.log || exit 1
done
cat $O/probe.log
exit 0
