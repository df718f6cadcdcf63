# Round 5: the share of the epilogue in the bench's two big fp32 GEMMs (gate/up + SwiGLU planes, down + fp32
# residual): the production build against a probe build whose 4W epilogues return before any load or store
# (build/probe/libedge_kernels_noepi_all.so, -DEDGE_PROBE_NOEPI_ALL on a scratch copy; not in the committed tree).
set -o pipefail
O=gpurun_out/${OUT:-r05s}
mkdir -p $O
for r in 1 2; do
  for op in gateup down; do
    timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 12 2>/dev/null | sed "s/^/prod  /" >> $O/probe.log || exit 1
    timeout -k 10 120 env EDGE_KERNEL_LIB=$PWD/build/probe/libedge_kernels_noepi_all.so python tools/kernel_probe.py --op $op --iters 12 2>/dev/null | sed "s/^/noepi /" >> $O/probe.log || exit 1
  done
done
cat $O/probe.log
exit 0
