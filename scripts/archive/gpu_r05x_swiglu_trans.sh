# Round 5: the SwiGLU epilogue's transcendentals: probe builds (scratch copies of gemm.hip, macros not committed)
# with the exp2 / rcp replaced by plain VALU (NOTRANS: wrong values, the cost bound) and with one rcp per output pair
# (ONERCP: 1 / (e0 e1) shared), against production; gate/up at the bench shape, sustained, interleaved.
set -o pipefail
O=gpurun_out/${OUT:-r05x}
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 120 python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/prod    /" >> $O/probe.log || exit 1
  for v in NOTRANS ONERCP; do
    timeout -k 10 120 env EDGE_KERNEL_LIB=$PWD/build/probe/libedge_kernels_$v.so python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/$v /" >> $O/probe.log || exit 1
  done
done
cat $O/probe.log
exit 0
