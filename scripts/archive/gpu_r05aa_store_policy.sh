# Round 5: the SwiGLU epilogue's plane stores with the nontemporal (nt) and the write-through (sc1) cache policies
# (probe builds from scratch copies of gemm.hip; macros not committed) against production: outputs bit-identical,
# gate/up sustained, interleaved.
set -o pipefail
O=gpurun_out/${OUT:-r05aa}
mkdir -p $O
T=${TMPDIR:-/tmp}
timeout -k 10 120 python tools/kernel_probe.py --op gateup --iters 1 --save $T/gu.pt > $O/save.log 2>&1 || { tail -5 $O/save.log; exit 1; }
for v in NT SC1; do
  timeout -k 10 120 env EDGE_KERNEL_LIB=$PWD/build/probe/libedge_kernels_$v.so python tools/kernel_probe.py --op gateup --iters 1 --compare $T/gu.pt > $O/cmp_$v.log 2>&1 || { tail -5 $O/cmp_$v.log; exit 1; }
  grep bit_identical $O/cmp_$v.log | sed "s/^/$v /" >> $O/bitexact.log
done
rm -f $T/gu.pt
cat $O/bitexact.log
for r in 1 2 3; do
  timeout -k 10 120 python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/prod /" >> $O/probe.log || exit 1
  for v in NT SC1; do
    timeout -k 10 120 env EDGE_KERNEL_LIB=$PWD/build/probe/libedge_kernels_$v.so python tools/kernel_probe.py --op gateup --iters 12 2>/dev/null | sed "s/^/$v  /" >> $O/probe.log || exit 1
  done
done
cat $O/probe.log
exit 0
