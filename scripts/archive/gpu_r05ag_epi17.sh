# Round 5: the AttnLRP dm-rule epilogue (EPI_H3_LRP_SWIGLU) with 16-byte plane stores (gate / up halves exchanged
# between lanes) written nontemporal, against the same with plain stores (build/probe/libedge_kernels_plain.so) and
# the 8-byte-store HEAD (build/probe/libedge_kernels_head.so): bit-identical outputs, the fused GEMM per call, the
# fp32 AttnLRP, interleaved; then the LRP tests.
set -o pipefail
O=gpurun_out/${OUT:-r05ag}
mkdir -p $O
T=${TMPDIR:-/tmp}
P=$PWD/build/probe
timeout -k 10 120 env EDGE_KERNEL_LIB=$P/libedge_kernels_head.so python tools/kernel_probe.py --op lrpmlp --iters 1 --save $T/m.pt > $O/save.log 2>&1 || { tail -5 $O/save.log; exit 1; }
for v in new plain; do
  if [ $v = new ]; then L=""; else L=$P/libedge_kernels_$v.so; fi
  EDGE_KERNEL_LIB=$L timeout -k 10 120 python tools/kernel_probe.py --op lrpmlp --iters 1 --compare $T/m.pt > $O/cmp_$v.log 2>&1 || { tail -5 $O/cmp_$v.log; exit 1; }
  grep bit_identical $O/cmp_$v.log | sed "s/^/$v /" >> $O/bitexact.log
done
rm -f $T/m.pt
cat $O/bitexact.log
for r in 1 2; do
  for v in head plain new; do
    if [ $v = new ]; then L=""; else L=$P/libedge_kernels_$v.so; fi
    EDGE_KERNEL_LIB=$L timeout -k 10 120 python tools/kernel_probe.py --op lrpmlp --iters 12 2>/dev/null | sed "s/^/$v /" >> $O/probe.log || exit 1
    EDGE_KERNEL_LIB=$L timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $O/lrp_${v}_$r.json > $O/lrp_${v}_$r.log 2>&1 || { tail -5 $O/lrp_${v}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/lrp_${v}_$r.json')); print('$v lrp fp32', d['tokens_per_s'])"
  done
done
cat $O/probe.log
timeout -k 10 500 python -u -m pytest tests/test_lrp_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
exit 0
