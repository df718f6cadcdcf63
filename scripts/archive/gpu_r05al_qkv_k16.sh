# Round 5: the fp32 QKV epilogue's K planes as 16-byte stores (lane exchange) against HEAD
# (build/probe/libedge_kernels_head.so): bit-identical outputs, time per call interleaved, then the fp32 tests.
set -o pipefail
O=gpurun_out/${OUT:-r05al}
mkdir -p $O
T=${TMPDIR:-/tmp}
HL=$PWD/build/probe/libedge_kernels_head.so
EDGE_KERNEL_LIB=$HL timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 1 --save $T/q.pt > $O/save.log 2>&1 || { tail -5 $O/save.log; exit 1; }
timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 1 --compare $T/q.pt > $O/cmp.log 2>&1 || { tail -5 $O/cmp.log; exit 1; }
rm -f $T/q.pt
grep bit_identical $O/cmp.log
for r in 1 2 3; do
  EDGE_KERNEL_LIB=$HL timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 200 2>/dev/null | sed "s/^/head /" >> $O/probe.log || exit 1
  timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 200 2>/dev/null | sed "s/^/new  /" >> $O/probe.log || exit 1
done
cat $O/probe.log
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
exit 0
