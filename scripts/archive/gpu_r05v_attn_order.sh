# Round 5: the fp32 attention forward with its MFMAs issued product-major over the four independent accumulators
# (no MFMA waits on the previous one's result) against the HEAD build (build/ab_attn/libedge_kernels_head.so):
# bit-identical outputs, time per call interleaved, then the fp32 GPU tests and the bench.
set -o pipefail
O=gpurun_out/${OUT:-r05v}
mkdir -p $O
HEAD_LIB=$PWD/build/ab_attn/libedge_kernels_head.so
T=${TMPDIR:-/tmp}
for kv in 1 0; do
  timeout -k 10 120 env EDGE_KERNEL_LIB=$HEAD_LIB python tools/kernel_probe.py --op attn --kv-planes $kv --iters 2 --save $T/attn_head_$kv.pt > $O/save_$kv.log 2>&1 || { tail -5 $O/save_$kv.log; exit 1; }
  timeout -k 10 120 python tools/kernel_probe.py --op attn --kv-planes $kv --iters 2 --compare $T/attn_head_$kv.pt > $O/cmp_$kv.log 2>&1 || { tail -5 $O/cmp_$kv.log; exit 1; }
  grep bit_identical $O/cmp_$kv.log >> $O/bitexact.log
  rm -f $T/attn_head_$kv.pt
done
cat $O/bitexact.log
for r in 1 2 3; do
  timeout -k 10 120 env EDGE_KERNEL_LIB=$HEAD_LIB python tools/kernel_probe.py --op attn --kv-planes 1 --iters 20 2>/dev/null | sed "s/^/head /" >> $O/probe.log || exit 1
  timeout -k 10 120 python tools/kernel_probe.py --op attn --kv-planes 1 --iters 20 2>/dev/null | sed "s/^/new  /" >> $O/probe.log || exit 1
done
cat $O/probe.log
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_f32.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_f32.log; exit 1; }
tail -1 $O/pytest_f32.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32-weights --no-hf-compare --json-out $O/bench.json > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d.get('value_bf16'))"
exit 0
