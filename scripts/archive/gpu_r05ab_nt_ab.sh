# Round 5: nontemporal stores for the SwiGLU planes (and the AttnLRP forward's raw pre-activations) - end to end:
# the driver-argument bench and the fp32 AttnLRP, HEAD build (build/probe/libedge_kernels_head.so) vs this tree,
# interleaved twice; then the fp32 / LRP GPU tests.
set -o pipefail
O=gpurun_out/${OUT:-r05ab}
mkdir -p $O
HL=$PWD/build/probe/libedge_kernels_head.so
for r in 1 2; do
  for v in head new; do
    if [ $v = head ]; then L=$HL; else L=""; fi
    EDGE_KERNEL_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32-weights --no-hf-compare \
      --json-out $O/bench_${v}_$r.json > $O/bench_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_${v}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v bench', d['value'], d.get('value_bf16'))"
    EDGE_KERNEL_LIB=$L timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $O/lrp_${v}_$r.json \
      > $O/lrp_${v}_$r.log 2>&1 || { echo "lrp $v failed"; tail -5 $O/lrp_${v}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/lrp_${v}_$r.json')); print('$v lrp fp32', d['tokens_per_s'])"
  done
done
timeout -k 10 500 python -u -m pytest tests/test_f32_gpu.py tests/test_lrp_gpu.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
exit 0
