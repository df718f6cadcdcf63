# Round 5: nontemporal stores on the remaining streams larger than the Infinity Cache - the AttnLRP dm rule's planes
# (637 MB), the bf16 SwiGLU output (318 MB) and the bf16 AttnLRP raw pre-activations (637 MB): HEAD build
# (build/probe/libedge_kernels_head.so) vs this tree, bench (fp32 + bf16) and AttnLRP fp32 / bf16, interleaved twice;
# then the GPU suite.
set -o pipefail
O=gpurun_out/${OUT:-r05ad}
mkdir -p $O
HL=$PWD/build/probe/libedge_kernels_head.so
for r in 1 2; do
  for v in head new; do
    if [ $v = head ]; then L=$HL; else L=""; fi
    EDGE_KERNEL_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32-weights --no-hf-compare \
      --json-out $O/bench_${v}_$r.json > $O/bench_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_${v}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v bench', d['value'], d.get('value_bf16'))"
    for dt in fp32 bf16; do
      EDGE_KERNEL_LIB=$L timeout -k 10 300 python tools/relevance_bench.py --dtype $dt --batch 64 --json-out $O/lrp_${dt}_${v}_$r.json \
        > $O/lrp_${dt}_${v}_$r.log 2>&1 || { echo "lrp $v failed"; tail -5 $O/lrp_${dt}_${v}_$r.log; exit 1; }
      python -c "import json; d=json.load(open('$O/lrp_${dt}_${v}_$r.json')); print('$v lrp $dt', d['tokens_per_s'])"
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
exit 0
