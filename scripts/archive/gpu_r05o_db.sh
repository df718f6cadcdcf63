# Round 5: double-buffered fp16-plane AttnLRP sweeps vs the single-buffered build (build/ab_raw/libedge_kernels_prev.so
# via EDGE_KERNEL_LIB), interleaved; LRP tests; fp32 AttnLRP throughput.
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
PREV=$PWD/build/ab_raw/libedge_kernels_prev.so
timeout -k 10 500 python -u -m pytest tests/test_lrp_gpu.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_lrp.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_lrp.log; exit 1; }
tail -1 $O/pytest_lrp.log
for r in 1 2 3; do
  timeout -k 10 120 env EDGE_KERNEL_LIB=$PREV python tools/kernel_probe.py --op lrpattn --iters 10 2>/dev/null | sed "s/^/prev /" >> $O/probe.log || exit 1
  timeout -k 10 120 python tools/kernel_probe.py --op lrpattn --iters 10 2>/dev/null | sed "s/^/new  /" >> $O/probe.log || exit 1
done
cat $O/probe.log
timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $O/rel_fp32.json > $O/rel.log 2>&1 || { echo "relbench failed"; tail -5 $O/rel.log; exit 1; }
python -c "import json; d=json.load(open('$O/rel_fp32.json')); print('lrp fp32', d['tokens_per_s'])"
exit 0
