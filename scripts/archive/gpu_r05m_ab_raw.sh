# Round 5: same-process-type A/B of the full-line raw pre-activation stores (AttnLRP forward gate/up) against the
# previous build (build/ab_raw/libedge_kernels_prev.so via EDGE_KERNEL_LIB), interleaved; the bench gate/up path too;
# then the raw-output test and the fp32 AttnLRP throughput of the new build.
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
PREV=$PWD/build/ab_raw/libedge_kernels_prev.so
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py tests/test_lrp_gpu.py -x -q \
  -k "swiglu_raw or qkv_kv_planes or engine_h3 or calibration" --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "tests failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for op in gateupraw gateup; do
    timeout -k 10 120 env EDGE_KERNEL_LIB=$PREV python tools/kernel_probe.py --op $op --iters 20 2>/dev/null | sed "s/^/prev /" >> $O/probe.log || exit 1
    timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 20 2>/dev/null | sed "s/^/new  /" >> $O/probe.log || exit 1
  done
done
cat $O/probe.log
timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $O/rel_fp32.json > $O/rel.log 2>&1 || { echo "relbench failed"; tail -5 $O/rel.log; exit 1; }
python -c "import json; d=json.load(open('$O/rel_fp32.json')); print('lrp fp32', d['tokens_per_s'])"
exit 0
