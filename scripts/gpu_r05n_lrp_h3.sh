# Round 5: the AttnLRP attention backward on scaled fp16 planes (h3) - tests against fp64 / autograd, the full-Qwen2
# table against CPU fp32, the sweeps' time (the x6 A/B: profiles/r05/lrp_attn_h3/probe.log) and the fp32 AttnLRP throughput.
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_lrp_gpu.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_lrp.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_lrp.log; exit 1; }
tail -1 $O/pytest_lrp.log
for r in 1 2; do
  for op in lrpattn; do
    timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 10 2>/dev/null >> $O/probe.log || exit 1
  done
done
cat $O/probe.log
timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $O/rel_fp32.json > $O/rel.log 2>&1 || { echo "relbench failed"; tail -5 $O/rel.log; exit 1; }
python -c "import json; d=json.load(open('$O/rel_fp32.json')); print('lrp fp32', d['tokens_per_s'])"
exit 0
