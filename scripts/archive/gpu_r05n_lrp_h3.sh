# Round 5: the AttnLRP attention backward on scaled fp16 planes (h3) - tests against fp64 / autograd, the full-Qwen2
# table against CPU fp32, the sweeps' time (the x6 A/B: profiles/history/r05/lrp_attn_h3/probe.log) and the fp32 AttnLRP throughput.
set -o pipefail
O=gpurun_out/${OUT:-r05n}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_lrp_gpu.py tests/test_f32_gpu.py -x -q --timeout 300 --timeout-method thread \
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
if [ "${PROF:-0}" = 1 ]; then
  R=$PWD
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lrp -o run --output-format csv -- \
    python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 --iters 3 --warmup 1 > $R/$O/lrp_prof.log 2>&1) \
    || { echo "prof failed"; tail -5 $O/lrp_prof.log; exit 1; }
  python tools/prof_summary.py $(ls $O/prof_lrp/*kernel_stats.csv $O/prof_lrp/*/*kernel_stats.csv 2>/dev/null | head -1) \
    "fp32 AttnLRP, round 5 (h3 attention sweeps), Qwen2-0.5B, 64 windows x 512" > $O/lrp_kernel_stats.md || true
  head -30 $O/lrp_kernel_stats.md
fi
exit 0
