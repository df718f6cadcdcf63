# Round 5 end-of-round check: smoke(), the whole GPU suite, the driver-argument bench, and a same-box A/B of the bench
# and the fp32 AttnLRP against the round-4 tree (ab_r04/, a worktree of its last commit with its own build).
set -o pipefail
O=gpurun_out/${OUT:-r05_final}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 180 python -c "import time, __graft_entry__ as g; t=time.time(); g.smoke(); print('smoke s', round(time.time()-t, 1))" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['value_bf16'], d['value_fp32_weights'], d.get('vs_same_node_reference_batch1'))"
if [ -d ab_r04 ]; then
  for t in r04 r05 r04 r05; do
    if [ $t = r04 ]; then D=$R/ab_r04; else D=$R; fi
    (cd $D && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32-weights --no-hf-compare \
      --json-out $R/$O/ab_bench_$t.json > $R/$O/ab_bench_$t.log 2>&1) || { echo "ab bench $t failed"; exit 1; }
    python -c "import json; d=json.load(open('$O/ab_bench_$t.json')); print('$t bench', d['value'], d.get('value_bf16'))"
    (cd $D && timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $R/$O/ab_lrp_$t.json \
      > $R/$O/ab_lrp_$t.log 2>&1) || { echo "ab lrp $t failed"; exit 1; }
    python -c "import json; d=json.load(open('$O/ab_lrp_$t.json')); print('$t lrp fp32', d['tokens_per_s'])"
  done
fi
exit 0
