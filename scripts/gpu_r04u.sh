# Round 4: fp32 AttnLRP dQ sweep from K / V pre-split into bf16 planes once per layer (x6_split_rows_kernel) vs split
# while staging: LRP GPU tests, then interleaved A/B in one tree (EDGE_LRP_KV_PRESPLIT=0/1), three rounds.
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for i in 1 2 3; do
  for v in 0 1; do
    EDGE_TUNING=1 EDGE_LRP_KV_PRESPLIT=$v timeout -k 10 240 python tools/relevance_bench.py --dtype fp32 --batch 64 \
      --json-out $O/rel_ps$v$i.json > $O/rel_ps$v$i.log 2>&1 || { echo "relevance bench ps$v$i failed"; tail -20 $O/rel_ps$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/rel_ps$v$i.json')); print('presplit=$v $i', d['tokens_per_s'], d['ms_per_batch'])"
  done
done
exit 0
