# Round 4: the bf16 AttnLRP engine with the last layer's O-proj / MLP on the seeded rows only (as the fp32 engine):
# LRP GPU tests, then same-box A/B against the unrestricted last layer (EDGE_TUNING=1 EDGE_LRP_LAST_ROWS=0), bf16 and
# fp32 engines, three interleaved rounds.
set -o pipefail
O=gpurun_out/r04z3
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for i in 1 2 3; do
  for dt in bf16 fp32; do
    for v in 0 1; do
      EDGE_TUNING=1 EDGE_LRP_LAST_ROWS=$v timeout -k 10 240 python tools/relevance_bench.py --dtype $dt --batch 64 \
        --json-out $O/rel_${dt}_lr$v$i.json > $O/rel_${dt}_lr$v$i.log 2>&1 || { echo "bench $dt $v $i failed"; tail -20 $O/rel_${dt}_lr$v$i.log; exit 1; }
      python -c "import json; d=json.load(open('$O/rel_${dt}_lr$v$i.json')); print('$dt last_rows=$v $i', d['tokens_per_s'], d['ms_per_batch'])"
    done
  done
done
exit 0
