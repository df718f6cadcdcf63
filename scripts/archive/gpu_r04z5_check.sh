# Round 4 re-entry check (rebuilt container): the whole GPU suite (one process per file, each under its own limit), smoke(), and the bench with the driver's arguments.
set -o pipefail
O=gpurun_out/r04z5
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu"
for f in tests/*gpu*.py; do
  n=$(basename $f .py)
  timeout -k 10 900 $T $f > $O/$n.log 2>&1 || { echo "$n failed"; tail -40 $O/$n.log; exit 1; }
  echo "$n: $(tail -1 $O/$n.log)"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for d in fp32 bf16; do
  timeout -k 10 240 python tools/relevance_bench.py --dtype $d --batch 64 --json-out $O/rel_$d.json > $O/rel_$d.log 2>&1 || { echo "relevance $d failed"; tail -20 $O/rel_$d.log; exit 1; }
  python -c "import json; d=json.load(open('$O/rel_$d.json')); print('relevance $d', d['tokens_per_s'], d['ms_per_batch'])"
done
exit 0
