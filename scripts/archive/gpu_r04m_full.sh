# Round 4: the whole GPU suite (one process per file, each under its own limit), smoke(), and the 1-GPU bench.
set -o pipefail
O=gpurun_out/r04m
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
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
exit 0
