# Full GPU test suite + N bench runs (A/B: set AB_ENV="VAR=0" to interleave a second configuration).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "[pytest gpu] rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$i.log 2>&1 || { tail gpurun_out/bench_$i.log; exit 1; }
  echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$i.log)"
  if [ -n "$AB_ENV" ]; then
    env $AB_ENV timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_ab_$i.log 2>&1 || { tail gpurun_out/bench_ab_$i.log; exit 1; }
    echo "bench [$AB_ENV]: $(grep -o '"value": [0-9.]*' gpurun_out/bench_ab_$i.log)"
  fi
done
