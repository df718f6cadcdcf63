set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_kernels_gpu.py -x -q -k "pipeline or flash or graph or sweep or ppl or scored" --timeout 120 --timeout-method thread > gpurun_out/pytest_e2e.log 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -4 gpurun_out/pytest_e2e.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo "[bench] rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
EDGE_LAST_LAYER_ALL_ROWS=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_full.log 2>&1; rc=$?; echo "[bench all-rows] rc=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
