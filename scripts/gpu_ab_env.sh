# A/B an env var on bench.py: bash scripts/gpu_ab_env.sh VAR=value   (alternating runs, same box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
if [ -n "$TESTS" ]; then
  env $1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "[pytest with $1] rc=$rc"; tail -2 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab0.log 2>&1; rc=$?; echo "[base] rc=$rc $(grep -o '"value": [0-9.]*\|"ppl_random_weights": [0-9.]*' gpurun_out/ab0.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
  env $1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab1.log 2>&1; rc=$?; echo "[$1] rc=$rc $(grep -o '"value": [0-9.]*\|"ppl_random_weights": [0-9.]*' gpurun_out/ab1.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
