set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "flash or models or importance" > gpurun_out/pytest_attn.log 2>&1; rc=$?
echo "[pytest] rc=$rc"; tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_bench.py --rounds 3 > gpurun_out/attn_bench.log 2>&1; rc=$?
echo "[attn_bench] rc=$rc"; grep -v amdgpu gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 3 4; do
  EDGE_ATTN_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_a$v.log 2>&1 || { tail gpurun_out/bench_a$v.log; exit 1; }
  echo "attn=$v $(grep -o '"value": [0-9.]*' gpurun_out/bench_a$v.log) $(grep -o '"ppl_random_weights": [0-9.]*' gpurun_out/bench_a$v.log)"
done; done
