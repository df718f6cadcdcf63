set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -q -x -k "gemm or qkv or tiny or graph or ssq or fused" > gpurun_out/pytest_quick.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py --rounds 3 --iters 10 --only qkv --no-lib 2>&1 | grep -v amdgpu
for cfg in "--batch 32 --microbatches 4" "--batch 64 --microbatches 2" "--batch 16 --microbatches 8"; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 $cfg > gpurun_out/bq.log 2>&1 || { tail gpurun_out/bq.log; exit 1; }
  echo "$cfg: $(grep -o '"value": [0-9.]*' gpurun_out/bq.log)"
done
