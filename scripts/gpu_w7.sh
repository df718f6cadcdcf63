# 256x224 GEMM: numerics, microbench vs the 256x256 kernels, end-to-end A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "w7 or fused_norm_and_ssq or gemm_inplace" > gpurun_out/pytest_w7.log 2>&1; rc=$?
echo "[pytest w7] rc=$rc"; tail -4 gpurun_out/pytest_w7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --rounds 5 --iters 10 --only down_b64,o_proj_b64 --tiles 0,256,256s > gpurun_out/gemm_w7.log 2>&1; rc=$?
echo "[gemm_bench] rc=$rc"; grep -v amdgpu gpurun_out/gemm_w7.log | tail -12; [ $rc -eq 0 ] || exit $rc
for w in 1 0 1 0; do
  EDGE_GEMM_W7=$w timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_w7_$w.log 2>&1 || { tail gpurun_out/bench_w7_$w.log; exit 1; }
  echo "W7=$w $(grep -o '"value": [0-9.]*' gpurun_out/bench_w7_$w.log) $(grep -o '"ppl_random_weights": [0-9.]*' gpurun_out/bench_w7_$w.log)"
done
