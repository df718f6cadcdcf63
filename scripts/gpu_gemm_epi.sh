set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py tests/test_lrp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -4 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py --rounds 3 --iters 10 --only gate_up_b64,down_b64,o_proj_b64,qkv > gpurun_out/gemm_bench.log 2>&1; rc=$?; echo "[gemm_bench] rc=$rc"; grep -v amdgpu gpurun_out/gemm_bench.log | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo "[bench] rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench.log) $(grep -o '"ppl_random_weights": [0-9.]*' gpurun_out/bench.log)"; [ $rc -eq 0 ] || exit $rc
done
