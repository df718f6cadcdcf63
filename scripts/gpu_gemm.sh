set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -rf -k "gemm or qkv or head_nll or tiny or fused or ssq" > gpurun_out/pytest_gemm.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gemm.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py --rounds 3 --iters 10 --tiles ${TILES:-128,256,256r} --only ${SHAPES:-down_b64,o_proj_b64,gate_up_b64} > gpurun_out/gemm_bench2.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/gemm_bench2.log; exit $rc
