set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "flash or importance" --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "[pytest_attn] rc=$rc"; tail -4 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?; echo "[attn_bench] rc=$rc"; tail -2 gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo "[bench] rc=$rc"; tail -1 gpurun_out/bench.log
