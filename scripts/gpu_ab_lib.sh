# A/B of two kernel-library builds on one box: the in-tree build vs _native/ab/libedge_kernels.so (EDGE_KERNEL_LIB),
# alternating bench.py runs; GPU kernel tests on the in-tree build first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB=$PWD/llm_inference_in_distributed_edge_networks_amd/_native/ab/libedge_kernels.so
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/pytest_ablib.log 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -2 gpurun_out/pytest_ablib.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_new.log 2>&1; rc=$?; echo "[new] rc=$rc $(grep -o '"value": [0-9.]*\|"ppl_random_weights": [0-9.]*' gpurun_out/ab_new.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
  EDGE_KERNEL_LIB=$AB timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_old.log 2>&1; rc=$?; echo "[old] rc=$rc $(grep -o '"value": [0-9.]*\|"ppl_random_weights": [0-9.]*' gpurun_out/ab_old.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
