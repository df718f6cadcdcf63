# Iteration check: selected GPU tests (PYTEST_K), GEMM shapes (GEMM_ONLY, tile specs GEMM_TILES) and the fp32 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAIL:-4}
  return $rc
}
if [ -n "$PYTEST_K" ]; then
  step pytest_sel 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" || exit $?
fi
if [ -n "$GEMM_ONLY" ]; then
  TAIL=40 step gemm 300 python tools/gemm_bench.py --only "$GEMM_ONLY" --tiles "${GEMM_TILES:-0}" --rounds 3 || exit $?
fi
TAIL=1 step bench_fp32 300 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/bench_iter.json || exit $?
exit 0
