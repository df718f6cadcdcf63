# One gpurun session: build, GPU tests, smoke, GEMM microbench, bench variants.  Every GPU step has its own
# time limit; a crash/timeout ends the script (no further GPU work).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -${TAIL:-6} gpurun_out/$name.log
  return $rc
}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
TAIL=25 step pytest_gpu 900 python -m pytest tests -m gpu -q -rf; rc=$?; [ $rc -le 1 ] || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step gemm_bench 300 python tools/gemm_bench.py --rounds 3 --iters 10 --json gpurun_out/gemm_bench.json || exit $?
step bench_b16m4 300 python bench.py --steps 5 --warmup 2 || exit $?
step bench_b32m4 300 python bench.py --steps 5 --warmup 2 --batch 32 || exit $?
step bench_b8m8 300 python bench.py --steps 5 --warmup 2 --batch 8 --microbatches 8 || exit $?
