# One gpurun session: build, GPU tests, smoke, GEMM microbench, bench + profile.  Every GPU step has its own
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
if [ -n "$GEMM" ]; then step gemm_bench 300 python tools/gemm_bench.py --rounds 3 --iters 10 --tiles 128,256 || exit $?; fi
step bench 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/bench.json || exit $?
if [ -n "$PROF" ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1); echo "[prof] rc=$?"
fi
if [ -n "$SWEEP" ]; then step sweep_bench 600 python tools/sweep_bench.py --windows ${SWEEP_WINDOWS:-256} --batch 8 --json-out gpurun_out/sweep_bench.json || exit $?; fi
exit 0
