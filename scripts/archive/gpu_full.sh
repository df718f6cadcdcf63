# Full round check: build, all GPU tests, smoke, bench x2, kernel profile, sweep bench, relevance bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAIL:-3}
  return $rc
}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAIL=1 step bench_1 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/bench.json || exit $?
TAIL=1 step bench_2 300 python bench.py --steps 10 --warmup 3 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1); echo "[prof] rc=$?"
TAIL=1 step sweep_bench 400 python tools/sweep_bench.py --windows 256 --batch 8 --json-out gpurun_out/sweep_bench.json || exit $?
TAIL=1 step relevance_bench 300 python tools/relevance_bench.py --batch 64 --json-out gpurun_out/relevance_bench_b64.json || exit $?
exit 0
