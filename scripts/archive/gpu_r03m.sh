# Session check after a fresh container rebuild: all GPU tests, smoke, bench, kernel profile of the fp32 bench,
# bf16 LRP engine error probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAIL:-3}
  return $rc
}
TAIL=8 step lrp_bf16_err 300 python tools/probes/lrp_bf16_err.py || exit $?
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAIL=1 step bench_1 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/bench.json || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 2 --no-bf16 --no-fp32-weights > $R/gpurun_out/prof.log 2>&1); rc=$?
echo "[prof] rc=$rc"; tail -2 gpurun_out/prof.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1); echo "$f"
python tools/prof_summary.py "$f" "bench fp32 N=1" > gpurun_out/prof_summary.md && head -24 gpurun_out/prof_summary.md
exit 0
