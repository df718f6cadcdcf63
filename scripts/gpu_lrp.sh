# fp32 / bf16 AttnLRP engines: GPU tests + throughput
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
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
TAIL=12 step pytest_lrp 600 python -u -m pytest tests/test_lrp_gpu.py tests/test_f32_gpu.py tests/test_fidelity_gpu.py -x -v -s --timeout 300 --timeout-method thread -k "peaked or fidelity or lo_class or importance_stats or (lrp and (f32 or fp32 or h3))" || exit $?
TAIL=1 step relbench_fp32_b16 300 python tools/relevance_bench.py --dtype fp32 --batch 16 --json-out gpurun_out/relevance_bench_fp32_b16.json || exit $?
TAIL=1 step relbench_fp32_b64 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out gpurun_out/relevance_bench_fp32_b64.json || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_lrp -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/relevance_bench.py --dtype fp32 --batch 16 --iters 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_lrp.log 2>&1); echo "[prof] rc=$?"
exit 0
