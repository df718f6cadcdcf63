# Session check: all GPU tests, smoke, one bench run, then the gate/up epilogue-burst stagger timing experiment.
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
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAIL=1 step bench_1 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/bench.json || exit $?
export EDGE_KERNEL_LIB=$GRAFT_REPO_ROOT/build/tuning/libedge_kernels.so
TAIL=40 step stagger 300 python tools/gemm_bench.py --no-lib --rounds 5 --only h3_2t_gate_up_b64,h3_2t_down_b64 \
  --tiles 0,0/st4,0/st8,0/st16,0/st24,0/sq8,0/sq16,0/noepi,0/nostore || exit $?
exit 0
