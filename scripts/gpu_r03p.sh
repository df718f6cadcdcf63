# fp32 K from the QKV GEMM only where the importance scorers read it (EDGE_QKV_K32=1 = the previous behaviour), and
# the four-wave GEMMs' start stagger (EDGE_TUNING=1 EDGE_GEMM_STAGGER=k, default off): GEMM probe timings, all GPU
# tests, same-box bench A/B/C, kernel profile.
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
ST="env EDGE_TUNING=1 EDGE_GEMM_STAGGER"
for op in gateup down qkv; do
  for r in 1 2; do
    for k in 0 4 8; do
      TAIL=1 step ${op}_st${k}_$r 120 $ST=$k python tools/kernel_probe.py --op $op --kv-planes 1 --iters 30 || exit $?
    done
  done
done
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for i in 1 2; do
  TAIL=1 step ab_new_$i 300 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/ab_new_$i.json || exit $?
  TAIL=1 step ab_k32_$i 300 env EDGE_QKV_K32=1 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/ab_k32_$i.json || exit $?
  TAIL=1 step ab_st8_$i 300 $ST=8 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/ab_st8_$i.json || exit $?
done
TAIL=1 step bench 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/bench.json || exit $?
exit 0
