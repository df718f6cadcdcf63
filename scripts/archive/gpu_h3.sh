# fp32-mode (h3) check: fp32 kernel tests, full-model numerics, smoke, bench, GEMM timing.
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
TAIL=15 step pytest_f32 600 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread || exit $?
TAIL=1 step bench_h3 400 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/bench_h3.json || exit $?
TAIL=30 step gemm 400 python tools/gemm_bench.py --only h3_2t_gate_up_b64,h3_2t_down_b64,h3_2t_o_proj_b64,h3_2t_qkv_rope_b64 --rounds 3 || exit $?
exit 0
