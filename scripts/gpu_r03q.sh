# KVP fp32 attention with four waves x two query tiles (EDGE_TUNING=1 EDGE_ATTN_RT2=1) against the eight-wave kernel:
# bit-identity, timing, the fp32 attention GPU tests under the new kernel, same-box bench A/B.
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
RT2="env EDGE_TUNING=1 EDGE_ATTN_RT2=1"
P="python tools/kernel_probe.py --op attn --kv-planes 1 --iters 50"
step attn_rt1_save 120 $P --save /tmp/attn_rt1.pt || exit $?
TAIL=2 step attn_rt2_cmp 120 $RT2 $P --compare /tmp/attn_rt1.pt || exit $?
rm -f /tmp/attn_rt1.pt
for r in 1 2 3; do
  TAIL=1 step attn_rt1_$r 120 $P || exit $?
  TAIL=1 step attn_rt2_$r 120 $RT2 $P || exit $?
done
step pytest_attn_rt2 600 $RT2 python -u -m pytest tests/test_f32_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
for i in 1 2; do
  TAIL=1 step ab_rt1_$i 300 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/ab_rt1_$i.json || exit $?
  TAIL=1 step ab_rt2_$i 300 $RT2 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/ab_rt2_$i.json || exit $?
done
exit 0
