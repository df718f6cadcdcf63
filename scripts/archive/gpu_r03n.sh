# fp32 attention probability split on v_fma_mix + raw row max, QKV V^T planes by quad-transposed 8-byte stores:
# bit-identity and timing vs the HEAD build (build/base); fp32 GPU tests; QKV epilogue ablations (tuning build).
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
BASE="env EDGE_KERNEL_LIB=$PWD/build/base/libedge_kernels.so"
for op in attn qkv; do
  P="python tools/kernel_probe.py --op $op --kv-planes 1 --iters 50"
  step ${op}_base_save 120 $BASE $P --save gpurun_out/${op}_base.pt || exit $?
  step ${op}_new_cmp 120 $P --compare gpurun_out/${op}_base.pt || exit $?
  for r in 1 2 3; do
    TAIL=1 step ${op}_base_$r 120 $BASE $P || exit $?
    TAIL=1 step ${op}_new_$r 120 $P || exit $?
  done
done
step pytest_f32 900 python -u -m pytest tests/test_f32_gpu.py tests/test_kernels_gpu.py tests/test_fidelity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
TAIL=12 step qkv_ablation 300 env EDGE_KERNEL_LIB=$PWD/build/tuning/libedge_kernels.so python tools/gemm_bench.py --no-lib --rounds 5 --only h3_2t_qkv_rope_kvp_b64 --tiles 0,0/noepi,0/nostore,0/novp || exit $?
TAIL=1 step bench 300 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --json-out gpurun_out/bench.json || exit $?
rm -f gpurun_out/*.pt
exit 0
