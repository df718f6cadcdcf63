# Pair splits on v_fma_mix in every h3-plane epilogue + the four-wave GEMMs' epilogue desync (odd workgroups start
# with half of their last tile): bit-identity vs the base build (build/base), timing base / new / new without the
# desync (EDGE_GEMM_SPLIT=0); all GPU tests; same-box bench A/B.
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
NOSPLIT="env EDGE_TUNING=1 EDGE_GEMM_SPLIT=0"
for op in gateup down qkv norm attn; do
  P="python tools/kernel_probe.py --op $op --kv-planes 1 --iters 30"
  step ${op}_base_save 120 $BASE $P --save /tmp/${op}_base.pt || exit $?
  TAIL=2 step ${op}_new_cmp 120 $P --compare /tmp/${op}_base.pt || exit $?
  for r in 1 2; do
    TAIL=1 step ${op}_base_$r 120 $BASE $P || exit $?
    TAIL=1 step ${op}_new_$r 120 $P || exit $?
    TAIL=1 step ${op}_nosplit_$r 120 $NOSPLIT $P || exit $?
  done
done
rm -f /tmp/*_base.pt
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
TAIL=1 step bench 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/bench.json || exit $?
AB_LIB=build/base/libedge_kernels.so TAIL=8 step ab 900 bash scripts/gpu_ab.sh || exit $?
exit 0
