# Post-epilogue wait change of the four-wave GEMMs: GEMM timing vs the HEAD build (build/base) and the gate/up-only
# build (build/mid), all GPU tests,
# interleaved same-box bench A/B (A = in-tree, B = build/base).
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
G="python tools/gemm_bench.py --no-lib --rounds 5 --only h3_2t_gate_up_b64,h3_2t_down_b64,h3_2t_o_proj_b64,h3_gate_up_b64"
TAIL=12 step gemm_new1 300 $G || exit $?
TAIL=12 step gemm_base1 300 env EDGE_KERNEL_LIB=$PWD/build/base/libedge_kernels.so $G || exit $?
TAIL=12 step gemm_mid1 300 env EDGE_KERNEL_LIB=$PWD/build/mid/libedge_kernels.so $G || exit $?
TAIL=12 step gemm_new2 300 $G || exit $?
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
AB_LIB=build/base/libedge_kernels.so TAIL=8 step ab 900 bash scripts/gpu_ab.sh || exit $?
exit 0
