# Pair splits on v_fma_mix in every h3-plane epilogue: bit-identity and timing vs the base build (build/base);
# all GPU tests; bench; same-box bench A/B against the base build; kernel profile.
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
BASE="env EDGE_KERNEL_LIB=$PWD/build/base/libedge_kernels.so"
for op in gateup qkv norm attn; do
  P="python tools/kernel_probe.py --op $op --kv-planes 1 --iters 30"
  step ${op}_base_save 120 $BASE $P --save /tmp/${op}_base.pt || exit $?
  TAIL=2 step ${op}_new_cmp 120 $P --compare /tmp/${op}_base.pt || exit $?
  for r in 1 2; do
    TAIL=1 step ${op}_base_$r 120 $BASE $P || exit $?
    TAIL=1 step ${op}_new_$r 120 $P || exit $?
  done
  rm -f /tmp/${op}_base.pt
done
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
TAIL=1 step bench 300 python bench.py --steps 10 --warmup 3 --json-out gpurun_out/bench.json || exit $?
AB_LIB=build/base/libedge_kernels.so TAIL=8 step ab 900 bash scripts/gpu_ab.sh || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 2 --no-bf16 --no-fp32-weights > $R/gpurun_out/prof.log 2>&1); rc=$?
echo "[prof] rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py "$f" "bench fp32 N=1" > gpurun_out/prof_summary.md && head -14 gpurun_out/prof_summary.md
t=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python tools/trace_gaps.py "$t" --last-ms 130 --top 10 > gpurun_out/trace_gaps.md; rm -f "$t"
exit 0
