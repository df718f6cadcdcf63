# Throughput of the reference's own sweep workloads at fp32 (its precision) on one GPU: the Qwen2-0.5B notebook sweep
# (tools/sweep_bench.py, 4 methods x 5 layers x 5 ratios per window) and the Pythia last_row / initial and Qwen2
# channel drivers through their entry points (synthetic tokens, random-init weights, windows/s in the JSON outputs).
set -o pipefail
mkdir -p gpurun_out/sweeps
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAIL:-2}
  return $rc
}
step sweep_fp32 400 python tools/sweep_bench.py --dtype fp32 --windows 256 --json-out gpurun_out/sweeps/sweep_bench_fp32.json || exit $?
step sweep_bf16 400 python tools/sweep_bench.py --dtype bf16 --windows 256 --json-out gpurun_out/sweeps/sweep_bench_bf16.json || exit $?
step pythia_last_row 400 python Experiments/Pythia-70M/main.py --params scripts/sweep_params/pythia_last_row.json --max-windows 512 || exit $?
step pythia_initial 400 python Experiments/Pythia-70M/main.py --params scripts/sweep_params/pythia_initial.json --max-windows 512 || exit $?
step qwen2_channel 400 python Experiments/Qwen2-0.5B/main.py --params scripts/sweep_params/qwen2_channel.json --max-windows 512 || exit $?
ls gpurun_out/sweeps
exit 0
