# Full-size (Qwen2-0.5B, 64-window micro-batches) rehearsal of the driver's N-GPU bench launch on ONE GPU:
# EDGE_SHARED_GPU=1 puts every rank on cuda:0 over gloo with host-staged p2p (throughput is not meaningful).
# Cases: N=2 (pp2), N=4 (pp2 x dp2), N=8 (pp2 x dp4) - the bench defaults the driver runs - and N=4 --pp 4 and
# N=8 --pp 8 (BASELINE configs 4-5).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 30; do date +%T >> gpurun_out/rehearse_heartbeat; done ) &   # long cases print nothing for minutes
HB=$!
trap "kill $HB 2>/dev/null" EXIT
run() {  # n extra-args...
  local n=$1; shift
  local tag=$n$(echo "$@" | tr -d ' -')
  EDGE_SHARED_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29$((500 + RANDOM % 400)) bench.py --gpus $n --steps 2 --warmup 1 --no-bf16 --no-fp32-weights "$@" > gpurun_out/rehearse_$tag.log 2>&1; local rc=$?
  echo "[N=$n $*] rc=$rc"; grep "^{" gpurun_out/rehearse_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','n_gpus','ms_per_step','ppl_random_weights')}, d['config']['parallelism'], d['config']['global_batch'], [(s['rank'], round(s.get('compute_ms', 0), 1)) for s in d.get('stages', [])])" || tail -20 gpurun_out/rehearse_$tag.log
  return $rc
}
run 2 && run 4 && run 8 && run 4 --pp 4 && run 8 --pp 8
