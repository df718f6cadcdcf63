# Full-size (Qwen2-0.5B, 64-window micro-batches) rehearsal of the driver's N-GPU bench launch on ONE GPU:
# EDGE_SHARED_GPU=1 puts every rank on cuda:0 over gloo with host-staged p2p (throughput is not meaningful).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
for n in 2 4; do
  EDGE_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2950$n bench.py --gpus $n --steps 3 --warmup 1 > gpurun_out/rehearse_$n.log 2>&1; rc=$?
  echo "[N=$n] rc=$rc"; grep "^{" gpurun_out/rehearse_$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','n_gpus','ms_per_step','ppl_random_weights')}, d['config']['parallelism'], d['config']['global_batch'])" || tail -20 gpurun_out/rehearse_$n.log
  [ $rc -eq 0 ] || exit $rc
done
