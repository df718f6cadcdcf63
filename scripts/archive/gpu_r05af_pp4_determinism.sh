# Round 5: determinism of the 4-rank shared-GPU pipeline (the rehearsal test's pp4 case failed once: 509.05 vs
# 503.23): the local pp4 and the 4-rank pp4 bench (tiny-qwen2, the test's arguments), three times each, PPL printed.
set -o pipefail
O=gpurun_out/${OUT:-r05af}
mkdir -p $O
A="bench.py --model tiny-qwen2 --batch 4 --microbatches 2 --steps 3 --warmup 1 --max-length 256 --split 1 --pp 4"
export EDGE_SHARED_GPU=1
for r in 1 2 3; do
  timeout -k 10 200 python $A > $O/local_$r.log 2>&1 || { echo "local failed"; tail -5 $O/local_$r.log; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/local_$r.log') if l.startswith('{')][-1]; print('local', d['ppl_random_weights'], d.get('ppl_random_weights_bf16'))"
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port $((29600 + r)) \
    $A --gpus 4 > $O/four_$r.log 2>&1 || { echo "four failed"; tail -5 $O/four_$r.log; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/four_$r.log') if l.startswith('{')][-1]; print('four ', d['ppl_random_weights'], d.get('ppl_random_weights_bf16'))"
done
exit 0
