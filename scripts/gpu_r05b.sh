# Round 5: the GPU suite on the pruned kernel set (one variant per op), then the driver-argument bench.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['value_bf16'], d['value_fp32_weights'], d.get('vs_same_node_reference_batch1'))"
exit 0
