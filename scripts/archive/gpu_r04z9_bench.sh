# Round 4 end: two more bench runs with the driver's arguments on the rebuilt tree (box-to-box range of the headline).
set -o pipefail
O=gpurun_out/r04z9
mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench$i.json > $O/bench$i.log 2>&1 || { echo "bench $i failed"; tail -20 $O/bench$i.log; exit 1; }
  python -c "import json; d=json.load(open('$O/bench$i.json')); print($i, d['value'], d['value_bf16'], d.get('vs_same_node_reference_batch1'))"
done
exit 0
