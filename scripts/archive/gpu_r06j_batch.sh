# Round 6: same-box A/B of the micro-batch size (windows per micro-batch) on the fp32 bench step: 64 (the default
# so far) against 96 and 128, interleaved twice.
set -o pipefail
O=gpurun_out/${OUT:-r06j}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in 64 128 96; do
    timeout -k 10 300 python bench.py --steps 12 --warmup 3 --batch $b --no-bf16 --no-fp32-weights --no-hf-compare \
      --no-sweep --json-out $O/bench_b${b}_$r.json > $O/bench_b${b}_$r.log 2>&1 \
      || { echo "bench b$b failed"; tail -5 $O/bench_b${b}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_b${b}_$r.json')); print('batch $b run $r', d['value'], d['ms_per_step'], d.get('box_calibration', {}).get('hipblaslt_fp16_tflops'))"
  done
done
exit 0
