# Round 5: the GPU suite on the pruned kernel set (one variant per op), then the driver-argument bench.
set -o pipefail
O=gpurun_out/${OUT:-r05b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['value_bf16'], d['value_fp32_weights'], d.get('vs_same_node_reference_batch1'))"
if [ "${PROF:-0}" = 1 ]; then
  R=$PWD
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/bench_prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-bf16 --no-fp32-weights --no-hf-compare > $R/$O/bench_prof.log 2>&1) \
    || { echo "prof failed"; tail -5 $O/bench_prof.log; exit 1; }
  python tools/prof_summary.py $(ls $O/bench_prof/*kernel_stats.csv $O/bench_prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
    "fp32 bench step, round 5 (Qwen2-0.5B 2-stage split, 64-window micro-batches)" > $O/bench_kernel_stats.md || true
  head -14 $O/bench_kernel_stats.md
fi
exit 0
