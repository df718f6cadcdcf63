# Round 4: bf16 QKV on the four-wave 256x192 tiles (EDGE_GEMM_QKV192_BF16=1) vs the 128x128 kernel (0): GPU tests, then
# the bf16 bench interleaved (EDGE_TUNING=1), three rounds, and a kernel profile of the 192 variant.
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "qkv" > $O/test_qkv.log 2>&1 || { echo "qkv tests failed"; tail -30 $O/test_qkv.log; exit 1; }
tail -1 $O/test_qkv.log
for i in 1 2 3; do
  for v in 0 1; do
    EDGE_TUNING=1 EDGE_GEMM_QKV192_BF16=$v timeout -k 10 300 python bench.py --dtype bf16 --steps 10 --warmup 3 --no-bf16 \
      --no-fp32-weights --json-out $O/bench_q$v$i.json > $O/bench_q$v$i.log 2>&1 || { echo "bench q$v$i failed"; tail -20 $O/bench_q$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_q$v$i.json')); print('qkv192_bf16=$v $i', d['value'], d['ms_per_step'])"
  done
done
cd /tmp
EDGE_TUNING=1 EDGE_GEMM_QKV192_BF16=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python3 $R/bench.py --dtype bf16 --steps 5 --warmup 2 --no-bf16 --no-fp32-weights > $R/$O/prof.log 2>&1 \
  || { echo "profile failed"; tail -20 $R/$O/prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "bf16 bench step, QKV on 256x192 four-wave tiles" > $O/kernel_stats.md || true
head -12 $O/kernel_stats.md
exit 0
