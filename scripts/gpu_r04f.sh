# Round 4: (1) fp32 AttnLRP attention backward on bf16 planes (x6): tests vs fp64, equivariance, full-size table;
# throughput x6 vs f32 MFMA at 64 windows, kernel profile.  (2) bf16 regression cause (bisect: 81fc4b5, the graph
# capture with the collector off): same-box A/B of the collector during capture, fp32 + bf16.
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_lrp_gpu.py -k "lrp_attn_bwd or calibration_table" > $O/test_lrp.log 2>&1 \
  || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for x in 1 0 1; do
  EDGE_TUNING=1 EDGE_LRP_ATTN_X6=$x timeout -k 10 240 python tools/relevance_bench.py --dtype fp32 --batch 64 \
    --json-out $O/relevance_fp32_b64_x6$x.json > $O/relevance_fp32_b64_x6$x.log 2>&1 \
    || { echo "relevance bench failed"; tail -20 $O/relevance_fp32_b64_x6$x.log; exit 1; }
  echo "x6=$x $(tail -1 $O/relevance_fp32_b64_x6$x.log | cut -c1-200)"
done
for i in 1 2; do
  for gc in 1 0; do
    EDGE_TUNING=1 EDGE_GRAPH_GC_OFF=$gc timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights \
      --json-out $O/gc${gc}_$i.json > $O/gc${gc}_$i.log 2>&1 || { echo "bench gc$gc failed"; tail -20 $O/gc${gc}_$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/gc${gc}_$i.json')); print('gc_off=$gc $i', d['value'], d['value_bf16'])"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/lrp_prof -o run -- \
  python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 --iters 3 --warmup 1 > $R/$O/lrp_prof.log 2>&1 \
  || { echo "lrp profile failed"; tail -20 $R/$O/lrp_prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls $O/lrp_prof/*kernel_stats.csv $O/lrp_prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "fp32 AttnLRP (x6 attention backward), Qwen2-0.5B, 64 windows x 512" > $O/lrp_kernel_stats.md || true
head -30 $O/lrp_kernel_stats.md
exit 0
