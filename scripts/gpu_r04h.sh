# Round 4: (1) LRP: column-scaled transposed GEMMs (two products) + the prefetching x6 attention backward: tests, then
# throughput x6 vs f32 MFMA at 64 windows and a kernel profile; (2) the graph-capture collector A/B (bf16 regression).
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_f32_gpu.py -k "colscale" > $O/test_colscale.log 2>&1 || { echo "colscale tests failed"; tail -30 $O/test_colscale.log; exit 1; }
tail -1 $O/test_colscale.log
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for x in 1 0 1; do
  EDGE_TUNING=1 EDGE_LRP_ATTN_X6=$x timeout -k 10 240 python tools/relevance_bench.py --dtype fp32 --batch 64 \
    --json-out $O/relevance_fp32_b64_x6$x.json > $O/relevance_fp32_b64_x6$x.log 2>&1 \
    || { echo "relevance bench failed"; tail -20 $O/relevance_fp32_b64_x6$x.log; exit 1; }
  python -c "import json; d=json.load(open('$O/relevance_fp32_b64_x6$x.json')); print('x6=$x', d['tokens_per_s'], d['ms_per_batch'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/lrp_prof -o run -- \
  python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 --iters 3 --warmup 1 > $R/$O/lrp_prof.log 2>&1 \
  || { echo "lrp profile failed"; tail -20 $R/$O/lrp_prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls $O/lrp_prof/*kernel_stats.csv $O/lrp_prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "fp32 AttnLRP (x6 attention backward, column-scaled two-product transposes), Qwen2-0.5B, 64 windows x 512" \
  > $O/lrp_kernel_stats.md || true
head -16 $O/lrp_kernel_stats.md
for i in 1 2 3; do
  for v in A B C; do
    case $v in
      A) envs="EDGE_TUNING=1" ;;
      B) envs="EDGE_TUNING=1 EDGE_GRAPH_GC_COLLECT=0" ;;
      C) envs="EDGE_TUNING=1 EDGE_GRAPH_GC_COLLECT=0 EDGE_GRAPH_GC_OFF=0" ;;
    esac
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights --json-out $O/gc_$v$i.json \
      > $O/gc_$v$i.log 2>&1 || { echo "bench $v$i failed"; tail -20 $O/gc_$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/gc_$v$i.json')); print('gc $v$i', d['value'], d['value_bf16'])"
  done
done
exit 0
