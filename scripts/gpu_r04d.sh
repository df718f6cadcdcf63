# Round 4: (1) desync as a compile-time kernel variant: bit-identity tests on the checked and production builds;
# (2) same-box bench A/B of the default path: HEAD build vs this build (fp32 + bf16);
# (3) bf16 regression bisect: bench --dtype bf16 from each round-3 tree, interleaved.
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
EDGE_KERNEL_LIB=$R/build/tuning/libedge_kernels.so timeout -k 10 300 $T tests/test_gemm_desync_gpu.py > $O/test_checked.log 2>&1 \
  || { echo "checked tests failed"; tail -30 $O/test_checked.log; exit 1; }
tail -1 $O/test_checked.log
timeout -k 10 300 $T tests/test_gemm_desync_gpu.py > $O/test_prod.log 2>&1 || { echo "prod tests failed"; tail -30 $O/test_prod.log; exit 1; }
tail -1 $O/test_prod.log
for i in 1 2; do
  for v in head new; do
    envs=""; [ $v = head ] && envs="EDGE_KERNEL_LIB=$R/build/ab_head/libedge_kernels.so"
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights --json-out $O/ab_${v}$i.json \
      > $O/ab_${v}$i.log 2>&1 || { echo "bench $v$i failed"; tail -20 $O/ab_${v}$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/ab_${v}$i.json')); print('ab $v$i', d['value'], d['value_bf16'])"
  done
done
for i in 1 2; do
  for t in 7a31976 82a69b0 b548016 81fc4b5 94ba5ac e675ad7 head; do
    d=$R/build/bisect/$t; [ $t = head ] && d=$R
    (cd $d && timeout -k 10 300 python bench.py --dtype bf16 --steps 10 --warmup 3 --no-fp32-weights \
      --json-out $R/$O/bisect_${t}_$i.json > $R/$O/bisect_${t}_$i.log 2>&1) \
      || { echo "bisect $t $i failed"; tail -20 $O/bisect_${t}_$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bisect_${t}_$i.json')); print('bisect $t $i', d['value'], d['ppl_random_weights'])"
  done
done
# (4) fp32 AttnLRP at the 64-window benchmark size: the bf16-plane (x6) attention backward tested against fp64,
# the full-size calibration table against the CPU, throughput x6 vs f32 MFMA, kernel profile
timeout -k 10 600 $T tests/test_lrp_gpu.py -k "lrp_attn_bwd or calibration_table" > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for x in 1 0 1; do
  EDGE_TUNING=1 EDGE_LRP_ATTN_X6=$x timeout -k 10 240 python tools/relevance_bench.py --dtype fp32 --batch 64 \
    --json-out $O/relevance_fp32_b64_x6$x.json > $O/relevance_fp32_b64_x6$x.log 2>&1 \
    || { echo "relevance bench failed"; tail -20 $O/relevance_fp32_b64_x6$x.log; exit 1; }
  echo "x6=$x $(tail -1 $O/relevance_fp32_b64_x6$x.log)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/lrp_prof -o run -- \
  python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 --iters 3 --warmup 1 > $R/$O/lrp_prof.log 2>&1 \
  || { echo "lrp profile failed"; tail -20 $R/$O/lrp_prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls $O/lrp_prof/*kernel_stats.csv $O/lrp_prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "fp32 AttnLRP, Qwen2-0.5B, 64 windows x 512" > $O/lrp_kernel_stats.md || true
head -20 $O/lrp_kernel_stats.md
exit 0
