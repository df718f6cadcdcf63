# Round 4: x6 AttnLRP attention backward with row-major staging only, transposed operands by ds_read_b64_tr_b16
# (the last layer on the seeded rows): tests, then throughput x6 vs f32 MFMA at 64 windows (interleaved) and a profile.
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_f32_gpu.py -k "swiglu_raw or colscale" > $O/test_raw.log 2>&1 || { echo "swiglu raw tests failed"; tail -30 $O/test_raw.log; exit 1; }
tail -1 $O/test_raw.log
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
  "fp32 AttnLRP (x6 attention backward, tr_b16 transposed reads), Qwen2-0.5B, 64 windows x 512" \
  > $O/lrp_kernel_stats.md || true
head -16 $O/lrp_kernel_stats.md
exit 0
