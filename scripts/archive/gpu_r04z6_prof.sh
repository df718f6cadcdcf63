# Round 4 end, rebuilt tree: kernel profiles (rocprofv3 --kernel-trace --stats) of the fp32 bench step and of the fp32
# AttnLRP engine at the 64-window benchmark size.
set -o pipefail
O=gpurun_out/r04z6
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/bench_prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-bf16 --no-fp32-weights --no-hf-compare > $R/$O/bench_prof.log 2>&1 \
  || { echo "bench profile failed"; tail -20 $R/$O/bench_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/lrp_prof -o run -- \
  python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 > $R/$O/lrp_prof.log 2>&1 \
  || { echo "lrp profile failed"; tail -20 $R/$O/lrp_prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls $O/bench_prof/*kernel_stats.csv $O/bench_prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "fp32 bench step, round-4 end (Qwen2-0.5B 2-stage split, 64-window micro-batches)" > $O/bench_kernel_stats.md || true
python tools/prof_summary.py $(ls $O/lrp_prof/*kernel_stats.csv $O/lrp_prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "fp32 AttnLRP, round-4 end, Qwen2-0.5B, 64 windows x 512" > $O/lrp_kernel_stats.md || true
head -14 $O/bench_kernel_stats.md
head -24 $O/lrp_kernel_stats.md
exit 0
