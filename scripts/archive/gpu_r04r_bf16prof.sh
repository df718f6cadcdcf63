# Round 4: kernel profile of the bf16 bench step (rocprofv3 --kernel-trace --stats), 5 steps.
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
  python3 $R/bench.py --dtype bf16 --steps 5 --warmup 2 --no-bf16 --no-fp32-weights > $R/$O/prof.log 2>&1 \
  || { echo "profile failed"; tail -20 $R/$O/prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "bf16 bench step (Qwen2-0.5B 2-stage split, 64-window micro-batches)" > $O/kernel_stats.md || true
head -24 $O/kernel_stats.md
exit 0
