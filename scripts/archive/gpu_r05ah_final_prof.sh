# Round 5 final kernel profiles: the driver-argument fp32 bench step (5 steps) and the fp32 AttnLRP (64 windows, 3
# passes) under rocprofv3 --kernel-trace --stats; summaries for profiles/history/r05/final_prof/.  Then the LRP tests.
set -o pipefail
O=gpurun_out/${OUT:-r05ah}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_bench -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-fp32-weights --no-bf16 --no-hf-compare > $R/$O/bench_prof.log 2>&1) \
  || { echo "bench prof failed"; tail -5 $O/bench_prof.log; exit 1; }
python tools/prof_summary.py $(ls $O/prof_bench/*kernel_stats.csv $O/prof_bench/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "fp32 bench step, round 5 final (Qwen2-0.5B 2-stage split, 64-window micro-batches, nontemporal SwiGLU planes)" > $O/bench_kernel_stats.md
head -16 $O/bench_kernel_stats.md
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lrp -o run --output-format csv -- \
  python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 --iters 3 --warmup 1 > $R/$O/lrp_prof.log 2>&1) \
  || { echo "lrp prof failed"; tail -5 $O/lrp_prof.log; exit 1; }
python tools/prof_summary.py $(ls $O/prof_lrp/*kernel_stats.csv $O/prof_lrp/*/*kernel_stats.csv 2>/dev/null | head -1) \
  "fp32 AttnLRP, round 5 final, Qwen2-0.5B, 64 windows x 512" > $O/lrp_kernel_stats.md
head -16 $O/lrp_kernel_stats.md
rm -rf $O/prof_bench $O/prof_lrp
timeout -k 10 500 python -u -m pytest tests/test_lrp_gpu.py tests/test_f32_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
exit 0
