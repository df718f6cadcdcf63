# Round-4 baseline on this round's box: bench (fp32 + bf16) twice, kernel stats of one fp32 run, then the PMC passes
# left pending at the end of round 3 (scripts/gpu_pmc_r03s.sh).
set -o pipefail
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights --json-out gpurun_out/r04a/bench$i.json \
    > gpurun_out/r04a/bench$i.log 2>&1 || { tail -20 gpurun_out/r04a/bench$i.log; exit 1; }
  tail -1 gpurun_out/r04a/bench$i.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04a/prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-bf16 --no-fp32-weights > $R/gpurun_out/r04a/prof.log 2>&1 \
  || { tail -20 $R/gpurun_out/r04a/prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls gpurun_out/r04a/prof/*kernel_stats.csv gpurun_out/r04a/prof/*/*kernel_stats.csv 2>/dev/null | head -1) "r04a fp32 bench kernels" > gpurun_out/r04a/kernel_stats.md 2>&1 || true
head -30 gpurun_out/r04a/kernel_stats.md
bash scripts/gpu_pmc_r03s.sh
