# Round 6: same-box kernel profiles of the fp32 bench step with the separate RMSNorm-2 pass (default) and with it fused
# into the O-projection epilogue (EDGE_FUSED_NORM_F32=1): where the fused step's extra time goes.
set -o pipefail
O=gpurun_out/${OUT:-r06i}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
for f in 0 1; do
  (cd /tmp && EDGE_FUSED_NORM_F32=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_f$f -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep > $R/$O/prof_f$f.log 2>&1) || { echo "prof $f failed"; tail -5 $O/prof_f$f.log; exit 1; }
done
python tools/step_breakdown.py $O/prof_f0/run_kernel_trace.csv $O/prof_f1/run_kernel_trace.csv > $O/pair.md && cat $O/pair.md
exit 0
