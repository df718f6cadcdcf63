# Round 6: (1) the bench step's per-window NLL bit-identity while a second process floods the
# GPU with copies + GEMMs; (2) the 4-rank pp4 rehearsal repeated with the same hog as a fifth process; (3) rocprofv3
# kernel statistics of the fp32 bench step.
set -o pipefail
O=gpurun_out/${OUT:-r06f}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u tools/contention_check.py --repeats 4 --hog-seconds 150 --out $O/contention.json \
  > $O/contention.log 2>&1 || { echo "contention rc=$?"; tail -20 $O/contention.log; exit 1; }
tail -1 $O/contention.log
timeout -k 10 500 python -u tools/rehearsal_stress.py --runs 6 --hog-seconds 200 --out $O/stress_hog \
  > $O/stress_hog.log 2>&1 || { echo "stress rc=$?"; tail -20 $O/stress_hog.log; exit 1; }
tail -1 $O/stress_hog.log | cut -c1-300
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep > $R/$O/prof.log 2>&1) || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); echo "stats: $f"
python tools/prof_summary.py "$f" "fp32 bench step, round 6" > $O/prof_summary.md && head -16 $O/prof_summary.md
exit 0
