# Round 5: same-box A/B of this tree against the round-4 tree (ab_r04/: a git worktree of e869cdf with its own build),
# interleaved: the driver-argument bench (fp32 headline + bf16 secondary) and the fp32 AttnLRP pass at 64 windows.
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
for rnd in 1 2; do
  for t in r04 r05; do
    if [ $t = r04 ]; then D=$R/ab_r04; else D=$R; fi
    (cd $D && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32-weights --no-hf-compare \
      --json-out $R/$O/bench_${t}_$rnd.json > $R/$O/bench_${t}_$rnd.log 2>&1) || { echo "bench $t failed"; tail -5 $O/bench_${t}_$rnd.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${t}_$rnd.json')); print('$t round $rnd bench fp32', d['value'], 'bf16', d.get('value_bf16'))"
  done
done
for rnd in 1 2; do
  for t in r04 r05; do
    if [ $t = r04 ]; then D=$R/ab_r04; else D=$R; fi
    (cd $D && timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $R/$O/lrp_${t}_$rnd.json \
      > $R/$O/lrp_${t}_$rnd.log 2>&1) || { echo "lrp $t failed"; tail -5 $O/lrp_${t}_$rnd.log; exit 1; }
    python -c "import json; d=json.load(open('$O/lrp_${t}_$rnd.json')); print('$t round $rnd lrp fp32', d['tokens_per_s'])"
  done
done
exit 0
