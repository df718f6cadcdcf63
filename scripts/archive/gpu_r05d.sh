# Round 5: the SwiGLU LRP rule in the dm GEMM's epilogue.  Tests of the fused kernel and the fp32
# engine, same-box A/B of the fused vs split MLP backward (kernel_probe), the fp32 AttnLRP throughput and its kernel
# profile.
set -o pipefail
O=gpurun_out/${OUT:-r05d}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_lrp_gpu.py -x -q ${TESTK:+-k "$TESTK"} --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_lrp.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_lrp.log; exit 1; }
tail -2 $O/pytest_lrp.log
for r in 1 2; do
  for op in lrpmlp_split lrpmlp; do
    timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 20 >> $O/probe.log 2>&1 || { echo "probe failed"; tail -5 $O/probe.log; exit 1; }
  done
done
cat $O/probe.log
timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $O/rel_fp32.json > $O/rel_fp32.log 2>&1 \
  || { echo "relbench failed"; tail -20 $O/rel_fp32.log; exit 1; }
python -c "import json; d=json.load(open('$O/rel_fp32.json')); print('lrp fp32', d['tokens_per_s'], d['ms_per_batch'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lrp -o run --output-format csv -- \
  python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 --iters 3 --warmup 1 > $R/$O/lrp_prof.log 2>&1 \
  || { echo "prof failed"; tail -5 $R/$O/lrp_prof.log; exit 1; }
cd $R
python tools/prof_summary.py $(ls $O/prof_lrp/*kernel_stats.csv $O/prof_lrp/*/*kernel_stats.csv 2>/dev/null | head -1) "fp32 AttnLRP, round 5 (SwiGLU rule fused into the dm GEMM), Qwen2-0.5B, 64 windows x 512" > $O/lrp_kernel_stats.md 2>/dev/null || true
head -16 $O/lrp_kernel_stats.md
exit 0
