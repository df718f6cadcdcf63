# Round 4: bf16 AttnLRP forward with one gate|up GEMM for the SwiGLU activation and the saved pre-activations
# (edge_gemm_swiglu_raw): GPU tests, then same-box A/B against the separate GEMM + SwiGLU pass
# (EDGE_TUNING=1 EDGE_LRP_FUSED_SWIGLU=0), three interleaved rounds.
set -o pipefail
O=gpurun_out/r04z4
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "swiglu" > $O/test_swiglu.log 2>&1 || { echo "swiglu tests failed"; tail -30 $O/test_swiglu.log; exit 1; }
tail -1 $O/test_swiglu.log
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for i in 1 2 3; do
  for v in 0 1; do
    EDGE_TUNING=1 EDGE_LRP_FUSED_SWIGLU=$v timeout -k 10 240 python tools/relevance_bench.py --dtype bf16 --batch 64 \
      --json-out $O/rel_fs$v$i.json > $O/rel_fs$v$i.log 2>&1 || { echo "bench $v $i failed"; tail -20 $O/rel_fs$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/rel_fs$v$i.json')); print('fused_swiglu=$v $i', d['tokens_per_s'], d['ms_per_batch'])"
  done
done
exit 0
