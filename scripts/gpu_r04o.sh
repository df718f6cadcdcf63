# Round 4: x6 AttnLRP attention backward, double-buffered staging (one barrier per tile, EDGE_LRP_ATTN_X6=2) vs
# single-buffered (1): tests, interleaved throughput at 64 windows.
set -o pipefail
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_f32_gpu.py -k "swiglu_raw or colscale or rmsnorm" > $O/test_raw.log 2>&1 || { echo "swiglu raw tests failed"; tail -30 $O/test_raw.log; exit 1; }
tail -1 $O/test_raw.log
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for x in 1 2 1 2; do
  EDGE_TUNING=1 EDGE_LRP_ATTN_X6=$x timeout -k 10 240 python tools/relevance_bench.py --dtype fp32 --batch 64 \
    --json-out $O/relevance_fp32_b64_x6$x.json > $O/relevance_fp32_b64_x6$x.log 2>&1 \
    || { echo "relevance bench failed"; tail -20 $O/relevance_fp32_b64_x6$x.log; exit 1; }
  python -c "import json; d=json.load(open('$O/relevance_fp32_b64_x6$x.json')); print('x6=$x', d['tokens_per_s'], d['ms_per_batch'])"
done

exit 0
