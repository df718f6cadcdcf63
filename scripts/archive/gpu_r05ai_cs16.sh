# Round 5: the column-scaled GEMM epilogue's dy planes as 16-byte stores (column groups exchanged between lanes;
# build/probe/libedge_kernels_cs16.so, the change not yet in the tree) against this tree: the planes test and the
# LRP tests on the probe build, then the fp32 AttnLRP interleaved.
set -o pipefail
O=gpurun_out/${OUT:-r05ai}
mkdir -p $O
CS=$PWD/build/probe/libedge_kernels_cs16.so
EDGE_KERNEL_LIB=$CS timeout -k 10 500 python -u -m pytest tests/test_f32_gpu.py -k "colscale" tests/test_lrp_gpu.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/pytest_cs16.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_cs16.log; exit 1; }
tail -1 $O/pytest_cs16.log
for r in 1 2; do
  for v in cur cs16; do
    if [ $v = cur ]; then L=""; else L=$CS; fi
    EDGE_KERNEL_LIB=$L timeout -k 10 300 python tools/relevance_bench.py --dtype fp32 --batch 64 --json-out $O/lrp_${v}_$r.json > $O/lrp_${v}_$r.log 2>&1 || { tail -5 $O/lrp_${v}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/lrp_${v}_$r.json')); print('$v lrp fp32', d['tokens_per_s'])"
  done
done
exit 0
