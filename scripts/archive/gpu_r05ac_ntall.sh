# Round 5: nontemporal stores on the bench's other large outputs too (the residual GEMMs' fp32 rows, the QKV
# epilogue's q / k, the attention's O planes, the RMSNorm planes; each 117 MB, small enough for the Infinity Cache):
# probe build NTALL (scratch copies, macro not committed) against this tree, end-to-end bench, interleaved twice.
set -o pipefail
O=gpurun_out/${OUT:-r05ac}
mkdir -p $O
for r in 1 2; do
  for v in new NTALL; do
    if [ $v = new ]; then L=""; else L=$PWD/build/probe/libedge_kernels_NTALL.so; fi
    EDGE_KERNEL_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32-weights --no-hf-compare \
      --json-out $O/bench_${v}_$r.json > $O/bench_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -5 $O/bench_${v}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v bench', d['value'], d.get('value_bf16'))"
  done
done
exit 0
