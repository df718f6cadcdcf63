# The fp32 bench with the spread-DMA ring per GEMM family (EDGE_GEMM_RING = 0 none, 1 all paired-B GEMMs, 2 the
# 256x224 O-projection / down tiles, 3 all but the QKV), interleaved three times on one box.
set -o pipefail
O=gpurun_out/ring_modes
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for r in 0 1 2 3; do
    EDGE_GEMM_RING=$r timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights \
      --no-hf-compare --no-sweep > $O/bench_r${r}_$i.log 2>&1 || exit $?
    echo "ring=$r #$i $(grep '^{' $O/bench_r${r}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])')"
  done
done
exit 0
