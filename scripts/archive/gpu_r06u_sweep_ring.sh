# The notebook sweep (tools/sweep_bench.py: 256 windows, fp32) under the paired-B GEMM DMA schedules
# EDGE_GEMM_RING 000 / 010 / 022, interleaved twice on one box (the bench's single 64-window sweep timing moved
# 0.955 -> 1.139 s between two boxes).
set -o pipefail
O=gpurun_out/sweep_ring
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for c in 000 010 022; do
    EDGE_GEMM_RING=$c timeout -k 10 200 python tools/sweep_bench.py --windows 256 --json-out $O/sweep_${c}_$i.json > $O/sweep_${c}_$i.log 2>&1 || exit $?
    echo "ring $c #$i $(python -c "import json; d=json.load(open('$O/sweep_${c}_$i.json')); print({k: v for k, v in d.items() if 'per' in k or 'second' in k or k == 'windows'})")"
  done
done
exit 0
