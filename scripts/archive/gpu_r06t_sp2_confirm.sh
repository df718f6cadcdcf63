# DMA schedules per tile width, confirmation round: EDGE_GEMM_RING (QKV / 224 / 256 digits; 0 two buffers, 1 ring,
# 2 two buffers with B spread) 010 (the default), 020, 022, 002, fp32 bench interleaved three times on one box.
set -o pipefail
O=gpurun_out/sp2_confirm
mkdir -p $O
export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep"
val() { grep '^{' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])'; }
for i in 1 2 3; do
  for c in 010 020 022 002; do
    EDGE_GEMM_RING=$c timeout -k 10 200 python bench.py $B > $O/ring${c}_$i.log 2>&1 || exit $?
    echo "ring $c #$i $(val $O/ring${c}_$i.log)"
  done
done
exit 0
