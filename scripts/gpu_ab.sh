# Same-box A/B of two kernel library builds on the fp32 bench: AB_LIB (B) against the in-tree library (A),
# interleaved A B A B A B (box-to-box variance is larger than the differences measured).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then export EDGE_KERNEL_LIB=$PWD/$AB_LIB; else unset EDGE_KERNEL_LIB; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights > gpurun_out/ab_$v$i.log 2>&1 || exit $?
    echo "$v$i $(grep '^{' gpurun_out/ab_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])')"
  done
done
exit 0
