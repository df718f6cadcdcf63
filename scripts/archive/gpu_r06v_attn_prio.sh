# fp32 attention (plane-staged, 8 waves) with the younger wave half at s_setprio 1 (EDGE_ATTN_PRIO=1) against the
# default: bench-shape probe (output bit-compared), three interleaved pairs, then the fp32 bench, two pairs.
set -o pipefail
O=gpurun_out/attn_prio
mkdir -p $O
export TMPDIR=/tmp
EDGE_ATTN_PRIO=0 timeout -k 10 120 python tools/kernel_probe.py --op attn --kv-planes 1 --iters 100 --save /tmp/ap.pt > $O/probe_0_0.log 2>&1 || exit $?
EDGE_ATTN_PRIO=1 timeout -k 10 120 python tools/kernel_probe.py --op attn --kv-planes 1 --iters 100 --compare /tmp/ap.pt > $O/probe_1_0.log 2>&1 || exit $?
for i in 1 2 3; do
  for p in 0 1; do
    EDGE_ATTN_PRIO=$p timeout -k 10 120 python tools/kernel_probe.py --op attn --kv-planes 1 --iters 100 > $O/probe_${p}_$i.log 2>&1 || exit $?
  done
done
for f in $O/probe_*.log; do echo "$f $(grep -h '^{' $f | tr '\n' ' ')"; done
B="--steps 10 --warmup 3 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep"
for i in 1 2; do
  for p in 0 1; do
    EDGE_ATTN_PRIO=$p timeout -k 10 200 python bench.py $B > $O/bench_${p}_$i.log 2>&1 || exit $?
    echo "prio=$p #$i $(grep '^{' $O/bench_${p}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])')"
  done
done
exit 0
