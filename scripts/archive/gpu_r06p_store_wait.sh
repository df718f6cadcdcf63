# The four-wave GEMMs with a full tile's last epilogue stores left in flight across the next tile's first wait
# (EDGE_GEMM_STORE_WAIT=1, GemmArgs::store_wait) against the draining wait, on one box: the bit-identity tests (ring
# and store-wait knobs), the bench-shape GEMMs (QKV, gate/up, down; outputs compared bit for bit) and the fp32 bench,
# interleaved 0 1 0 1 (0 1 0 1 0 1 for the bench).
set -o pipefail
mkdir -p gpurun_out/store_wait
export TMPDIR=/tmp
O=gpurun_out/store_wait
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_f32_gpu.py \
  -k "ring" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for op in qkv gateup down; do
  EDGE_GEMM_STORE_WAIT=0 timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 50 --save /tmp/sw_$op.pt \
    > $O/probe_${op}_0a.log 2>&1 || exit $?
  EDGE_GEMM_STORE_WAIT=1 timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 50 --compare /tmp/sw_$op.pt \
    > $O/probe_${op}_1a.log 2>&1 || exit $?
  EDGE_GEMM_STORE_WAIT=0 timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 50 > $O/probe_${op}_0b.log 2>&1 || exit $?
  EDGE_GEMM_STORE_WAIT=1 timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 50 > $O/probe_${op}_1b.log 2>&1 || exit $?
  for f in $O/probe_${op}_*.log; do echo "$f $(tail -2 $f | tr '\n' ' ')"; done
done
for i in 1 2 3; do
  for r in 0 1; do
    EDGE_GEMM_STORE_WAIT=$r timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights \
      > $O/bench_r${r}_$i.log 2>&1 || exit $?
    echo "store_wait=$r #$i $(grep '^{' $O/bench_r${r}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])')"
  done
done
exit 0
