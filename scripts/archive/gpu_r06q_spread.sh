# The three-slot A ring with the DMA SPREAD over both K-halves (EDGE_GEMM_RING=1: M(u,0) stages K-tile u+2's A pieces,
# M(u,1) its B pieces) against the two-buffer kernels, and the QKV GEMM's tile walk (EDGE_GEMM_WALK=0 strided /
# 1 XCD-chunked, its default), on one box: bit-identity tests, bench-shape probes (outputs compared bit for bit),
# fp32 bench, interleaved.
set -o pipefail
O=gpurun_out/spread
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_f32_gpu.py \
  -k "ring" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
probe() {  # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 120 python tools/kernel_probe.py $PARGS > $O/probe_$tag.log 2>&1 || return $?
  echo "$tag $(grep -h '^{' $O/probe_$tag.log | tr '\n' ' ')"
}
for op in qkv gateup down; do
  PARGS="--op $op --iters 50 --save /tmp/sp_$op.pt" probe ${op}_r0a EDGE_GEMM_RING=0 || exit $?
  PARGS="--op $op --iters 50 --compare /tmp/sp_$op.pt" probe ${op}_r1a EDGE_GEMM_RING=1 || exit $?
  PARGS="--op $op --iters 50" probe ${op}_r0b EDGE_GEMM_RING=0 || exit $?
  PARGS="--op $op --iters 50" probe ${op}_r1b EDGE_GEMM_RING=1 || exit $?
done
for i in a b; do
  PARGS="--op qkv --iters 50" probe qkv_walk0$i EDGE_GEMM_WALK=0 || exit $?
  PARGS="--op qkv --iters 50" probe qkv_walk1$i EDGE_GEMM_WALK=1 || exit $?
done
for i in 1 2 3; do
  for r in 0 1; do
    EDGE_GEMM_RING=$r timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights \
      > $O/bench_r${r}_$i.log 2>&1 || exit $?
    echo "ring=$r #$i $(grep '^{' $O/bench_r${r}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])')"
  done
done
exit 0
