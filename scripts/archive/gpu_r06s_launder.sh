# (1) the row-scale launder (no compiler vmcnt(0) at the SwiGLU epilogue's start) A/B: previous library
# (build_ab/libedge_kernels_prev.so) vs the in-tree one, fp32 bench, interleaved three times; (2) DMA schedules per
# tile width with the in-tree library (EDGE_GEMM_RING digits QKV / 224 / 256: 0 two buffers, 1 ring, 2 B-spread).
set -o pipefail
O=gpurun_out/launder
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_f32_gpu.py \
  -k "ring" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="--steps 10 --warmup 3 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep"
val() { grep '^{' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])'; }
for i in 1 2 3; do
  EDGE_KERNEL_LIB=$PWD/build_ab/libedge_kernels_prev.so timeout -k 10 200 python bench.py $B > $O/prev_$i.log 2>&1 || exit $?
  echo "prev #$i $(val $O/prev_$i.log)"
  timeout -k 10 200 python bench.py $B > $O/new_$i.log 2>&1 || exit $?
  echo "new  #$i $(val $O/new_$i.log)"
done
for i in 1 2; do
  for c in 010 012 212 020; do
    EDGE_GEMM_RING=$c timeout -k 10 200 python bench.py $B > $O/ring${c}_$i.log 2>&1 || exit $?
    echo "ring $c #$i $(val $O/ring${c}_$i.log)"
  done
done
exit 0
