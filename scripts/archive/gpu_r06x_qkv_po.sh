# Planes-only QKV instantiation (EPI_F32_QKV_PLANES: unused fp32 K / V^T / V paths compiled out, bias loaded once per
# tile, V^T plane rows from one base pointer): the QKV / plane / attention / full-model GPU tests, the bench-shape
# probe bit-compared against the previous build (AB_LIB), then probe and fp32 bench interleaved: A = new default,
# G = new library with EDGE_QKV_GENERIC=1 (generic instantiation), B = previous build.
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
export TMPDIR=/tmp
AB_LIB=${AB_LIB:-build/ab/lib_base.so}
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "qkv or kv_planes or attention or full_model" > $O/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EDGE_KERNEL_LIB=$PWD/$AB_LIB timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 2 --iters 5 \
  --save /tmp/qkv_base.pt > $O/probe_save.log 2>&1 || { echo "probe save failed"; tail $O/probe_save.log; exit 1; }
timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 2 --iters 5 --compare /tmp/qkv_base.pt \
  > $O/probe_compare.log 2>&1 || { echo "probe compare failed"; tail $O/probe_compare.log; exit 1; }
tail -1 $O/probe_compare.log
run_v() {   # $1 = A | G | B
  unset EDGE_KERNEL_LIB EDGE_QKV_GENERIC
  if [ $1 = B ]; then export EDGE_KERNEL_LIB=$PWD/$AB_LIB; fi
  if [ $1 = G ]; then export EDGE_QKV_GENERIC=1; fi
}
for i in 1 2 3; do
  for v in A G B; do
    run_v $v
    timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 2 --iters 50 > $O/probe_$v$i.log 2>&1 || exit 1
    echo "probe $v$i $(tail -1 $O/probe_$v$i.log)"
  done
done
for i in 1 2 3; do
  for v in A G B; do
    run_v $v
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep \
      > $O/bench_$v$i.log 2>&1 || { echo "bench $v$i failed"; tail $O/bench_$v$i.log; exit 1; }
    echo "bench $v$i $(grep '^{' $O/bench_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ppl_random_weights"])')"
  done
done
exit 0
