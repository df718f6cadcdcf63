# (archived: run from the repo root as scripts/archive/gpu_r06w_vt_quad.sh against a build of the reverted change)
# V^T planes by quad-transposed 8-byte stores in the 256x192 QKV epilogues (fp32 h3 planes + bf16 V^T): the QKV / plane
# / attention / full-model GPU tests on the new in-tree library, the bench-shape QKV probe bit-compared and timed
# against the previous build (AB_LIB), and the fp32 bench interleaved A (new) / B (previous) three times.
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
export TMPDIR=/tmp
AB_LIB=${AB_LIB:-build/ab/lib_base.so}
timeout -k 10 400 python -u -m pytest tests/test_f32_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "qkv or kv_planes or attention or full_model" > $O/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
EDGE_KERNEL_LIB=$PWD/$AB_LIB timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 5 \
  --save /tmp/qkv_base.pt > $O/probe_save.log 2>&1 || { echo "probe save failed"; tail $O/probe_save.log; exit 1; }
timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 5 --compare /tmp/qkv_base.pt \
  > $O/probe_compare.log 2>&1 || { echo "probe compare failed"; tail $O/probe_compare.log; exit 1; }
tail -2 $O/probe_compare.log
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then export EDGE_KERNEL_LIB=$PWD/$AB_LIB; else unset EDGE_KERNEL_LIB; fi
    timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 50 > $O/probe_$v$i.log 2>&1 || exit 1
    echo "probe $v$i $(tail -1 $O/probe_$v$i.log)"
  done
done
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then export EDGE_KERNEL_LIB=$PWD/$AB_LIB; else unset EDGE_KERNEL_LIB; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-fp32-weights --no-hf-compare --no-sweep \
      > $O/bench_$v$i.log 2>&1 || { echo "bench $v$i failed"; tail $O/bench_$v$i.log; exit 1; }
    echo "bench $v$i $(grep '^{' $O/bench_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("value_bf16"), d["ppl_random_weights"])')"
  done
done
exit 0
