# Round 4: GEMM epilogue desync re-landed (hazard-padded park / restore, persistent per-device workspace).
#  1. bit-identity tests on the CHECKED tuning build (device-side bounds checks of every segment / park area)
#  2. the same tests on the production build
#  3. kernel timings, desync off vs on, interleaved in one process
#  4. same-box bench A/B (fp32 and bf16): HEAD build vs this build (desync off) vs this build (desync on)
set -o pipefail
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
EDGE_KERNEL_LIB=$PWD/build/tuning/libedge_kernels.so timeout -k 10 300 $T tests/test_gemm_desync_gpu.py \
  > gpurun_out/r04b/test_checked.log 2>&1 || { echo "checked tests failed"; tail -30 gpurun_out/r04b/test_checked.log; exit 1; }
tail -2 gpurun_out/r04b/test_checked.log
timeout -k 10 300 $T tests/test_gemm_desync_gpu.py > gpurun_out/r04b/test_prod.log 2>&1 \
  || { echo "prod tests failed"; tail -30 gpurun_out/r04b/test_prod.log; exit 1; }
tail -2 gpurun_out/r04b/test_prod.log
timeout -k 10 200 python tools/desync_bench.py --rounds 5 > gpurun_out/r04b/desync_bench.log 2>&1 \
  || { echo "desync bench failed"; tail -20 gpurun_out/r04b/desync_bench.log; exit 1; }
cat gpurun_out/r04b/desync_bench.log
for i in 1 2; do
  for v in head off on; do
    case $v in
      head) envs="EDGE_KERNEL_LIB=$PWD/build/ab_head/libedge_kernels.so" ;;
      off) envs="" ;;
      on) envs="EDGE_TUNING=1 EDGE_GEMM_SPLIT=-1" ;;
    esac
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights \
      --json-out gpurun_out/r04b/bench_${v}$i.json > gpurun_out/r04b/bench_${v}$i.log 2>&1 \
      || { echo "bench $v$i failed"; tail -20 gpurun_out/r04b/bench_${v}$i.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r04b/bench_${v}$i.json')); print('$v$i', d['value'], d['value_bf16'], d['ppl_random_weights'], d['ppl_random_weights_bf16'])"
  done
done
exit 0
