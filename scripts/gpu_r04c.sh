# Round 4: desync kernel timings (off vs on, interleaved) + same-box bench A/B (HEAD build / desync off / desync on),
# fp32 and bf16.  (The bit-identity tests passed on the checked and production builds: gpu_r04b.sh.)
set -o pipefail
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
timeout -k 10 200 python tools/desync_bench.py --rounds 5 > gpurun_out/r04b/desync_bench.log 2>&1 \
  || { echo "desync bench failed"; tail -20 gpurun_out/r04b/desync_bench.log; exit 1; }
grep '^{' gpurun_out/r04b/desync_bench.log
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
