# Round 4: (1) desync as a compile-time kernel variant: bit-identity tests on the checked and production builds;
# (2) same-box bench A/B of the default path: HEAD build vs this build (fp32 + bf16);
# (3) bf16 regression bisect: bench --dtype bf16 from each round-3 tree, interleaved.
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
EDGE_KERNEL_LIB=$R/build/tuning/libedge_kernels.so timeout -k 10 300 $T tests/test_gemm_desync_gpu.py > $O/test_checked.log 2>&1 \
  || { echo "checked tests failed"; tail -30 $O/test_checked.log; exit 1; }
tail -1 $O/test_checked.log
timeout -k 10 300 $T tests/test_gemm_desync_gpu.py > $O/test_prod.log 2>&1 || { echo "prod tests failed"; tail -30 $O/test_prod.log; exit 1; }
tail -1 $O/test_prod.log
for i in 1 2; do
  for v in head new; do
    envs=""; [ $v = head ] && envs="EDGE_KERNEL_LIB=$R/build/ab_head/libedge_kernels.so"
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights --json-out $O/ab_${v}$i.json \
      > $O/ab_${v}$i.log 2>&1 || { echo "bench $v$i failed"; tail -20 $O/ab_${v}$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/ab_${v}$i.json')); print('ab $v$i', d['value'], d['value_bf16'])"
  done
done
for i in 1 2; do
  for t in 7a31976 82a69b0 b548016 81fc4b5 94ba5ac e675ad7 head; do
    d=$R/build/bisect/$t; [ $t = head ] && d=$R
    (cd $d && timeout -k 10 300 python bench.py --dtype bf16 --steps 10 --warmup 3 --no-fp32-weights \
      --json-out $R/$O/bisect_${t}_$i.json > $R/$O/bisect_${t}_$i.log 2>&1) \
      || { echo "bisect $t $i failed"; tail -20 $O/bisect_${t}_$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bisect_${t}_$i.json')); print('bisect $t $i', d['value'], d['ppl_random_weights'])"
  done
done
exit 0
