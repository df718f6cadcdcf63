# Round 4: same-box A/B of the x6 AttnLRP staging: transposed images (conflict-free, build/ab_lrp = 795c7b9) vs
# row-major images + ds_read_b64_tr_b16 (build/ab_tr = d93fe95) vs that + the vectorized RoPE / GQA pack (this tree),
# three interleaved rounds at 64 windows, after the LRP GPU tests.
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for i in 1 2 3; do
  for v in img tr cur; do
    case $v in
      img) envs="EDGE_KERNEL_LIB=$PWD/build/ab_lrp/libedge_kernels.so" ;;
      tr) envs="EDGE_KERNEL_LIB=$PWD/build/ab_tr/libedge_kernels.so" ;;
      cur) envs="" ;;
    esac
    env $envs timeout -k 10 240 python tools/relevance_bench.py --dtype fp32 --batch 64 \
      --json-out $O/rel_$v$i.json > $O/rel_$v$i.log 2>&1 || { echo "relevance bench $v$i failed"; tail -20 $O/rel_$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/rel_$v$i.json')); print('$v$i', d['tokens_per_s'], d['ms_per_batch'])"
  done
done
exit 0
