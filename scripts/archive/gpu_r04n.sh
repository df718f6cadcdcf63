# Round 4: bf16 AttnLRP attention backward staged like the fp32 x6 kernels (swizzled row-major tiles, transposed
# operands by ds_read_b64_tr_b16, tile-ahead prefetch): LRP GPU tests, then same-box A/B at 64 windows (bf16 engine)
# against build/ab_lrpb (the padded-row + transposed-copy staging), three interleaved rounds.  Then the fp32 bench
# at the same global batch (256 windows) with 64 / 128 / 256-window micro-batches, two interleaved rounds.
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for i in 1 2 3; do
  for v in old new; do
    case $v in
      old) envs="EDGE_KERNEL_LIB=$PWD/build/ab_lrpb/libedge_kernels.so" ;;
      new) envs="" ;;
    esac
    env $envs timeout -k 10 240 python tools/relevance_bench.py --dtype bf16 --batch 64 \
      --json-out $O/rel_$v$i.json > $O/rel_$v$i.log 2>&1 || { echo "relevance bench $v$i failed"; tail -20 $O/rel_$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/rel_$v$i.json')); print('$v$i', d['tokens_per_s'], d['ms_per_batch'])"
  done
done
for i in 1 2; do
  for mb in 64 128 256; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights --no-bf16 --batch $mb \
      --microbatches $((256 / mb)) --json-out $O/bench_b${mb}_$i.json > $O/bench_b${mb}_$i.log 2>&1 \
      || { echo "bench b$mb $i failed"; tail -20 $O/bench_b${mb}_$i.log; exit 1; }
    tail -1 $O/bench_b${mb}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('b$mb $i', d['value'], d['ms_per_step'])"
  done
done
exit 0
