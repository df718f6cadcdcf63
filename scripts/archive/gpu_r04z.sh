# Round 4: bf16 AttnLRP delta kernel with 8 lanes per row (coalesced rows, shuffle reduction): LRP GPU tests, then
# same-box A/B at 64 windows (bf16 engine) against build/ab_lrpb (the previous commit), three rounds.
set -o pipefail
O=gpurun_out/r04z
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
exit 0
