# Round 4: x6 AttnLRP sweeps with the v_exp_f32 exponential and an unmasked fast path on off-diagonal tiles: LRP GPU
# tests, then same-box A/B against build/ab_lrp (176ae3f: IEEE expf, masking on every tile), three interleaved rounds.
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_lrp_gpu.py > $O/test_lrp.log 2>&1 || { echo "lrp tests failed"; tail -30 $O/test_lrp.log; exit 1; }
tail -1 $O/test_lrp.log
for i in 1 2 3; do
  for v in old new; do
    case $v in
      old) envs="EDGE_KERNEL_LIB=$PWD/build/ab_lrp/libedge_kernels.so" ;;
      new) envs="" ;;
    esac
    env $envs timeout -k 10 240 python tools/relevance_bench.py --dtype fp32 --batch 64 \
      --json-out $O/rel_$v$i.json > $O/rel_$v$i.log 2>&1 || { echo "relevance bench $v$i failed"; tail -20 $O/rel_$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/rel_$v$i.json')); print('$v$i', d['tokens_per_s'], d['ms_per_batch'])"
  done
done
exit 0
