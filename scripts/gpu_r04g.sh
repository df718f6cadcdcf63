# Round 4: the bf16 regression (bisect: 81fc4b5 = explicit gc.collect() before each graph capture + collector off
# during capture).  Same-box interleaved A/B of the three graph-capture variants, fp32 + bf16, 3 rounds.
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in A B C; do
    case $v in
      A) envs="EDGE_TUNING=1" ;;                                              # collect + off (round-3 default)
      B) envs="EDGE_TUNING=1 EDGE_GRAPH_GC_COLLECT=0" ;;                      # off only
      C) envs="EDGE_TUNING=1 EDGE_GRAPH_GC_COLLECT=0 EDGE_GRAPH_GC_OFF=0" ;;  # neither (before 81fc4b5)
    esac
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32-weights --json-out $O/$v$i.json \
      > $O/$v$i.log 2>&1 || { echo "bench $v$i failed"; tail -20 $O/$v$i.log; exit 1; }
    python -c "import json; d=json.load(open('$O/$v$i.json')); print('$v$i', d['value'], d['value_bf16'])"
  done
done
exit 0
