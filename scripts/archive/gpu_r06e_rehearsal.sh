# Round 6: the shared-GPU rehearsal tests one by one (-v, durations), then the instrumented 4-rank pp4 repeat
# (per-window NLL bit-compare + checked transport), then the driver-argument bench.  A heartbeat line every 30 s
# keeps a long multi-process test from reading as silence.
set -o pipefail
O=gpurun_out/${OUT:-r06e}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 30; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_rehearsal_gpu.py -v --durations=0 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/rehearsal.log 2>&1 || { echo "rehearsal rc=$?"; tail -40 $O/rehearsal.log; exit 1; }
grep -E "PASSED|FAILED|ERROR|s call" $O/rehearsal.log
timeout -k 10 600 python -u tools/rehearsal_stress.py --runs ${RUNS:-6} --out $O/stress > $O/stress.log 2>&1 \
  || { echo "stress rc=$?"; tail -20 $O/stress.log; exit 1; }
tail -8 $O/stress.log | cut -c1-400
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['value_bf16'], d['value_fp32_weights'], d.get('vs_same_node_reference_batch1'), 'sweep', d.get('sweep_windows_per_s'), d.get('sweep_speedup_vs_t4'))"
exit 0
