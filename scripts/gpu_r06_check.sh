# Round 6 end-to-end check: smoke(), the whole GPU suite in one process, the driver-argument bench (with the N = 1
# notebook-sweep timing), and a rocprofv3 kernel profile of a short bench under profiles-ready CSV.
set -o pipefail
O=gpurun_out/${OUT:-r06_check}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 180 python -c "import time, __graft_entry__ as g; t=time.time(); g.smoke(); print('smoke s', round(time.time()-t, 1))" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
grep -E "smoke" $O/smoke.log
if [ "${SUITE:-1}" = 1 ]; then
( while sleep 30; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit 1; }
grep -cE " PASSED" $O/pytest_gpu.log; tail -18 $O/pytest_gpu.log
fi
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $O/bench.json > $O/bench.log 2>&1 \
  || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['value_bf16'], d['value_fp32_weights'], d.get('vs_same_node_reference_batch1'), 'sweep', d.get('sweep_windows_per_s'), d.get('sweep_speedup_vs_t4'), d['notebook_sweep'].get('wall_s_incl_build'))"
if [ "${PROF:-1}" = 1 ]; then
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep > $R/$O/prof.log 2>&1) || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); echo "stats: $f"; head -12 "$f" | cut -c1-150
fi
exit 0
