# Round 6: (1) instrumented repeat of the 4-rank pp4 rehearsal (per-window NLL bit-compare + checked transport);
# (2) rocprof kernel trace proving EDGE_POISON=2 launches the LDS/register poisoner before every kernel;
# (3) the new N>1 transports record on 2 ranks sharing the GPU (RCCL must be an error entry, not a crash).
set -o pipefail
O=gpurun_out/${OUT:-r06c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python tools/rehearsal_stress.py --runs 8 --out $O/stress > $O/stress.log 2>&1 || { echo "stress rc=$?"; tail -20 $O/stress.log; exit 1; }
tail -9 $O/stress.log
cd /tmp && EDGE_POISON=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/poison_prof -o p -- python3 -c "import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT'); import __graft_entry__ as g; g.smoke()" > $GRAFT_REPO_ROOT/$O/poison_prof.log 2>&1 || { echo "poison prof failed"; tail -20 $GRAFT_REPO_ROOT/$O/poison_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/poison_prof -name "*kernel_stats.csv" | head -1); echo "stats: $f"; head -12 "$f" | cut -c1-160
EDGE_SHARED_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --model tiny-qwen2 --batch 4 --microbatches 2 --steps 3 --warmup 1 --max-length 256 --split 1 --gpus 2 --no-bf16 --no-fp32-weights --deep-pp-timeout 120 --json-out $O/transports2.json > $O/transports2.log 2>&1 || { echo "transports rc=$?"; tail -30 $O/transports2.log; exit 1; }
python -c "import json; d=json.load(open('$O/transports2.json')); print(json.dumps(d['transports'])[:2500])"
exit 0
