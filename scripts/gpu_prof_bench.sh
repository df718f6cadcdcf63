set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
for cfg in "--batch 64 --microbatches 2" "--batch 32 --microbatches 4" "--batch 128 --microbatches 1"; do
timeout -k 10 300 python bench.py --steps 10 --warmup 3 $cfg > gpurun_out/bq.log 2>&1; rc=$?; echo "[$cfg] rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bq.log)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo "[prof] rc=$?"
