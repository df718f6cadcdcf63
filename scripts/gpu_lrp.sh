# LRP kernels: GPU tests, relevance bench, kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_lrp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_lrp.log 2>&1
rc=$?; echo "[pytest_lrp] rc=$rc"; tail -4 gpurun_out/pytest_lrp.log; [ $rc -eq 0 ] || exit $rc
for b in 16 64; do
timeout -k 10 300 python tools/relevance_bench.py --batch $b --json-out gpurun_out/relevance_bench_b$b.json > gpurun_out/relevance_bench.log 2>&1
rc=$?; echo "[relevance_bench b$b] rc=$rc"; tail -1 gpurun_out/relevance_bench.log; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_lrp -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/relevance_bench.py --batch 64 --iters 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_lrp.log 2>&1
echo "[prof_lrp] rc=$?"
