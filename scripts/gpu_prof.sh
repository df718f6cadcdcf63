# rocprofv3 kernel-trace + stats of the N=1 bench (summary -> profiles/ by tools/prof_summary.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; rc=$?
echo "[prof] rc=$rc"; grep -o '"value": [0-9.]*' $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit $rc
